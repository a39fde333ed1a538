#!/bin/bash
# One GPU session for the current change set: targeted parity tests, then the single-GPU legs
# and a kernel-trace profile of the convertor leg.  Every GPU step has its own time limit and the
# first failure ends the script.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== pytest ${TESTS:-}"
timeout -k 10 900 python -m pytest ${TESTS:-tests} -m gpu -x -q > gpurun_out/pytest_round.log 2>&1 || { tail -60 gpurun_out/pytest_round.log; exit 1; }
tail -2 gpurun_out/pytest_round.log
if [ "${LEGS:-}" != "" ]; then
  echo "== legs $LEGS"
  bash tools/gpu_legs.sh || exit 1
fi
