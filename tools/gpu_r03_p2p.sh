#!/bin/bash
# Round 3: streamed host payloads (p2p fragment pipeline): the point-to-point GPU tests, then the
# two-process host -> host rates with and without the pipeline (printed by the test, -s).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest "tests/test_coll_ipc_gpu.py::test_host_p2p_between_processes" -m gpu -x -v -s \
    --timeout 200 --timeout-method thread > gpurun_out/host_p2p.log 2>&1
rc=$?
grep -E '^\{|passed|failed' gpurun_out/host_p2p.log
exit $rc
