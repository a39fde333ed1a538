#!/bin/bash
# small allreduce latency from C (no Python), with the engine's step clock, done words off / on
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for dw in 0 1; do
  echo "== C caller, MI355X_DONE_WORDS=$dw"
  MI355X_DONE_WORDS=$dw MI355X_LAT_PROFILE=1 timeout -k 10 120 ./tools/build/small_ar_c 2 2000 || exit 1
done
