#!/bin/bash
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TESTS="tests/test_coll_ipc_gpu.py::test_done_words" bash tools/gpu_tests.sh || exit 1
echo "== C caller"
MI355X_LAT_PROFILE=1 timeout -k 10 120 ./tools/build/small_ar_c 2 3000 > gpurun_out/small_c.jsonl 2> gpurun_out/small_c.err || { cat gpurun_out/small_c.err; exit 1; }
cat gpurun_out/small_c.jsonl gpurun_out/small_c.err
echo "== python caller"
PROF=0 PORT=29711 ARGS="--reps 1000" bash tools/gpu_small_prof.sh
