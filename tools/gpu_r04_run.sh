#!/bin/bash
set -uo pipefail
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
MI355X_SVC_RS=1 timeout -k 10 600 python -u -m pytest tests/test_coll_ipc_gpu.py -k "ipc_ranks or resident_service" -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04_rs_tests.log 2>&1 || { tail -60 gpurun_out/r04_rs_tests.log; exit 1; }
tail -5 gpurun_out/r04_rs_tests.log
timeout -k 10 300 bash tools/gpu_r03_pull_rs.sh > gpurun_out/r04_pull_rs.log 2>&1 || { tail -30 gpurun_out/r04_pull_rs.log; exit 1; }
cat gpurun_out/r04_pull_rs.log
