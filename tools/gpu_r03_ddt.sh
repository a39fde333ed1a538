#!/bin/bash
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TESTS="tests/test_ddt_gpu.py" bash tools/gpu_tests.sh || exit 1
timeout -k 10 200 ./tools/build/unpack_ceiling 20 > gpurun_out/unpack_ceiling3.jsonl 2>&1 || { cat gpurun_out/unpack_ceiling3.jsonl; exit 1; }
grep -E "TRI|engine" gpurun_out/unpack_ceiling3.jsonl
