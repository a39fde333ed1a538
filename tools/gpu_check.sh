#!/bin/bash
# One GPU session: launch-shape sweep, bench, rocprof kernel stats, then parity tests and smoke.
# Every GPU step has its own time limit; the first failure ends the script.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${SKIP_TUNE:-0}" != "1" ]; then
echo "== op_tune"; timeout -k 10 600 python tools/op_tune.py > gpurun_out/op_tune.log 2>&1; grep -E "RESULT|torch add" gpurun_out/op_tune.log
fi
echo "== bench"; timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 5 > gpurun_out/bench.log 2>&1; tail -1 gpurun_out/bench.log
echo "== rocprof"; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof.log 2>&1
echo "== pytest -m gpu"; timeout -k 10 1200 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; tail -1 gpurun_out/smoke.log
