#!/bin/bash
# Round-3 check on one GPU: the parity suite + smoke, the N=1 bench, and the bare
# `bench.py --gpus 2` self-launch (ranks share device 0: a rehearsal line).  Every step bounded;
# the first failure ends the script.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${SUITE:-1}" = "1" ]; then
  bash tools/gpu_suite.sh || exit 1
fi
echo "== bench N=1"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r03_bench_n1.json 2> gpurun_out/r03_bench_n1.err \
  || { tail -20 gpurun_out/r03_bench_n1.err; exit 1; }
cat gpurun_out/r03_bench_n1.json
echo "== bench --gpus 2 (self-launch)"
timeout -k 10 500 python bench.py --gpus 2 --steps 5 --warmup 2 ${ARGS2:-} > gpurun_out/r03_bench_n2.json 2> gpurun_out/r03_bench_n2.err
rc=$?
echo "rc=$rc"
tail -5 gpurun_out/r03_bench_n2.err
head -c 1500 gpurun_out/r03_bench_n2.json
exit $rc
