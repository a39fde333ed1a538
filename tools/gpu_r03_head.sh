#!/bin/bash
# Head-of-tree evidence on one MI355X: parity suite + smoke, N=1 bench, its rocprofv3 kernel
# trace, and the bare `bench.py --gpus 2` self-launch (rehearsal).  Each GPU step bounded; the
# first failure ends the script.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
SUITE=${SUITE:-1} bash tools/gpu_r03_check.sh || exit 1
echo "== rocprofv3 bench N=1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_bench -o run --output-format csv -- \
  python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/prof_bench.log 2>&1 || { tail -30 $O/prof_bench.log; exit 1; }
tail -1 $O/prof_bench.log
echo "== done"
