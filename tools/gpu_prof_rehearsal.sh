#!/bin/bash
# Kernel trace (rocprofv3 --kernel-trace --stats) of rank 0 of an N-rank allreduce rehearsal on the
# box's one GPU, every rank on the engine's default flow (--no-autotune), so the profiled kernel's
# average duration can be set against the line's roofline.kernel_avg_ms (HIP events on the same
# launches).  Ranks are started directly (no launcher under the profiler).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
N=${N:-8}
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1 WORLD_SIZE=$N MASTER_PORT=${PORT:-29691}
O=gpurun_out
mkdir -p $O
ARGS="--gpus $N --steps ${STEPS:-20} --warmup 3 --no-legs --no-cpu-baseline --no-autotune"
pids=()
for r in $(seq 1 $((N - 1))); do
  RANK=$r LOCAL_RANK=$r timeout -k 10 400 python bench.py $ARGS > $O/prof_n${N}_r$r.log 2>&1 &
  pids+=($!)
done
RANK=0 LOCAL_RANK=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_n$N -o run --output-format csv -- \
  python bench.py $ARGS > $O/prof_n${N}_r0.log 2>&1
rc0=$?
rcs=0
for p in "${pids[@]}"; do wait $p || rcs=1; done
echo "rank0 rc=$rc0 others rc=$rcs"
[ $rc0 -eq 0 ] && [ $rcs -eq 0 ] || { tail -20 $O/prof_n${N}_r0.log; exit 1; }
grep '^{' $O/prof_n${N}_r0.log | tail -1 | cut -c1-1500
head -4 $O/prof_n$N/run_kernel_stats.csv | cut -c1-200
