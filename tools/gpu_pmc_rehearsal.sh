#!/bin/bash
# HBM traffic (rocprofv3 PMC, FETCH_SIZE and WRITE_SIZE in separate passes) of the N>1 allreduce
# kernels in an N-rank rehearsal on the box's one GPU (N=2 by default; N=8 is the driver's np).  Each rank is its own process started
# directly (no launcher under rocprofv3); rank 0 runs under the profiler.  The samples attribute
# each of rank 0's dispatches its own traffic (measured: k_fold 1.00005x and k_pipe_allreduce
# 1.0000x of ONE rank's algorithmic bytes, profiles/r02_pmc_rehearsal_n2.json), which is what the
# rehearsal line's roofline.alg_bytes_per_launch counts.  Then the
# ordinary torchrun rehearsal of `bench.py --gpus 2`, which picks the summary up as
# roofline.traffic.  Every GPU step has a time limit; the first failure ends the script.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
N=${N:-2}
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1 WORLD_SIZE=$N MI355X_TIMEOUT_S=60
O=gpurun_out
mkdir -p $O
ARGS="--gpus $N --steps ${STEPS:-10} --warmup 3 --no-legs --no-cpu-baseline"
port=29611
for c in FETCH_SIZE WRITE_SIZE; do
  port=$((port + 1))
  echo "== pmc $c (n=$N)"
  pids=()
  for r in $(seq 1 $((N - 1))); do
    MASTER_PORT=$port RANK=$r LOCAL_RANK=$r timeout -k 10 400 python bench.py $ARGS > $O/pmc_reh_n${N}_r${r}_$c.log 2>&1 &
    pids+=($!)
  done
  MASTER_PORT=$port RANK=0 LOCAL_RANK=0 timeout -k 10 400 rocprofv3 --pmc $c -d $O/pmc_reh_n${N}_$c -o run \
    --output-format csv -- python bench.py $ARGS > $O/pmc_reh_n${N}_r0_$c.log 2>&1
  rc0=$?
  rcs=0
  for p in "${pids[@]}"; do wait $p || rcs=1; done
  echo "rank0 rc=$rc0 others rc=$rcs"
  tail -c 600 $O/pmc_reh_n${N}_r0_$c.log
  [ $rc0 -eq 0 ] && [ $rcs -eq 0 ] || exit 1
done
python tools/pmc_summary.py $O/pmc_reh_n${N}_FETCH_SIZE $O/pmc_reh_n${N}_WRITE_SIZE $O/r02_pmc_rehearsal_n$N.json \
  "k_pipe_allreduce=k_pipe_allreduce_rehearsal_n$N" "k_fold=k_fold_rehearsal_n$N" || exit 1
cp $O/r02_pmc_rehearsal_n$N.json profiles/r02_pmc_rehearsal_n$N.json
[ "${BENCH:-1}" = "1" ] || exit 0
unset MASTER_ADDR WORLD_SIZE
echo "== bench N=$N rehearsal"
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
  --master-port 29641 bench.py --gpus $N --steps 10 --warmup 3 > $O/bench_n$N.json 2> $O/bench_n$N.err || { tail -30 $O/bench_n$N.err; exit 1; }
tail -c 2500 $O/bench_n$N.json
