#!/bin/bash
# HBM traffic (rocprofv3 PMC, FETCH_SIZE and WRITE_SIZE in separate passes) of the N>1 allreduce
# kernels in a 2-rank rehearsal on the box's one GPU.  Each rank is its own process started
# directly (no launcher under rocprofv3); rank 0 runs under the profiler.  The samples attribute
# each of rank 0's dispatches its own traffic (measured: k_fold 1.00005x and k_pipe_allreduce
# 1.0000x of ONE rank's algorithmic bytes, profiles/r02_pmc_rehearsal.json), which is what the
# rehearsal line's roofline.alg_bytes_per_launch counts.  Then the
# ordinary torchrun rehearsal of `bench.py --gpus 2`, which picks the summary up as
# roofline.traffic.  Every GPU step has a time limit; the first failure ends the script.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1 WORLD_SIZE=2 MI355X_TIMEOUT_S=60
O=gpurun_out
mkdir -p $O
ARGS="--gpus 2 --steps ${STEPS:-10} --warmup 3 --no-legs --no-cpu-baseline"
port=29611
for c in FETCH_SIZE WRITE_SIZE; do
  port=$((port + 1))
  echo "== pmc $c"
  MASTER_PORT=$port RANK=1 LOCAL_RANK=1 timeout -k 10 400 python bench.py $ARGS > $O/pmc_reh_r1_$c.log 2>&1 &
  p1=$!
  MASTER_PORT=$port RANK=0 LOCAL_RANK=0 timeout -k 10 400 rocprofv3 --pmc $c -d $O/pmc_reh_$c -o run \
    --output-format csv -- python bench.py $ARGS > $O/pmc_reh_r0_$c.log 2>&1
  rc0=$?
  wait $p1
  rc1=$?
  echo "rank0 rc=$rc0 rank1 rc=$rc1"
  tail -c 600 $O/pmc_reh_r0_$c.log
  [ $rc0 -eq 0 ] && [ $rc1 -eq 0 ] || { tail -20 $O/pmc_reh_r1_$c.log; exit 1; }
done
python tools/pmc_summary.py $O/pmc_reh_FETCH_SIZE $O/pmc_reh_WRITE_SIZE $O/r02_pmc_rehearsal.json \
  "k_pipe_allreduce=k_pipe_allreduce_rehearsal" "k_fold=k_fold_rehearsal" || exit 1
cp $O/r02_pmc_rehearsal.json profiles/r02_pmc_rehearsal.json
echo "== bench N=2 rehearsal"
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29641 bench.py --gpus 2 --steps 10 --warmup 3 > $O/bench_n2.json 2> $O/bench_n2.err || { tail -30 $O/bench_n2.err; exit 1; }
tail -c 2500 $O/bench_n2.json
