#!/bin/bash
# Round-2 measurement evidence on one MI355X: the N=1 headline line + its rocprofv3 kernel trace,
# the single-GPU legs (op sweep, convertor, CPU ring) + the convertor kernel trace, and a kernel
# trace of rank 0 of a 2-rank allreduce rehearsal (ranks started directly, no launcher under the
# profiler).  Every GPU step has its own limit; the first failure ends the script.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1 || { echo "FAILED $name rc=$?"; tail -40 "$O/$name.log"; exit 1; }; }
step bench 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 10
tail -1 $O/bench.log
step prof_bench 300 rocprofv3 --kernel-trace --stats -d $O/prof_bench -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline
step legs 600 python tools/bench_legs.py --legs op,ddt,cpu_ar --out $O/legs.jsonl
step prof_ddt 300 rocprofv3 --kernel-trace --stats -d $O/prof_ddt -o run --output-format csv -- python tools/bench_legs.py --legs ddt --no-cpu-baseline --out $O/legs_ddt_prof.jsonl
export MASTER_ADDR=127.0.0.1 WORLD_SIZE=2 MASTER_PORT=29677
echo "== prof_n2 (rank 0 under rocprofv3 --kernel-trace --stats)"
RANK=1 LOCAL_RANK=1 timeout -k 10 400 python bench.py --gpus 2 --steps 10 --warmup 3 --no-legs --no-cpu-baseline > $O/prof_n2_r1.log 2>&1 &
p1=$!
RANK=0 LOCAL_RANK=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_n2 -o run --output-format csv -- python bench.py --gpus 2 --steps 10 --warmup 3 --no-legs --no-cpu-baseline > $O/prof_n2_r0.log 2>&1
rc0=$?
wait $p1
rc1=$?
echo "rank0 rc=$rc0 rank1 rc=$rc1"
[ $rc0 -eq 0 ] && [ $rc1 -eq 0 ] || { tail -20 $O/prof_n2_r0.log $O/prof_n2_r1.log; exit 1; }
unset MASTER_ADDR WORLD_SIZE MASTER_PORT
step bench_n2 700 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29681 bench.py --gpus 2 --steps 10 --warmup 3
tail -c 400 $O/bench_n2.log
echo "== done"
