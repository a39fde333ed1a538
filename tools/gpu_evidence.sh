#!/bin/bash
# Round evidence on one MI355X: full GPU parity suite, headline bench + kernel trace, single-GPU
# legs + convertor kernel trace, PMC traffic passes (separate FETCH_SIZE / WRITE_SIZE runs), a
# 2-rank rehearsal of the N>1 bench, and smoke().  Each GPU step has its own time limit; the
# first failure ends the script.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1 || { echo "FAILED $name rc=$?"; tail -40 "$O/$name.log"; exit 1; }; }
step pytest_gpu 1200 python -m pytest tests -m gpu -x -q
tail -2 $O/pytest_gpu.log
step bench 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 10
tail -1 $O/bench.log
step prof_bench 300 rocprofv3 --kernel-trace --stats -d $O/prof_bench -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline
step legs 600 python tools/bench_legs.py --legs op,ddt,cpu_ar --out $O/legs.jsonl
step prof_ddt 300 rocprofv3 --kernel-trace --stats -d $O/prof_ddt -o run --output-format csv -- python tools/bench_legs.py --legs ddt --no-cpu-baseline --out $O/legs_ddt_prof.jsonl
step pmc_f 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_f -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline
step pmc_w 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_w -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline
step pmc_ddt_f 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_ddt_f -o run --output-format csv -- python tools/bench_legs.py --legs ddt --steps 5 --warmup 1 --no-cpu-baseline --out $O/legs_pmc_f.jsonl
step pmc_ddt_w 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_ddt_w -o run --output-format csv -- python tools/bench_legs.py --legs ddt --steps 5 --warmup 1 --no-cpu-baseline --out $O/legs_pmc_w.jsonl
python tools/pmc_summary.py $O/pmc_f $O/pmc_w $O/pmc_op.json "k_chunk<mi355x::OpSum<float>, true=op_3buff_sum_float" > /dev/null
python tools/pmc_summary.py $O/pmc_ddt_f $O/pmc_ddt_w $O/pmc_ddt.json "k_ddt_rows<true, false=ddt_pack_vector" "k_ddt_rows<false, false=ddt_unpack_vector" > /dev/null
step bench_n2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2
tail -1 $O/bench_n2.log
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
echo "== done"
