#!/bin/bash
# Round-2 closing evidence on one MI355X: the GPU parity suite + smoke, the N=1 headline line and
# its rocprofv3 kernel trace, PMC traffic passes (FETCH_SIZE and WRITE_SIZE in separate runs) for
# the op kernel and the new convertor kernels, and the single-GPU legs.  Every GPU step has its own
# time limit; the first failure ends the script.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1 || { echo "FAILED $name rc=$?"; tail -40 "$O/$name.log"; exit 1; }; }
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
tail -2 $O/pytest_gpu.log
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 10
tail -1 $O/bench.log | cut -c1-300
step prof_bench 300 rocprofv3 --kernel-trace --stats -d $O/prof_bench -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline
step pmc_f 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_f -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline
step pmc_w 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_w -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline
step pmc_ddt_f 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_ddt_f -o run --output-format csv -- python tools/bench_legs.py --legs ddt_narrow,ddt_runs --steps 3 --warmup 1 --no-cpu-baseline --out $O/legs_pmc_f.jsonl
step pmc_ddt_w 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_ddt_w -o run --output-format csv -- python tools/bench_legs.py --legs ddt_narrow,ddt_runs --steps 3 --warmup 1 --no-cpu-baseline --out $O/legs_pmc_w.jsonl
python tools/pmc_summary.py $O/pmc_f $O/pmc_w $O/pmc_op.json "k_chunk<mi355x::OpSum<float>, true=op_3buff_sum_float" > /dev/null
python tools/pmc_summary.py $O/pmc_ddt_f $O/pmc_ddt_w $O/pmc_ddt.json \
  "k_ddt_rows<true, false, 3, 8, 8>=ddt_pack_rows_w8" "k_ddt_rows<false, false, 3, 8, 8>=ddt_unpack_rows_w8" \
  "k_ddt_rows<true, false, 3, 8, 4>=ddt_pack_rows_w4" "k_ddt_rows<false, false, 3, 8, 4>=ddt_unpack_rows_w4" \
  "k_ddt_units<true, false, 8>=ddt_pack_units_w8" "k_ddt_units<false, false, 8>=ddt_unpack_units_w8" \
  "k_ddt_units<true, false, 4>=ddt_pack_units_w4" "k_ddt_units<false, false, 4>=ddt_unpack_units_w4" > /dev/null
step legs 600 python tools/bench_legs.py --legs op,ddt,ddt_narrow,ddt_runs,cpu_ar --out $O/legs.jsonl
echo "== done"
