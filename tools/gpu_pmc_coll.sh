#!/bin/bash
# PMC traffic passes for the op bench kernel + a 2-rank rehearsal of the N>1 allreduce bench
# (both ranks on the box's single GPU -> exercises the IPC path; the 8-GPU run is the driver's).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== pmc FETCH_SIZE"; timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_f -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/pmc_f.log 2>&1
echo "== pmc WRITE_SIZE"; timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_w -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/pmc_w.log 2>&1
python tools/pmc_summary.py gpurun_out/pmc_f gpurun_out/pmc_w gpurun_out/r01_pmc.json "k_chunk<mi355x::OpSum<float>, true=op_3buff_sum_float"
echo "== bench N=2 rehearsal"; timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/bench_n2.log 2>&1; tail -1 gpurun_out/bench_n2.log
echo "== bench N=1"; timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 5 > gpurun_out/bench.log 2>&1; tail -1 gpurun_out/bench.log
