#!/bin/bash
# Single-GPU legs (op sweep, convertor) + a kernel-trace profile of the convertor leg.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python tools/bench_legs.py --legs "${LEGS:-op,ddt}" --out gpurun_out/legs.jsonl > gpurun_out/legs.log 2>&1 || { tail -30 gpurun_out/legs.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ddt -o run --output-format csv -- python tools/bench_legs.py --legs ddt --no-cpu-baseline --out gpurun_out/legs_ddt_prof.jsonl > gpurun_out/prof_ddt.log 2>&1 || { tail -30 gpurun_out/prof_ddt.log; exit 1; }
tail -3 gpurun_out/legs.log
