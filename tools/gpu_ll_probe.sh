#!/bin/bash
# LL vs host latency probe (2 ranks on one GPU), plain and under rocprofv3 kernel traces (one
# profiler per rank process, no launcher in between).  Bounded; outputs in gpurun_out/.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
export TMPDIR=/tmp
mkdir -p gpurun_out
N=${N:-2}
K=llp$$
for r in $(seq 0 $((N-1))); do
  timeout -k 10 120 python tools/ll_probe2.py $r $N ${K}a 300 > gpurun_out/llprobe_plain_r$r.txt 2>&1 &
done
wait
cat gpurun_out/llprobe_plain_r0.txt | grep -v amdgpu.ids
if [ "${PROF:-1}" = "1" ]; then
  for r in $(seq 0 $((N-1))); do
    timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/llprof_r$r" -o run --output-format csv \
      -- python "$R/tools/ll_probe2.py" $r $N ${K}b 100 > gpurun_out/llprobe_prof_r$r.txt 2>&1 &
  done
  wait
  find gpurun_out/llprof_r0 -name "*kernel_stats.csv" | head -1 | xargs -r cat | cut -c1-160 | head -20
fi
