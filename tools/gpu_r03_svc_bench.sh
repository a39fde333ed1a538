#!/bin/bash
# resident-service tests + C latency (tools/gpu_r03_svc_c.sh), then the self-launched np=2 bench
# line (its allreduce sweep carries the us_svc column)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_r03_svc_c.sh || exit 1
timeout -k 10 500 python bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/r03_bench_n2.json 2> gpurun_out/r03_bench_n2.err \
  || { tail -20 gpurun_out/r03_bench_n2.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r03_bench_n2.json").read().strip().splitlines()[-1])
print("value", d["value"], "ms_per_step", d["ms_per_step"])
for r in d["legs"]["allreduce_sweep_f32"]:
    print({k: r.get(k) for k in ("bytes", "us", "us_svc", "us_pull", "us_host", "us_ll", "us_host_2phase", "exact")})
PY
