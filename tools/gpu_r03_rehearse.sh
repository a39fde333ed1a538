#!/bin/bash
# N-rank bench rehearsals on one GPU through bench.py's self-launch (no external launcher)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for N in ${NS:-2 8}; do
  echo "== bench.py --gpus $N"
  timeout -k 10 ${TMO:-420} python bench.py --gpus $N --steps ${STEPS:-10} --warmup 3 ${ARGS:-} \
      > gpurun_out/r03_bench_n$N.json 2> gpurun_out/r03_bench_n$N.err
  rc=$?
  echo "rc=$rc"
  tail -3 gpurun_out/r03_bench_n$N.err
  python - "$N" <<'PY'
import json, sys
n = sys.argv[1]
for l in open(f"gpurun_out/r03_bench_n{n}.json"):
    if l.startswith("{"):
        d = json.loads(l)
        legs = d.get("legs") or {}
        print(json.dumps({k: d.get(k) for k in ("value", "ms_per_step", "n_gpus")}), d["config"].get("data_flow"),
              d["config"].get("exact_check"), json.dumps(d["config"].get("best")))
        print("legs:", {k: (v if not isinstance(v, list) else len(v)) for k, v in legs.items() if k != "allreduce_sweep_f32"})
        for row in legs.get("allreduce_sweep_f32", []):
            print(" sweep", json.dumps(row))
PY
  [ $rc -eq 0 ] || exit $rc
done
