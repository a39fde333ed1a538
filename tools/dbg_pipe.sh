#!/bin/bash
# Debug run of the multi-process worker (2 ranks) with engine traces; each rank's output in
# gpurun_out/.  Bounded: the workers' own faulthandler ends them, the outer timeout ends the rest.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MI355X_DEBUG=1 MI355X_TIMEOUT_S=${TMO:-20}
K=dbg$$
for r in 0 1; do
  timeout -k 5 ${RT:-60} python -u tests/ipc_worker.py $K $r 2 0 > gpurun_out/dbg_r$r.log 2>&1 &
done
wait
tail -n 5 gpurun_out/dbg_r0.log gpurun_out/dbg_r1.log
