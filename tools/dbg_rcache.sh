#!/bin/bash
# Exploratory (round 6): the bounded-cache churn worker (ipc_worker.py::rcache, 3 ranks) with engine
# traces, repeated until it fails once; logs under gpurun_out/dbg/ (see profiles/r06_rcache_churn_trace_r0.txt)
# (exploratory) run the bounded-cache churn worker with engine traces until it fails once
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/dbg
for a in 1 2 3 4 5 6; do
  key="dbg$RANDOM$a"
  pids=()
  for r in 0 1 2; do
    MI355X_DEBUG=1 MI355X_TIMEOUT_S=60 RCACHE_ROUNDS=2 timeout -k 10 120 python tests/ipc_worker.py $key $r 3 0 rcache > gpurun_out/dbg/a${a}_r$r.log 2>&1 &
    pids+=($!)
  done
  fail=0
  for p in "${pids[@]}"; do wait $p || fail=1; done
  echo "attempt $a fail=$fail"
  if [ $fail = 1 ]; then break; fi
  rm -f gpurun_out/dbg/a${a}_r*.log
done
