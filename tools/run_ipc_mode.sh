#!/bin/bash
# Run one tests/ipc_worker.py mode as N plain processes, each rank's output in gpurun_out/i<rank>.log
#   bash tools/run_ipc_mode.sh MODE [N] [SECONDS]   (extra environment passes through)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
MODE=${1:?mode}; N=${2:-2}; T=${3:-150}
mkdir -p gpurun_out
K=i$RANDOM$RANDOM
for ((r = 0; r < N; r++)); do
  MI355X_TIMEOUT_S=${MI355X_TIMEOUT_S:-60} timeout -k 5 $T python -u tests/ipc_worker.py $K $r $N 0 $MODE > gpurun_out/i$r.log 2>&1 &
done
rc=0
for job in $(jobs -p); do wait $job || rc=1; done
for ((r = 0; r < N; r++)); do tail -n 4 gpurun_out/i$r.log; done
exit $rc
