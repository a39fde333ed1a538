#!/bin/bash
# Run one tests/coll_worker.py mode as N plain processes (no pytest) with each rank's output in
# gpurun_out/w<rank>.log -- for watching a multi-process GPU test rank by rank.
#   bash tools/run_worker.sh MODE [N] [SECONDS]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
MODE=${1:?mode}; N=${2:-2}; T=${3:-150}
mkdir -p gpurun_out
K=w$RANDOM$RANDOM
for ((r = 0; r < N; r++)); do
  OMPI_COMM_WORLD_SIZE=$N OMPI_COMM_WORLD_LOCAL_SIZE=$N OMPI_COMM_WORLD_RANK=$r OMPI_COMM_WORLD_LOCAL_RANK=$r \
  MI355X_TIMEOUT_S=60 timeout -k 5 $T python -u tests/coll_worker.py $r $N $K $MODE > gpurun_out/w$r.log 2>&1 &
done
rc=0
for job in $(jobs -p); do wait $job || rc=1; done
for ((r = 0; r < N; r++)); do tail -n 3 gpurun_out/w$r.log; done
exit $rc
