#!/bin/bash
# small-message allreduce latency, completion words on vs off (MI355X_DONE_WORDS), np=2 on one GPU
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for dw in 1 0; do
  echo "== MI355X_DONE_WORDS=$dw"
  MI355X_DONE_WORDS=$dw PROF=0 PORT=$((29700 + dw)) ARGS="--reps 1000" bash tools/gpu_small_prof.sh || exit 1
done
