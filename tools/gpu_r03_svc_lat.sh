#!/bin/bash
# Small-message allreduce latency on one GPU: host-synchronised path vs per-call LL kernels vs the
# resident LL service, np = 2, 4 and 8 (ranks share the GPU: a rehearsal)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for n in ${NS:-2 4 8}; do
  echo "== np=$n"
  N=$n PROF=0 PORT=$((29710 + n)) ARGS="--reps ${REPS:-1000} --sizes 8,1024,16384,65536,262144,1048576 --paths host,ll,svc" \
    bash tools/gpu_small_prof.sh || exit 1
done
