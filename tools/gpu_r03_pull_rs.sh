#!/bin/bash
# reduce_scatter_block (MPI_FLOAT SUM, bytes per rank's block): the resident service's pull form
# (LL_PULL_RS) vs the host-synchronised flow, np = 2 and 4 on one GPU (C caller)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for n in 2 4; do
  MI355X_SVC_RS=1 SMALL_COLL=reduce_scatter_block SMALL_SIZES=8,1024,16384,65536,131072 \
    timeout -k 10 100 ./tools/build/small_ar_c $n 1000 host | grep us_per_call | sed 's/"host"/"svc_pull"/' || exit 1
  SMALL_COLL=reduce_scatter_block SMALL_SIZES=8,1024,16384,65536,131072 MI355X_SVC_PULL_MAX_BYTES=0 \
    timeout -k 10 100 ./tools/build/small_ar_c $n 1000 host | grep us_per_call || exit 1
done
