#!/bin/bash
# allgather / bcast: LL form (svc) vs pull-copy form at small sizes, and the pull-copy form up to
# 1 MiB vs the host-synchronised flow, np = 2 and 4 on one GPU (C caller)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for coll in allgather bcast; do
  for n in 2 4; do
    SMALL_COLL=$coll SMALL_SIZES=8,1024,4096,16384 timeout -k 10 100 ./tools/build/small_ar_c $n 1000 svc | grep us_per_call || exit 1
    SMALL_COLL=$coll SMALL_SIZES=8,1024,4096,16384,262144,524288,1048576 MI355X_SVC_PULL_MAX_BYTES=1048576 \
      timeout -k 10 100 ./tools/build/small_ar_c $n 1000 host | grep us_per_call | sed 's/"host"/"pull_or_host"/' || exit 1
    SMALL_COLL=$coll SMALL_SIZES=262144,524288,1048576 MI355X_SVC_PULL_MAX_BYTES=0 \
      timeout -k 10 100 ./tools/build/small_ar_c $n 1000 host | grep us_per_call || exit 1
  done
done
