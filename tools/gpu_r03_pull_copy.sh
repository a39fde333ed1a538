#!/bin/bash
# allgather / bcast 32-128 KiB: the resident service's pull-copy form vs the host-synchronised
# pull (MI355X_SVC_PULL_MAX_BYTES=0), np = 2 and 4 on one GPU (C caller)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export SMALL_SIZES=16384,65536,131072,262144
for coll in allgather bcast; do
  for n in 2 4; do
    for pm in 0 131072; do
      SMALL_COLL=$coll MI355X_SVC_PULL_MAX_BYTES=$pm timeout -k 10 100 ./tools/build/small_ar_c $n 1000 host | \
        grep us_per_call | sed "s/^{/{\"svc_pull_max\": $pm, /" || exit 1
    done
  done
done
