#!/bin/bash
# the resident service's pull form (one-phase ring from the mapped inputs) against the host-
# synchronised one-phase flow, np = 2 and 4, with 8 and 16 service workgroups (C caller)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export SMALL_SIZES=65536,131072,262144,524288,1048576
for n in 2 4; do
  for wg in 8 16; do
    echo "== np=$n wgs=$wg"
    MI355X_SVC_WGS=$wg MI355X_SVC_PULL_MAX_BYTES=0 timeout -k 10 100 ./tools/build/small_ar_c $n 1000 host || exit 1
    MI355X_SVC_WGS=$wg MI355X_SVC_PULL_MAX_BYTES=1048576 timeout -k 10 100 ./tools/build/small_ar_c $n 1000 host || exit 1
  done
done
