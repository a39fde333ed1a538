#!/bin/bash
# HIP API trace (rocprofv3 --hip-trace --kernel-trace --stats, no counters) of rank 0 of a 2-rank
# small-message probe (tools/ll_probe2.py: 8 B..64 KiB allreduce / allgather / bcast), to see where
# the host-synchronised path spends its time.  Ranks started directly.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
K=small$$
timeout -k 10 300 python tools/ll_probe2.py 1 2 $K 200 > $O/small_r1.log 2>&1 &
p1=$!
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --stats -d $O/small_trace -o run --output-format csv -- \
  python tools/ll_probe2.py 0 2 $K 200 > $O/small_r0.log 2>&1
rc0=$?
wait $p1
rc1=$?
echo "rank0 rc=$rc0 rank1 rc=$rc1"
tail -12 $O/small_r0.log
