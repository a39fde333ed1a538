#!/bin/bash
# Small-message allreduce latency at N ranks on the box's one GPU, rank 0 under rocprofv3
# --hip-trace --kernel-trace --stats (HIP API and kernel time per call); ranks started directly.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
N=${N:-2}
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1 WORLD_SIZE=$N MASTER_PORT=${PORT:-29693}
O=gpurun_out
mkdir -p $O
pids=()
for r in $(seq 1 $((N - 1))); do
  RANK=$r LOCAL_RANK=$r timeout -k 10 200 python tools/small_ar.py ${ARGS:-} > $O/small_r$r.log 2>&1 &
  pids+=($!)
done
if [ "${PROF:-1}" = "1" ]; then
  RANK=0 LOCAL_RANK=0 timeout -k 10 200 rocprofv3 --hip-trace --kernel-trace --stats -d $O/small_prof -o run \
    --output-format csv -- python tools/small_ar.py ${ARGS:-} > $O/small_r0.log 2>&1
else
  RANK=0 LOCAL_RANK=0 timeout -k 10 200 python tools/small_ar.py ${ARGS:-} > $O/small_r0.log 2>&1
fi
rc0=$?
rcs=0
for p in "${pids[@]}"; do wait $p || rcs=1; done
echo "rank0 rc=$rc0 others rc=$rcs"
grep '^{' $O/small_r0.log
[ $rc0 -eq 0 ] && [ $rcs -eq 0 ] || { tail -20 $O/small_r0.log; exit 1; }
