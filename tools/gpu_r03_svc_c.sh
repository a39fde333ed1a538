#!/bin/bash
# resident-service tests, then small-message allreduce latency from C (no Python in the loop):
# host-synchronised path vs per-call LL kernels vs the resident LL service, np = 2 and 4 on one GPU,
# and the service's stage trace at 8 B and 64 KiB
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 400 python -u -m pytest tests/test_coll_ipc_gpu.py -k "resident_service or ipc_ranks" -x -v -s \
    --timeout 300 --timeout-method thread > gpurun_out/svc_tests.log 2>&1 || { tail -60 gpurun_out/svc_tests.log; exit 1; }
  grep -E "PASSED|FAILED|svc:|resident service" gpurun_out/svc_tests.log
fi
export SMALL_SIZES=${SMALL_SIZES:-8,256,1024,4096,16384,65536,262144}
for n in ${NS:-2 4}; do
  timeout -k 10 200 ./tools/build/small_ar_c $n ${REPS:-2000} ${PATHS:-host,ll,svc} || exit 1
done
for sz in 8 65536; do
  SMALL_SIZES=$sz MI355X_SVC_TRACE=1 timeout -k 10 60 ./tools/build/small_ar_c 2 2000 svc 2>&1 | grep -E "traced|us_per_call" || exit 1
done
