#!/bin/bash
# Selected GPU tests (TESTS="file::name ..."), bounded; output in gpurun_out/pytest_sel.log.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 ${TMO:-900} python -u -m pytest ${TESTS} -m gpu -x -v --timeout ${PER:-300} --timeout-method thread \
    > gpurun_out/pytest_sel.log 2>&1
rc=$?
tail -40 gpurun_out/pytest_sel.log
exit $rc
