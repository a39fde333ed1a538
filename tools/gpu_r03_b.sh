#!/bin/bash
# round-3 batch: concurrency + tuned-variable tests, then the unpack ceiling probe
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TESTS="tests/test_coll_ipc_gpu.py::test_concurrent_communicators tests/test_components_gpu.py::test_tuned_variables_through_mca_var_system" \
  bash tools/gpu_tests.sh || exit 1
echo "== unpack ceiling"
timeout -k 10 300 ./tools/build/unpack_ceiling 20 > gpurun_out/unpack_ceiling.jsonl 2> gpurun_out/unpack_ceiling.err || { cat gpurun_out/unpack_ceiling.err; exit 1; }
cat gpurun_out/unpack_ceiling.jsonl
