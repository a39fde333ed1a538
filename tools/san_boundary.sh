#!/bin/bash
# The boundary tests (tests/test_boundary.py: C-ABI exports, component headers and ABI offsets, op
# selection and host routing, coll comm_query, the harness's host channel, PML hook, MCA
# variables) and the engine host-code tests (datatype compiler, rules parser, schedule compiler)
# and the admission-token holder protocol (tests/test_tokens.py, real processes killed mid-hold),
# with every host-side library built under AddressSanitizer + UBSan
# (ompi-release_amd/csrc/Makefile.san -> ompi-release_amd/lib_san), run by a Python linked against
# the sanitizer runtime (tests/c/san_python.c).  CPU only: device code is not instrumented and no
# GPU is touched.  A sanitizer report fails the run (halt_on_error).
set -euo pipefail
cd "$(dirname "$0")/.."
make -s -C ompi-release_amd/csrc -f Makefile.san -j8
make -s -C tests/c build/san_python
export MI355X_LIB_DIR="$PWD/ompi-release_amd/lib_san"
# leaks: the interpreter and torch keep their allocations until exit by design
export ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:abort_on_error=0:exitcode=99"
export UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1:exitcode=98"
exec tests/c/build/san_python -m pytest tests/test_boundary.py tests/test_ddt_host.py tests/test_rules.py \
    tests/test_sched.py tests/test_oracle_ddt.py tests/test_tokens.py -q -x -p no:cacheprovider "$@"
