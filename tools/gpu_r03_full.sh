#!/bin/bash
# full GPU parity suite + smoke, then the small-message latency A/B (completion words on / off)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_suite.sh || exit 1
bash tools/gpu_r03_lat.sh
