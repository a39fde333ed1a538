#!/bin/bash
# What an extra hardware queue / a resident kernel costs HIP launch-to-completion: one process
# (queue created after HIP's queues, and before them), two processes on the GPU (the rehearsal's case)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
O=gpurun_out/r03_queue_probe.jsonl
: > $O
tag() { sed "s/^{/{\"case\": \"$1\", /" >> $O; }
timeout -k 10 60 ./tools/build/queue_probe 2000 | tag one_process || exit 1
Q_EARLY=1 timeout -k 10 60 ./tools/build/queue_probe 2000 | tag one_process_queue_first || exit 1
Q_STREAMS=8 timeout -k 10 60 ./tools/build/queue_probe 2000 | tag one_process_8_streams || exit 1
(Q_EARLY=1 timeout -k 10 60 ./tools/build/queue_probe 2000 > gpurun_out/qa.txt &
 Q_EARLY=1 timeout -k 10 60 ./tools/build/queue_probe 2000 > gpurun_out/qb.txt; wait) || exit 1
tag two_processes_queue_first_a < gpurun_out/qa.txt
tag two_processes_queue_first_b < gpurun_out/qb.txt
(Q_STREAMS=8 timeout -k 10 60 ./tools/build/queue_probe 2000 > gpurun_out/qa.txt &
 Q_STREAMS=8 timeout -k 10 60 ./tools/build/queue_probe 2000 > gpurun_out/qb.txt; wait) || exit 1
tag two_processes_8_streams_a < gpurun_out/qa.txt
tag two_processes_8_streams_b < gpurun_out/qb.txt
grep launch_sync $O
