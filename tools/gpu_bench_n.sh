#!/bin/bash
# N-rank bench rehearsal on one GPU (ranks share device 0), bounded; output in gpurun_out/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
N=${N:-2}
timeout -k 10 ${TMO:-500} python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
  --master-port ${PORT:-29555} bench.py --gpus $N --steps ${STEPS:-10} --warmup ${WARM:-3} ${ARGS:-} \
  > gpurun_out/bench_n$N.json 2> gpurun_out/bench_n$N.err
rc=$?
tail -n 3 gpurun_out/bench_n$N.err
tail -c 3000 gpurun_out/bench_n$N.json
exit $rc
