#!/bin/bash
# One parameterised GPU runner for the measurements and checks of this repo (it replaces the
# per-round tools/gpu_r0*_*.sh scripts).  Usage, on the GPU box:
#   bash tools/gpu_run.sh STEP [STEP ...]
# Every step runs under its own time limit with its output under gpurun_out/; the first failure
# ends the script (no GPU step runs after a failed, faulted or timed-out one).  Steps:
#   suite          pytest -m gpu (whole suite) + smoke()               -> pytest_gpu.log, smoke.log
#   tests          pytest -m gpu on $TESTS (node ids / files), -k "$K" -> pytest_sel.log
#   smoke          __graft_entry__.smoke()
#   bench          python bench.py (N = 1 headline line)               -> bench_n1.json
#   prof_bench     rocprofv3 --kernel-trace --stats of the N = 1 bench -> prof_bench/
#   pmc            FETCH_SIZE / WRITE_SIZE passes (separate runs) of the N = 1 bench -> pmc_op.json
#   legs           tools/bench_legs.py --legs $LEGS (default op,ddt)   -> legs.jsonl
#   prof_ddt       rocprofv3 kernel trace of the convertor legs         -> prof_ddt/
#   rehearse       bench.py --gpus N self-launch for N in $NS (default "2 8"; ranks share the GPU)
#   small          small collectives from C (tools/build/small_ar_c), np in $NS (default "2 4"),
#                  $SMALL_COLL (allreduce), $SMALL_SIZES, $PATHS (host,ll,svc), $REPS -> small.jsonl
#   svc_trace      the service's per-stage times at 8 B and 64 KiB (MI355X_SVC_TRACE=1)
#   pull           the service's pull form vs the host-synchronised one-phase flow, 64 KiB-1 MiB
#   pull_copy      allgather / bcast: the service's pull copy vs the host flow, to 1 MiB
#   pull_rs        reduce_scatter_block: the service's LL_PULL_RS form vs the host flow
#   queue_probe    what a resident kernel costs HIP launch-to-completion   -> queue_probe.jsonl
#   unpack_ceiling tools/build/unpack_ceiling (convertor unpack ceiling)   -> unpack_ceiling.jsonl
#   host_p2p       host -> host point-to-point rates between two processes -> host_p2p.log
#   op_overhead    what op/hip adds to host-buffer reductions (tools/build/op_host_overhead) -> op_overhead.jsonl
#                  and an 8 B host-buffer allreduce with / without the components (small_ar_c host_mini)
#   p2p_lat        point-to-point ping-pong latency, host and device buffers, 8 B - 64 KiB -> p2p_lat.jsonl
#   interference   the resident service beside compute streams (tools/svc_interference.py) -> svc_interference.jsonl
#   ab_host        host-synchronised small-call latency, this tree vs a build staged in ab_old/ (A/B)
#   prof_rehearsal rocprofv3 kernel trace of rank 0 of an N-rank (N=${N:-8}) allreduce rehearsal on the
#                  default flow (--no-autotune): kernel average vs the line's kernel_avg_ms -> prof_n$N/
#   pmc_rehearsal  FETCH_SIZE / WRITE_SIZE (separate passes) of rank 0 of an N-rank (N=${N:-2})
#                  rehearsal -> pmc_rehearsal_n$N.json (what bench_coll.py reads as roofline.traffic)
# (multi-rank profiles start every rank directly -- no launcher under the profiler -- with rank 0
# under rocprofv3 and the others as plain processes)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
PYT="python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread"

run() {  # run NAME LIMIT CMD...: output to $O/NAME.log, tail on failure, exit on failure
    local name=$1 lim=$2
    shift 2
    echo "== $name"
    timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
    local rc=$?
    if [ $rc -ne 0 ]; then
        echo "FAILED $name rc=$rc"
        tail -60 "$O/$name.log"
        exit 1
    fi
}

ranks_bench() {  # ranks_bench NAME PROFILER_ARGS... -- rank 0 of an N-rank bench.py run under rocprofv3
    local name=$1
    shift
    local args="--gpus $N --steps ${STEPS:-10} --warmup 3 --no-legs --no-cpu-baseline ${EXTRA:-}"
    local pids=() rcs=0 r
    port=$((port + 1))
    for r in $(seq 1 $((N - 1))); do
        MASTER_ADDR=127.0.0.1 WORLD_SIZE=$N MASTER_PORT=$port RANK=$r LOCAL_RANK=$r MI355X_TIMEOUT_S=60 \
            timeout -k 10 400 python bench.py $args > $O/${name}_r$r.log 2>&1 &
        pids+=($!)
    done
    MASTER_ADDR=127.0.0.1 WORLD_SIZE=$N MASTER_PORT=$port RANK=0 LOCAL_RANK=0 MI355X_TIMEOUT_S=60 \
        timeout -k 10 400 rocprofv3 "$@" -d $O/$name -o run --output-format csv -- python bench.py $args > $O/${name}_r0.log 2>&1
    local rc0=$?
    for p in "${pids[@]}"; do wait $p || rcs=1; done
    echo "== $name: rank0 rc=$rc0 others rc=$rcs"
    [ $rc0 -eq 0 ] && [ $rcs -eq 0 ] || { tail -20 $O/${name}_r0.log; exit 1; }
}
port=29700

small_c() {  # small_c NP REPS PATHS [sed tag]: one small_ar_c run, JSON lines appended to small.jsonl
    local n=$1 reps=$2 paths=$3
    timeout -k 10 200 ./tools/build/small_ar_c "$n" "$reps" "$paths" > $O/small_one.log 2>&1 || { cat $O/small_one.log; exit 1; }
    grep us_per_call $O/small_one.log | sed "s/^{/{\"tag\": \"${4:-}\", /" | tee -a $O/small.jsonl
}

for step in "$@"; do
    case $step in
    suite)
        run pytest_gpu 1100 $PYT tests
        tail -3 $O/pytest_gpu.log
        run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
        tail -2 $O/smoke.log ;;
    tests)
        run pytest_sel 1000 $PYT -rP ${TESTS:-tests} ${K:+-k "$K"}
        grep -E "PASSED|FAILED|SKIPPED|ERROR|passed|failed" $O/pytest_sel.log | tail -40 ;;
    op_overhead)
        run op_overhead 120 ./tools/build/op_host_overhead
        grep '^{' $O/op_overhead.log | tee $O/op_overhead.jsonl
        for n in 2 4; do
            run host8_n$n 200 bash tools/run_worker.sh host8 $n 150
            grep -h '^{' $O/w0.log | tee -a $O/op_overhead.jsonl
        done ;;
    smoke)
        run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
        tail -2 $O/smoke.log ;;
    bench)
        run bench_n1 300 python bench.py --steps ${STEPS:-20} --warmup ${WARM:-5}
        grep '^{' $O/bench_n1.log | tail -1 > $O/bench_n1.json
        cut -c1-600 $O/bench_n1.json ;;
    bench_ab)  # N = 1: the K timed launches issued one by one vs replayed as one HIP graph, alternated
        for i in 1 2 3; do
            for g in "" --graph; do
                timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup ${WARM:-5} --no-cpu-baseline $g > $O/bench_ab.log 2>&1 \
                    || { tail -20 $O/bench_ab.log; exit 1; }
                grep '^{' $O/bench_ab.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'graph': '$g' != '', 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'frac': d['roofline']['frac'], 'kernel_avg_ms': d['roofline']['kernel_avg_ms']}))" | tee -a $O/bench_ab.jsonl
            done
        done ;;
    prof_bench)
        run prof_bench 300 rocprofv3 --kernel-trace --stats -d $O/prof_bench -o run --output-format csv -- \
            python bench.py --steps 20 --warmup 5 --no-cpu-baseline
        head -3 $O/prof_bench/run_kernel_stats.csv | cut -c1-200 ;;
    pmc)
        run pmc_f 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_f -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline
        run pmc_w 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_w -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline
        python tools/pmc_summary.py $O/pmc_f $O/pmc_w $O/pmc_op.json "k_chunk<mi355x::OpSum<float>, true=op_3buff_sum_float" ;;
    legs)
        run legs 600 python tools/bench_legs.py --legs "${LEGS:-op,ddt}" --out $O/legs.jsonl
        tail -3 $O/legs.log ;;
    prof_ddt)
        run prof_ddt 300 rocprofv3 --kernel-trace --stats -d $O/prof_ddt -o run --output-format csv -- \
            python tools/bench_legs.py --legs ddt --no-cpu-baseline --out $O/legs_ddt_prof.jsonl ;;
    rehearse)
        for N in ${NS:-2 8}; do
            run bench_n$N ${TMO:-420} python bench.py --gpus $N --steps ${STEPS:-10} --warmup 3 ${ARGS:-}
            grep '^{' $O/bench_n$N.log | tail -1 > $O/bench_n$N.json
            cut -c1-800 $O/bench_n$N.json
        done ;;
    small)
        for n in ${NS:-2 4}; do small_c $n ${REPS:-2000} ${PATHS:-host,ll,svc} small; done ;;
    svc_trace)
        for sz in 8 65536; do
            SMALL_SIZES=$sz MI355X_SVC_TRACE=1 small_c 2 2000 svc svc_trace_$sz
            grep traced $O/small_one.log || true
        done ;;
    pull)
        for n in 2 4; do
            SMALL_SIZES=65536,131072,262144,524288,1048576 MI355X_SVC_PULL_MAX_BYTES=0 small_c $n 1000 host pull_off
            SMALL_SIZES=65536,131072,262144,524288,1048576 MI355X_SVC_PULL_MAX_BYTES=1048576 small_c $n 1000 host pull_on
        done ;;
    pull_copy)
        for coll in allgather bcast; do
            for n in 2 4; do
                SMALL_COLL=$coll SMALL_SIZES=8,1024,4096,16384 small_c $n 1000 svc ll_form
                SMALL_COLL=$coll SMALL_SIZES=16384,65536,262144,524288,1048576 small_c $n 1000 host pull_copy
                SMALL_COLL=$coll SMALL_SIZES=16384,65536,262144,524288,1048576 MI355X_SVC_PULL_COPY_MAX_BYTES=0 small_c $n 1000 host host_flow
            done
        done ;;
    pull_rs)
        for n in 2 4; do
            SMALL_COLL=reduce_scatter_block SMALL_SIZES=8,1024,16384,65536,131072 small_c $n 1000 host svc_rs
            SMALL_COLL=reduce_scatter_block SMALL_SIZES=8,1024,16384,65536,131072 MI355X_SVC_RS=0 small_c $n 1000 host host_flow
        done ;;
    queue_probe)
        : > $O/queue_probe.jsonl
        for mode in one_process:Q_X one_process_queue_first:Q_EARLY one_process_8_streams:Q_STREAMS; do
            case=${mode%%:*}; var=${mode##*:}
            env $var=$([ $var = Q_STREAMS ] && echo 8 || echo 1) timeout -k 10 60 ./tools/build/queue_probe 2000 \
                | sed "s/^{/{\"case\": \"$case\", /" >> $O/queue_probe.jsonl || exit 1
        done
        grep launch_sync $O/queue_probe.jsonl ;;
    unpack_ceiling)
        timeout -k 10 300 ./tools/build/unpack_ceiling 20 > $O/unpack_ceiling.jsonl 2> $O/unpack_ceiling.err \
            || { cat $O/unpack_ceiling.err; exit 1; }
        cat $O/unpack_ceiling.jsonl ;;
    host_p2p)
        run host_p2p 400 python -u -m pytest "tests/test_coll_ipc_gpu.py::test_host_p2p_between_processes" -m gpu -x -v -s \
            --timeout 200 --timeout-method thread
        grep -E '^\{|passed|failed' $O/host_p2p.log ;;
    p2p_lat)
        : > $O/p2p_lat.jsonl
        for kind in p2p_host p2p_dev p2p_dev:single_offer p2p_dev:unregistered; do
            reg=1; [ "${kind#*:}" = unregistered ] && reg=0
            dual=1; [ "${kind#*:}" = single_offer ] && dual=0
            MI355X_P2P_DUAL=$dual MI355X_P2P_REGISTER=$reg SMALL_COLL=${kind%%:*} SMALL_SIZES=8,64,512,1024,4096,16384,65536 \
                timeout -k 10 120 ./tools/build/small_ar_c 2 ${REPS:-5000} host > $O/small_one.log 2>&1 || { cat $O/small_one.log; exit 1; }
            grep one_way_us $O/small_one.log | sed "s/^{/{\"host_arena_registered\": $reg, \"dual_offer\": $dual, /" | tee -a $O/p2p_lat.jsonl
        done
        run p2p_lat_py 300 python tools/p2p_latency.py --out $O/p2p_lat.jsonl
        grep python $O/p2p_lat.jsonl ;;
    ab_host)  # host-synchronised small-call latency: this tree vs the build in ab_old/ (if present)
        for n in 2 4; do
            for coll in allgather allreduce; do
                SMALL_COLL=$coll SMALL_SIZES=16384,65536 MI355X_SVC_PULL_COPY_MAX_BYTES=0 MI355X_SVC_PULL_MAX_BYTES=0 \
                    small_c $n 1000 host host_new
                SMALL_COLL=$coll SMALL_SIZES=16384,65536 MI355X_SVC_PULL_COPY_MAX_BYTES=0 MI355X_SVC_PULL_MAX_BYTES=0 \
                    MI355X_SELFTEST=0 small_c $n 1000 host host_new_noselftest
                if [ -x ab_old/small_ar_c_old ]; then
                    SMALL_COLL=$coll SMALL_SIZES=16384,65536 MI355X_SVC_PULL_COPY_MAX_BYTES=0 MI355X_SVC_PULL_MAX_BYTES=0 \
                        timeout -k 10 200 ./ab_old/small_ar_c_old $n 1000 host > $O/small_one.log 2>&1 || { cat $O/small_one.log; exit 1; }
                    grep us_per_call $O/small_one.log | sed 's/^{/{"tag": "host_old", /' | tee -a $O/small.jsonl
                fi
            done
        done ;;
    ab_prep)  # the 4-process host-flow latency vs parts of the service's creation done at creation
        for prep in 0 1 2 8 16 4 27; do
            MI355X_SVC_PREP=$prep SMALL_COLL=allgather SMALL_SIZES=16384 MI355X_SVC_PULL_COPY_MAX_BYTES=0 \
                timeout -k 10 200 ./tools/build/small_ar_c 4 1000 host > $O/small_one.log 2>&1 || { cat $O/small_one.log; exit 1; }
            grep us_per_call $O/small_one.log | sed "s/^{/{\"svc_prep\": $prep, /" | tee -a $O/small.jsonl
        done ;;
    ab_host4)  # the 4-process host-flow latency: which setting matters (service / pipelined flow off)
        for env in "" MI355X_SVC=0 MI355X_PIPE=0 "MI355X_SVC=0 MI355X_PIPE=0"; do
            tag=$(echo "new ${env:-default}" | tr ' =' '__')
            env $env SMALL_COLL=allgather SMALL_SIZES=16384 MI355X_SVC_PULL_COPY_MAX_BYTES=0 \
                timeout -k 10 200 ./tools/build/small_ar_c 4 1000 host > $O/small_one.log 2>&1 || { cat $O/small_one.log; exit 1; }
            grep us_per_call $O/small_one.log | sed "s/^{/{\"tag\": \"$tag\", /" | tee -a $O/small.jsonl
            tag=$(echo "old ${env:-default}" | tr ' =' '__')
            env $env SMALL_COLL=allgather SMALL_SIZES=16384 MI355X_SVC_PULL_COPY_MAX_BYTES=0 \
                timeout -k 10 200 ./ab_old/small_ar_c_old 4 1000 host > $O/small_one.log 2>&1 || { cat $O/small_one.log; exit 1; }
            grep us_per_call $O/small_one.log | sed "s/^{/{\"tag\": \"$tag\", /" | tee -a $O/small.jsonl
        done ;;
    interference)
        run interference 900 python tools/svc_interference.py --out $O/svc_interference.jsonl
        cat $O/svc_interference.jsonl ;;
    prof_rehearsal)
        N=${N:-8} STEPS=${STEPS:-20} EXTRA=--no-autotune ranks_bench prof_n${N:-8} --kernel-trace --stats
        grep '^{' $O/prof_n${N:-8}_r0.log | tail -1 | cut -c1-1500
        head -4 $O/prof_n${N:-8}/run_kernel_stats.csv | cut -c1-200 ;;
    pmc_rehearsal)
        n=${N:-2}
        for c in FETCH_SIZE WRITE_SIZE; do N=$n ranks_bench pmc_reh_n${n}_$c --pmc $c; done
        python tools/pmc_summary.py $O/pmc_reh_n${n}_FETCH_SIZE $O/pmc_reh_n${n}_WRITE_SIZE $O/pmc_rehearsal_n$n.json \
            "k_pipe_allreduce=k_pipe_allreduce_rehearsal_n$n" "k_fold=k_fold_rehearsal_n$n" || exit 1
        cat $O/pmc_rehearsal_n$n.json ;;
    *)
        echo "unknown step $step"
        exit 2 ;;
    esac
done
echo "== done"
