"""N > 1 leg of bench.py: MPI_Allreduce MPI_SUM fp32, 1 GiB per rank, through the coll/mi355x
engine (libmi355x_rt, IPC-mapped peers over xGMI), one process per GPU.

Launched by `python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N`.
torch.distributed (gloo, CPU) is used only for the launcher's rendezvous, the timing barrier and
the max-over-ranks reduction; every byte of the collective moves through the HIP engine.
value = busbw = (S / t) * 2 (n - 1) / n with S = 1 GiB and t = max over ranks per step.
"""
from __future__ import annotations

import datetime
import json
import os
import threading
import sys
import time
import uuid

GIB = 1 << 30
# MI355X Infinity Fabric: 7 links per GPU, 153.6 GB/s per link (spec, both directions)
# -> 76.8 GB/s per link per direction.  Ring peak busbw with R concurrent rings = R x 76.8.
XGMI_LINK_DIR_GBS = 76.8


def _log(rank, msg):
    """progress on stderr (rank 0), so a long multi-GPU run is visibly alive"""
    if rank == 0:
        print(f"[bench_coll {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def _timed(dist, torch, fn, reps, warm=1):
    """max-over-ranks seconds per call of fn (barrier + synchronize around the timed calls)"""
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    t = torch.tensor([(time.perf_counter() - t0) / reps], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t[0])


def extra_legs(args, pkg, torch, comm, world, rank, dev, legs, key):
    """The other multi-GPU BASELINE configs, measured on the same communicator after the headline
    (not part of `value`): configs[2] size sweep, configs[3] reduce_scatter_block + allgather fp64
    (4 GiB per rank), configs[4] 4 GiB bcast and the vector-datatype bcast / allreduce through the
    GPU convertor.  Every leg checks an exact-integer result."""
    import torch.distributed as dist
    f32, f64, SUM = pkg.T["FLOAT"], pkg.T["DOUBLE"], pkg.OP["SUM"]
    want = world * (world + 1) / 2
    # configs[2]: latency / busbw over message sizes (ring vs recursive-doubling regions)
    sweep = []
    for nbytes in (8, 1024, 8192, 65536, 1 << 20, 16 << 20, 256 << 20):
        _log(rank, f"leg allreduce_sweep {nbytes} B")
        cnt = nbytes // 4
        x = torch.full((cnt,), float(rank + 1), device=dev)
        y = torch.empty_like(x)
        run = lambda: comm.allreduce(x.data_ptr(), y.data_ptr(), cnt, f32, SUM)
        reps = 20 if nbytes <= (1 << 20) else 5
        sec = _timed(dist, torch, run, reps, 2)
        row = {"bytes": nbytes, "us": round(sec * 1e6, 2), "alg": comm.last_algorithm(),
               "busbw_GBs": round(nbytes / sec * 2 * (world - 1) / world / 1e9, 3),
               "exact": bool(torch.all(y == want).item()),
               "svc_resident": comm.get("SVC_RESIDENT"), "svc_launches": comm.get("SVC_LAUNCHES")}
        if nbytes <= (1 << 20):
            # every data flow at this size, for the thresholds: one-shot LL, host-synchronised with
            # ring orders in one phase (k_ring_all, below ONE_PHASE_MAX_BYTES) and in two
            # and the resident LL service (coll_svc.hip; reads 0 where this communicator has none)
            # the resident service's two forms (coll_svc.hip; read 0 where this communicator has
            # none): LL granules (us_svc) and the one-phase ring pulled from the mapped inputs (us_pull)
            one_phase, svc_max = comm.get("ONE_PHASE_MAX_BYTES"), comm.get("SVC_MAX_BYTES")
            pull_max = comm.get("SVC_PULL_MAX_BYTES")
            flows = [("us_ll", 1 << 20, one_phase, 0, 0), ("us_host", 0, 1 << 20, 0, 0), ("us_host_2phase", 0, 0, 0, 0)]
            if svc_max or pull_max:
                flows += [("us_svc", 0, one_phase, 1 << 20, 0), ("us_pull", 0, 1 << 20, 0, 1 << 20)]
            for name, llmax, op1, svc, pull in flows:
                comm.set("LL_MAX_BYTES", llmax)
                comm.set("ONE_PHASE_MAX_BYTES", op1)
                comm.set("SVC_MAX_BYTES", svc)
                comm.set("SVC_PULL_MAX_BYTES", pull)
                y.zero_()
                row[name] = round(_timed(dist, torch, run, reps, 2) * 1e6, 2)
                row["exact"] = row["exact"] and bool(torch.all(y == want).item())
            comm.set("LL_MAX_BYTES", 0)  # the defaults
            comm.set("ONE_PHASE_MAX_BYTES", one_phase)
            comm.set("SVC_MAX_BYTES", svc_max)
            comm.set("SVC_PULL_MAX_BYTES", pull_max)
        sweep.append(row)
        del x, y
    legs["allreduce_sweep_f32"] = sweep
    # what coll/mi355x's buffer-kind vote (mi355x_comm_vote) adds to every component collective
    # of the mixed-buffer set: in a window after device calls a device-buffer rank only publishes,
    # after host-only calls a host-buffer rank does; every 32nd call every rank waits (the sweep
    # above calls the engine directly, without the vote)
    legs["buffer_kind_vote_us"] = {
        "device_rank": round(_timed(dist, torch, lambda: comm.vote(True), 200, 5) * 1e6, 3),
        "host_ranks": round(_timed(dist, torch, lambda: comm.vote(False), 200, 5) * 1e6, 3)}
    # configs[3]: reduce_scatter_block + allgather, fp64, 4 GiB per rank
    _log(rank, "leg rsb_allgather_f64_4GiB")
    total = (4 << 30) // 8
    rcount = total // world
    x = torch.full((rcount * world,), float(rank + 1), dtype=torch.float64, device=dev)
    r = torch.empty((rcount,), dtype=torch.float64, device=dev)
    g = torch.empty((rcount * world,), dtype=torch.float64, device=dev)
    S = rcount * world * 8
    t_rs = _timed(dist, torch, lambda: comm.reduce_scatter_block(x.data_ptr(), r.data_ptr(), rcount, f64, SUM), 3)
    ok_rs = bool(torch.all(r == want).item())
    t_ag = _timed(dist, torch, lambda: comm.allgather(r.data_ptr(), g.data_ptr(), rcount * 8), 3)
    ok_ag = bool(torch.all(g == want).item())
    legs["rsb_allgather_f64_4GiB"] = {
        "rsb_ms": round(t_rs * 1e3, 3), "rsb_busbw_GBs": round(S / t_rs * (world - 1) / world / 1e9, 2),
        "rsb_alg": comm.last_algorithm(), "allgather_ms": round(t_ag * 1e3, 3),
        "allgather_busbw_GBs": round(S / t_ag * (world - 1) / world / 1e9, 2), "exact": ok_rs and ok_ag}
    del r, g
    # configs[4]: 4 GiB bcast (as MPI_FLOAT count 2^30), root 0
    _log(rank, "leg bcast_4GiB")
    xb = x.view(torch.uint8)
    nb = xb.numel()
    if rank != 0:
        x.zero_()
    torch.cuda.synchronize()
    t_b = _timed(dist, torch, lambda: comm.bcast(xb.data_ptr(), nb, 0), 3)
    ok_b = bool(torch.all(x == 1.0).item())
    legs["bcast_4GiB"] = {"ms": round(t_b * 1e3, 3), "busbw_GBs": round(nb / t_b / 1e9, 2), "exact": ok_b}
    del x, xb
    # configs[4]: vector(2^22, 64, 128, MPI_FLOAT) over a 2 GiB extent: root packs, 1 GiB packed
    # bytes broadcast, the others unpack (what coll/mi355x does for a derived datatype)
    _log(rank, "leg bcast_vector")
    nblk = 1 << 22
    d = pkg.Ddt.vector(nblk, 64, 128, 4)
    buf = torch.full((nblk, 128), float(rank + 1), device=dev)
    packed = torch.empty((nblk, 64), device=dev)

    def vbcast():
        if rank == 0:
            d.pack(1, buf.data_ptr(), 0, packed.data_ptr(), d.size)
        comm.bcast(packed.data_ptr(), d.size, 0)
        if rank != 0:
            d.unpack(1, buf.data_ptr(), 0, packed.data_ptr(), d.size)
    t_vb = _timed(dist, torch, vbcast, 3)
    ok_vb = bool(torch.all(buf[:, :64] == 1.0).item()) and bool(torch.all(buf[:, 64:] == rank + 1).item())
    legs["bcast_vector_1GiB_packed"] = {"ms": round(t_vb * 1e3, 3), "busbw_GBs": round(d.size / t_vb / 1e9, 2),
                                        "exact": ok_vb}
    # MPI_Allreduce of the vector's elements: pack -> contiguous allreduce -> unpack (the reference
    # rejects an intrinsic op on a derived type, op.h:490-501, so this is the parity definition)
    _log(rank, "leg allreduce_vector")
    buf.fill_(float(rank + 1))
    red = torch.empty_like(packed)

    def vallreduce():
        d.pack(1, buf.data_ptr(), 0, packed.data_ptr(), d.size)
        comm.allreduce(packed.data_ptr(), red.data_ptr(), nblk * 64, f32, SUM)
        d.unpack(1, buf.data_ptr(), 0, red.data_ptr(), d.size)
    t_va = _timed(dist, torch, vallreduce, 1, 0)
    ok_va = bool(torch.all(buf[:, :64] == want).item()) and bool(torch.all(buf[:, 64:] == rank + 1).item())
    t_va = _timed(dist, torch, vallreduce, 3, 0)
    legs["allreduce_vector_1GiB_packed"] = {
        "ms": round(t_va * 1e3, 3), "busbw_GBs": round(d.size / t_va * 2 * (world - 1) / world / 1e9, 2),
        "exact": ok_va}
    del buf, packed, red
    d.destroy()
    torch.cuda.empty_cache()
    # the callers either side of the path: MPI_Alltoall of 1 GiB per rank (pairwise blocks of
    # 1 GiB / n, each rank pulls n-1 blocks over n-1 links at once), and device point-to-point
    # (MPI_Sendrecv ring of 256 MiB: each rank pulls its predecessor's buffer)
    _log(rank, "leg alltoall_1GiB")
    try:
        blk = (1 << 30) // world
        a_s = torch.empty((blk * world,), dtype=torch.uint8, device=dev)
        for q in range(world):
            a_s[q * blk:(q + 1) * blk].fill_((rank * 16 + q) & 0xFF)
        a_r = torch.empty_like(a_s)
        torch.cuda.synchronize()
        t_a = _timed(dist, torch, lambda: comm.alltoall(a_s.data_ptr(), a_r.data_ptr(), blk), 3)
        ok_a = all(int(a_r[q * blk]) == ((q * 16 + rank) & 0xFF) and int(a_r[(q + 1) * blk - 1]) == ((q * 16 + rank) & 0xFF)
                   for q in range(world))
        legs["alltoall_1GiB"] = {"ms": round(t_a * 1e3, 3),
                                 "busbw_GBs": round(blk * world / t_a * (world - 1) / world / 1e9, 2), "exact": ok_a}
        del a_s, a_r
    except Exception as e:
        legs["alltoall_1GiB"] = {"error": repr(e)[:300]}
    _log(rank, "leg sendrecv_256MiB")
    try:
        nb = 256 << 20
        p_s = torch.full((nb,), rank + 1, dtype=torch.uint8, device=dev)
        p_r = torch.zeros_like(p_s)
        torch.cuda.synchronize()
        nxt, prv = (rank + 1) % world, (rank - 1) % world
        t_p = _timed(dist, torch, lambda: comm.sendrecv(p_s.data_ptr(), nb, nxt, 0, p_r.data_ptr(), nb, prv, 0), 3)
        ok_p = int(p_r.min()) == prv + 1 and int(p_r.max()) == prv + 1
        legs["sendrecv_ring_256MiB"] = {"ms": round(t_p * 1e3, 3), "GBs_per_rank": round(nb / t_p / 1e9, 2),
                                        "exact": ok_p}
        del p_s, p_r
    except Exception as e:
        legs["sendrecv_ring_256MiB"] = {"error": repr(e)[:300]}
    torch.cuda.empty_cache()
    # comparison point only (BASELINE north star): RCCL's allreduce on the same device buffers,
    # through torch.distributed's "nccl" backend (= RCCL on ROCm).  Needs one GPU per rank.
    if torch.cuda.device_count() >= world:
        _log(rank, "leg rccl_allreduce")
        try:
            pg = dist.new_group(backend="nccl")
            rows = []
            for nbytes in (8, 65536, 1 << 20, 16 << 20, 256 << 20, 1 << 30):
                cnt = max(1, nbytes // 4)
                x = torch.full((cnt,), float(rank + 1), device=dev)
                sec = _timed(dist, torch, lambda: dist.all_reduce(x, group=pg), 20 if nbytes <= (1 << 20) else 5, 2)
                rows.append({"bytes": nbytes, "us": round(sec * 1e6, 2),
                             "busbw_GBs": round(nbytes / sec * 2 * (world - 1) / world / 1e9, 3)})
                del x
            legs["rccl_allreduce_f32"] = rows
            dist.destroy_process_group(pg)
        except Exception as e:  # comparison only: never fails the run
            legs["rccl_allreduce_f32"] = {"error": repr(e)[:300]}
        torch.cuda.empty_cache()
    return legs


def measure_link(pkg, torch, dist, world, rank, dev, key):
    """xGMI link bandwidth, the roofline denominator (SURVEY.md §8(d) C3 and BASELINE.md §2: "must
    be measured"): ranks 0 and 1 alone, each pulling 256 MiB from the other over their one link
    (both directions at once) through the engine's own copy kernel.  Every rank returns the same
    dict (max over ranks)."""
    nb = 256 << 20
    try:
        if rank < 2:
            pair = pkg.Comm.create(f"{key}_pair", rank, 2, dev.index)
            pair.set("TIMEOUT_S", 120)
            src = torch.full((nb,), rank + 1, dtype=torch.uint8, device=dev)
            dst = torch.empty((2 * nb,), dtype=torch.uint8, device=dev)
            for _ in range(2):
                pair.allgather(src.data_ptr(), dst.data_ptr(), nb)
            torch.cuda.synchronize()
            pair.barrier()
            t0 = time.perf_counter()
            for _ in range(5):
                pair.allgather(src.data_ptr(), dst.data_ptr(), nb)
            torch.cuda.synchronize()
            t_l = (time.perf_counter() - t0) / 5
            ok_l = int(dst[:nb].max()) == 1 and int(dst[nb:].min()) == 2
            pair.destroy()
            del src, dst
        else:
            t_l, ok_l = 0.0, True
        err = 0.0
    except Exception:  # noqa: BLE001 -- reported as an error entry, the spec peak is used then
        t_l, ok_l, err = 0.0, False, 1.0
    t = torch.tensor([t_l, 0.0 if ok_l else 1.0, err], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    torch.cuda.empty_cache()
    if t[2] > 0 or t[0] <= 0:
        return {"error": "link measurement failed on some rank"}
    return {"ms": round(float(t[0]) * 1e3, 3), "GBs_per_direction": round(nb / float(t[0]) / 1e9, 2),
            "exact": float(t[1]) == 0.0, "note": "ranks 0,1 only; each pulls 256 MiB from the other"}


def run(args, pkg, torch):
    import torch.distributed as dist

    if "WORLD_SIZE" not in os.environ or "MASTER_ADDR" not in os.environ:
        # bench.py --gpus N spawns its ranks itself (bench.spawn_ranks); reaching here without the
        # launcher's environment means this module was driven some other way
        raise SystemExit("bench_coll needs a launcher environment (WORLD_SIZE, MASTER_ADDR): "
                         "run `python bench.py --gpus N` or torch.distributed.run")
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    # a measurement run bounds its waits (communicator creation included) at minutes, not the
    # engine's default of a day: a rank that failed before creating a communicator ends the run
    os.environ.setdefault("MI355X_TIMEOUT_S", "300")
    if world < 2:
        raise SystemExit("bench_coll needs WORLD_SIZE >= 2")
    local = local % max(1, torch.cuda.device_count())  # one-GPU rehearsal: ranks share device 0
    torch.cuda.set_device(local)
    if not dist.is_initialized():
        # bounded waits: a failing rank surfaces as an error on the others, not a hang
        dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=300))
    # node-unique rendezvous key: rank 0 picks it, the launcher's process group spreads it
    key = [f"bench_{os.getpid()}_{uuid.uuid4().hex[:12]}" if rank == 0 else None]
    dist.broadcast_object_list(key, src=0)
    key = key[0]
    comm = pkg.Comm.create(key, rank, world, local)
    comm.set("TIMEOUT_S", 120)

    n = GIB // 4
    dev = torch.device("cuda", local)
    ty, op = pkg.T["FLOAT"], pkg.OP["SUM"]
    # data-flow / launch-shape autotune on the real size, with an exactness check on every
    # candidate (check_calls: data that changes per call, rbuf poisoned first).  Candidates: the pipelined
    # flow (one launch: fold + pulls with device-side chunk flags; workgroups per CU x chunk size:
    # the engine's own (~512 chunks per block, >= 64 KiB: 256 KiB at n = 8), 512 KiB and 2 MiB, so
    # separate GPUs' link latency picks its own overlap granularity)
    # and the two-phase flow (fold -> host barrier -> pull; grid cap).  All ranks see the same
    # max-over-ranks times, so they pick the same candidate.  Push is not a candidate: its remote
    # writes land behind the owner's L2 (coarse-grained memory is not probed) -- single device only.
    x = torch.full((n,), float(rank + 1), device=dev)
    y = torch.empty_like(x)
    want = world * (world + 1) / 2
    ok = True
    cands = [{"pipe": 1, "pipe_wg_per_cu": wg, "pipe_chunk_kib": ck, "pipe_wt": wt}
             for wt in (0, 1) for wg in (1, 2, 4, 8) for ck in (0, 512, 2048)]
    cands += [{"pipe": 0, "blocks_per_cu": bpc, "copy_block_kib": 4} for bpc in (8, 1024)]
    if getattr(args, "no_autotune", False):  # the engine's defaults only
        cands = [{"pipe": comm.get("PIPE"), "pipe_wg_per_cu": comm.get("PIPE_WG_PER_CU"),
                  "pipe_chunk_kib": comm.get("PIPE_CHUNK_KIB"), "pipe_wt": comm.get("PIPE_WT"),
                  "blocks_per_cu": comm.get("BLOCKS_PER_CU"), "copy_block_kib": comm.get("COPY_BLOCK_KIB")}]

    comm, key, tried, ok, best = autotune(comm, key, cands, pkg=pkg, dist=dist, rank=rank, world=world,
                                          local=local, x=x, y=y, n=n, ty=ty, op=op, want=want,
                                          sync=torch.cuda.synchronize, ok=ok)
    # timed data: N(0,1), order-dependent (the engine replicates the segmented-ring order)
    _log(rank, f"timed: {args.steps} steps, best {best}")
    x.normal_()
    torch.cuda.synchronize()
    for _ in range(args.warmup):
        comm.allreduce(x.data_ptr(), y.data_ptr(), n, ty, op)
    alg = comm.last_algorithm()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        comm.allreduce(x.data_ptr(), y.data_ptr(), n, ty, op)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    dist.barrier()
    t = torch.tensor([dt, 0.0 if ok else 1.0], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt, bad = float(t[0]), float(t[1])
    per = dt / args.steps
    busbw = (n * 4 / per) * 2 * (world - 1) / world / 1e9
    # dominant kernel (phase 1, k_fold: the owner folds its block from all n ranks), timed with
    # HIP events on the call's stream over 5 untimed-region calls; max over ranks
    comm.set("TIME_PHASES", 1)
    p1 = p2 = 0.0
    for _ in range(5):
        comm.allreduce(x.data_ptr(), y.data_ptr(), n, ty, op)
        a1, a2 = comm.phase_ms()
        p1 += a1 / 5
        p2 += a2 / 5
    comm.set("TIME_PHASES", 0)
    tk = torch.tensor([p1, p2], dtype=torch.float64)
    dist.all_reduce(tk, op=dist.ReduceOp.MAX)
    p1, p2 = float(tk[0]), float(tk[1])
    blk = n * 4 / world                              # bytes of one ring block
    pipe = bool(best["pipe"])
    # algorithmic bytes of the dominant launch.  xGMI (ingress per rank): pipelined = the fold's
    # n-1 remote block reads + the n-1 pulled blocks; two-phase phase 1 = the n-1 remote blocks.
    # Rehearsal (every rank on one GPU, concurrent launches): the chip's HBM reads + writes of all
    # ranks' launches -- pipelined (3n-1) blocks per rank (fold n reads + 1 write, pulls n-1 reads
    # + n-1 writes), phase 1 (n+1) blocks per rank.
    xgmi_bytes = (2 if pipe else 1) * (world - 1) * blk
    hbm_bytes = world * ((3 * world - 1) if pipe else (world + 1)) * blk
    fold_xgmi = xgmi_bytes / (p1 * 1e-3) / 1e9
    fold_hbm = hbm_bytes / (p1 * 1e-3) / 1e9
    kname = "k_pipe_allreduce (fold + pulls, one launch)" if pipe else "k_fold (allreduce phase 1)"
    # ranks sharing one GPU (a rehearsal on a 1-GPU box): the traffic never leaves local HBM
    shared = torch.cuda.device_count() < world
    # the denominator: the measured per-direction link rate x (n-1) links; the spec rate rides along
    link = None if shared else measure_link(pkg, torch, dist, world, rank, dev, key)
    link_gbs = link.get("GBs_per_direction") if link and link.get("exact") else None
    peak_spec = (world - 1) * XGMI_LINK_DIR_GBS
    peak_all = (world - 1) * link_gbs if link_gbs else peak_spec
    res = {
        "metric": "MPI_Allreduce busbw GB/s (1 GiB fp32, np=8) + op/hip reduce HBM GB/s",
        "value": round(busbw, 2),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(per * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (torch normal_ on device)",
        "config": {"workload": f"MPI_Allreduce MPI_SUM MPI_FLOAT 1 GiB per rank, np={world} (BASELINE configs[2])",
                   "count": n, "algorithm": {3: "recursive_doubling", 4: "ring", 5: "segmented_ring"}.get(alg, alg),
                   "exact_check": "ok" if bad == 0 else "FAILED",
                   "data_flow": "pipelined (fold + pulls, device flags)" if pipe else "two-phase pull",
                   "best": best, "autotune_ms_per_call": tried},
        "roofline": ({"bound": "xgmi", "achieved": round(fold_xgmi, 2), "peak": round(peak_all, 1), "unit": "GB/s",
                      "frac": round(fold_xgmi / peak_all, 4), "traffic": pmc_traffic(pipe, shared=False, world=world),
                      "traffic_note": "HBM bytes per launch from a committed rocprofv3 PMC summary of this "
                                      "kernel on separate GPUs, or null: only the one-GPU rehearsal's "
                                      "(profiles/r02_pmc_rehearsal_n*.json) exists so far",
                      "kernel": kname, "kernel_avg_ms": round(p1, 4),
                      "alg_bytes_per_launch": int(xgmi_bytes), "phase2_ms": round(p2, 4),
                      "busbw_frac": round(busbw / peak_all, 4),
                      # against one ring (one link per direction) as well as all n-1
                      "busbw_frac_ring1": round(busbw / (link_gbs or XGMI_LINK_DIR_GBS), 4),
                      "peak_spec": round(peak_spec, 1), "frac_spec": round(fold_xgmi / peak_spec, 4),
                      "link": link,
                      "peak_note": (f"(n-1) links x {link_gbs} GB/s per direction, measured (link.GBs_per_direction)"
                                    if link_gbs else f"(n-1) links x {XGMI_LINK_DIR_GBS} GB/s per direction (spec; "
                                    "the link measurement failed)") + "; achieved = the remote bytes one launch "
                                   "reads over xGMI / its event time"} if not shared else
                     {"bound": "hbm", "achieved": round(fold_hbm, 2), "peak": 8000.0, "unit": "GB/s",
                      "frac": round(fold_hbm / 8000.0, 4), "traffic": pmc_traffic(pipe, shared=True, world=world),
                      "kernel": kname, "kernel_avg_ms": round(p1, 4),
                      "alg_bytes_per_launch": int(hbm_bytes / world), "phase2_ms": round(p2, 4),
                      "peak_note": "REHEARSAL: all ranks share one GPU, no xGMI traffic: the n concurrent "
                                   "launches' HBM reads + writes (n x alg_bytes_per_launch) against the "
                                   "chip's HBM; busbw not valid"}),
        "cpu_baseline": None,
        "legs": None,
    }
    if not args.no_legs:
        del x, y
        torch.cuda.empty_cache()
        legs = {}
        # watchdog: a leg that never returns must not take the headline line with it
        done = threading.Event()

        def watchdog():
            if not done.wait(args.legs_timeout):
                if rank == 0:
                    legs["error"] = f"legs exceeded {args.legs_timeout:.0f} s; partial results above"
                    res["legs"] = legs
                    print(json.dumps(res), flush=True)
                os._exit(3)  # a hung leg is a failed run, whatever the headline said
        threading.Thread(target=watchdog, daemon=True).start()
        try:
            extra_legs(args, pkg, torch, comm, world, rank, dev, legs, key)
        except Exception as e:  # a failing extra leg must not hide the headline line
            legs["error"] = repr(e)[:300]
        done.set()
        res["legs"] = legs
    comm.destroy()
    if rank != 0:
        dist.destroy_process_group()
        return None
    dist.destroy_process_group()
    if not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline_ring(world, args.cpu_seconds)
    if bad != 0:  # a wrong result is not a measurement
        res["error"] = "allreduce result differs from the exact sum"
        res["value"] = None
    return res


def apply_cand(comm, cand):
    """set a candidate's knobs on the engine communicator"""
    comm.set("PUSH", 0)
    comm.set("PIPE", cand["pipe"])
    for k, knob in (("pipe_wg_per_cu", "PIPE_WG_PER_CU"), ("pipe_chunk_kib", "PIPE_CHUNK_KIB"), ("pipe_wt", "PIPE_WT"),
                    ("blocks_per_cu", "BLOCKS_PER_CU"), ("copy_block_kib", "COPY_BLOCK_KIB")):
        if k in cand:
            comm.set(knob, cand[k])


def check_calls(comm, x, y, n, ty, op, *, rank, world, want, ks):
    """exactness on data that changes every call, with rbuf poisoned (NaN) before each call: a
    stale hand-off -- a peer's block read before its owner's result reached memory -- shows here,
    where constant data (the same sum every call) cannot.  x_r = r + 1 + 3k -> want + 3k*world."""
    import torch
    good = True
    for k in ks:
        x.fill_(float(rank + 1 + 3 * k))
        y.fill_(float("nan"))
        comm.allreduce(x.data_ptr(), y.data_ptr(), n, ty, op)
        good = good and bool(torch.all(y == want + 3 * k * world).item())
    # and once in place (MPI_IN_PLACE: a rank's block boundaries share cache lines between the
    # peers' inputs it folds and the results it pulls)
    k = ks[-1] + 1
    y.fill_(float(rank + 1 + 3 * k))
    comm.allreduce(None, y.data_ptr(), n, ty, op)
    good = good and bool(torch.all(y == want + 3 * k * world).item())
    return good


def autotune(comm, key, cands, *, pkg, dist, rank, world, local, x, y, n, ty, op, want, sync, ok=True):
    """time every candidate (3 calls, max over ranks) after an exactness check on changing data.
    A candidate that fails -- e.g. a flag never seen over this machine's links: the engine's
    bounded wait turns it into an error on every rank, or on some -- is dropped with its flow;
    every rank agrees on the outcome first, then the communicator is rebuilt under a new key and
    the search goes on.  A candidate whose result is wrong on any rank (a stale hand-off) is
    dropped alone.  The winner is re-checked on fresh data; if that fails the next best is taken.
    Returns (comm, key, tried, ok, best); best is applied, ok is False only when no candidate
    passed the re-check."""
    import torch
    tried = []
    failed_flows = set()
    comm.set("TIMEOUT_S", 30)
    for ci, cand in enumerate(cands):
        if cand["pipe"] in failed_flows:
            continue
        _log(rank, f"autotune {cand}")
        err = None
        cand_ok = True
        try:
            apply_cand(comm, cand)
            sync()
            cand_ok = check_calls(comm, x, y, n, ty, op, rank=rank, world=world, want=want, ks=(2 * ci, 2 * ci + 1))
            t0 = time.perf_counter()
            for _ in range(3):
                comm.allreduce(x.data_ptr(), y.data_ptr(), n, ty, op)
            el = (time.perf_counter() - t0) / 3
        except pkg.MI355XError as e:
            err, el = repr(e)[:240], float("inf")
        agree = torch.tensor([el, 1.0 if err else 0.0, 0.0 if cand_ok else 1.0])
        dist.all_reduce(agree, op=dist.ReduceOp.MAX)
        if agree[1] > 0:
            failed_flows.add(cand["pipe"])
            tried.append(dict(cand, ms=None, error=err or "failed on another rank"))
            sync()
            dist.barrier()
            comm.destroy()
            key = f"{key}_r"
            comm = pkg.Comm.create(key, rank, world, local)
            comm.set("TIMEOUT_S", 30)
            continue
        if agree[2] > 0:
            tried.append(dict(cand, ms=None, error="wrong result" + ("" if not cand_ok else " on another rank")))
            continue
        tried.append(dict(cand, ms=round(float(agree[0]) * 1e3, 4)))
    comm.set("TIMEOUT_S", 120)
    ranked = sorted((c for c in tried if c["ms"] is not None), key=lambda c: c["ms"])
    if not ranked:
        raise SystemExit("every allreduce candidate failed: " + json.dumps(tried))
    for i, best in enumerate(ranked):
        apply_cand(comm, best)
        sync()
        good = check_calls(comm, x, y, n, ty, op, rank=rank, world=world, want=want,
                           ks=range(1000 + 4 * i, 1004 + 4 * i))
        agree = torch.tensor([0.0 if good else 1.0])
        dist.all_reduce(agree, op=dist.ReduceOp.MAX)
        if agree[0] == 0:
            return comm, key, tried, ok, best
        best["recheck"] = "wrong result on fresh data: dropped"
    apply_cand(comm, ranked[0])
    return comm, key, tried, False, ranked[0]


def pmc_traffic(pipe, shared, world):
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3 PMC summary
    (profiles/*pmc*.json, FETCH_SIZE x 2 + WRITE_SIZE per MI355X_MICROARCH.md) measured at this
    world size, or None"""
    import pathlib
    key = ("k_pipe_allreduce" if pipe else "k_fold") + ("_rehearsal" if shared else "") + f"_n{world}"
    for p in sorted((pathlib.Path(__file__).resolve().parent / "profiles").glob("*pmc*.json"), reverse=True):
        try:
            ent = json.loads(p.read_text()).get("kernels", {}).get(key)
        except Exception:
            continue
        if ent and "hbm_bytes_per_launch" in ent:
            return ent["hbm_bytes_per_launch"]
    return None


def cpu_baseline_ring(n, seconds):
    """BASELINE configs[0] on this host: the reference CPU path (coll/tuned segmented ring, 1 MiB
    segments, over sm-BTL-style 32 KiB shared-memory fragments; oracle/cpu_ring.c), n ranks as n
    threads pinned to n distinct host cores, MPI_SUM MPI_FLOAT 16 M elements (64 MiB) per rank --
    the configs[0] message size, a bounded sample of the same metric.  busbw = S/t * 2(n-1)/n."""
    import ctypes
    import pathlib
    import numpy as np
    so = pathlib.Path(__file__).resolve().parent / "oracle" / "build" / "liboracle.so"
    if not so.exists():
        return None
    lib = ctypes.CDLL(str(so))
    vp = ctypes.c_void_p
    lib.oracle_cpu_allreduce.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_uint32,
                                         ctypes.POINTER(vp), ctypes.POINTER(vp), ctypes.c_int, ctypes.c_int,
                                         ctypes.POINTER(ctypes.c_double)]
    count = 1 << 24
    xs = [np.full(count, float(r + 1), dtype=np.float32) for r in range(n)]
    outs = [np.empty(count, dtype=np.float32) for _ in range(n)]
    P = lambda arrs: (vp * n)(*[a.ctypes.data for a in arrs])
    cores = sorted(os.sched_getaffinity(0))
    core0 = cores[0] if len(cores) >= n and cores[n - 1] - cores[0] == n - 1 else -1
    t = ctypes.c_double()
    if lib.oracle_cpu_allreduce(n, count, 14, 3, 1 << 20, P(xs), P(outs), 1, core0, ctypes.byref(t)) != 0:
        return None
    reps = max(1, min(200, int(seconds / max(t.value, 1e-6))))
    t0 = time.perf_counter()
    lib.oracle_cpu_allreduce(n, count, 14, 3, 1 << 20, P(xs), P(outs), reps, core0, ctypes.byref(t))
    wall = time.perf_counter() - t0
    S = count * 4
    exact = all(bool(np.all(o == n * (n + 1) / 2)) for o in outs)
    return {"value": round(S / t.value * 2 * (n - 1) / n / 1e9, 3), "unit": "GB/s", "cores": n, "kind": "port",
            "pinned": core0 >= 0, "exact": exact,
            "sample": f"configs[0] CPU path at np={n}: segmented ring (1 MiB segments, 32 KiB shm fragments), "
                      f"16 M fp32 (64 MiB) per rank, {reps} calls, {wall:.1f} s; busbw"}
