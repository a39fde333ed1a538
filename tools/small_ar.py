#!/usr/bin/env python3
"""Small-message MPI_Allreduce latency through the engine (one process per rank, ranks started by
the caller with RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT set, or under torch.distributed.run).
Prints one JSON line per size from rank 0: mean microseconds per call over --reps calls (a host
barrier between the calls is part of every call, as in MPI).  Used to take apart where the
host-synchronised path spends its ~18 us (run rank 0 under rocprofv3 --hip-trace --kernel-trace)."""
from __future__ import annotations

import argparse
import datetime
import json
import os
import pathlib
import sys
import time
import uuid

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="8,1024,65536,1048576")
    ap.add_argument("--reps", type=int, default=500)
    ap.add_argument("--paths", default="host", help="comma list of host (per-call launch + host sync), "
                    "ll (per-call LL kernels), svc (resident LL service)")
    ap.add_argument("--sched", type=int, default=-1, help="hipSetDeviceFlags schedule (1 spin, 2 yield, 4 blocking)")
    args = ap.parse_args()
    if args.sched >= 0:  # before any other HIP call of this process
        import ctypes
        hip = ctypes.CDLL("libamdhip64.so")
        print("hipSetDeviceFlags", hip.hipSetDeviceFlags(args.sched), file=sys.stderr)
    import torch
    import torch.distributed as dist
    import bench
    pkg = bench.load_pkg()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", rank)) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=120))
    key = [f"small_{os.getpid()}_{uuid.uuid4().hex[:8]}" if rank == 0 else None]
    dist.broadcast_object_list(key, src=0)
    comm = pkg.Comm.create(key[0], rank, world, local)
    comm.set("TIMEOUT_S", 60)
    sizes = [int(s) for s in args.sizes.split(",")]

    def run_path(path):
        comm.set("SVC_MAX_BYTES", max(sizes) if path == "svc" else 0)
        comm.set("LL_MAX_BYTES", max(sizes) if path == "ll" else 0)
        if path == "svc" and comm.get("SVC_MAX_BYTES") == 0:
            if rank == 0:
                print(json.dumps({"path": "svc", "error": "no resident service on this communicator"}), flush=True)
            return
        for nbytes in sizes:
            cnt = nbytes // 4
            x = torch.full((cnt,), float(rank + 1), device="cuda")
            y = torch.empty_like(x)
            for _ in range(20):
                comm.allreduce(x.data_ptr(), y.data_ptr(), cnt, pkg.T["FLOAT"], pkg.OP["SUM"])
            torch.cuda.synchronize()
            dist.barrier()
            t0 = time.perf_counter()
            for _ in range(args.reps):
                comm.allreduce(x.data_ptr(), y.data_ptr(), cnt, pkg.T["FLOAT"], pkg.OP["SUM"])
            dt = (time.perf_counter() - t0) / args.reps
            ok = bool(torch.all(y == world * (world + 1) / 2).item())
            if rank == 0:
                print(json.dumps({"path": path, "bytes": nbytes, "us_per_call": round(dt * 1e6, 2),
                                  "alg": comm.last_algorithm(), "n": world, "exact": ok,
                                  "svc_calls": comm.get("SVC_CALLS"), "svc_launches": comm.get("SVC_LAUNCHES")}),
                      flush=True)

    try:
        for path in args.paths.split(","):
            run_path(path)
        # the buffer-kind vote coll/mi355x adds to every component collective (mi355x_comm_vote):
        # a device-buffer rank only publishes; a host-buffer rank waits for every vote
        for kind, dev in (("vote_device_us", True), ("vote_host_us", False)):
            for _ in range(20):
                comm.vote(dev)
            dist.barrier()
            t0 = time.perf_counter()
            for _ in range(args.reps):
                comm.vote(dev)
            dt = (time.perf_counter() - t0) / args.reps
            if rank == 0:
                print(json.dumps({kind: round(dt * 1e6, 3), "n": world}), flush=True)
    finally:
        comm.destroy()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
