"""LL (one-shot, device flags) vs host-synchronised latency of small collectives, one process per
rank WITHOUT a launcher (each rank can run under its own rocprofv3): ranks meet through the
engine's own control segment (key from argv) and time with its barrier.

usage: python tools/ll_probe2.py <rank> <size> <key> [calls]
Rank 0 prints one line per (collective, size, flow): mean us per call over `calls` calls.
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

rank, size, key = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
calls = int(sys.argv[4]) if len(sys.argv) > 4 else 200
pkg = bench.load_pkg()
pkg.rt()
dev = rank % torch.cuda.device_count()
torch.cuda.set_device(dev)
comm = pkg.Comm.create(key, rank, size, dev)
comm.set("TIMEOUT_S", 30)
f32, SUM = pkg.T["FLOAT"], pkg.OP["SUM"]


def timed(fn):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    comm.barrier()
    t0 = time.perf_counter()
    for _ in range(calls):
        fn()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / calls
    comm.barrier()
    return dt


rows = []
for nbytes in (8, 4096, 65536):
    cnt = max(1, nbytes // 4)
    x = torch.full((cnt,), float(rank + 1), device="cuda")
    y = torch.empty_like(x)
    g = torch.empty(cnt * size, device="cuda")
    b = torch.empty(cnt, device="cuda")
    for flow, llmax in (("ll", 1 << 20), ("host", 0)):
        comm.set("LL_MAX_BYTES", llmax)
        t_ar = timed(lambda: comm.allreduce(x.data_ptr(), y.data_ptr(), cnt, f32, SUM))
        ok = bool(torch.all(y == size * (size + 1) / 2))
        t_ag = timed(lambda: comm.allgather(x.data_ptr(), g.data_ptr(), cnt * 4))
        ok = ok and all(bool(torch.all(g[q * cnt:(q + 1) * cnt] == q + 1)) for q in range(size))
        b.fill_(float(rank))
        t_bc = timed(lambda: comm.bcast(b.data_ptr(), cnt * 4, 0))
        ok = ok and bool(torch.all(b == 0))
        rows.append((nbytes, flow, t_ar, t_ag, t_bc, ok))
comm.set("LL_MAX_BYTES", 0)
comm.destroy()
if rank == 0:
    print(f"# tools/ll_probe2.py, {size} ranks, device {dev} of {torch.cuda.device_count()}, {calls} calls per row")
    print(f"{'bytes':>8} {'flow':5s} {'allreduce_us':>13} {'allgather_us':>13} {'bcast_us':>9} exact")
    for nbytes, flow, a, g_, c, ok in rows:
        print(f"{nbytes:>8} {flow:5s} {a * 1e6:13.2f} {g_ * 1e6:13.2f} {c * 1e6:9.2f} {ok}", flush=True)
