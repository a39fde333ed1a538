"""Device point-to-point ping-pong between two ranks (engine p2p, rendezvous + pull): one-way
latency per message size, one process per rank without a launcher.

usage: python tools/p2p_latency.py <rank> <key> [iters]      (run rank 0 and rank 1)
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

rank, key = int(sys.argv[1]), sys.argv[2]
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 200
pkg = bench.load_pkg()
pkg.rt()
dev = rank % torch.cuda.device_count()
torch.cuda.set_device(dev)
comm = pkg.Comm.create(key, rank, 2, dev)
comm.set("TIMEOUT_S", 30)
peer = 1 - rank
rows = []
for nbytes in (8, 1024, 8192, 65536, 1 << 20, 16 << 20):
    buf = torch.full((nbytes,), rank + 1, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    for phase in ("warm", "timed"):
        n = 10 if phase == "warm" else iters
        comm.barrier()
        t0 = time.perf_counter()
        for _ in range(n):
            if rank == 0:
                comm.send(buf.data_ptr(), nbytes, peer, 5)
                comm.recv(buf.data_ptr(), nbytes, peer, 6)
            else:
                comm.recv(buf.data_ptr(), nbytes, peer, 5)
                comm.send(buf.data_ptr(), nbytes, peer, 6)
        dt = (time.perf_counter() - t0) / n / 2
    rows.append((nbytes, dt))
comm.destroy()
if rank == 0:
    print(f"# tools/p2p_latency.py, 2 ranks on device(s) {dev} of {torch.cuda.device_count()}, {iters} round trips per size")
    for nbytes, dt in rows:
        print(f"{nbytes:>10} B  one-way {dt * 1e6:9.2f} us  {nbytes / dt / 1e9:8.2f} GB/s", flush=True)
