"""Point-to-point ping-pong between two processes through the engine (the path every MPI_Send /
MPI_Recv on an engine communicator takes, host or device buffer): one-way latency per message
size, for host buffers (the sm BTL's domain in the reference: 4 KiB eager, 1 us advertised,
btl_sm_component.c:243-253) and device buffers.

usage: python tools/p2p_latency.py [--out FILE] [--iters N] [--kinds host,dev]
       (starts both ranks itself; each rank is `python tools/p2p_latency.py --rank R --key K`)
"""
import argparse
import json
import os
import subprocess
import sys
import time
import uuid

HERE = os.path.dirname(os.path.abspath(__file__))
SIZES_HOST = (8, 64, 512, 1024, 4096, 16384, 65536)
SIZES_DEV = (8, 1024, 4096, 65536, 1 << 20, 16 << 20)


def rank_main(rank, key, iters, kinds):
    import numpy as np
    import torch
    sys.path.insert(0, os.path.dirname(HERE))
    import bench
    pkg = bench.load_pkg()
    pkg.rt()
    dev = rank % torch.cuda.device_count()
    torch.cuda.set_device(dev)
    comm = pkg.Comm.create(key, rank, 2, dev)
    comm.set("TIMEOUT_S", 30)
    peer = 1 - rank
    rows = []
    for kind in kinds:
        for nbytes in (SIZES_HOST if kind == "host" else SIZES_DEV):
            if kind == "host":
                buf = np.full(nbytes, rank + 1, dtype=np.uint8)
                ptr = buf.ctypes.data
            else:
                buf = torch.full((nbytes,), rank + 1, dtype=torch.uint8, device="cuda")
                torch.cuda.synchronize()
                ptr = buf.data_ptr()
            samples = []
            for phase in ("warm", "timed"):
                n = 20 if phase == "warm" else iters
                comm.barrier()
                t0 = time.perf_counter()
                for _ in range(n):
                    if rank == 0:
                        comm.send(ptr, nbytes, peer, 5)
                        comm.recv(ptr, nbytes, peer, 6)
                    else:
                        comm.recv(ptr, nbytes, peer, 5)
                        comm.send(ptr, nbytes, peer, 6)
                samples.append((time.perf_counter() - t0) / n / 2)
            dt = samples[-1]
            rows.append({"leg": "p2p_pingpong", "kind": kind, "bytes": nbytes, "one_way_us": round(dt * 1e6, 2),
                         "GBs": round(nbytes / dt / 1e9, 3), "iters": iters, "caller": "python"})
    comm.barrier()
    comm.destroy()
    if rank == 0:
        for r in rows:
            print(json.dumps(r), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rank", type=int, default=-1)
    ap.add_argument("--key", default="")
    ap.add_argument("--iters", type=int, default=2000)
    ap.add_argument("--kinds", default="host,dev")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    kinds = [k for k in a.kinds.split(",") if k]
    if a.rank >= 0:
        return rank_main(a.rank, a.key, a.iters, kinds)
    key = "p2p" + uuid.uuid4().hex[:10]
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__), "--rank", str(r), "--key", key, "--iters",
                               str(a.iters), "--kinds", a.kinds], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
             for r in range(2)]
    outs = [p.communicate(timeout=600)[0] for p in procs]
    if any(p.returncode for p in procs):
        sys.stderr.write("\n".join(outs))
        sys.exit(1)
    lines = [ln for ln in outs[0].splitlines() if ln.startswith("{")]
    if a.out:
        with open(a.out, "a") as f:
            for ln in lines:
                f.write(ln + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
