"""A/B of the coll kernels' launch shapes on one box (2 ranks sharing the GPU): 1 GiB allreduce
phase times and a 1 GiB allgather for each (blocks_per_cu, copy_block_kib) pair, max over ranks."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import torch.distributed as dist
    from __graft_entry__ import _load_pkg
    pkg = _load_pkg()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    torch.cuda.set_device(0)
    comm = pkg.Comm.create(f"ab_{os.environ.get('MASTER_PORT')}", rank, world, 0)
    n = (1 << 30) // 4
    x = torch.full((n,), float(rank + 1), device="cuda")
    y = torch.empty_like(x)
    g = torch.empty((world * (1 << 30),), dtype=torch.uint8, device="cuda")
    rows = []
    for bpc in (64, 1024):
        for kib in (4, 16, 64):
            comm.set("BLOCKS_PER_CU", bpc)
            comm.set("COPY_BLOCK_KIB", kib)
            comm.set("TIME_PHASES", 1)
            p = [0.0, 0.0]
            for i in range(6):
                comm.allreduce(x.data_ptr(), y.data_ptr(), n, pkg.T["FLOAT"], pkg.OP["SUM"])
                if i:
                    a, b = comm.phase_ms()
                    p[0] += a / 5
                    p[1] += b / 5
            comm.allgather(x.data_ptr(), g.data_ptr(), 1 << 30)
            torch.cuda.synchronize()
            dist.barrier()
            t0 = time.perf_counter()
            for _ in range(3):
                comm.allgather(x.data_ptr(), g.data_ptr(), 1 << 30)
            torch.cuda.synchronize()
            t = torch.tensor([p[0], p[1], (time.perf_counter() - t0) / 3 * 1e3], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            rows.append({"blocks_per_cu": bpc, "copy_kib": kib, "fold_ms": round(float(t[0]), 4),
                         "pull_ms": round(float(t[1]), 4), "allgather_1GiB_ms": round(float(t[2]), 4)})
    if rank == 0:
        print(json.dumps(rows))
    comm.destroy()


if __name__ == "__main__":
    main()
