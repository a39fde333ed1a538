"""Probe: LL vs host-synchronised allreduce latency per size (multi-process, run under
torch.distributed.run).  Prints one line per (size, flow) on rank 0."""
import datetime, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, torch.distributed as dist
import bench
pkg = bench.load_pkg(); pkg.rt()
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=90))
dev = rank % torch.cuda.device_count()
torch.cuda.set_device(dev)
comm = pkg.Comm.create("llp_" + os.environ.get("MASTER_PORT", "0"), rank, world, dev)
comm.set("TIMEOUT_S", 30)
f32, SUM = pkg.T["FLOAT"], pkg.OP["SUM"]
for nbytes in (8, 4096, 65536, 262144, 1 << 20):
    cnt = nbytes // 4
    x = torch.full((cnt,), float(rank + 1), device="cuda")
    y = torch.empty_like(x)
    for name, llmax in (("ll", 1 << 20), ("host", 0)):
        comm.set("LL_MAX_BYTES", llmax)
        for _ in range(5):
            comm.allreduce(x.data_ptr(), y.data_ptr(), cnt, f32, SUM)
        torch.cuda.synchronize(); dist.barrier()
        t0 = time.perf_counter()
        for _ in range(200):
            comm.allreduce(x.data_ptr(), y.data_ptr(), cnt, f32, SUM)
        dt = (time.perf_counter() - t0) / 200
        ok = bool(torch.all(y == world * (world + 1) / 2))
        if rank == 0:
            print(f"{nbytes:>8} B {name:5s} {dt*1e6:8.2f} us ok={ok}", flush=True)
comm.destroy()
dist.destroy_process_group()
