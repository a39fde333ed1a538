"""Debug: reduce_scatter_block / allgather at growing sizes, 2 ranks (one-GPU rehearsal)."""
import datetime, faulthandler, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, torch.distributed as dist
import bench
pkg = bench.load_pkg(); pkg.rt()
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
faulthandler.dump_traceback_later(60, exit=True)
dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=90))
torch.cuda.set_device(0)
comm = pkg.Comm.create("dbg_" + os.environ.get("MASTER_PORT", "0"), rank, world, 0)
comm.set("TIMEOUT_S", 40)
f64, SUM = pkg.T["DOUBLE"], pkg.OP["SUM"]
def log(m):
    print(f"[r{rank} {time.strftime('%H:%M:%S')}] {m}", file=sys.stderr, flush=True)
for gib in [float(g) for g in os.environ.get("DBG_GIB", "0.25,1,2,3,4").split(",")]:
    total = int(gib * (1 << 30)) // 8
    rcount = total // world
    x = torch.full((rcount * world,), float(rank + 1), dtype=torch.float64, device="cuda")
    r = torch.empty((rcount,), dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    log(f"rsb {gib} GiB start")
    comm.reduce_scatter_block(x.data_ptr(), r.data_ptr(), rcount, f64, SUM)
    torch.cuda.synchronize()
    log(f"rsb {gib} GiB done alg={comm.last_algorithm()} ok={bool(torch.all(r == 3).item())}")
    g = torch.empty((rcount * world,), dtype=torch.float64, device="cuda")
    comm.allgather(r.data_ptr(), g.data_ptr(), rcount * 8)
    torch.cuda.synchronize()
    log(f"allgather {gib} GiB ok={bool(torch.all(g == 3).item())}")
    faulthandler.dump_traceback_later(60, exit=True)
    del x, r, g
    torch.cuda.empty_cache()
comm.destroy()
dist.destroy_process_group()
