"""Debug: which hipMalloc sizes hipIpcOpenMemHandle imports (2 ranks, one-GPU rehearsal).
One fresh communicator per size; each rank exports a hipMalloc'd buffer of that size as the
allgather source."""
import ctypes, datetime, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, torch.distributed as dist
import bench
pkg = bench.load_pkg(); lib = pkg.rt()
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=60))
torch.cuda.set_device(0)
for kib in [int(v) for v in os.environ.get("DBG_KIB", "1,4,64,512,1024,2048,4096").split(",")]:
    comm = pkg.Comm.create(f"dbgs_{os.environ.get('MASTER_PORT', '0')}_{kib}", rank, world, 0)
    comm.set("TIMEOUT_S", 15)
    comm.set("LL_MAX_BYTES", 0)
    nb = kib * 1024
    p = ctypes.c_void_p()
    assert lib.mi355x_malloc(ctypes.byref(p), nb) == 0
    assert lib.mi355x_memset_async(p, rank + 1, nb, None) == 0
    dst = torch.zeros(nb * world, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    try:
        comm.allgather(p.value, dst.data_ptr(), nb)
        ok = all(int(dst[r * nb:(r + 1) * nb].min()) == r + 1 for r in range(world))
        msg = f"ok={ok}"
    except Exception as e:
        msg = f"ERROR {e}"
    print(f"[r{rank}] {kib} KiB hipMalloc: {msg}", file=sys.stderr, flush=True)
    dist.barrier()
    lib.mi355x_free(p)
    comm.destroy()
dist.destroy_process_group()
