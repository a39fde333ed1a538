"""Debug: two hipMalloc'd buffers of one rank exported in the same call (allreduce sbuf + rbuf,
direct pull path) -- does the importer map both?  2 ranks, one-GPU rehearsal."""
import ctypes, datetime, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, torch.distributed as dist
import bench
pkg = bench.load_pkg(); lib = pkg.rt()
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=60))
torch.cuda.set_device(0)
for kib in [int(v) for v in os.environ.get("DBG_KIB", "128,512,1024,2048,4096").split(",")]:
    comm = pkg.Comm.create(f"dbgp_{os.environ.get('MASTER_PORT', '0')}_{kib}", rank, world, 0)
    comm.set("TIMEOUT_S", 15)
    comm.set("LL_MAX_BYTES", 0)
    nb = kib * 1024
    s, r = ctypes.c_void_p(), ctypes.c_void_p()
    assert lib.mi355x_malloc(ctypes.byref(s), nb) == 0 and lib.mi355x_malloc(ctypes.byref(r), nb) == 0
    x = torch.full((nb // 4,), float(rank + 1), device="cuda")
    assert lib.mi355x_memcpy(s, ctypes.c_void_p(x.data_ptr()), nb) == 0
    try:
        comm.allreduce(s.value, r.value, nb // 4, pkg.T["FLOAT"], pkg.OP["SUM"])
        y = torch.empty_like(x)
        assert lib.mi355x_memcpy(ctypes.c_void_p(y.data_ptr()), r, nb) == 0
        msg = f"ok={bool(torch.all(y == 3))} s={s.value:#x} r={r.value:#x}"
    except Exception as e:
        msg = f"ERROR {e}"
    print(f"[r{rank}] {kib} KiB sbuf+rbuf: {msg}", file=sys.stderr, flush=True)
    dist.barrier()
    lib.mi355x_free(s); lib.mi355x_free(r)
    comm.destroy()
dist.destroy_process_group()
