"""Debug: which allocation sizes hipIpcOpenMemHandle maps (2 ranks, one-GPU rehearsal)."""
import datetime, faulthandler, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, torch.distributed as dist
import bench
pkg = bench.load_pkg(); pkg.rt()
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=90))
torch.cuda.set_device(0)
comm = pkg.Comm.create("dbgipc_" + os.environ.get("MASTER_PORT", "0"), rank, world, 0)
comm.set("TIMEOUT_S", 40)
for mib in [int(v) for v in os.environ.get("DBG_MIB", "2046,2048").split(",")]:
    faulthandler.dump_traceback_later(30, exit=True)
    big = torch.zeros((mib << 20,), dtype=torch.uint8, device="cuda")
    src = torch.full((8,), rank + 1, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    comm.allgather(src.data_ptr(), big.data_ptr(), 8)
    torch.cuda.synchronize()
    print(f"[r{rank}] {mib} MiB ok={big[:16].tolist()}", file=sys.stderr, flush=True)
    del big
    torch.cuda.empty_cache()
comm.destroy()
dist.destroy_process_group()
