#!/usr/bin/env python3
"""Event-record perturbation probe for the N = 1 bench loop: ms per step with HIP events around
every launch, every 4th launch and none (1 GiB 3-buff SUM fp32)."""
import sys, time, torch
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
import bench
pkg = bench.load_pkg(); pkg.rt()
n = (1 << 30) // 4
a = torch.randn(n, device='cuda'); b = torch.randn(n, device='cuda'); o = torch.empty_like(a)
s = torch.cuda.current_stream(); sh = s.cuda_stream
op, ty = pkg.OP["SUM"], pkg.T["FLOAT"]
def run(K, every):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for k in range(K):
        inst = every and k % every == 0
        if inst: ev[k][0].record(s)
        pkg.op_reduce_3buff(op, ty, a.data_ptr(), b.data_ptr(), o.data_ptr(), n, sh)
        if inst: ev[k][1].record(s)
    torch.cuda.synchronize(); wall = time.perf_counter() - t0
    km = [x.elapsed_time(y) for k,(x,y) in enumerate(ev) if every and k % every == 0]
    return wall*1e3/K, (sum(km)/len(km) if km else None)
for _ in range(3): run(20, 1)
for rep in range(3):
    for every in (1, 4, 0):
        print(every, run(20, every))
for every in (1, 4, 0):
    print('K=200', every, run(200, every))
