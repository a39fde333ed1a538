"""What the resident LL service costs a PyTorch-like process, and what it gains it.

Each rank process keeps 4 streams busy with compute (alternating a bandwidth-bound 128 MiB copy and
a compute-bound 4096^3 bf16 matmul, queued ahead) while its main thread issues a small (8 B) allreduce
every `interval` microseconds through the engine -- the pattern of a training loop that
interleaves small collectives (loss / grad-norm scalars) with compute.  Measured per variant and
interval: the compute streams' throughput (kernels per second over their own span, HIP events)
relative to a window of the same compute with no allreduce at all (measured in the same process
pair at the start of every repetition), and the allreduce latency (median / p90), beside the same
calls without compute.

Variants, interleaved in ONE process pair (both ranks on the box's one GPU, so the two processes
also contend with each other; on separate GPUs each process has its GPU to itself), repeated:
  svc_off        SVC_MAX_BYTES = 0: every small call takes the host-synchronised flow
  idle_<t>ms     the service on, leaving after t ms without a call (MI355X_KNOB_SVC_IDLE_US), its
                 workgroups but the first leaving after 100 us (the default, MI355X_KNOB_SVC_SHRINK_US)
  idle_<t>ms_full  the same with the whole grid resident until it leaves (SVC_SHRINK_US = 0)

usage: python tools/svc_interference.py [--out FILE] [--variants svc_off,idle_0.1ms,idle_1ms,idle_5ms]
       [--intervals 50,200,500] [--reps 3]   (default variants: svc_off,idle_0.1ms,idle_1ms,idle_1ms_full,idle_5ms)
"""
import argparse
import json
import os
import subprocess
import sys
import time
import uuid

HERE = os.path.dirname(os.path.abspath(__file__))


def rank_main(rank, key, variants, intervals, window_ms, reps):
    import numpy as np
    import torch
    sys.path.insert(0, os.path.dirname(HERE))
    import bench
    pkg = bench.load_pkg()
    pkg.rt()
    torch.cuda.set_device(0)
    comm = pkg.Comm.create(key, rank, 2, 0)
    f32, SUM = pkg.T["FLOAT"], pkg.OP["SUM"]
    svc_max = comm.get("SVC_MAX_BYTES")
    shrink_default = comm.get("SVC_SHRINK_US")
    streams = [torch.cuda.Stream() for _ in range(4)]
    big = [torch.empty(32 << 20, device="cuda") for _ in range(8)]  # 128 MiB each
    a = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
    outs = [torch.empty(4096, 4096, device="cuda", dtype=torch.bfloat16) for _ in range(4)]
    x = torch.ones(2, device="cuda")
    y = torch.empty_like(x)
    torch.cuda.synchronize()

    def one_kernel(i, k):
        if k % 2:
            big[2 * i + 1].copy_(big[2 * i])
        else:
            torch.matmul(a, b, out=outs[i])

    # kernels per stream for a window of ~window_ms: warm the kernels up (library initialisation),
    # then time whole rounds (one kernel on every stream) with the device synchronised
    for k in range(6):
        for i, st in enumerate(streams):
            with torch.cuda.stream(st):
                one_kernel(i, k)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(10):
        for i, st in enumerate(streams):
            with torch.cuda.stream(st):
                one_kernel(i, k)
    torch.cuda.synchronize()
    per_round_ms = (time.perf_counter() - t0) * 1e3 / 10
    nk = max(20, int(window_ms / per_round_ms))

    def ar_loop(interval, n_ar):
        lat = []
        comm.barrier()  # both ranks start their schedules together
        tstart = time.perf_counter()
        for j in range(n_ar):
            target = tstart + j * interval * 1e-6
            while time.perf_counter() < target:
                pass
            t1 = time.perf_counter()
            comm.allreduce(x.data_ptr(), y.data_ptr(), 2, f32, SUM)
            lat.append((time.perf_counter() - t1) * 1e6)
        return lat, (time.perf_counter() - tstart) * 1e3

    def window(interval):
        comm.barrier()
        ev = []
        for i, st in enumerate(streams):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(st):
                e0.record(st)
                for k in range(nk):
                    one_kernel(i, k)
                e1.record(st)
            ev.append((e0, e1))
        n_ar = int(0.8 * window_ms * 1e3 / interval) if interval else 0
        lat, loop_ms = ar_loop(interval, n_ar) if interval else ([], 0.0)
        torch.cuda.synchronize()
        assert float(y[0].item()) == 2.0 or not interval
        first = ev[0][0]
        span = max(first.elapsed_time(e1) for _, e1 in ev) - min(first.elapsed_time(e0) for e0, _ in ev)
        return 4 * nk / span * 1e3, span, lat, loop_ms

    def apply(var):
        if var == "svc_off":
            comm.set("SVC_MAX_BYTES", 0)
        else:
            full = var.endswith("_full")
            comm.set("SVC_MAX_BYTES", svc_max)
            comm.set("SVC_SHRINK_US", 0 if full else shrink_default)
            comm.set("SVC_IDLE_US", int(float(var[len("idle_"):].split("ms")[0]) * 1000))

    rows = []
    for rep in range(reps):
        base, _, _, _ = window(0)
        for var in (variants if rep % 2 == 0 else variants[::-1]):
            apply(var)
            for interval in intervals:
                alone = ar_loop(interval, min(int(0.8 * window_ms * 1e3 / interval), 1000))[0]
                l0 = comm.get("SVC_LAUNCHES")
                kps, span, lat, loop_ms = window(interval)
                rows.append({"rep": rep, "variant": var, "interval_us": interval, "compute_rel": round(kps / base, 4),
                             "kernels_per_s": round(kps, 1), "baseline_kernels_per_s": round(base, 1),
                             "span_ms": round(span, 2), "ar_loop_ms": round(loop_ms, 2), "ar_calls": len(lat),
                             "ar_us_median": round(float(np.median(lat)), 2), "ar_us_p90": round(float(np.percentile(lat, 90)), 2),
                             "ar_us_median_no_compute": round(float(np.median(alone)), 2),
                             "svc_launches_in_window": comm.get("SVC_LAUNCHES") - l0})
    comm.barrier()
    comm.destroy()
    if rank == 0:
        for r in rows:
            print(json.dumps(r), flush=True)
        for var in variants:
            for interval in intervals:
                sel = [r for r in rows if r["variant"] == var and r["interval_us"] == interval]
                print(json.dumps({"summary": True, "variant": var, "interval_us": interval, "reps": len(sel),
                                  "compute_rel_mean": round(float(np.mean([r["compute_rel"] for r in sel])), 4),
                                  "ar_us_median_mean": round(float(np.mean([r["ar_us_median"] for r in sel])), 2),
                                  "ar_us_p90_mean": round(float(np.mean([r["ar_us_p90"] for r in sel])), 2)}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rank", type=int, default=-1)
    ap.add_argument("--key", default="")
    ap.add_argument("--intervals", default="50,200,500")
    ap.add_argument("--window-ms", type=float, default=400.0)
    ap.add_argument("--variants", default="svc_off,idle_0.1ms,idle_1ms,idle_1ms_full,idle_5ms")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    variants = [v for v in a.variants.split(",") if v]
    intervals = [int(v) for v in a.intervals.split(",") if v]
    if a.rank >= 0:
        return rank_main(a.rank, a.key, variants, intervals, a.window_ms, a.reps)
    key = "int" + uuid.uuid4().hex[:10]
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__), "--rank", str(r), "--key", key,
                               "--intervals", a.intervals, "--window-ms", str(a.window_ms), "--variants", a.variants,
                               "--reps", str(a.reps)],
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True) for r in range(2)]
    outs = [p.communicate(timeout=900)[0] for p in procs]
    if any(p.returncode for p in procs):
        sys.stderr.write("\n".join(outs))
        sys.exit(1)
    lines = [ln for ln in outs[0].splitlines() if ln.startswith("{")]
    if a.out:
        with open(a.out, "a") as f:
            f.write("\n".join(lines) + "\n")
    print("\n".join(lines), flush=True)


if __name__ == "__main__":
    main()
