#!/usr/bin/env python3
"""Benchmark of the MI355X collective-reduction path.

Metric (BASELINE.json): "MPI_Allreduce busbw GB/s (1 GiB fp32, np=8) + op/hip reduce HBM GB/s".

  N = 1  (configs[1]): op/hip 3-buff MPI_SUM over MPI_FLOAT, 1 GiB per operand, device-resident.
         value = algorithmic HBM GB/s = 3 x 2^30 B x steps / time.
  N > 1  (configs[2] at 1 GiB): MPI_Allreduce MPI_SUM fp32 1 GiB per rank through coll/mi355x's
         engine over IPC-mapped peers; value = busbw = (S/t) x 2(n-1)/n, max time over ranks.

Launch: `python bench.py --gpus N --steps K --warmup W`.  N > 1 runs one rank per GPU: under
torch.distributed.run as the driver launches it, or -- with no launcher environment -- bench.py starts
torch.distributed.run itself as a child process and forwards rank 0's line (spawn_ranks).
Rank 0 prints ONE JSON line.  Timed region = exactly K steps between barrier+synchronize pairs.
"""
from __future__ import annotations

import argparse
import ctypes
import importlib.util
import json
import os
import pathlib
import sys
import time

REPO = pathlib.Path(__file__).resolve().parent
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md
GIB = 1 << 30


def load_pkg():
    name = "ompi_release_amd"
    if name in sys.modules:
        return sys.modules[name]
    spec = importlib.util.spec_from_file_location(name, REPO / "ompi-release_amd" / "__init__.py")
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def pmc_traffic(kernel_key: str):
    """(HBM bytes per launch, the profiles/ file it is read from) from the newest committed
    rocprofv3 PMC summary holding the kernel (corrected per MI355X_MICROARCH.md §HBM: FETCH_SIZE x 2
    for 16-B streaming reads), or (None, None)."""
    for p in sorted((REPO / "profiles").glob("*pmc*.json"), reverse=True):
        try:
            d = json.loads(p.read_text())
        except Exception:
            continue
        ent = d.get("kernels", {}).get(kernel_key)
        if ent and "hbm_bytes_per_launch" in ent:
            return ent["hbm_bytes_per_launch"], f"profiles/{p.name}"
    return None, None


def cpu_baseline_op(target_s: float = 10.0):
    """oracle (restated reference op loop, -O3 like the reference build) timed on this host:
    3-buff MPI_SUM fp32, single core, on a 64 MiB-per-operand sample of the same workload."""
    so = REPO / "oracle" / "build" / "liboracle.so"
    if not so.exists():
        return None
    import numpy as np
    lib = ctypes.CDLL(str(so))
    lib.oracle_op_3buff.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_void_p, ctypes.c_size_t]
    n = 1 << 24
    rng = np.random.default_rng(1)
    a = rng.standard_normal(n, dtype=np.float32)
    b = rng.standard_normal(n, dtype=np.float32)
    o = np.empty_like(a)
    lib.oracle_op_3buff(3, 14, a.ctypes.data, b.ctypes.data, o.ctypes.data, n)  # warm
    reps, t0 = 0, time.perf_counter()
    while True:
        lib.oracle_op_3buff(3, 14, a.ctypes.data, b.ctypes.data, o.ctypes.data, n)
        reps += 1
        el = time.perf_counter() - t0
        if el >= target_s:
            break
    gbs = 3.0 * n * 4 * reps / el / 1e9
    out = {"value": round(gbs, 3), "unit": "GB/s", "cores": 1, "kind": "port",
           "sample": f"oracle_op_3buff SUM FLOAT, 2^24 elems (64 MiB/operand) x {reps} reps, {el:.1f} s"}
    # the same loop on the host cores this box grants a GPU job (16; BASELINE.md section 3, C2
    # "single-core and all-cores"), on 256 MiB operands (beyond the host caches)
    try:
        lib.oracle_op_3buff_mt.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        threads = max(1, min(16, os.cpu_count() or 1))
        n2 = 1 << 26
        a2 = np.resize(a, n2)
        b2 = np.resize(b, n2)
        o2 = np.empty_like(a2)
        lib.oracle_op_3buff_mt(3, 14, a2.ctypes.data, b2.ctypes.data, o2.ctypes.data, n2, threads)
        reps2, t0 = 0, time.perf_counter()
        while True:
            lib.oracle_op_3buff_mt(3, 14, a2.ctypes.data, b2.ctypes.data, o2.ctypes.data, n2, threads)
            reps2 += 1
            el2 = time.perf_counter() - t0
            if el2 >= target_s / 2:
                break
        out["all_cores"] = {"value": round(3.0 * n2 * 4 * reps2 / el2 / 1e9, 3), "cores": threads,
                            "sample": f"oracle_op_3buff_mt, 2^26 elems (256 MiB/operand) x {reps2} reps, {el2:.1f} s"}
    except Exception as e:  # baseline detail only
        out["all_cores"] = {"error": repr(e)[:200]}
    return out


def bench_op(args, pkg, torch):
    """N = 1: op/hip 3-buff SUM fp32, 1 GiB per operand."""
    n = GIB // 4
    dev = torch.device("cuda", 0)
    a = torch.randn(n, device=dev, dtype=torch.float32)
    b = torch.randn(n, device=dev, dtype=torch.float32)
    o = torch.empty_like(a)
    s = torch.cuda.current_stream()
    sh = s.cuda_stream
    op, ty = pkg.OP["SUM"], pkg.T["FLOAT"]
    pa, pb, po = a.data_ptr(), b.data_ptr(), o.data_ptr()
    for _ in range(args.warmup):
        pkg.op_reduce_3buff(op, ty, pa, pb, po, n, sh)
    torch.cuda.synchronize()
    # parity spot-check of the measured kernel on the real size (size-independent property)
    assert torch.equal(o, a + b), "op/hip SUM result differs from a + b"
    # One HIP event pair on the launch stream brackets the K launches of the timed region; the
    # kernel's average = their span / K (it includes the ~1.5 us launch boundaries, so it bounds
    # the kernel's own time from above; rocprofv3's per-launch average agrees within 1 %).  An
    # event pair around every launch would add ~7 us per step to the wall clock (0.500 vs 0.493 ms,
    # tools/ev_probe.py) and slow the bracketed launches themselves by ~1 %.
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    graph = None
    if args.graph:
        # --graph: the K launches captured once into a HIP graph (one kernel node per step, every
        # step the full 1 GiB reduction) and replayed as one submission in the timed region
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            gs = torch.cuda.current_stream().cuda_stream
            for _ in range(args.steps):
                pkg.op_reduce_3buff(op, ty, pa, pb, po, n, gs)
        graph.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record(s)
    if graph is not None:
        graph.replay()
    else:
        for _ in range(args.steps):
            pkg.op_reduce_3buff(op, ty, pa, pb, po, n, sh)
    e1.record(s)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    avg_ms = e0.elapsed_time(e1) / args.steps
    alg_bytes = 3 * n * 4
    value = alg_bytes * args.steps / wall / 1e9
    achieved = alg_bytes / (avg_ms * 1e-3) / 1e9
    traffic, traffic_from = pmc_traffic("op_3buff_sum_float")
    u, bpc, nt = pkg.get_tune()
    config = {"workload": "op/hip 3-buff MPI_SUM MPI_FLOAT, 1 GiB per operand (BASELINE configs[1])",
              "count": n, "bytes_per_operand": n * 4, "launch": {"unroll": u, "blocks_per_cu": bpc,
                                                                  "nontemporal": nt}}
    if not args.no_sweep:
        # the rest of configs[1] (every slot, both forms), timed after the headline's region
        config["sweep"] = sweep_op(pkg, torch, a, b, o)
    return {
        "metric": "MPI_Allreduce busbw GB/s (1 GiB fp32, np=8) + op/hip reduce HBM GB/s",
        "value": round(value, 2),
        "unit": "GB/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(wall * 1e3 / args.steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (torch.randn on device)",
        "config": config,
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_from": traffic_from,
                     "kernel_avg_ms": round(avg_ms, 5),
                     "kernel_avg_from": "HIP events around the K launches / K" + (" (one HIP graph replay)" if graph is not None else ""),
                     "alg_bytes_per_launch": alg_bytes},
    }


# 2 reads + 1 write cannot beat 3 / (2/6.9 + 1/6.2) TB/s on this machine: the measured read-only
# and write-only stream rates (tools/op_ceiling.hip, profiles/r02_op_ceiling.jsonl)
OP_CEILING_GBS = 6640.0


def fill_x87(torch, bufs):
    """Valid x87 extended values in every 16-B unit: significand with its integer bit set, exponent
    0x3fff +- 16, random sign (the padding bytes 10..15 zero).  Used for the long double slots, whose
    integer-arithmetic kernels take a different path for the invalid encodings random bits produce."""
    g = torch.Generator(device=bufs[0].device)
    g.manual_seed(87)
    for t in bufs:
        w = t.view(torch.int64).view(-1, 2)
        w[:, 0] = torch.randint(-2**63, 2**63 - 1, (w.shape[0],), device=t.device, dtype=torch.int64,
                                generator=g) | (-2**63)
        e = torch.randint(0x3fff - 16, 0x3fff + 17, (w.shape[0],), device=t.device, dtype=torch.int64,
                          generator=g)
        sgn = torch.randint(0, 2, (w.shape[0],), device=t.device, dtype=torch.int64, generator=g)
        w[:, 1] = e | (sgn << 15)
    torch.cuda.synchronize()


def sweep_op(pkg, torch, a, b, o, reps: int = 5):
    """BASELINE configs[1] as a whole: every op/hip GPU slot (op x predefined type), 2-buff and
    3-buff, on 1 GiB per operand (the headline's buffers re-typed), after the headline's timed
    region.  Per slot and form: one untimed launch, then `reps` launches between one HIP event pair
    on the launch stream (span / reps).  Algorithmic bytes = 3 x 2^30 per launch for both forms
    (2-buff: read in, read + write inout; op_base_functions.c:39-103 / 606-683)."""
    s = torch.cuda.current_stream()
    sh = s.cuda_stream
    pa, pb, po = a.data_ptr(), b.data_ptr(), o.data_ptr()
    nbytes = a.numel() * a.element_size()
    rows = []
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    x87 = [i for i, t in enumerate(pkg.TYPES) if "LONG_DOUBLE" in t]
    order = [t for t in range(len(pkg.TYPES)) if t not in x87] + x87
    refilled = False
    for ty in order:
        for op in range(1, len(pkg.OPS)):
            if not pkg.op_supported(op, ty):
                continue
            if ty in x87 and not refilled:
                fill_x87(torch, (a, b, o))
                refilled = True
            n = nbytes // pkg.type_size(ty)
            res = {}
            for form in ("2buff", "3buff"):
                if form == "3buff":
                    f = lambda: pkg.op_reduce_3buff(op, ty, pa, pb, po, n, sh)
                else:
                    f = lambda: pkg.op_reduce(op, ty, pa, po, n, sh)
                f()
                e0.record(s)
                for _ in range(reps):
                    f()
                e1.record(s)
                e1.synchronize()
                ms = e0.elapsed_time(e1) / reps
                res[form] = round(3 * n * pkg.type_size(ty) / (ms * 1e-3) / 1e9, 1)
            rows.append((pkg.OPS[op], pkg.TYPES[ty], pkg.type_size(ty), res["2buff"], res["3buff"]))

    def summary(idx):
        vals = sorted(r[idx] for r in rows)
        worst = min(rows, key=lambda r: r[idx])
        med = vals[len(vals) // 2] if len(vals) % 2 else 0.5 * (vals[len(vals) // 2 - 1] + vals[len(vals) // 2])
        return {"min_GBps": vals[0], "median_GBps": round(med, 1), "max_GBps": vals[-1],
                "worst": {"slot": f"{worst[0]}/{worst[1]}", "GBps": worst[idx],
                          "frac_peak": round(worst[idx] / HBM_PEAK_GBS, 4),
                          "frac_ceiling": round(worst[idx] / OP_CEILING_GBS, 4)},
                "slots_below_0.90_ceiling": [f"{r[0]}/{r[1]}" for r in rows if r[idx] < 0.9 * OP_CEILING_GBS]}

    return {"slots": len(rows), "bytes_per_operand": nbytes, "reps": reps,
            "x87_data": "the long double slots run last, on operands refilled with valid x87 encodings "
                        "(explicit integer bit, exponent within 2^+-16, random sign and significand): "
                        "the headline's fp32 bits read as x87 values are half invalid encodings",
            "ceiling_2r1w_GBps": OP_CEILING_GBS, "ceiling_from": "profiles/r02_op_ceiling.jsonl",
            "two_buff": summary(3), "three_buff": summary(4),
            "table": {f"{r[0]}/{r[1]}": [r[3], r[4]] for r in rows},
            "table_columns": ["GBps_2buff", "GBps_3buff"]}


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(nproc: int, script: str, script_args: list[str]) -> int:
    """`bench.py --gpus N` (N > 1) started without a launcher: start the N ranks the way the driver
    does (`python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1`),
    as a CHILD process -- never an exec, and before this process has touched the GPU -- forward rank
    0's JSON line to stdout and return the child's exit code.  mpirun launches its own ranks the
    same way (orte/tools/orterun/orterun.c:611)."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", script, *script_args]
    env = dict(os.environ)
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, env=env, text=True, bufsize=1)
    for line in proc.stdout:  # rank 0 prints the one JSON line; anything else is progress
        s = line.strip()
        if s.startswith("{") and '"metric"' in s:
            print(s, flush=True)
        elif s:
            print(s, file=sys.stderr, flush=True)
    return proc.wait()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--graph", action="store_true", help="N = 1: replay the K timed launches as one HIP graph")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-sweep", action="store_true", help="N = 1: skip the configs[1] slot sweep")
    ap.add_argument("--no-legs", action="store_true", help="N > 1: skip the other configs' legs")
    ap.add_argument("--no-autotune", action="store_true",
                    help="N > 1: time the engine's default allreduce flow only (for profiling one configuration)")
    ap.add_argument("--legs-timeout", type=float, default=300.0,
                    help="N > 1: seconds after which the legs are abandoned and the headline printed")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no launcher: start the ranks ourselves (child process, nothing GPU-side touched yet)
        sys.exit(spawn_ranks(args.gpus, str(pathlib.Path(__file__).resolve()), sys.argv[1:]))

    import torch
    pkg = load_pkg()
    pkg.rt()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1 or args.gpus > 1:
        import bench_coll  # allreduce engine bench (N > 1)
        res = bench_coll.run(args, pkg, torch)
        if res is None:
            return
    else:
        res = bench_op(args, pkg, torch)
        res["cpu_baseline"] = None if args.no_cpu_baseline else cpu_baseline_op(args.cpu_seconds)
    print(json.dumps(res), flush=True)
    if res.get("value") is None:  # a failed exactness check or a hung leg: not a valid measurement
        sys.exit(2)


if __name__ == "__main__":
    main()
