#!/usr/bin/env python3
"""Single-GPU legs of BASELINE.json beyond bench.py's headline line:

  op     configs[1] sweep: op/hip 3-buff (and 2-buff) over every (op, type) the config names,
         1 GiB per operand; roofline bound HBM, algorithmic bytes = 3 x 1 GiB per launch.
  ddt    configs[4] convertor: MPI_Type_vector(2^22, 64, 128, MPI_FLOAT) (1 GiB packed, 2 GiB
         extent) pack / unpack / pack+checksum; algorithmic bytes = 2 x packed bytes per launch.

Each measurement is one JSON object (one per line) on stdout and in --out.  Kernel time is taken
with HIP events on the stream the kernel is launched on (torch's current stream, passed to the C
ABI explicitly).  CPU baselines time the oracle (the restated reference loop) on a bounded sample.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import pathlib
import sys
import time

REPO = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
HBM_PEAK_GBS = 8000.0
GIB = 1 << 30

SWEEP = {
    "SUM": ["INT8", "UINT8", "INT16", "UINT16", "INT32", "UINT32", "INT64", "UINT64",
            "FLOAT", "DOUBLE", "C_FLOAT_COMPLEX", "C_DOUBLE_COMPLEX"],
    "PROD": ["INT8", "INT32", "INT64", "FLOAT", "DOUBLE", "C_FLOAT_COMPLEX", "C_DOUBLE_COMPLEX"],
    "MAX": ["INT8", "INT16", "INT32", "INT64", "UINT64", "FLOAT", "DOUBLE"],
    "MIN": ["INT32", "FLOAT", "DOUBLE"],
    "BAND": ["INT8", "INT32", "INT64", "BYTE"],
    "MAXLOC": ["FLOAT_INT", "DOUBLE_INT", "LONG_INT", "2INT", "SHORT_INT"],
}


def timed(torch, fn, steps, warmup):
    s = torch.cuda.current_stream()
    for _ in range(warmup):
        fn(s.cuda_stream)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    torch.cuda.synchronize()
    for a, b in ev:
        a.record(s)
        fn(s.cuda_stream)
        b.record(s)
    torch.cuda.synchronize()
    ms = sorted(a.elapsed_time(b) for a, b in ev)
    return sum(ms) / len(ms), ms[len(ms) // 2]


def leg_op(pkg, torch, args, emit):
    a = torch.empty(GIB, dtype=torch.uint8, device="cuda")
    b = torch.empty_like(a)
    o = torch.empty_like(a)
    a.view(torch.float32).normal_()
    b.view(torch.float32).normal_()
    for opname, types in SWEEP.items():
        for tname in types:
            op, ty = pkg.OP[opname], pkg.T[tname]
            esz = pkg.type_size(ty)
            n = GIB // esz
            avg, med = timed(torch, lambda s: pkg.op_reduce_3buff(op, ty, a.data_ptr(), b.data_ptr(), o.data_ptr(),
                                                                  n, s), args.steps, args.warmup)
            alg = 3 * n * esz
            emit({"leg": "op_3buff", "op": opname, "type": tname, "count": n, "alg_bytes": alg,
                  "kernel_avg_ms": round(avg, 5), "kernel_med_ms": round(med, 5),
                  "achieved_GBs": round(alg / (avg * 1e-3) / 1e9, 1),
                  "frac": round(alg / (avg * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)})
    for tname in ["FLOAT", "DOUBLE", "INT32"]:
        op, ty = pkg.OP["SUM"], pkg.T[tname]
        n = GIB // pkg.type_size(ty)
        avg, med = timed(torch, lambda s: pkg.op_reduce(op, ty, a.data_ptr(), o.data_ptr(), n, s),
                         args.steps, args.warmup)
        alg = 3 * GIB
        emit({"leg": "op_2buff", "op": "SUM", "type": tname, "count": n, "alg_bytes": alg,
              "kernel_avg_ms": round(avg, 5), "kernel_med_ms": round(med, 5),
              "achieved_GBs": round(alg / (avg * 1e-3) / 1e9, 1),
              "frac": round(alg / (avg * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)})
    # torch's own elementwise add on the same bytes, as a reference point for the machine
    af, bf, of = a.view(torch.float32), b.view(torch.float32), o.view(torch.float32)
    avg, med = timed(torch, lambda s: torch.add(af, bf, out=of), args.steps, args.warmup)
    emit({"leg": "torch_add_ref", "type": "FLOAT", "alg_bytes": 3 * GIB, "kernel_avg_ms": round(avg, 5),
          "achieved_GBs": round(3 * GIB / (avg * 1e-3) / 1e9, 1)})
    del a, b, o


def leg_ddt(pkg, torch, args, emit, oracle):
    nblk = 1 << 22
    d = pkg.Ddt.vector(nblk, 64, 128, 4)
    x = torch.randn(nblk, 128, device="cuda")
    p = torch.empty(nblk, 64, device="cuda")
    y = torch.zeros_like(x)
    size = d.size
    assert size == GIB
    alg = 2 * size

    def pack(s):
        d.pack(1, x.data_ptr(), 0, p.data_ptr(), size, s)

    def unpack(s):
        d.unpack(1, y.data_ptr(), 0, p.data_ptr(), size, s)

    for name, fn in [("pack", pack), ("unpack", unpack)]:
        avg, med = timed(torch, fn, args.steps, args.warmup)
        emit({"leg": "ddt_" + name, "type": "vector(2^22,64,128,FLOAT)", "alg_bytes": alg,
              "kernel_avg_ms": round(avg, 5), "kernel_med_ms": round(med, 5),
              "achieved_GBs": round(alg / (avg * 1e-3) / 1e9, 1),
              "frac": round(alg / (avg * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)})
    assert torch.equal(p, x[:, :64]) and torch.equal(y[:, :64], x[:, :64])
    # with the convertor checksum (one host round trip per call: the checksum is returned)
    for _ in range(2):  # warm-up: the first call sets up the checksum workspace
        d.pack(1, x.data_ptr(), 0, p.data_ptr(), size, torch.cuda.current_stream().cuda_stream, checksum=True)
    t0 = time.perf_counter()
    reps = max(5, args.steps // 2)
    for _ in range(reps):
        d.pack(1, x.data_ptr(), 0, p.data_ptr(), size, torch.cuda.current_stream().cuda_stream, checksum=True)
    dt = (time.perf_counter() - t0) / reps
    # device time of the same call (events bracket the launch on the call's stream; the call
    # itself waits for its kernel, so the host round trip is not inside the bracket)
    kavg, _ = timed(torch, lambda s: d.pack(1, x.data_ptr(), 0, p.data_ptr(), size, s, checksum=True), reps, 1)
    emit({"leg": "ddt_pack_checksum", "type": "vector(2^22,64,128,FLOAT)", "alg_bytes": alg,
          "wall_ms": round(dt * 1e3, 4), "achieved_GBs": round(alg / dt / 1e9, 1),
          "kernel_avg_ms": round(kavg, 5), "kernel_GBs": round(alg / (kavg * 1e-3) / 1e9, 1),
          "frac": round(alg / (kavg * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)})
    # torch strided copy of the same view, as a reference point
    avg, _ = timed(torch, lambda s: p.copy_(x[:, :64]), args.steps, args.warmup)
    emit({"leg": "torch_strided_copy_ref", "alg_bytes": alg, "kernel_avg_ms": round(avg, 5),
          "achieved_GBs": round(alg / (avg * 1e-3) / 1e9, 1)})
    avg, _ = timed(torch, lambda s: y[:, :64].copy_(p), args.steps, args.warmup)  # the unpack direction
    emit({"leg": "torch_strided_unpack_ref", "alg_bytes": alg, "kernel_avg_ms": round(avg, 5),
          "achieved_GBs": round(alg / (avg * 1e-3) / 1e9, 1)})
    del x, p, y
    if oracle is not None and not args.no_cpu_baseline:
        import numpy as np
        nb = 1 << 18  # 64 MiB packed sample of the same layout
        od = oracle.oracle_ddt_vector(nb, 64, 128, 4)
        src = np.random.default_rng(3).standard_normal(nb * 128, dtype=np.float32)
        dst = np.empty(nb * 64, dtype=np.float32)
        oracle.oracle_ddt_pack_runs(od, 1, src.ctypes.data, dst.ctypes.data)
        reps, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < args.cpu_seconds:
            oracle.oracle_ddt_pack_runs(od, 1, src.ctypes.data, dst.ctypes.data)
            reps += 1
        el = time.perf_counter() - t0
        emit({"leg": "ddt_pack_cpu_baseline", "kind": "port", "cores": 1,
              "sample": f"oracle_ddt_pack_runs vector(2^18,64,128,FLOAT) 64 MiB packed x {reps}",
              "achieved_GBs": round(2 * nb * 256 * reps / el / 1e9, 2)})
        oracle.oracle_ddt_free(od)


def leg_ddt_narrow(pkg, torch, args, emit):
    """vector layouts whose runs are not 16-B multiples (a column of doubles, 3-float blocks),
    256 MiB packed: the row kernel with narrow slots (mi355x_ddt_tune_rows 2) vs the general
    kernel (0) vs torch's strided copy of the same view.  alg_bytes = 2 x packed; the strided side
    moves whole 128-B lines, so a column's reads cost 2 x its packed bytes of HBM traffic."""
    cases = [("vector(2^25,1,2,DOUBLE)", (1 << 25, 1, 2, 8), torch.float64, 2, 1),
             ("vector(22369621,3,4,FLOAT)", (22369621, 3, 4, 4), torch.float32, 4, 3)]
    for name, vargs, dt, width, take in cases:
        d = pkg.Ddt.vector(*vargs)
        x = torch.randn(vargs[0], width, device="cuda", dtype=dt)
        p = torch.empty(vargs[0], take, device="cuda", dtype=dt)
        y = torch.zeros_like(x)
        size = d.size
        alg = 2 * size
        for mode in (2, 0):
            pkg.ddt_tune_rows(mode)
            for dirn, fn in (("pack", lambda s: d.pack(1, x.data_ptr(), 0, p.data_ptr(), size, s)),
                             ("unpack", lambda s: d.unpack(1, y.data_ptr(), 0, p.data_ptr(), size, s))):
                avg, med = timed(torch, fn, args.steps, args.warmup)
                emit({"leg": "ddt_narrow_" + dirn, "type": name, "kernel": "rows" if mode == 2 else "general",
                      "alg_bytes": alg, "kernel_avg_ms": round(avg, 5), "kernel_med_ms": round(med, 5),
                      "achieved_GBs": round(alg / (avg * 1e-3) / 1e9, 1),
                      "frac": round(alg / (avg * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)})
            assert torch.equal(p, x[:, :take]) and torch.equal(y[:, :take], x[:, :take]), (name, mode)
            y.zero_()
        pkg.ddt_tune_rows(2)
        for dirn, fn in (("pack", lambda s: p.copy_(x[:, :take])), ("unpack", lambda s: y[:, :take].copy_(p))):
            avg, _ = timed(torch, fn, args.steps, args.warmup)
            emit({"leg": "torch_strided_ref_" + dirn, "type": name, "alg_bytes": alg, "kernel_avg_ms": round(avg, 5),
                  "achieved_GBs": round(alg / (avg * 1e-3) / 1e9, 1)})
        del x, p, y


def leg_ddt_runs(pkg, torch, args, emit):
    """run-list layouts (several runs per block), 256 MiB packed: the unit kernel (LDS-staged run
    tables; mi355x_ddt_tune_rows 2) vs the general kernel (0).  Upper triangle of a 256 x 256
    double matrix (indexed, 256 runs per instance) and a 7-run indexed float layout."""
    import numpy as np
    tri_bl = [256 - i for i in range(256)]
    tri_dp = [257 * i for i in range(256)]
    f7_bl, f7_dp = [1, 3, 2, 7, 1, 1, 4], [0, 2, 9, 13, 25, 27, 40]
    cases = [("indexed upper-triangle 256x256 DOUBLE", tri_bl, tri_dp, 8),
             ("indexed 7 runs of FLOAT (19 of 44 elements)", f7_bl, f7_dp, 4)]
    for name, bl, dp, esz in cases:
        d = pkg.Ddt.indexed(bl, dp, esz)
        ext = (max(a + b for a, b in zip(dp, bl)) - min(dp)) * esz
        count = (256 << 20) // d.size
        x = torch.randint(0, 255, (count * ext,), dtype=torch.uint8, device="cuda")
        p = torch.empty(count * d.size, dtype=torch.uint8, device="cuda")
        y = torch.zeros_like(x)
        size = count * d.size
        alg = 2 * size
        outs = {}
        for mode in (2, 3, 0):
            pkg.ddt_tune_rows(mode)
            for dirn, fn in (("pack", lambda s: d.pack(count, x.data_ptr(), 0, p.data_ptr(), size, s)),
                             ("unpack", lambda s: d.unpack(count, y.data_ptr(), 0, p.data_ptr(), size, s))):
                avg, med = timed(torch, fn, args.steps, args.warmup)
                emit({"leg": "ddt_runs_" + dirn, "type": name, "kernel": {2: "units", 3: "units_w", 0: "general"}[mode],
                      "count": count, "alg_bytes": alg, "kernel_avg_ms": round(avg, 5), "kernel_med_ms": round(med, 5),
                      "achieved_GBs": round(alg / (avg * 1e-3) / 1e9, 1),
                      "frac": round(alg / (avg * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)})
            outs[mode] = (p.clone(), y.clone())
            y.zero_()
        for mode in (2, 3):
            assert torch.equal(outs[mode][0], outs[0][0]) and torch.equal(outs[mode][1], outs[0][1]), (name, mode)
        pkg.ddt_tune_rows(2)
        # the same unpack through 4 convertor windows (set_position fragments at unaligned run
        # offsets: the wave-per-run kernel clips the first and last run of each window)
        cuts = [0] + [(size * i // 4) // (2 * esz) * (2 * esz) + esz for i in (1, 2, 3)] + [size]

        def windows(s):
            for lo, hi in zip(cuts[:-1], cuts[1:]):
                d.unpack(count, y.data_ptr(), lo, p.data_ptr() + lo, hi - lo, s)
        for mode in (2, 3):  # 3: W-byte units only (what windows took before the wave-per-run kernel clipped runs)
            pkg.ddt_tune_rows(mode)
            y.zero_()
            avg, med = timed(torch, windows, args.steps, args.warmup)
            emit({"leg": "ddt_runs_unpack_windows4", "type": name, "kernel": {2: "units", 3: "units_w"}[mode],
                  "count": count, "alg_bytes": alg, "kernel_avg_ms": round(avg, 5), "kernel_med_ms": round(med, 5),
                  "achieved_GBs": round(alg / (avg * 1e-3) / 1e9, 1),
                  "frac": round(alg / (avg * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)})
            assert torch.equal(y, outs[0][1]), (name, "windows", mode)
        pkg.ddt_tune_rows(2)
        del x, p, y, outs


def leg_cpu_allreduce(args, emit, oracle):
    """BASELINE configs[0]: the reference CPU path (coll/tuned segmented ring over sm-BTL-style
    32 KiB shared-memory fragments), 4 ranks on 4 distinct host cores, MPI_SUM MPI_FLOAT 16 M
    elements (64 MiB) per rank; busbw = S/t * 2(n-1)/n."""
    import os
    import numpy as np
    n, count = 4, 16 * 1024 * 1024
    xs = []
    for r in range(n):  # exactly representable values -> order-independent, checkable sum
        i = np.arange(count, dtype=np.uint64)
        xs.append(((((i * 2654435761 + r * 40503) & 0xFFFF).astype(np.int64) - 32768) / 256.0).astype(np.float32))
    outs = [np.empty_like(xs[0]) for _ in range(n)]
    P = lambda arrs: (ctypes.c_void_p * n)(*[a.ctypes.data for a in arrs])
    cores = sorted(os.sched_getaffinity(0))
    core0 = cores[0] if len(cores) >= n and cores[n - 1] - cores[0] == n - 1 else -1
    t = ctypes.c_double()
    rc = oracle.oracle_cpu_allreduce(n, count, 14, 3, 1 << 20, P(xs), P(outs), args.cpu_reps, core0, ctypes.byref(t))
    assert rc == 0
    want = xs[0] + xs[1] + xs[2] + xs[3]
    ok = all(np.array_equal(o, want) for o in outs)
    S = count * 4
    emit({"leg": "cpu_allreduce_baseline", "config": "BASELINE configs[0]", "kind": "port", "cores": n,
          "pinned": core0 >= 0, "sample": f"np=4 segmented ring 1 MiB segments, 32 KiB fragments, {args.cpu_reps} calls",
          "count": count, "sec_per_call": round(t.value, 5), "algbw_GBs": round(S / t.value / 1e9, 3),
          "busbw_GBs": round(S / t.value * 2 * (n - 1) / n / 1e9, 3), "exact": ok,
          "cpu": _cpu_model()})


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--legs", default="op,ddt")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--out", default="gpurun_out/legs.jsonl")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=5.0)
    ap.add_argument("--cpu-reps", type=int, default=5)
    args = ap.parse_args()
    legs = args.legs.split(",")
    import bench
    pkg = bench.load_pkg()
    torch = None
    if "op" in legs or any(l.startswith("ddt") for l in legs):
        import torch
        pkg.rt()
    oracle = None
    so = REPO / "oracle" / "build" / "liboracle.so"
    if so.exists():
        sys.path.insert(0, str(REPO / "tests"))
        from conftest import load_oracle
        oracle = load_oracle()
    out = pathlib.Path(args.out)
    out.parent.mkdir(parents=True, exist_ok=True)
    fh = out.open("w")

    def emit(rec):
        line = json.dumps(rec)
        print(line, flush=True)
        fh.write(line + "\n")
        fh.flush()

    if "op" in legs:
        leg_op(pkg, torch, args, emit)
    if "ddt" in legs:
        leg_ddt(pkg, torch, args, emit, oracle)
    if "ddt_narrow" in legs:
        leg_ddt_narrow(pkg, torch, args, emit)
    if "ddt_runs" in legs:
        leg_ddt_runs(pkg, torch, args, emit)
    if "cpu_ar" in legs:
        leg_cpu_allreduce(args, emit, oracle)
    fh.close()


if __name__ == "__main__":
    main()
