#!/usr/bin/env python3
"""Launch-shape sweep of the row pack/unpack kernel on the configs[4] layout
(MPI_Type_vector(2^22, 64, 128, MPI_FLOAT), 1 GiB packed): unroll x non-temporal mask."""
from __future__ import annotations

import json
import pathlib
import sys

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
sys.path.insert(0, str(pathlib.Path(__file__).resolve().parent))


def main():
    import torch
    import bench
    from bench_legs import timed
    pkg = bench.load_pkg()
    pkg.rt()
    nblk = 1 << 22
    d = pkg.Ddt.vector(nblk, 64, 128, 4)
    x = torch.randn(nblk, 128, device="cuda")
    p = torch.empty(nblk, 64, device="cuda")
    y = torch.zeros_like(x)
    alg = 2 * d.size
    best = {}
    for threads in (256, 512, 1024):
        for unroll in (2, 4, 8):
            for nt in (0, 1, 2, 3):
                pkg.ddt_tune(unroll, unroll, threads, nt)
                for name, fn in (("pack", lambda s: d.pack(1, x.data_ptr(), 0, p.data_ptr(), d.size, s)),
                                 ("unpack", lambda s: d.unpack(1, y.data_ptr(), 0, p.data_ptr(), d.size, s))):
                    avg, _ = timed(torch, fn, 20, 3)
                    gbs = alg / (avg * 1e-3) / 1e9
                    print(json.dumps({"dir": name, "threads": threads, "unroll": unroll, "nt": nt,
                                      "ms": round(avg, 5), "GBs": round(gbs, 1)}), flush=True)
                    if gbs > best.get(name, (0,))[0]:
                        best[name] = (gbs, threads, unroll, nt)
    assert torch.equal(p, x[:, :64]) and torch.equal(y[:, :64], x[:, :64])
    print("BEST", json.dumps(best))


if __name__ == "__main__":
    main()
