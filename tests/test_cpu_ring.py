"""The CPU baseline of BASELINE configs[0] (oracle/cpu_ring.c: the segmented ring over 32 KiB
shared-memory fragments, n concurrent ranks) computes exactly what the schedule simulation
oracle_allreduce computes -- two independent restatements of coll_tuned_allreduce.c agree."""
from __future__ import annotations

import ctypes

import numpy as np
import pytest

import opdata


@pytest.mark.parametrize("n,count,segsize,alg", [(4, 3_000_001, 1 << 20, 5), (4, 70_001, 1 << 20, 4),
                                                  (3, 1_500_000, 1 << 18, 5), (2, 17, 0, 4), (5, 999_999, 0, 4)])
@pytest.mark.parametrize("opname,tname", [("SUM", "FLOAT"), ("MAX", "INT32"), ("PROD", "DOUBLE")])
def test_cpu_ring_matches_schedule(oracle, pkg, n, count, segsize, alg, opname, tname):
    op, ty = pkg.OP[opname], pkg.T[tname]
    xs = [opdata.make(tname, count, 900 + r) for r in range(n)]
    want = [np.zeros_like(xs[0]) for _ in range(n)]
    got = [np.zeros_like(xs[0]) for _ in range(n)]
    P = lambda arrs: (ctypes.c_void_p * n)(*[a.ctypes.data for a in arrs])
    assert oracle.oracle_allreduce(alg, n, count, ty, op, segsize, P(xs), P(want)) == alg
    t = ctypes.c_double()
    assert oracle.oracle_cpu_allreduce(n, count, ty, op, segsize, P(xs), P(got), 1, -1, ctypes.byref(t)) == 0
    for r in range(n):
        opdata.assert_same(tname, opname, got[r], want[r], f"cpu ring rank {r}")
    assert t.value > 0
