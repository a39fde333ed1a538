"""CPU checks of the scan / exscan oracle (oracle/coll_oracle_scan.c) against a direct restatement
of coll/basic's chain with the oracle's own 2-buff op, and the property that the float order matters
(so the GPU parity test is order-sensitive)."""
from __future__ import annotations

import ctypes

import numpy as np
import pytest

import opdata


def _ptrs(arrs):
    return (ctypes.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])


@pytest.mark.parametrize("n", [1, 2, 3, 7])
@pytest.mark.parametrize("opname,tname", [("SUM", "FLOAT"), ("MAXLOC", "FLOAT_INT"), ("PROD", "C_FLOAT_COMPLEX")])
def test_scan_chain(pkg, oracle, n, opname, tname):
    op, ty = pkg.OP[opname], pkg.T[tname]
    count = 513
    xs = [opdata.make(tname, count, 5 + r) for r in range(n)]
    out = [np.zeros_like(xs[0]) for _ in range(n)]
    assert oracle.oracle_scan(0, n, count, ty, op, _ptrs(xs), _ptrs(out)) == 0
    acc = xs[0].copy()
    opdata.assert_same(tname, opname, out[0], acc, "rank 0")
    for r in range(1, n):
        t = xs[r].copy()
        oracle.oracle_op_2buff(op, ty, acc.ctypes.data, t.ctypes.data, count)  # rbuf = prior (op) rbuf
        acc = t
        opdata.assert_same(tname, opname, out[r], acc, f"rank {r}")
    ex = [np.full_like(xs[0], 0) for _ in range(n)]
    assert oracle.oracle_scan(1, n, count, ty, op, _ptrs(xs), _ptrs(ex)) == 0
    assert not ex[0].view(np.uint8).any(), "exscan must not touch rank 0"
    for r in range(1, n):
        opdata.assert_same(tname, opname, ex[r], out[r - 1], f"exscan rank {r}")


def test_scan_order_matters(pkg, oracle):
    n, count = 8, 4096
    xs = [np.nan_to_num(opdata.make("FLOAT", count, 70 + r), nan=0.0, posinf=1.0, neginf=-1.0) for r in range(n)]
    out = [np.zeros_like(xs[0]) for _ in range(n)]
    oracle.oracle_scan(0, n, count, pkg.T["FLOAT"], pkg.OP["SUM"], _ptrs(xs), _ptrs(out))
    rev = np.zeros_like(xs[0])
    for x in reversed(xs):
        rev = (rev + x).astype(np.float32)
    assert (out[-1].view(np.uint32) != rev.view(np.uint32)).sum() > 50
