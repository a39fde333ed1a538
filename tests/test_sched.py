"""CPU tests of coll/mi355x's schedule compiler (host logic of libmi355x_rt, no GPU).

For every reference algorithm and communicator size, the per-element program the engine would run
on the device (mi355x_sched_program) is evaluated here with the oracle's op loops and must equal,
bit for bit, the oracle's full simulation of the reference schedule (which moves data the way
coll/tuned does).  Float SUM on N(0,1) data makes every order difference visible; MAX with NaNs and
signed zeros, and MAXLOC ties, make operand-role differences visible.
"""
from __future__ import annotations

import ctypes

import numpy as np
import pytest

import opdata


def _ptrs(arrs):
    return (ctypes.c_void_p * len(arrs))(*[a.ctypes.data if a is not None else None for a in arrs])


def eval_program(oracle, prog, op, ty, xs):
    """evaluate a serialized engine program on host arrays xs[rank] with the oracle ops"""
    if prog[0] == 1:
        L = prog[2]
        order, roles = prog[3:3 + L], prog[3 + L:3 + 2 * L]
        acc = xs[order[0]].copy()
        for j in range(1, L):
            x = xs[order[j]]
            if roles[j]:   # acc is the `out` operand
                oracle.oracle_op_2buff(op, ty, x.ctypes.data, acc.ctypes.data, len(acc))
            else:          # the rank's value is `out`, acc is `in`
                t = x.copy()
                oracle.oracle_op_2buff(op, ty, acc.ctypes.data, t.ctypes.data, len(acc))
                acc = t
        return acc
    nsteps, result = prog[2], prog[3]
    R = [x.copy() for x in xs]
    for k in range(nsteps):
        d, o, i = prog[4 + 3 * k: 7 + 3 * k]
        t = R[o].copy()
        oracle.oracle_op_2buff(op, ty, R[i].ctypes.data, t.ctypes.data, len(t))
        R[d] = t
    return R[result]


CASES = [("SUM", "FLOAT"), ("MAX", "DOUBLE"), ("MAXLOC", "FLOAT_INT"), ("PROD", "C_FLOAT_COMPLEX")]


@pytest.mark.parametrize("n", [2, 3, 4, 5, 6, 7, 8, 11, 16])
@pytest.mark.parametrize("alg", [3, 4, 5])
def test_allreduce_programs(pkg, oracle, n, alg):
    count = 37 * n + 5 if alg != 3 else 257   # ring: uneven early/late blocks
    for opname, tname in CASES:
        op, ty = pkg.OP[opname], pkg.T[tname]
        xs = [opdata.make(tname, count, 10 + r) for r in range(n)]
        outs = [np.zeros_like(xs[0]) for _ in range(n)]
        seg = 4 * 16 if alg == 5 else 0          # tiny segments: many phases
        got_alg = oracle.oracle_allreduce(alg, n, count, ty, op, seg, _ptrs(xs), _ptrs(outs))
        assert got_alg >= 0
        for r in range(1, n):
            opdata.assert_same(tname, opname, outs[r], outs[0], f"ranks agree n={n}")
        if alg == 3:
            prog = pkg.sched_program(1, n, 3, 0)
            got = eval_program(oracle, prog, op, ty, xs)
            opdata.assert_same(tname, opname, got, outs[0], f"recdbl n={n}")
        else:
            for b in range(n):
                lo, ln = _ring_block(count, n, b)
                prog = pkg.sched_program(1, n, alg, b)
                got = eval_program(oracle, prog, op, ty, [x[lo:lo + ln] for x in xs])
                opdata.assert_same(tname, opname, got, outs[0][lo:lo + ln], f"ring n={n} b={b}")


def _ring_block(count, n, b):
    early = late = count // n
    split = count % n
    if split:
        early += 1
    off = b * early if b < split else b * late + split
    return off, (early if b < split else late)


@pytest.mark.parametrize("n", [2, 3, 4, 5, 7, 8, 13])
@pytest.mark.parametrize("ralg", [1, 2, 3, 4, 5])
def test_reduce_programs(pkg, oracle, n, ralg):
    count = 101
    for opname, tname in CASES:
        op, ty = pkg.OP[opname], pkg.T[tname]
        xs = [opdata.make(tname, count, 30 + r) for r in range(n)]
        for root in sorted({0, n // 2, n - 1}):
            want = np.zeros_like(xs[0])
            assert oracle.oracle_reduce(ralg, n, root, count, ty, op, 0, _ptrs(xs), want.ctypes.data) == ralg
            prog = pkg.sched_program(2, n, ralg, root)
            got = eval_program(oracle, prog, op, ty, xs)
            opdata.assert_same(tname, opname, got, want, f"reduce alg={ralg} n={n} root={root}")


@pytest.mark.parametrize("n", [3, 5, 6, 8, 13, 16])
@pytest.mark.parametrize("fanout", [1, 2, 3, 4, 7, 32])
def test_reduce_chain_fanouts(pkg, oracle, n, fanout):
    """ompi_coll_tuned_topo_build_chain with every shape of chains (even and uneven splits)"""
    count = 64
    xs = [opdata.make("FLOAT", count, 60 + r) for r in range(n)]
    want = np.zeros_like(xs[0])
    assert oracle.oracle_reduce_fo(2, n, 0, fanout, count, pkg.T["FLOAT"], pkg.OP["SUM"], _ptrs(xs),
                                   want.ctypes.data) == 2
    got = eval_program(oracle, pkg.sched_program(5, n, 0, fanout), pkg.OP["SUM"], pkg.T["FLOAT"], xs)
    opdata.assert_same("FLOAT", "SUM", got, want, f"chain n={n} fanout={fanout}")


def test_chain_fanout_changes_the_order(pkg, oracle):
    """the forced chain (alg 2) is NOT the pipeline when the fan-out is > 1 (default 4)"""
    n, count = 9, 4096
    xs = [np.nan_to_num(opdata.make("FLOAT", count, 80 + r), nan=0.0, posinf=1.0, neginf=-1.0) for r in range(n)]
    a, b = np.zeros_like(xs[0]), np.zeros_like(xs[0])
    oracle.oracle_reduce_fo(2, n, 0, 4, count, 14, 3, _ptrs(xs), a.ctypes.data)
    oracle.oracle_reduce_fo(2, n, 0, 1, count, 14, 3, _ptrs(xs), b.ctypes.data)
    assert (a.view(np.uint32) != b.view(np.uint32)).sum() > 100


@pytest.mark.parametrize("n", [2, 3, 4, 5, 6, 7, 8, 12])
@pytest.mark.parametrize("rsalg", [1, 2, 3])
def test_reduce_scatter_programs(pkg, oracle, n, rsalg):
    """coll/tuned ids: 1 non-overlapping (reduce to 0 + scatterv), 2 recursive halving, 3 ring"""
    rng = np.random.default_rng(n)
    rcounts = [int(v) for v in rng.integers(0, 9, n)]
    rcounts[0] = max(rcounts[0], 1)
    total = sum(rcounts)
    disp = np.concatenate([[0], np.cumsum(rcounts)])
    for opname, tname in CASES:
        op, ty = pkg.OP[opname], pkg.T[tname]
        xs = [opdata.make(tname, total, 50 + r) for r in range(n)]
        outs = [np.zeros(max(c, 1), dtype=xs[0].dtype) for c in rcounts]
        rc = (ctypes.c_int * n)(*rcounts)
        assert oracle.oracle_reduce_scatter_alg(rsalg, n, rc, ty, op, _ptrs(xs), _ptrs(outs)) == rsalg
        for b in range(n):
            if rcounts[b] == 0:
                continue
            if rsalg == 1:   # every block carries the reduce tree (decision on the total count)
                ralg = oracle.oracle_reduce_decision(n, total, ty, None)
                prog = pkg.sched_program(2, n, ralg, 0)
            else:
                prog = pkg.sched_program(3 if rsalg == 3 else 4, n, 0, b)
            lo, hi = disp[b], disp[b + 1]
            got = eval_program(oracle, prog, op, ty, [x[lo:hi] for x in xs])
            opdata.assert_same(tname, opname, got, outs[b][:rcounts[b]], f"rs alg={rsalg} n={n} b={b}")


def test_recdbl_ring_orders_differ(pkg, oracle):
    """the two allreduce orders really differ on fp32 (so order replication is load-bearing)"""
    n, count = 8, 4096
    xs = [opdata.make("FLOAT", count, 70 + r) for r in range(n)]
    xs = [np.nan_to_num(x, nan=0.0, posinf=1.0, neginf=-1.0) for x in xs]
    a = [np.zeros_like(xs[0]) for _ in range(n)]
    b = [np.zeros_like(xs[0]) for _ in range(n)]
    oracle.oracle_allreduce(3, n, count, 14, 3, 0, _ptrs(xs), _ptrs(a))
    oracle.oracle_allreduce(4, n, count, 14, 3, 0, _ptrs(xs), _ptrs(b))
    assert (a[0].view(np.uint32) != b[0].view(np.uint32)).sum() > 100


def test_decisions(pkg, oracle):
    """allreduce decision thresholds (coll_tuned_decision_fixed.c:42-85)"""
    d = oracle.oracle_allreduce_decision
    assert d(8, 2499, 14, None) == 3          # 9996 B < 10000
    assert d(8, 2500, 14, None) == 4          # ring up to np * 1 MiB
    assert d(8, 2 * 1024 * 1024, 14, None) == 4
    assert d(8, 2 * 1024 * 1024 + 1, 14, None) == 5
    assert d(8, 1 << 28, 14, None) == 5       # 1 GiB fp32 np=8: segmented ring
