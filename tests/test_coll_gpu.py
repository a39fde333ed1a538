"""coll/mi355x engine on one MI355X: loopback communicators (n virtual ranks, one thread each,
one device) vs the oracle's simulation of the reference schedules.

Covers MPI_Allreduce (decision + every forced tuned algorithm), MPI_Reduce_scatter_block,
MPI_Reduce_scatter (recursive halving + ring), MPI_Allgather and MPI_Bcast, in place and not,
odd counts, and element types whose results expose operand order (fp32 SUM on N(0,1), MAX with
NaN/signed zeros, MAXLOC ties, complex PROD).  Bar: bit-exact (NaN payloads of float SUM/PROD
excepted, see opdata.py).  The multi-process IPC path is covered by test_coll_ipc_gpu.py.
"""
from __future__ import annotations

import ctypes
import threading

import numpy as np
import pytest

import opdata

pytestmark = pytest.mark.gpu

CASES = [("SUM", "FLOAT"), ("SUM", "DOUBLE"), ("MAX", "DOUBLE"), ("MAXLOC", "FLOAT_INT"),
         ("PROD", "C_DOUBLE_COMPLEX"), ("BAND", "INT64"), ("SUM", "INT8"), ("MINLOC", "DOUBLE_INT")]


def _ptrs(arrs):
    return (ctypes.c_void_p * len(arrs))(*[a.ctypes.data if a is not None else None for a in arrs])


def run_ranks(n, fn):
    """run fn(rank) on n threads, re-raising the first failure"""
    errs = [None] * n

    def body(r):
        try:
            fn(r)
        except BaseException as e:  # noqa: BLE001
            errs[r] = e

    th = [threading.Thread(target=body, args=(r,)) for r in range(n)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    for e in errs:
        if e is not None:
            raise e


def to_dev(torch, a: np.ndarray):
    return torch.from_numpy(a.view(np.uint8).copy()).cuda()


def from_dev(t, like: np.ndarray, n=None):
    n = len(like) if n is None else n
    return t[: n * like.dtype.itemsize].cpu().numpy().view(like.dtype).copy()


@pytest.fixture(scope="module")
def comms(gpu, pkg):
    made = {}

    def get(n):
        if n not in made:
            made[n] = pkg.Comm.loopback(n, 0)
        return made[n]

    yield get
    for cs in made.values():
        for c in cs:
            c.destroy()


@pytest.mark.parametrize("n", [2, 3, 4, 8])
@pytest.mark.parametrize("alg", [0, 3, 4, 5])
@pytest.mark.parametrize("inplace", [False, True])
@pytest.mark.parametrize("push", [0, 1])
def test_allreduce(gpu, pkg, oracle, comms, n, alg, inplace, push):
    torch = gpu
    cs = comms(n)
    for c in cs:  # (a per-communicator knob: the same value on every rank)
        c.set("PUSH", push)
    try:
        _allreduce_cases(torch, pkg, oracle, cs, n, alg, inplace)
    finally:
        for c in cs:
            c.set("PUSH", 0)


def _allreduce_cases(torch, pkg, oracle, cs, n, alg, inplace):
    for opname, tname in CASES:
        op, ty = pkg.OP[opname], pkg.T[tname]
        esz = pkg.type_size(ty)
        for count in (1, 7, 2500 // esz + 3, 40_001):
            xs = [opdata.make(tname, count, 100 + r) for r in range(n)]
            outs = [np.zeros_like(xs[0]) for _ in range(n)]
            ran = oracle.oracle_allreduce(alg, n, count, ty, op, 0, _ptrs(xs), _ptrs(outs))
            assert ran >= 0
            dx = [to_dev(torch, x) for x in xs]
            dr = [t.clone() if inplace else torch.zeros_like(t) for t in dx]
            torch.cuda.synchronize()
            for c in cs:
                c.set("ALLREDUCE_ALG", alg)

            def rank(r):
                cs[r].allreduce(None if inplace else dx[r].data_ptr(), dr[r].data_ptr(), count, ty, op)

            run_ranks(n, rank)
            torch.cuda.synchronize()
            for r in range(n):
                opdata.assert_same(tname, opname, from_dev(dr[r], outs[r]), outs[r],
                                   f"allreduce n={n} alg={alg} count={count} rank={r}")
            assert cs[0].last_algorithm() == ran


@pytest.mark.parametrize("n", [3, 4, 8])
def test_segmented_ring_region(gpu, pkg, oracle, comms, n):
    """the fixed decision's segmented-ring region at n >= 3 (counts above n x segcount, 1 MiB
    segments; coll_tuned_allreduce.c:635-873, coll_tuned_decision_fixed.c:64-80), where the ring's
    per-element fold order is order-sensitive: N(0,1) fp32 SUM and C_DOUBLE_COMPLEX PROD,
    one phase and three phases with a ragged remainder, compared bit-exact with the oracle's
    phase-by-phase simulation"""
    torch = gpu
    cs = comms(n)
    for c in cs:
        c.set("ALLREDUCE_ALG", 0)
    for opname, tname in (("SUM", "FLOAT"), ("PROD", "C_DOUBLE_COMPLEX")):
        op, ty = pkg.OP[opname], pkg.T[tname]
        seg = (1 << 20) // pkg.type_size(ty)
        ns = n * seg
        for count in (ns + seg // 2 + 7, 2 * ns + (3 * ns) // 5 + 13):
            xs = [opdata.make(tname, count, 4000 + 17 * n + r) for r in range(n)]
            outs = [np.zeros_like(xs[0]) for _ in range(n)]
            assert oracle.oracle_allreduce(0, n, count, ty, op, 0, _ptrs(xs), _ptrs(outs)) == 5
            dx = [to_dev(torch, x) for x in xs]
            dr = [torch.zeros_like(t) for t in dx]
            torch.cuda.synchronize()
            run_ranks(n, lambda r: cs[r].allreduce(dx[r].data_ptr(), dr[r].data_ptr(), count, ty, op))
            torch.cuda.synchronize()
            assert cs[0].last_algorithm() == 5
            for r in range(n):
                opdata.assert_same(tname, opname, from_dev(dr[r], outs[r]), outs[r],
                                   f"segmented ring n={n} count={count} rank={r}")
            # the result really is order-sensitive: a naive rank-order fold differs somewhere
            if opname == "SUM":
                naive = xs[0].copy()
                with np.errstate(over="ignore", invalid="ignore"):  # the inputs carry ±Inf / NaN specials
                    for q in range(1, n):
                        naive = (naive + xs[q]).astype(np.float32)
                assert len(opdata.mismatches("FLOAT", "SUM", naive, outs[0])) > 0
            del dx, dr


@pytest.mark.parametrize("n", [2, 3, 5, 8])
@pytest.mark.parametrize("alg", [0, 1, 2, 3, 4, 5])
def test_reduce(gpu, pkg, oracle, comms, n, alg):
    """MPI_Reduce: every tuned reduce tree (forced) and the decision, roots 0 and n-1, in place at
    the root and not; non-roots pass no rbuf; small messages in one phase (the root evaluates
    everything) and, with ONE_PHASE_MAX_BYTES 0, owner-computes + pull"""
    torch = gpu
    cs = comms(n)
    oracle.oracle_reduce.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_size_t, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_uint32, ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p]
    for c in cs:
        c.set("REDUCE_ALG", alg)
    try:
        for opname, tname in CASES[:6]:
            op, ty = pkg.OP[opname], pkg.T[tname]
            for count, one_phase in ((1, 1 << 20), (7, 1 << 20), (40_001, 1 << 20), (40_001, 0)):
                for c in cs:
                    c.set("ONE_PHASE_MAX_BYTES", one_phase)
                xs = [opdata.make(tname, count, 800 + r) for r in range(n)]
                for root in (0, n - 1):
                    want = np.zeros_like(xs[0])
                    ran = oracle.oracle_reduce(alg, n, root, count, ty, op, 0, _ptrs(xs), want.ctypes.data)
                    assert ran >= 0
                    for inplace in (False, True):
                        dx = [to_dev(torch, x) for x in xs]
                        dr = dx[root].clone() if inplace else torch.zeros_like(dx[root])
                        torch.cuda.synchronize()

                        def rank(r):
                            sb = None if (inplace and r == root) else dx[r].data_ptr()
                            cs[r].reduce(sb, dr.data_ptr() if r == root else None, count, ty, op, root)

                        run_ranks(n, rank)
                        torch.cuda.synchronize()
                        opdata.assert_same(tname, opname, from_dev(dr, want), want,
                                           f"reduce n={n} alg={alg} root={root} count={count} inplace={inplace}")
                        assert cs[0].last_algorithm() == ran
    finally:
        for c in cs:
            c.set("REDUCE_ALG", 0)
            c.set("ONE_PHASE_MAX_BYTES", 1 << 20)


@pytest.mark.parametrize("n", [2, 3, 4, 8])
@pytest.mark.parametrize("inplace", [False, True])
def test_reduce_scatter_block(gpu, pkg, oracle, comms, n, inplace):
    torch = gpu
    cs = comms(n)
    for opname, tname in CASES:
        op, ty = pkg.OP[opname], pkg.T[tname]
        for rcount in (1, 33, 5000):
            total = rcount * n
            xs = [opdata.make(tname, total, 200 + r) for r in range(n)]
            outs = [np.zeros(rcount, dtype=xs[0].dtype) for _ in range(n)]
            assert oracle.oracle_reduce_scatter_block(n, rcount, ty, op, _ptrs(xs), _ptrs(outs)) >= 0
            dx = [to_dev(torch, x) for x in xs]
            dr = [t.clone() for t in dx] if inplace else [torch.zeros(rcount * pkg.type_size(ty), dtype=torch.uint8, device="cuda") for _ in dx]
            torch.cuda.synchronize()

            def rank(r):
                cs[r].reduce_scatter_block(None if inplace else dx[r].data_ptr(), dr[r].data_ptr(), rcount, ty, op)

            run_ranks(n, rank)
            torch.cuda.synchronize()
            for r in range(n):
                opdata.assert_same(tname, opname, from_dev(dr[r], outs[r], rcount), outs[r],
                                   f"rsb n={n} rcount={rcount} rank={r}")


@pytest.mark.parametrize("n", [2, 3, 5, 8])
@pytest.mark.parametrize("rsalg", [0, 1, 2, 3])
def test_reduce_scatter(gpu, pkg, oracle, comms, n, rsalg):
    torch = gpu
    cs = comms(n)
    oracle.oracle_reduce_scatter_alg.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                                 ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p),
                                                 ctypes.POINTER(ctypes.c_void_p)]
    rng = np.random.default_rng(n * 10 + rsalg)
    for opname, tname in CASES:
        op, ty = pkg.OP[opname], pkg.T[tname]
        for scale in (3, 3000):
            rcounts = [int(v) for v in rng.integers(0, scale, n)]
            total = sum(rcounts)
            if total == 0:
                continue
            xs = [opdata.make(tname, total, 300 + r) for r in range(n)]
            outs = [np.zeros(max(c, 1), dtype=xs[0].dtype) for c in rcounts]
            rc = (ctypes.c_int * n)(*rcounts)
            assert oracle.oracle_reduce_scatter_alg(rsalg, n, rc, ty, op, _ptrs(xs), _ptrs(outs)) >= 0
            dx = [to_dev(torch, x) for x in xs]
            dr = [torch.zeros(max(c, 1) * pkg.type_size(ty), dtype=torch.uint8, device="cuda") for c in rcounts]
            torch.cuda.synchronize()
            for c in cs:
                c.set("REDUCE_SCATTER_ALG", rsalg)

            def rank(r):
                cs[r].reduce_scatter(dx[r].data_ptr(), dr[r].data_ptr(), rcounts, ty, op)

            run_ranks(n, rank)
            torch.cuda.synchronize()
            for r in range(n):
                if rcounts[r]:
                    opdata.assert_same(tname, opname, from_dev(dr[r], outs[r], rcounts[r]), outs[r][:rcounts[r]],
                                       f"rs alg={rsalg} n={n} rank={r} rcounts={rcounts}")
    for c in cs:
        c.set("REDUCE_SCATTER_ALG", 0)


@pytest.mark.parametrize("n", [2, 3, 8])
@pytest.mark.parametrize("nbytes", [1, 13, 4096, 1_000_003])
@pytest.mark.parametrize("inplace", [False, True])
@pytest.mark.parametrize("push", [0, 1])
def test_allgather(gpu, pkg, comms, n, nbytes, inplace, push):
    torch = gpu
    cs = comms(n)
    for c in cs:  # (a per-communicator knob: the same value on every rank)
        c.set("PUSH", push)
    src = [torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device="cuda") for _ in range(n)]
    dst = [torch.zeros(n * nbytes, dtype=torch.uint8, device="cuda") for _ in range(n)]
    if inplace:
        for r in range(n):
            dst[r][r * nbytes:(r + 1) * nbytes].copy_(src[r])
    torch.cuda.synchronize()
    run_ranks(n, lambda r: cs[r].allgather(None if inplace else src[r].data_ptr(), dst[r].data_ptr(), nbytes))
    torch.cuda.synchronize()
    for c in cs:
        c.set("PUSH", 0)
    want = torch.cat(src)
    for r in range(n):
        assert torch.equal(dst[r], want), r


@pytest.mark.parametrize("n", [2, 3, 8])
@pytest.mark.parametrize("nbytes", [1, 7, 65536, 1 << 20, 3_000_001])
def test_bcast(gpu, pkg, comms, n, nbytes):
    torch = gpu
    cs = comms(n)
    for root in (0, n - 1):
        bufs = [torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device="cuda") for _ in range(n)]
        want = bufs[root].clone()
        torch.cuda.synchronize()
        run_ranks(n, lambda r: cs[r].bcast(bufs[r].data_ptr(), nbytes, root))
        torch.cuda.synchronize()
        for r in range(n):
            assert torch.equal(bufs[r], want), (root, r)


def test_large_allreduce_exact_property(gpu, pkg, comms):
    """BASELINE size class on one device: 1 GiB fp32 per rank, n = 2, small-integer values (sum is
    exact in any order -> equals torch's sum), then the same call repeated: buffers reused (IPC
    registration cache path) and still correct."""
    torch = gpu
    cs = comms(2)
    n_el = 1 << 28
    xs = [torch.randint(-64, 64, (n_el,), device="cuda", dtype=torch.int32).float() for _ in range(2)]
    out = [torch.empty_like(xs[0]) for _ in range(2)]
    want = xs[0] + xs[1]
    torch.cuda.synchronize()
    for _ in range(2):
        run_ranks(2, lambda r: cs[r].allreduce(xs[r].data_ptr(), out[r].data_ptr(), n_el, pkg.T["FLOAT"], pkg.OP["SUM"]))
        torch.cuda.synchronize()
        assert torch.equal(out[0], want) and torch.equal(out[1], want)
    del xs, out, want
    torch.cuda.empty_cache()


@pytest.fixture(scope="module")
def staged_comms(gpu, pkg):
    """loopback communicators forced onto the staged data flow (every buffer treated as
    unexportable) with a 64 KiB staging buffer, so every call runs several windows"""
    made = {}

    def get(n):
        if n not in made:
            cs = pkg.Comm.loopback(n, 0)
            for c in cs:
                c.set("IPC_MAX_BYTES", 0)
                c.set("STAGE_BYTES", 64 << 10)
            made[n] = cs
        return made[n]

    yield get
    for cs in made.values():
        for c in cs:
            c.destroy()


@pytest.mark.parametrize("n", [2, 3, 8])
@pytest.mark.parametrize("alg", [0, 3, 5])
@pytest.mark.parametrize("inplace", [False, True])
def test_staged_allreduce(gpu, pkg, oracle, staged_comms, n, alg, inplace):
    """staged data flow (allocations too large to export): same bits as the reference schedule"""
    _allreduce_cases(gpu, pkg, oracle, staged_comms(n), n, alg, inplace)
    for c in staged_comms(n):
        c.set("ALLREDUCE_ALG", 0)


@pytest.mark.parametrize("n", [2, 5])
@pytest.mark.parametrize("inplace", [False, True])
def test_staged_reduce_scatter_block(gpu, pkg, oracle, staged_comms, n, inplace):
    torch = gpu
    cs = staged_comms(n)
    for opname, tname in CASES[:4]:
        op, ty = pkg.OP[opname], pkg.T[tname]
        for rcount in (1, 5000, 20_011):
            xs = [opdata.make(tname, rcount * n, 500 + r) for r in range(n)]
            outs = [np.zeros(rcount, dtype=xs[0].dtype) for _ in range(n)]
            assert oracle.oracle_reduce_scatter_block(n, rcount, ty, op, _ptrs(xs), _ptrs(outs)) >= 0
            dx = [to_dev(torch, x) for x in xs]
            dr = [t.clone() for t in dx] if inplace else [torch.zeros(rcount * pkg.type_size(ty), dtype=torch.uint8, device="cuda") for _ in dx]
            torch.cuda.synchronize()
            run_ranks(n, lambda r: cs[r].reduce_scatter_block(None if inplace else dx[r].data_ptr(), dr[r].data_ptr(),
                                                              rcount, ty, op))
            torch.cuda.synchronize()
            for r in range(n):
                opdata.assert_same(tname, opname, from_dev(dr[r], outs[r], rcount), outs[r],
                                   f"staged rsb n={n} rcount={rcount} rank={r}")


def test_staged_reduce(gpu, pkg, oracle, staged_comms):
    torch = gpu
    n = 3
    cs = staged_comms(n)
    oracle.oracle_reduce.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_size_t, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_uint32, ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p]
    for opname, tname in CASES[:4]:
        op, ty = pkg.OP[opname], pkg.T[tname]
        count = 30_011
        xs = [opdata.make(tname, count, 900 + r) for r in range(n)]
        for root in range(n):
            want = np.zeros_like(xs[0])
            assert oracle.oracle_reduce(0, n, root, count, ty, op, 0, _ptrs(xs), want.ctypes.data) >= 0
            dx = [to_dev(torch, x) for x in xs]
            dr = torch.zeros_like(dx[0])
            torch.cuda.synchronize()
            run_ranks(n, lambda r: cs[r].reduce(dx[r].data_ptr(), dr.data_ptr() if r == root else None, count, ty, op,
                                                root))
            torch.cuda.synchronize()
            opdata.assert_same(tname, opname, from_dev(dr, want), want, f"staged reduce root={root}")


@pytest.mark.parametrize("rsalg", [1, 2, 3])
def test_staged_reduce_scatter(gpu, pkg, oracle, staged_comms, rsalg):
    torch = gpu
    n = 4
    cs = staged_comms(n)
    oracle.oracle_reduce_scatter_alg.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                                 ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p),
                                                 ctypes.POINTER(ctypes.c_void_p)]
    rcounts = [9000, 0, 17, 30_000]
    total = sum(rcounts)
    for opname, tname in CASES[:4]:
        op, ty = pkg.OP[opname], pkg.T[tname]
        xs = [opdata.make(tname, total, 600 + r) for r in range(n)]
        outs = [np.zeros(max(c, 1), dtype=xs[0].dtype) for c in rcounts]
        rc = (ctypes.c_int * n)(*rcounts)
        assert oracle.oracle_reduce_scatter_alg(rsalg, n, rc, ty, op, _ptrs(xs), _ptrs(outs)) >= 0
        dx = [to_dev(torch, x) for x in xs]
        dr = [torch.zeros(max(c, 1) * pkg.type_size(ty), dtype=torch.uint8, device="cuda") for c in rcounts]
        torch.cuda.synchronize()
        for c in cs:
            c.set("REDUCE_SCATTER_ALG", rsalg)
        run_ranks(n, lambda r: cs[r].reduce_scatter(dx[r].data_ptr(), dr[r].data_ptr(), rcounts, ty, op))
        torch.cuda.synchronize()
        for r in range(n):
            if rcounts[r]:
                opdata.assert_same(tname, opname, from_dev(dr[r], outs[r], rcounts[r]), outs[r][:rcounts[r]],
                                   f"staged rs alg={rsalg} rank={r}")
    for c in cs:
        c.set("REDUCE_SCATTER_ALG", 0)


@pytest.mark.parametrize("n", [2, 3])
@pytest.mark.parametrize("nbytes", [13, 200_003])
@pytest.mark.parametrize("inplace", [False, True])
def test_staged_allgather(gpu, pkg, staged_comms, n, nbytes, inplace):
    torch = gpu
    cs = staged_comms(n)
    src = [torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device="cuda") for _ in range(n)]
    dst = [torch.zeros(n * nbytes, dtype=torch.uint8, device="cuda") for _ in range(n)]
    if inplace:
        for r in range(n):
            dst[r][r * nbytes:(r + 1) * nbytes].copy_(src[r])
    torch.cuda.synchronize()
    run_ranks(n, lambda r: cs[r].allgather(None if inplace else src[r].data_ptr(), dst[r].data_ptr(), nbytes))
    torch.cuda.synchronize()
    want = torch.cat(src)
    for r in range(n):
        assert torch.equal(dst[r], want), r


@pytest.mark.parametrize("n", [2, 3, 8])
@pytest.mark.parametrize("nbytes", [7, 65536, 3_000_001])
def test_staged_bcast(gpu, pkg, staged_comms, n, nbytes):
    """windows of >= 1 MiB take the scatter + allgather shape: a 1 MiB staging buffer covers it"""
    torch = gpu
    cs = staged_comms(n)
    for c in cs:
        c.set("STAGE_BYTES", 1 << 20)
    try:
        for root in (0, n - 1):
            bufs = [torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device="cuda") for _ in range(n)]
            want = bufs[root].clone()
            torch.cuda.synchronize()
            run_ranks(n, lambda r: cs[r].bcast(bufs[r].data_ptr(), nbytes, root))
            torch.cuda.synchronize()
            for r in range(n):
                assert torch.equal(bufs[r], want), (root, r)
    finally:
        for c in cs:
            c.set("STAGE_BYTES", 64 << 10)


@pytest.mark.parametrize("n", [2, 3, 5])
def test_nonblocking(gpu, pkg, oracle, comms, n):
    """MPI_I* collectives: several posted back to back on every rank, then a blocking allreduce
    (ordered after them), then all waited -- each result bit-identical to the oracle's schedule"""
    torch = gpu
    cs = comms(n)
    oracle.oracle_reduce.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_size_t, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_uint32, ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p]
    op, ty = pkg.OP["SUM"], pkg.T["FLOAT"]
    count, rcount, nb = 50_001, 7001, 100_003
    xa = [opdata.make("FLOAT", count, 1000 + r) for r in range(n)]
    wa = [np.zeros_like(xa[0]) for _ in range(n)]
    assert oracle.oracle_allreduce(0, n, count, ty, op, 0, _ptrs(xa), _ptrs(wa)) >= 0
    xb = [opdata.make("FLOAT", rcount * n, 1100 + r) for r in range(n)]
    wb = [np.zeros(rcount, dtype=np.float32) for _ in range(n)]
    assert oracle.oracle_reduce_scatter_block(n, rcount, ty, op, _ptrs(xb), _ptrs(wb)) >= 0
    wr = np.zeros_like(xa[0])
    assert oracle.oracle_reduce(0, n, n - 1, count, ty, op, 0, _ptrs(xa), wr.ctypes.data) >= 0
    xc = [opdata.make("FLOAT", count, 1200 + r) for r in range(n)]
    wc = [np.zeros_like(xc[0]) for _ in range(n)]
    assert oracle.oracle_allreduce(0, n, count, ty, op, 0, _ptrs(xc), _ptrs(wc)) >= 0
    da = [to_dev(torch, x) for x in xa]
    ra = [torch.zeros_like(t) for t in da]
    db = [to_dev(torch, x) for x in xb]
    rb = [torch.zeros(rcount * 4, dtype=torch.uint8, device="cuda") for _ in range(n)]
    rr = torch.zeros_like(da[0])
    gsrc = [torch.randint(0, 256, (nb,), dtype=torch.uint8, device="cuda") for _ in range(n)]
    gdst = [torch.zeros(n * nb, dtype=torch.uint8, device="cuda") for _ in range(n)]
    bb = [torch.randint(0, 256, (nb,), dtype=torch.uint8, device="cuda") for _ in range(n)]
    bwant = bb[0].clone()
    dc = [to_dev(torch, x) for x in xc]
    rc = [torch.zeros_like(t) for t in dc]
    torch.cuda.synchronize()

    def rank(r):
        c = cs[r]
        reqs = [c.iallreduce(da[r].data_ptr(), ra[r].data_ptr(), count, ty, op),
                c.ireduce_scatter_block(db[r].data_ptr(), rb[r].data_ptr(), rcount, ty, op),
                c.ireduce(da[r].data_ptr(), rr.data_ptr() if r == n - 1 else None, count, ty, op, n - 1),
                c.iallgather(gsrc[r].data_ptr(), gdst[r].data_ptr(), nb),
                c.ibcast(bb[r].data_ptr(), nb, 0)]
        c.allreduce(dc[r].data_ptr(), rc[r].data_ptr(), count, ty, op)  # waits for the posted ones
        assert all(q.test() for q in reqs)
        for q in reqs:
            q.wait()

    run_ranks(n, rank)
    torch.cuda.synchronize()
    want_g = torch.cat(gsrc)
    for r in range(n):
        opdata.assert_same("FLOAT", "SUM", from_dev(ra[r], wa[r]), wa[r], f"iallreduce rank={r}")
        opdata.assert_same("FLOAT", "SUM", from_dev(rb[r], wb[r], rcount), wb[r], f"ireduce_scatter_block rank={r}")
        opdata.assert_same("FLOAT", "SUM", from_dev(rc[r], wc[r]), wc[r], f"blocking after nonblocking rank={r}")
        assert torch.equal(gdst[r], want_g), r
        assert torch.equal(bb[r], bwant), r
    opdata.assert_same("FLOAT", "SUM", from_dev(rr, wr), wr, "ireduce")


def test_dynamic_rules(gpu, pkg, oracle, comms, tmp_path):
    """coll/tuned's dynamic rules file drives the choice per message size: allreduce recursive
    doubling below 4 KiB and ring above it for 4-rank communicators; reduce = chain with fan-out 2;
    reduce_scatter = ring.  Results equal the oracle's for the algorithm the rule names."""
    torch = gpu
    n = 4
    cs = comms(n)
    f = tmp_path / "rules.conf"
    f.write_text("""# collectives
3
2   # ALLREDUCE
1   # one communicator size
4 2 # size 4, two message sizes
0    3 0 0
4096 4 0 0
11  # REDUCE
1
2 1
0 2 2 0
12  # REDUCESCATTER
1
2 1
0 3 0 0
""")
    rules = pkg.Rules(str(f))
    assert rules.ncoll == 3
    for c in cs:
        c.set_rules(rules)
    try:
        op, ty = pkg.OP["SUM"], pkg.T["FLOAT"]
        for count, alg in ((100, 3), (5000, 4)):
            xs = [opdata.make("FLOAT", count, 1500 + r) for r in range(n)]
            outs = [np.zeros_like(xs[0]) for _ in range(n)]
            assert oracle.oracle_allreduce(alg, n, count, ty, op, 0, _ptrs(xs), _ptrs(outs)) == alg
            dx = [to_dev(torch, x) for x in xs]
            dr = [torch.zeros_like(t) for t in dx]
            torch.cuda.synchronize()
            run_ranks(n, lambda r: cs[r].allreduce(dx[r].data_ptr(), dr[r].data_ptr(), count, ty, op))
            torch.cuda.synchronize()
            assert cs[0].last_algorithm() == alg
            for r in range(n):
                opdata.assert_same("FLOAT", "SUM", from_dev(dr[r], outs[r]), outs[r], f"rules allreduce {count}")
        count = 3001
        xs = [opdata.make("FLOAT", count, 1600 + r) for r in range(n)]
        want = np.zeros_like(xs[0])
        assert oracle.oracle_reduce_fo(2, n, 1, 2, count, ty, op, _ptrs(xs), want.ctypes.data) == 2
        dx = [to_dev(torch, x) for x in xs]
        dr = torch.zeros_like(dx[0])
        torch.cuda.synchronize()
        run_ranks(n, lambda r: cs[r].reduce(dx[r].data_ptr(), dr.data_ptr() if r == 1 else None, count, ty, op, 1))
        torch.cuda.synchronize()
        assert cs[0].last_algorithm() == 2
        opdata.assert_same("FLOAT", "SUM", from_dev(dr, want), want, "rules reduce chain fan-out 2")
        rcounts = [100, 7, 0, 900]
        xs = [opdata.make("FLOAT", sum(rcounts), 1700 + r) for r in range(n)]
        outs = [np.zeros(max(k, 1), dtype=np.float32) for k in rcounts]
        rc = (ctypes.c_int * n)(*rcounts)
        assert oracle.oracle_reduce_scatter_alg(3, n, rc, ty, op, _ptrs(xs), _ptrs(outs)) == 3
        dx = [to_dev(torch, x) for x in xs]
        dr = [torch.zeros(max(k, 1) * 4, dtype=torch.uint8, device="cuda") for k in rcounts]
        torch.cuda.synchronize()
        run_ranks(n, lambda r: cs[r].reduce_scatter(dx[r].data_ptr(), dr[r].data_ptr(), rcounts, ty, op))
        torch.cuda.synchronize()
        assert cs[0].last_algorithm() == 3
        for r in range(n):
            if rcounts[r]:
                opdata.assert_same("FLOAT", "SUM", from_dev(dr[r], outs[r], rcounts[r]), outs[r][:rcounts[r]], "rules rs")
    finally:
        for c in cs:
            c.set_rules(None)
        rules.destroy()


def test_phase_timing(gpu, pkg, comms):
    """MI355X_KNOB_TIME_PHASES: both kernels of the direct allreduce timed with HIP events"""
    torch = gpu
    cs = comms(2)
    count = 1 << 22
    xs = [torch.full((count,), float(r + 1), device="cuda") for r in range(2)]
    ys = [torch.empty_like(x) for x in xs]
    for c in cs:
        c.set("TIME_PHASES", 1)
    torch.cuda.synchronize()
    run_ranks(2, lambda r: (torch.cuda.set_device(0),
                            cs[r].allreduce(xs[r].data_ptr(), ys[r].data_ptr(), count, pkg.T["FLOAT"], pkg.OP["SUM"])))
    for r, c in enumerate(cs):
        p1, p2 = c.phase_ms()
        c.set("TIME_PHASES", 0)
        assert 0.0 < p1 < 1000.0 and 0.0 < p2 < 1000.0, (p1, p2)
        assert bool(torch.all(ys[r] == 3.0))


@pytest.mark.parametrize("n", [3, 5, 8])
def test_one_phase_ring(gpu, pkg, oracle, comms, n):
    """ring-ordered allreduce below ONE_PHASE_MAX_BYTES: every rank evaluates every ring block
    (k_ring_all) -- bit-exact with the oracle's ring and with the two-phase flow (knob 0), on
    order-sensitive data, ragged block partitions (count % n != 0) included"""
    torch = gpu
    cs = comms(n)
    for c in cs:
        c.set("ALLREDUCE_ALG", 4)
    try:
        for opname, tname in (("SUM", "FLOAT"), ("PROD", "C_DOUBLE_COMPLEX"), ("MAXLOC", "DOUBLE_INT")):
            op, ty = pkg.OP[opname], pkg.T[tname]
            for count in (n, 3 * n + 1, 10_007, (200 << 10) // pkg.type_size(ty) + n - 1):
                xs = [opdata.make(tname, count, 7000 + 13 * n + r) for r in range(n)]
                outs = [np.zeros_like(xs[0]) for _ in range(n)]
                assert oracle.oracle_allreduce(4, n, count, ty, op, 0, _ptrs(xs), _ptrs(outs)) == 4
                dx = [to_dev(torch, x) for x in xs]
                for one_phase in (1 << 20, 0):
                    for c in cs:  # per communicator: every rank must take the same flow
                        c.set("ONE_PHASE_MAX_BYTES", one_phase)
                    dr = [torch.zeros_like(t) for t in dx]
                    torch.cuda.synchronize()
                    run_ranks(n, lambda r: cs[r].allreduce(dx[r].data_ptr(), dr[r].data_ptr(), count, ty, op))
                    torch.cuda.synchronize()
                    for r in range(n):
                        opdata.assert_same(tname, opname, from_dev(dr[r], outs[r]), outs[r],
                                           f"ring n={n} count={count} one_phase={one_phase} rank={r}")
    finally:
        for c in cs:
            c.set("ONE_PHASE_MAX_BYTES", 1 << 20)
            c.set("ALLREDUCE_ALG", 0)
