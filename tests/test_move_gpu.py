"""MPI_Scan / MPI_Exscan and the data-movement collectives (gather(v), scatter(v), allgatherv,
alltoall(v)) of coll_move.cpp on loopback communicators (n virtual ranks, one thread each).

Scan / Exscan must be bit-identical to the oracle's simulation of coll/basic's linear chain
(coll_basic_scan.c:40-120, coll_basic_exscan.c:40-110) for types whose results expose operand order
(fp32 SUM on N(0,1), MAXLOC ties, complex PROD), in place and not.  Data movement is byte-exact
against numpy's placement of the same blocks, ragged counts, zero-length blocks and MPI_IN_PLACE
included."""
from __future__ import annotations

import ctypes

import numpy as np
import pytest

import opdata
from test_coll_gpu import from_dev, run_ranks, to_dev

pytestmark = pytest.mark.gpu

SCAN_CASES = [("SUM", "FLOAT"), ("SUM", "DOUBLE"), ("MAXLOC", "FLOAT_INT"), ("PROD", "C_DOUBLE_COMPLEX"),
              ("BAND", "INT64"), ("MIN", "INT8")]


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


def _ptrs(arrs):
    return (ctypes.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])


@pytest.mark.parametrize("n", [1, 2, 3, 5, 8])
@pytest.mark.parametrize("exclusive", [False, True])
@pytest.mark.parametrize("inplace", [False, True])
def test_scan(gpu, pkg, oracle, comms, n, exclusive, inplace):
    torch = gpu
    cs = comms(n)
    for opname, tname in SCAN_CASES:
        op, ty = pkg.OP[opname], pkg.T[tname]
        count = 4099
        xs = [opdata.make(tname, count, 900 + r) for r in range(n)]
        fill = opdata.make(tname, count, 77)
        want = [fill.copy() for _ in range(n)]
        assert oracle.oracle_scan(int(exclusive), n, count, ty, op, _ptrs(xs), _ptrs(want)) == 0
        dx = [to_dev(torch, x) for x in xs]
        dr = [to_dev(torch, fill) for _ in range(n)]
        torch.cuda.synchronize()

        def rank(r):
            torch.cuda.set_device(0)
            fn = cs[r].exscan if exclusive else cs[r].scan
            if inplace:
                dr[r].copy_(dx[r])
                torch.cuda.synchronize()
                fn(None, dr[r].data_ptr(), count, ty, op)
            else:
                fn(dx[r].data_ptr(), dr[r].data_ptr(), count, ty, op)

        run_ranks(n, rank)
        for r in range(n):
            got = from_dev(dr[r], xs[0])
            if exclusive and r == 0:
                # rank 0's rbuf is untouched (in place: it still holds its input)
                expect = xs[0] if inplace else fill
                assert np.array_equal(got.view(np.uint8), expect.view(np.uint8)), "exscan rank 0 touched"
                continue
            opdata.assert_same(tname, opname, got, want[r], f"{'ex' if exclusive else ''}scan n={n} r={r}")


def _blocks(n, seed, lo=0, hi=5000):
    g = np.random.default_rng(seed)
    c = [int(v) for v in g.integers(lo, hi, n)]
    return c


@pytest.mark.parametrize("n", [2, 3, 8])
@pytest.mark.parametrize("inplace", [False, True])
def test_gather_scatter(gpu, pkg, comms, n, inplace):
    torch = gpu
    cs = comms(n)
    g = np.random.default_rng(n)
    nb = 12345
    for root in sorted({0, n - 1}):
        src = [torch.from_numpy(g.integers(0, 256, nb, dtype=np.uint8)).cuda() for _ in range(n)]
        out = torch.zeros(nb * n, dtype=torch.uint8, device="cuda")
        if inplace:
            out[root * nb:(root + 1) * nb].copy_(src[root])
        torch.cuda.synchronize()
        run_ranks(n, lambda r: (torch.cuda.set_device(0), cs[r].gather(
            None if (inplace and r == root) else src[r].data_ptr(), out.data_ptr() if r == root else None, nb, root)))
        assert torch.equal(out, torch.cat(src)), f"gather root={root}"
        # scatter back into fresh buffers
        dst = [torch.zeros(nb, dtype=torch.uint8, device="cuda") for _ in range(n)]
        run_ranks(n, lambda r: (torch.cuda.set_device(0), cs[r].scatter(
            out.data_ptr() if r == root else None, None if (inplace and r == root) else dst[r].data_ptr(), nb, root)))
        for r in range(n):
            if inplace and r == root:
                continue
            assert torch.equal(dst[r], src[r]), f"scatter root={root} r={r}"


@pytest.mark.parametrize("n", [2, 3, 8])
def test_gatherv_scatterv(gpu, pkg, comms, n):
    torch = gpu
    cs = comms(n)
    counts = _blocks(n, 10 + n)
    counts[0] = 0                     # an empty block
    displs = [int(v) + 7 * i for i, v in enumerate(np.concatenate([[0], np.cumsum(counts[:-1])]))]  # gaps
    total = displs[-1] + counts[-1] + 3
    g = np.random.default_rng(3)
    src = [torch.from_numpy(g.integers(0, 256, max(c, 1), dtype=np.uint8)).cuda() for c in counts]
    root = n // 2
    out = torch.full((total,), 0xEE, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    run_ranks(n, lambda r: (torch.cuda.set_device(0), cs[r].gatherv(
        src[r].data_ptr(), counts[r], out.data_ptr() if r == root else None, counts if r == root else None,
        displs if r == root else None, root)))
    want = np.full(total, 0xEE, dtype=np.uint8)
    for r in range(n):
        want[displs[r]:displs[r] + counts[r]] = src[r][:counts[r]].cpu().numpy()
    assert np.array_equal(out.cpu().numpy(), want), "gatherv"
    dst = [torch.zeros(max(c, 1), dtype=torch.uint8, device="cuda") for c in counts]
    run_ranks(n, lambda r: (torch.cuda.set_device(0), cs[r].scatterv(
        out.data_ptr() if r == root else None, counts if r == root else None, displs if r == root else None,
        dst[r].data_ptr(), counts[r], root)))
    for r in range(n):
        assert torch.equal(dst[r][:counts[r]], src[r][:counts[r]]), f"scatterv r={r}"


@pytest.mark.parametrize("n", [2, 3, 8])
@pytest.mark.parametrize("inplace", [False, True])
def test_allgatherv(gpu, pkg, comms, n, inplace):
    torch = gpu
    cs = comms(n)
    counts = _blocks(n, 20 + n)
    counts[-1] = 0
    displs = [int(v) + 5 * i for i, v in enumerate(np.concatenate([[0], np.cumsum(counts[:-1])]))]
    total = displs[-1] + counts[-1] + 1
    g = np.random.default_rng(4)
    src = [torch.from_numpy(g.integers(0, 256, max(c, 1), dtype=np.uint8)).cuda() for c in counts]
    outs = [torch.full((total,), 0x11, dtype=torch.uint8, device="cuda") for _ in range(n)]
    if inplace:
        for r in range(n):
            outs[r][displs[r]:displs[r] + counts[r]].copy_(src[r][:counts[r]])
    torch.cuda.synchronize()
    run_ranks(n, lambda r: (torch.cuda.set_device(0), cs[r].allgatherv(
        None if inplace else src[r].data_ptr(), counts[r], outs[r].data_ptr(), counts, displs)))
    want = np.full(total, 0x11, dtype=np.uint8)
    for r in range(n):
        want[displs[r]:displs[r] + counts[r]] = src[r][:counts[r]].cpu().numpy()
    for r in range(n):
        assert np.array_equal(outs[r].cpu().numpy(), want), f"allgatherv r={r}"


@pytest.mark.parametrize("n", [2, 3, 8])
@pytest.mark.parametrize("inplace", [False, True])
def test_alltoall(gpu, pkg, comms, n, inplace):
    torch = gpu
    cs = comms(n)
    nb = 3001
    g = np.random.default_rng(5)
    src = [torch.from_numpy(g.integers(0, 256, nb * n, dtype=np.uint8)).cuda() for _ in range(n)]
    outs = [s.clone() if inplace else torch.zeros(nb * n, dtype=torch.uint8, device="cuda") for s in src]
    torch.cuda.synchronize()
    run_ranks(n, lambda r: (torch.cuda.set_device(0), cs[r].alltoall(
        None if inplace else src[r].data_ptr(), outs[r].data_ptr(), nb)))
    for r in range(n):
        want = torch.cat([src[q][r * nb:(r + 1) * nb] for q in range(n)])
        assert torch.equal(outs[r], want), f"alltoall r={r}"


@pytest.mark.parametrize("n", [2, 3, 8])
def test_alltoallv(gpu, pkg, comms, n):
    torch = gpu
    cs = comms(n)
    g = np.random.default_rng(6 + n)
    # sizes[q][r] = bytes q sends to r (some zero)
    sizes = [[int(v) if (q + r) % 4 else 0 for r, v in enumerate(g.integers(1, 3000, n))] for q in range(n)]
    sdispls = [[int(v) + 3 * r for r, v in enumerate(np.concatenate([[0], np.cumsum(sizes[q][:-1])]))]
               for q in range(n)]
    rcounts = [[sizes[q][r] for q in range(n)] for r in range(n)]
    rdispls = [[int(v) + 11 * q for q, v in enumerate(np.concatenate([[0], np.cumsum(rcounts[r][:-1])]))]
               for r in range(n)]
    src = [torch.from_numpy(g.integers(0, 256, sdispls[q][-1] + sizes[q][-1] + 1, dtype=np.uint8)).cuda()
           for q in range(n)]
    outs = [torch.full((rdispls[r][-1] + rcounts[r][-1] + 1,), 0x33, dtype=torch.uint8, device="cuda")
            for r in range(n)]
    torch.cuda.synchronize()
    run_ranks(n, lambda r: (torch.cuda.set_device(0), cs[r].alltoallv(
        src[r].data_ptr(), sizes[r], sdispls[r], outs[r].data_ptr(), rcounts[r], rdispls[r])))
    for r in range(n):
        want = np.full(outs[r].numel(), 0x33, dtype=np.uint8)
        for q in range(n):
            ln = sizes[q][r]
            want[rdispls[r][q]:rdispls[r][q] + ln] = src[q][sdispls[q][r]:sdispls[q][r] + ln].cpu().numpy()
        assert np.array_equal(outs[r].cpu().numpy(), want), f"alltoallv r={r}"


def test_truncation(gpu, pkg, comms):
    torch = gpu
    a = torch.zeros(100, dtype=torch.uint8, device="cuda")
    out = torch.zeros(200, dtype=torch.uint8, device="cuda")
    errs = []

    def rank(r):
        torch.cuda.set_device(0)
        try:   # rank 1 sends 100 bytes, the root expects 50 from it
            cs[r].gatherv(a.data_ptr(), 100 if r == 1 else 50, out.data_ptr() if r == 0 else None,
                          [50, 50] if r == 0 else None, [0, 100] if r == 0 else None, 0)
        except pkg.MI355XError as e:
            errs.append((r, str(e)))

    import os
    os.environ["MI355X_TIMEOUT_S"] = "5"
    cs = c2 = pkg.Comm.loopback(2, 0)
    try:
        run_ranks(2, rank)
    finally:
        for c in c2:
            c.destroy()
        os.environ["MI355X_TIMEOUT_S"] = "60"
    assert any(r == 0 and "gatherv: rank 1 sends 100 bytes" in m for r, m in errs), errs


def test_nonblocking(gpu, pkg, oracle, comms):
    torch = gpu
    n = 4
    cs = comms(n)
    count = 1000
    xs = [opdata.make("FLOAT", count, 50 + r) for r in range(n)]
    want = [np.zeros_like(xs[0]) for _ in range(n)]
    oracle.oracle_scan(0, n, count, pkg.T["FLOAT"], pkg.OP["SUM"], _ptrs(xs), _ptrs(want))
    dx = [to_dev(torch, x) for x in xs]
    dr = [torch.zeros_like(d) for d in dx]
    nb = 500
    asrc = [torch.full((nb * n,), r, dtype=torch.uint8, device="cuda") for r in range(n)]
    aout = [torch.zeros(nb * n, dtype=torch.uint8, device="cuda") for _ in range(n)]
    torch.cuda.synchronize()

    def rank(r):
        torch.cuda.set_device(0)
        q1 = cs[r].iscan(dx[r].data_ptr(), dr[r].data_ptr(), count, pkg.T["FLOAT"], pkg.OP["SUM"])
        q2 = cs[r].ialltoall(asrc[r].data_ptr(), aout[r].data_ptr(), nb)
        q1.wait()
        q2.wait()

    run_ranks(n, rank)
    for r in range(n):
        opdata.assert_same("FLOAT", "SUM", from_dev(dr[r], xs[0]), want[r], f"iscan r={r}")
        assert torch.equal(aout[r].cpu(), torch.arange(n, dtype=torch.uint8).repeat_interleave(nb)), "ialltoall"
