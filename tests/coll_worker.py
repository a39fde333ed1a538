"""One rank of test_components_gpu.test_coll_component_processes: a mini-OMPI communicator whose
lower-priority module is a stub; coll/mi355x selected on top; collectives on device buffers must
match the oracle, host buffers must reach the stub."""
from __future__ import annotations

import ctypes
import os
import pathlib
import sys
import time

import numpy as np

sys.path.insert(0, str(pathlib.Path(__file__).parent))
from conftest import load_oracle  # noqa: E402
from mini import mini  # noqa: E402
import opdata  # noqa: E402
from ddtcases import OPAL_FLOAT4, OPAL_INT4, opal_strided_elems, opal_vector  # noqa: E402


SENT = 0xA5


def derived_bcast(m, comm, oracle, rank, size, torch):
    nblk, count = 1000, 2
    desc, used, tsize, lb, ub = opal_vector(nblk, 256, 512)  # vector(1000, 64, 128, MPI_FLOAT)
    dt = m.derived(desc, used, tsize, lb, ub)
    od = oracle.oracle_ddt_vector(nblk, 64, 128, 4)
    span = (count - 1) * (ub - lb) + ub
    root = size - 1
    rootbuf = np.random.default_rng(77).integers(0, 256, span, dtype=np.uint8)
    mine = rootbuf.copy() if rank == root else np.full(span, SENT, dtype=np.uint8)
    want = rootbuf.copy()
    if rank != root:  # expected: the type map's bytes from the root, the gaps untouched
        packed = np.zeros(count * tsize, dtype=np.uint8)
        oracle.oracle_ddt_pack(od, count, rootbuf.ctypes.data, 0, packed.ctypes.data, count * tsize)
        want = np.full(span, SENT, dtype=np.uint8)
        oracle.oracle_ddt_unpack(od, count, want.ctypes.data, 0, packed.ctypes.data, count * tsize)
    d = torch.from_numpy(mine).cuda()
    torch.cuda.synchronize()
    assert m.lib.mini_bcast(comm, d.data_ptr(), count, dt, root) == 0
    assert np.array_equal(d.cpu().numpy(), want), "derived bcast"
    m.lib.mini_datatype_destroy(dt)
    oracle.oracle_ddt_free(od)


def derived_allgather(m, comm, oracle, rank, size, torch):
    n = 300
    # rdtype = vector(300, 1, 2, MPI_FLOAT): one strided ELEM record
    desc, used, tsize, lb, ub = opal_strided_elems(n, OPAL_FLOAT4, 4, 8)
    rdt = m.derived(desc, used, tsize, lb, ub)
    ext = ub - lb
    od = oracle.oracle_ddt_vector(n, 1, 2, 4)
    fdt = m.dtype_for_slot(m.pkg.T["FLOAT"])
    contrib = [np.arange(n, dtype=np.float32) + 1000 * r for r in range(size)]
    want = np.full(size * ext, SENT, dtype=np.uint8)
    for r in range(size):
        oracle.oracle_ddt_unpack(od, 1, want.ctypes.data + r * ext, 0, contrib[r].ctypes.data, n * 4)
    for inplace in (False, True):
        rb = np.full(size * ext, SENT, dtype=np.uint8)
        if inplace:  # my block already sits in rbuf, laid out by rdtype
            oracle.oracle_ddt_unpack(od, 1, rb.ctypes.data + rank * ext, 0, contrib[rank].ctypes.data, n * 4)
        drb = torch.from_numpy(rb).cuda()
        dsb = torch.from_numpy(contrib[rank].copy()).cuda()
        torch.cuda.synchronize()
        sp = 1 if inplace else dsb.data_ptr()  # MPI_IN_PLACE == (void *)1
        assert m.lib.mini_allgather(comm, sp, n, fdt, drb.data_ptr(), 1, rdt) == 0
        assert np.array_equal(drb.cpu().numpy(), want), f"derived allgather inplace={inplace}"
    m.lib.mini_datatype_destroy(rdt)
    oracle.oracle_ddt_free(od)


def nonblocking_mixed_layouts(m, comm, oracle, rank, size, torch):
    """MPI_Iallgather / MPI_Ibcast where the LAYOUTS differ between ranks (only the type signatures
    match, as MPI allows): even ranks receive n floats per rank into vector(n, 1, 2, MPI_FLOAT)
    blocks and send dense, odd ranks receive dense and send out of a strided buffer; the bcast root
    uses the vector layout while the others use n dense floats, then the other way round.  Every
    rank must stay in the engine (derived layouts staged at initiation / unpacked at completion);
    a rank-local fallback to the previous component would leave the ranks in different protocols.
    Two calls are in flight before the first wait."""
    L = m.lib
    n = 300
    desc, used, tsize, lb, ub = opal_strided_elems(n, OPAL_FLOAT4, 4, 8)
    vec = m.derived(desc, used, tsize, lb, ub)
    ext = ub - lb
    fdt = m.dtype_for_slot(m.pkg.T["FLOAT"])
    contrib = [np.arange(n, dtype=np.float32) + 1000 * r for r in range(size)]
    strided = lambda a: np.stack([a, np.full(n, -1, np.float32)], 1).reshape(-1)[: 2 * n - 1]  # vector layout
    even = rank % 2 == 0
    # iallgather
    if even:
        send = torch.from_numpy(contrib[rank].copy()).cuda()
        rbuf = torch.full((size * ext // 4,), -5.0, device="cuda")
        sargs, rargs = (send.data_ptr(), n, fdt), (rbuf.data_ptr(), 1, vec)
    else:
        send = torch.from_numpy(strided(contrib[rank]).copy()).cuda()
        rbuf = torch.full((size * n,), -5.0, device="cuda")
        sargs, rargs = (send.data_ptr(), 1, vec), (rbuf.data_ptr(), n, fdt)
    # ibcast #1: the root's layout is the vector, the others dense; #2 the reverse
    root = size - 1
    b1 = torch.from_numpy(strided(contrib[root]).copy()).cuda() if rank == root else torch.full((n,), -3.0, device="cuda")
    b1args = (b1.data_ptr(), 1, vec) if rank == root else (b1.data_ptr(), n, fdt)
    torch.cuda.synchronize()
    reqs = [ctypes.c_void_p() for _ in range(2)]
    assert L.mini_iallgather(comm, *sargs, *rargs, ctypes.byref(reqs[0])) == 0
    assert L.mini_ibcast(comm, *b1args, root, ctypes.byref(reqs[1])) == 0
    for q in reqs:
        assert L.mini_wait(ctypes.byref(q)) == 0
    got = rbuf.cpu().numpy()
    for r in range(size):
        if even:
            blk = got[r * ext // 4: r * ext // 4 + 2 * n - 1]
            assert np.array_equal(blk[0::2], contrib[r]) and (blk[1::2] == -5).all(), ("iallgather into vector blocks", r)
        else:
            assert np.array_equal(got[r * n:(r + 1) * n], contrib[r]), ("iallgather dense", r)
    g1 = b1.cpu().numpy()
    assert np.array_equal(g1[0::2] if rank == root else g1, contrib[root]), "ibcast, vector at the root"
    b2 = torch.from_numpy(contrib[root].copy()).cuda() if rank == root else torch.full((2 * n - 1,), -4.0, device="cuda")
    b2args = (b2.data_ptr(), n, fdt) if rank == root else (b2.data_ptr(), 1, vec)
    torch.cuda.synchronize()
    req = ctypes.c_void_p()
    assert L.mini_ibcast(comm, *b2args, root, ctypes.byref(req)) == 0
    assert L.mini_wait(ctypes.byref(req)) == 0
    g2 = b2.cpu().numpy()
    if rank != root:
        assert np.array_equal(g2[0::2], contrib[root]) and (g2[1::2] == -4).all(), "ibcast into vectors off the root"
    L.mini_datatype_destroy(vec)


def mixed_buffers(m, comm, oracle, rank, size, torch):
    """coll/cuda lets ranks mix host and device buffers in one collective (coll_cuda_allreduce.c:
    30-77); here rank 0 passes host memory and the others device memory to MPI_Allreduce (also in
    place), MPI_Reduce (host root, device root), MPI_Reduce_scatter_block, MPI_Reduce_scatter,
    MPI_Allgather (also in place) and MPI_Bcast (host root, device root).  Every rank must end in the
    engine (rank 0 staging its buffers) with exact results; the previous (stub) component is never
    called (checked by the caller's stub count)."""
    L, pkg = m.lib, m.pkg
    fdt = m.dtype_for_slot(pkg.T["FLOAT"])
    op = m.select_op(pkg.OP["SUM"])
    host = rank == 0
    want = size * (size + 1) / 2

    def buf(vals):
        a = np.ascontiguousarray(vals, dtype=np.float32)
        return (a, a.ctypes.data) if host else (lambda t: (t, t.data_ptr()))(torch.from_numpy(a.copy()).cuda())

    def val(b):
        return b if host else b.cpu().numpy()

    n = 10_007
    x, px = buf(np.full(n, rank + 1))
    y, py = buf(np.zeros(n))
    torch.cuda.synchronize()
    assert L.mini_allreduce(comm, px, py, n, fdt, op) == 0
    assert (val(y) == want).all(), "mixed allreduce"
    z, pz = buf(np.full(n, rank + 1))
    torch.cuda.synchronize()
    assert L.mini_allreduce(comm, 1, pz, n, fdt, op) == 0  # MPI_IN_PLACE
    assert (val(z) == want).all(), "mixed allreduce in place"
    for root in (0, size - 1):
        r, pr = buf(np.zeros(n))
        torch.cuda.synchronize()
        assert L.mini_reduce(comm, px, pr if rank == root else None, n, fdt, op, root) == 0
        if rank == root:
            assert (val(r) == want).all(), ("mixed reduce", root)
    rc = 777
    s, ps = buf(np.full(rc * size, rank + 1))
    o, po = buf(np.zeros(rc))
    torch.cuda.synchronize()
    assert L.mini_reduce_scatter_block(comm, ps, po, rc, fdt, op) == 0
    assert (val(o) == want).all(), "mixed reduce_scatter_block"
    counts = [100 + 37 * q for q in range(size)]
    v, pv = buf(np.full(sum(counts), rank + 1))
    w, pw = buf(np.zeros(counts[rank]))
    torch.cuda.synchronize()
    assert L.mini_reduce_scatter(comm, pv, pw, (ctypes.c_int * size)(*counts), fdt, op) == 0
    assert (val(w) == want).all(), "mixed reduce_scatter"
    g, pg = buf(np.zeros(n * size))
    torch.cuda.synchronize()
    assert L.mini_allgather(comm, px, n, fdt, pg, n, fdt) == 0
    gv = val(g)
    assert all((gv[q * n:(q + 1) * n] == q + 1).all() for q in range(size)), "mixed allgather"
    gi, pgi = buf(np.concatenate([np.full(n, q + 1 if q == rank else -1) for q in range(size)]))
    torch.cuda.synchronize()
    assert L.mini_allgather(comm, 1, 0, fdt, pgi, n, fdt) == 0  # MPI_IN_PLACE
    gv = val(gi)
    assert all((gv[q * n:(q + 1) * n] == q + 1).all() for q in range(size)), "mixed allgather in place"
    for root in (0, size - 1):
        b, pb = buf(np.full(n, 5 + root if rank == root else -1))
        torch.cuda.synchronize()
        assert L.mini_bcast(comm, pb, n, fdt, root) == 0
        assert (val(b) == 5 + root).all(), ("mixed bcast", root)


def mixed_more(m, comm, oracle, rank, size, torch, ptrs):
    """ranks mixing host and device buffers in the collectives outside the reductions too (ob1
    decides per request on each side, pml_ob1_cuda.c:52-100): rank 0 host memory, the others device
    memory, in MPI_Gather / Gatherv / Scatter / Scatterv / Allgatherv / Alltoall / Alltoallv (rooted
    calls at a host and at a device root; a host rank's derived layout through the host convertor),
    and in the nonblocking MPI_Iallreduce / Ireduce / Ireduce_scatter_block / Iallgather / Ibcast,
    whose initiation cannot vote: every rank enters the engine, host ranks on device copies.  Exact
    against the oracle / the arithmetic, no timeout, nothing reaches the stub."""
    L, pkg = m.lib, m.pkg
    idt = m.dtype_for_slot(pkg.T["INT32"])
    host = rank == 0
    IA = lambda v: (ctypes.c_int * len(v))(*v)

    def buf(vals, on_host=host):
        a = np.ascontiguousarray(vals, dtype=np.int32).copy()
        if on_host:
            return a, a.ctypes.data, (lambda: a.copy())
        t = torch.from_numpy(a.copy()).cuda()
        return t, t.data_ptr(), (lambda: t.cpu().numpy())

    stub0 = [L.mini_stub_calls(w) for w in range(16)]
    n = 1003
    blocks = [np.arange(n, dtype=np.int32) * (q + 1) + 1000 * q for q in range(size)]
    for root in (0, size - 1):
        # gather
        mine, pm, _ = buf(blocks[rank])
        out, po, rd = buf(np.full(n * size, -1))
        torch.cuda.synchronize()
        assert L.mini_gather(comm, pm, n, idt, po if rank == root else None, n, idt, root) == 0
        if rank == root:
            assert np.array_equal(rd(), np.concatenate(blocks)), ("mixed gather", root)
        # gatherv (ragged, displaced)
        cnt = [n - 7 * q for q in range(size)]
        disp = [q * (n + 5) for q in range(size)]
        part, pp, _ = buf(blocks[rank][:cnt[rank]])
        gz, pgz, gread = buf(np.full(size * (n + 5), -1))
        torch.cuda.synchronize()
        assert L.mini_gatherv(comm, pp, cnt[rank], idt, pgz if rank == root else None, IA(cnt), IA(disp), idt, root) == 0
        if rank == root:
            g = gread()
            for q in range(size):
                assert np.array_equal(g[disp[q]:disp[q] + cnt[q]], blocks[q][:cnt[q]]), ("mixed gatherv", root, q)
                assert (g[disp[q] + cnt[q]:disp[q] + n + 5] == -1).all(), ("mixed gatherv gap", root, q)
        # scatter / scatterv
        src, ps, _ = buf(np.concatenate(blocks))
        rcv, pr, rread = buf(np.full(n, -1))
        torch.cuda.synchronize()
        assert L.mini_scatter(comm, ps if rank == root else None, n, idt, pr, n, idt, root) == 0
        assert np.array_equal(rread(), blocks[rank]), ("mixed scatter", root)
        src2, ps2, _ = buf(np.concatenate([np.concatenate([blocks[q][:cnt[q]], np.full(n + 5 - cnt[q], -9)])
                                           for q in range(size)]))
        rcv2, pr2, rread2 = buf(np.full(n, -1))
        torch.cuda.synchronize()
        assert L.mini_scatterv(comm, ps2 if rank == root else None, IA(cnt), IA(disp), idt, pr2, cnt[rank], idt,
                               root) == 0
        r2 = rread2()
        assert np.array_equal(r2[:cnt[rank]], blocks[rank][:cnt[rank]]) and (r2[cnt[rank]:] == -1).all(), \
            ("mixed scatterv", root)
    # allgatherv
    cnt = [n - 3 * q for q in range(size)]
    disp = [q * n for q in range(size)]
    part, pp, _ = buf(blocks[rank][:cnt[rank]])
    ag, pag, agread = buf(np.full(size * n, -1))
    torch.cuda.synchronize()
    assert L.mini_allgatherv(comm, pp, cnt[rank], idt, pag, IA(cnt), IA(disp), idt) == 0
    a = agread()
    for q in range(size):
        assert np.array_equal(a[disp[q]:disp[q] + cnt[q]], blocks[q][:cnt[q]]), ("mixed allgatherv", q)
    # alltoall / alltoallv: piece q of rank r = 10^6 r + 1000 q + i
    piece = lambda r, q, k: (np.arange(k, dtype=np.int32) + 1000 * q + 1_000_000 * r)
    k = 257
    sa, psa, _ = buf(np.concatenate([piece(rank, q, k) for q in range(size)]))
    ra, pra, raread = buf(np.full(k * size, -1))
    torch.cuda.synchronize()
    assert L.mini_alltoall(comm, psa, k, idt, pra, k, idt) == 0
    assert np.array_equal(raread(), np.concatenate([piece(q, rank, k) for q in range(size)])), "mixed alltoall"
    scnt = [k + q + rank for q in range(size)]          # rank -> q sends k + q + rank
    rcnt = [k + rank + q for q in range(size)]          # q -> rank sends k + rank + q
    sdisp = list(np.cumsum([0] + scnt[:-1]))
    rdisp = [int(x) + 2 * i for i, x in enumerate(np.cumsum([0] + rcnt[:-1]))]
    sv, psv, _ = buf(np.concatenate([piece(rank, q, scnt[q]) for q in range(size)]))
    rv, prv, rvread = buf(np.full(rdisp[-1] + rcnt[-1] + 2, -1))
    torch.cuda.synchronize()
    assert L.mini_alltoallv(comm, psv, IA(scnt), IA([int(x) for x in sdisp]), idt, prv, IA(rcnt), IA(rdisp), idt) == 0
    got = rvread()
    for q in range(size):
        assert np.array_equal(got[rdisp[q]:rdisp[q] + rcnt[q]], piece(q, rank, rcnt[q])), ("mixed alltoallv", q)
    # a host rank's derived layout (every other int) through the host convertor: gather to a device root
    desc, used, tsize, _, true_ub = opal_strided_elems(n, OPAL_INT4, 4, 8)   # vector(n, 1, 2, MPI_INT)
    vec = L.mini_datatype_create_raw(desc, used, tsize, 0, true_ub, 0, true_ub, 0)
    if True:
        spread = np.full(2 * n, -5, np.int32)
        spread[::2] = blocks[rank]
        sb, psb, _ = buf(spread)
        root = size - 1
        gg, pgg, ggread = buf(np.full(n * size, -1))
        torch.cuda.synchronize()
        assert L.mini_gather(comm, psb, 1, vec, pgg if rank == root else None, n, idt, root) == 0
        if rank == root:
            assert np.array_equal(ggread(), np.concatenate(blocks)), "mixed gather, host vector layout"
    # nonblocking: no vote; host ranks join the engine on device copies
    code, slot = pkg.OP["SUM"], pkg.T["DOUBLE"]
    dt = m.dtype_for_slot(slot)
    op = m.select_op(code)
    count, rcount = 20_001, 3001
    xa = [opdata.make("DOUBLE", count, 1500 + r) for r in range(size)]
    wa = [np.zeros_like(xa[0]) for _ in range(size)]
    oracle.oracle_allreduce(0, size, count, slot, code, 0, ptrs(xa), ptrs(wa))
    wr = np.zeros_like(xa[0])
    oracle.oracle_reduce(0, size, 0, count, slot, code, 0, ptrs(xa), wr.ctypes.data)
    xb = [opdata.make("DOUBLE", rcount * size, 1600 + r) for r in range(size)]
    wb = [np.zeros(rcount, dtype=np.float64) for _ in range(size)]
    oracle.oracle_reduce_scatter_block(size, rcount, slot, code, ptrs(xb), ptrs(wb))

    def fbuf(vals):
        a = np.ascontiguousarray(vals).copy()
        if host:
            return a, a.ctypes.data, (lambda: a.copy())
        t = torch.from_numpy(a.view(np.uint8).copy()).cuda()
        return t, t.data_ptr(), (lambda: t.cpu().numpy().view(a.dtype))

    da, pda, _ = fbuf(xa[rank])
    ra_, pra_, raread_ = fbuf(np.zeros_like(xa[0]))
    rr, prr, rrread = fbuf(np.zeros_like(xa[0]))
    ia, pia, iaread = fbuf(xa[rank])       # in place
    db, pdb, _ = fbuf(xb[rank])
    rb, prb, rbread = fbuf(np.zeros(rcount))
    gs, pgs, _ = buf(np.full(n, rank + 1))
    gd, pgd, gdread = buf(np.full(n * size, -1))
    bc, pbc, bcread = buf(np.full(n, 7 if rank == 0 else -1))
    torch.cuda.synchronize()
    reqs = [ctypes.c_void_p() for _ in range(6)]
    assert L.mini_iallreduce(comm, pda, pra_, count, dt, op, ctypes.byref(reqs[0])) == 0
    assert L.mini_iallreduce(comm, 1, pia, count, dt, op, ctypes.byref(reqs[1])) == 0
    assert L.mini_ireduce(comm, pda, prr if rank == 0 else None, count, dt, op, 0, ctypes.byref(reqs[2])) == 0
    assert L.mini_ireduce_scatter_block(comm, pdb, prb, rcount, dt, op, ctypes.byref(reqs[3])) == 0
    assert L.mini_iallgather(comm, pgs, n, idt, pgd, n, idt, ctypes.byref(reqs[4])) == 0
    assert L.mini_ibcast(comm, pbc, n, idt, 0, ctypes.byref(reqs[5])) == 0
    for q in reqs:
        assert L.mini_wait(ctypes.byref(q)) == 0
    opdata.assert_same("DOUBLE", "SUM", raread_(), wa[rank], "mixed iallreduce")
    opdata.assert_same("DOUBLE", "SUM", iaread(), wa[rank], "mixed iallreduce in place")
    if rank == 0:
        opdata.assert_same("DOUBLE", "SUM", rrread(), wr, "mixed ireduce (host root)")
    opdata.assert_same("DOUBLE", "SUM", rbread(), wb[rank], "mixed ireduce_scatter_block")
    g = gdread()
    assert all((g[q * n:(q + 1) * n] == q + 1).all() for q in range(size)), "mixed iallgather"
    assert (bcread() == 7).all(), "mixed ibcast (host root)"
    L.mini_op_destroy(op)
    assert [L.mini_stub_calls(w) for w in range(16)] == stub0, "a mixed call reached the stub"


def nonblocking(m, comm, oracle, rank, size, torch, ptrs):
    pkg = m.pkg
    code, slot = pkg.OP["SUM"], pkg.T["DOUBLE"]
    dt = m.dtype_for_slot(slot)
    op = m.select_op(code)
    count, rcount, nb = 20_001, 3001, 70_001
    xa = [opdata.make("DOUBLE", count, 1300 + r) for r in range(size)]
    wa = [np.zeros_like(xa[0]) for _ in range(size)]
    oracle.oracle_allreduce(0, size, count, slot, code, 0, ptrs(xa), ptrs(wa))
    xb = [opdata.make("DOUBLE", rcount * size, 1400 + r) for r in range(size)]
    wb = [np.zeros(rcount, dtype=np.float64) for _ in range(size)]
    oracle.oracle_reduce_scatter_block(size, rcount, slot, code, ptrs(xb), ptrs(wb))
    wr = np.zeros_like(xa[0])
    oracle.oracle_reduce.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_size_t, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_uint32, ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p]
    oracle.oracle_reduce(0, size, 0, count, slot, code, 0, ptrs(xa), wr.ctypes.data)
    da = torch.from_numpy(xa[rank].view(np.uint8).copy()).cuda()
    ra, rr = torch.zeros_like(da), torch.zeros_like(da)
    db = torch.from_numpy(xb[rank].view(np.uint8).copy()).cuda()
    rb = torch.zeros(rcount * 8, dtype=torch.uint8, device="cuda")
    bdt = m.dtype_for_slot(pkg.T["FLOAT"])
    assert bdt
    gs = torch.full((nb,), float(rank + 1), device="cuda")
    gd = torch.zeros(nb * size, device="cuda")
    bc = torch.full((nb,), float(rank + 7), device="cuda")
    torch.cuda.synchronize()
    reqs = [ctypes.c_void_p() for _ in range(5)]
    L = m.lib
    assert L.mini_iallreduce(comm, da.data_ptr(), ra.data_ptr(), count, dt, op, ctypes.byref(reqs[0])) == 0
    assert L.mini_ireduce_scatter_block(comm, db.data_ptr(), rb.data_ptr(), rcount, dt, op, ctypes.byref(reqs[1])) == 0
    assert L.mini_ireduce(comm, da.data_ptr(), rr.data_ptr() if rank == 0 else None, count, dt, op, 0,
                          ctypes.byref(reqs[2])) == 0
    assert L.mini_iallgather(comm, gs.data_ptr(), nb, bdt, gd.data_ptr(), nb, bdt, ctypes.byref(reqs[3])) == 0
    assert L.mini_ibcast(comm, bc.data_ptr(), nb, bdt, size - 1, ctypes.byref(reqs[4])) == 0
    assert L.mini_progress_callbacks() >= 1
    for q in reqs:
        assert L.mini_wait(ctypes.byref(q)) == 0
        assert L.mini_request_is_null(q), "MPI_Wait leaves MPI_REQUEST_NULL"
    opdata.assert_same("DOUBLE", "SUM", ra.cpu().numpy().view(np.float64), wa[rank], "component iallreduce")
    opdata.assert_same("DOUBLE", "SUM", rb.cpu().numpy().view(np.float64), wb[rank], "component ireduce_scatter_block")
    if rank == 0:
        opdata.assert_same("DOUBLE", "SUM", rr.cpu().numpy().view(np.float64), wr, "component ireduce")
    for r in range(size):
        assert int(gd[r * nb:(r + 1) * nb].min()) == r + 1 == int(gd[r * nb:(r + 1) * nb].max())
    assert int(bc.min()) == size - 1 + 7 == int(bc.max())
    assert dt
    # host buffers: a nonblocking initiation cannot vote (it may not wait for its peers), so the path
    # depends only on the op and type every rank shares -- the host ranks join the engine on device
    # copies (nb_host_join), nothing reaches the previous owner of the slot (the stub)
    hs = (np.arange(16, dtype=np.float64) + 3 * rank).copy()
    h = np.zeros(16, dtype=np.float64)
    q = ctypes.c_void_p()
    assert L.mini_iallreduce(comm, hs.ctypes.data, h.ctypes.data, 16, dt, op, ctypes.byref(q)) == 0
    assert L.mini_wait(ctypes.byref(q)) == 0
    assert np.array_equal(h, sum(np.arange(16, dtype=np.float64) + 3 * r for r in range(size))), h
    assert L.mini_stub_calls(6) == 0
    m.lib.mini_op_destroy(op)


def movement(m, comm, oracle, rank, size, torch, ptrs):
    """the callers' slots: gather(v) / scatter(v) / allgatherv / alltoall(v) on MPI_INT, scan / exscan
    on MPI_FLOAT SUM (oracle: coll/basic's chain), host buffers to the stub"""
    L, pkg = m.lib, m.pkg
    idt = m.dtype_for_slot(pkg.T["INT32"])
    fdt = m.dtype_for_slot(pkg.T["FLOAT"])
    IA = lambda v: (ctypes.c_int * len(v))(*v)
    n = 1000
    mine = torch.arange(n, dtype=torch.int32, device="cuda") + 10000 * rank
    allv = torch.cat([torch.arange(n, dtype=torch.int32) + 10000 * q for q in range(size)])
    root = size - 1
    out = torch.zeros(n * size, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    assert L.mini_gather(comm, mine.data_ptr(), n, idt, out.data_ptr() if rank == root else None, n, idt, root) == 0
    if rank == root:
        assert torch.equal(out.cpu(), allv), "component gather"
    back = torch.zeros(n, dtype=torch.int32, device="cuda")
    assert L.mini_scatter(comm, out.data_ptr() if rank == root else None, n, idt, back.data_ptr(), n, idt, root) == 0
    assert torch.equal(back, mine), "component scatter"
    # ragged v-variants: rank q contributes q + 1 ints
    cnt = [q + 1 for q in range(size)]
    dsp = [int(sum(cnt[:q])) + 2 * q for q in range(size)]
    tot = dsp[-1] + cnt[-1]
    part = torch.full((cnt[rank],), rank + 1, dtype=torch.int32, device="cuda")
    gv = torch.zeros(tot, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    assert L.mini_allgatherv(comm, part.data_ptr(), cnt[rank], idt, gv.data_ptr(), IA(cnt), IA(dsp), idt) == 0
    want = torch.zeros(tot, dtype=torch.int32)
    for q in range(size):
        want[dsp[q]:dsp[q] + cnt[q]] = q + 1
    assert torch.equal(gv.cpu(), want), "component allgatherv"
    gz = torch.zeros(tot, dtype=torch.int32, device="cuda")
    assert L.mini_gatherv(comm, part.data_ptr(), cnt[rank], idt, gz.data_ptr() if rank == 0 else None, IA(cnt),
                          IA(dsp), idt, 0) == 0
    if rank == 0:
        assert torch.equal(gz.cpu(), want), "component gatherv"
    sv = torch.zeros(cnt[rank], dtype=torch.int32, device="cuda")
    assert L.mini_scatterv(comm, gv.data_ptr() if rank == 0 else None, IA(cnt), IA(dsp), idt, sv.data_ptr(),
                           cnt[rank], idt, 0) == 0
    assert bool((sv == rank + 1).all()), "component scatterv"
    # alltoall: block for q = 100 * rank + q
    a2 = torch.cat([torch.full((7,), 100 * rank + q, dtype=torch.int32) for q in range(size)]).cuda()
    a2o = torch.zeros_like(a2)
    torch.cuda.synchronize()
    assert L.mini_alltoall(comm, a2.data_ptr(), 7, idt, a2o.data_ptr(), 7, idt) == 0
    assert torch.equal(a2o.cpu(), torch.cat([torch.full((7,), 100 * q + rank, dtype=torch.int32) for q in range(size)]))
    # alltoallv: rank -> q sends (rank + q) % 3 + 1 ints of value 1000 * rank + q
    sc = [(rank + q) % 3 + 1 for q in range(size)]
    sd = [int(sum(sc[:q])) for q in range(size)]
    rc = [(q + rank) % 3 + 1 for q in range(size)]
    rd = [int(sum(rc[:q])) + q for q in range(size)]
    sv2 = torch.cat([torch.full((sc[q],), 1000 * rank + q, dtype=torch.int32) for q in range(size)]).cuda()
    rv2 = torch.full((rd[-1] + rc[-1],), -1, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    assert L.mini_alltoallv(comm, sv2.data_ptr(), IA(sc), IA(sd), idt, rv2.data_ptr(), IA(rc), IA(rd), idt) == 0
    got = rv2.cpu()
    for q in range(size):
        assert bool((got[rd[q]:rd[q] + rc[q]] == 1000 * q + rank).all()), "component alltoallv"
    # scan / exscan, MPI_FLOAT SUM: bit-exact with coll/basic's chain
    op = m.select_op(pkg.OP["SUM"])
    count = 3001
    xs = [opdata.make("FLOAT", count, 700 + q) for q in range(size)]
    for exclusive in (0, 1):
        want = [np.zeros_like(xs[0]) for _ in range(size)]
        oracle.oracle_scan(exclusive, size, count, pkg.T["FLOAT"], pkg.OP["SUM"], ptrs(xs), ptrs(want))
        dx = torch.from_numpy(xs[rank].view(np.uint8).copy()).cuda()
        dr = torch.zeros_like(dx)
        torch.cuda.synchronize()
        fn = L.mini_exscan if exclusive else L.mini_scan
        assert fn(comm, dx.data_ptr(), dr.data_ptr(), count, fdt, op) == 0
        if not (exclusive and rank == 0):
            opdata.assert_same("FLOAT", "SUM", dr.cpu().numpy().view(np.float32), want[rank], "component scan")
    resized_column(m, comm, rank, size, torch)
    # host buffers -> the stub
    h = np.zeros(64, dtype=np.int32)
    before = L.mini_stub_calls(7)
    assert L.mini_gather(comm, h.ctypes.data, 4, idt, h.ctypes.data, 4, idt, 0) == L.mini_stub_marker()
    assert L.mini_stub_calls(7) == before + 1
    assert L.mini_scan(comm, h.ctypes.data, h.ctypes.data, 4, fdt, op) == L.mini_stub_marker()
    assert L.mini_alltoall(comm, h.ctypes.data, 4, idt, h.ctypes.data, 4, idt) == L.mini_stub_marker()
    m.lib.mini_op_destroy(op)


def resized_column(m, comm, rank, size, torch):
    """MPI_Gather where ONLY the root's layout is derived: the root receives rank q's n ints into
    column q of an n x size int matrix (vector(n, 1, size, MPI_INT) resized to extent 4), the others
    send plain MPI_INT -- the path must not depend on the rank-local layout (else the root would
    fall back while the others enter the engine).  Then MPI_Scatter back out of the columns and
    MPI_Alltoall with the same column type on the receive side only."""
    L, pkg = m.lib, m.pkg
    n = 257
    idt = m.dtype_for_slot(pkg.T["INT32"])
    desc, used, tsize, _, true_ub = opal_strided_elems(n, OPAL_INT4, 4, 4 * size)
    col = L.mini_datatype_create_raw(desc, used, tsize, 0, 4, 0, true_ub, 0)  # MPI_Type_create_resized(.., 0, 4)
    root = size - 1
    mine = torch.arange(n, dtype=torch.int32, device="cuda") * 100 + rank
    mat = torch.full((n * size,), -7, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    if rank == root:
        assert L.mini_gather(comm, mine.data_ptr(), n, idt, mat.data_ptr(), 1, col, root) == 0
        want = (torch.arange(n, dtype=torch.int32).view(n, 1) * 100 + torch.arange(size, dtype=torch.int32).view(1, size))
        assert torch.equal(mat.cpu().view(n, size), want), "gather into a resized column type at the root"
    else:
        assert L.mini_gather(comm, mine.data_ptr(), n, idt, None, 1, col, root) == 0
    back = torch.zeros(n, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    assert L.mini_scatter(comm, mat.data_ptr() if rank == root else None, 1, col, back.data_ptr(), n, idt, root) == 0
    assert torch.equal(back, mine), "scatter out of a resized column type at the root"
    # alltoall: rank r sends block q = n ints (r, q) dense; receives into columns of its matrix
    snd = torch.cat([torch.arange(n, dtype=torch.int32) * 1000 + rank * 10 + q for q in range(size)]).cuda()
    got = torch.full((n * size,), -1, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    assert L.mini_alltoall(comm, snd.data_ptr(), n, idt, got.data_ptr(), 1, col) == 0
    want = torch.arange(n, dtype=torch.int32).view(n, 1) * 1000 + torch.arange(size, dtype=torch.int32).view(1, size) * 10 + rank
    assert torch.equal(got.cpu().view(n, size), want), "alltoall into resized column types"
    L.mini_datatype_destroy(col)


def split_main():
    """MPI_Comm_split with two colors on one node: world ranks {0,1} and {2,3} form two
    2-rank communicators with the SAME job id and the SAME context id (Open MPI 1.8 allocates one
    cid over the parent for every color, comm.c:610); each group selects coll/mi355x and runs
    collectives at the same time as the other -- each must see only its own members"""
    wrank = int(sys.argv[1])
    group, rank, size = wrank // 2, wrank % 2, 2
    import torch
    torch.cuda.set_device(wrank % torch.cuda.device_count())
    m = mini()
    oracle = load_oracle()
    m.install_oracle_base(oracle)
    comm = m.lib.mini_comm_create(rank, size, 42)
    m.lib.mini_comm_set_channel(comm, f"{sys.argv[3]}_g{group}".encode())
    m.lib.mini_comm_install(comm, m.lib.mini_stub_module())
    assert m.lib.mini_coll_select(comm, m.component_ptr(m.coll, "mca_coll_mi355x_component")) == 90
    pkg = m.pkg
    fdt = m.dtype_for_slot(pkg.T["FLOAT"])
    op = m.select_op(pkg.OP["SUM"])
    for it in range(20):
        for count in (1000, 300_001):
            x = torch.full((count,), float(100 * group + rank + it), device="cuda")
            y = torch.empty_like(x)
            torch.cuda.synchronize()
            assert m.lib.mini_allreduce(comm, x.data_ptr(), y.data_ptr(), count, fdt, op) == 0
            want = float(2 * (100 * group + it) + 1)
            assert bool((y == want).all()), (group, it, count, float(y[0]), want)
        b = torch.full((5000,), float(1000 * group + rank), device="cuda")
        torch.cuda.synchronize()
        assert m.lib.mini_bcast(comm, b.data_ptr(), 5000, fdt, 1) == 0
        assert bool((b == 1000 * group + 1).all()), ("split bcast", group)
    m.lib.mini_op_destroy(op)
    m.lib.mini_comm_destroy(comm)
    print(f"rank {wrank} split OK", flush=True)


class Status(ctypes.Structure):  # ompi_status_public_t (mpi.h.in:344-356)
    _fields_ = [("MPI_SOURCE", ctypes.c_int), ("MPI_TAG", ctypes.c_int), ("MPI_ERROR", ctypes.c_int),
                ("_cancelled", ctypes.c_int), ("_ucount", ctypes.c_size_t)]


BSEND, SSEND, STANDARD = 2, 0, 4   # mca_pml_base_send_mode_t (pml.h:78-85)


def pml_mixed(m, comm, rank, size, torch, fdt):
    """MPI semantics across buffer kinds through the component: dev->host, host->dev, dev->dev,
    host->host (eager and rendezvous sizes, MPI_FLOAT and a derived vector type), MPI_ANY_SOURCE
    over senders of both kinds, same-tag order across kinds, MPI_Bsend(dev) -> MPI_Recv(dev), the
    small unsafe exchange (both ranks send first), persistent MPI_Send_init / MPI_Recv_init /
    MPI_Start, MPI_Mprobe + MPI_Mrecv / MPI_Improbe + MPI_Imrecv, MPI_Cancel, MPI_Probe"""
    L = m.lib
    st = Status()
    ANY = -1
    left, right = (rank - 1) % size, (rank + 1) % size

    def mk(kind, vals):
        a = np.asarray(vals, dtype=np.float32)
        if kind == "host":
            h = a.copy()
            return h.ctypes.data, (lambda: h.copy()), h
        d = torch.from_numpy(a.copy()).cuda()
        torch.cuda.synchronize()
        return d.data_ptr(), (lambda: d.cpu().numpy()), d

    # a) every kind pairing around the ring, sizes either side of the 4 KiB eager limit
    for skind in ("dev", "host"):
        for rkind in ("dev", "host"):
            for n in (0, 5, 1024, 1025, 300_001):
                sp, _, ks = mk(skind, np.arange(n) + 1000 * rank)
                rp, read, kr = mk(rkind, np.full(n + 3, -1.0))
                rq, sq = ctypes.c_void_p(), ctypes.c_void_p()
                assert L.mini_irecv(rp, n + 3, fdt, left, 30, comm, ctypes.byref(rq)) == 0
                assert L.mini_isend(sp, n, fdt, right, 30, comm, ctypes.byref(sq)) == 0
                assert L.mini_wait_status(ctypes.byref(rq), ctypes.byref(st)) == 0
                assert L.mini_wait_status(ctypes.byref(sq), None) == 0
                assert (st.MPI_SOURCE, st.MPI_TAG, st._ucount) == (left, 30, 4 * n), (skind, rkind, n)
                got = read()
                assert np.array_equal(got[:n], np.arange(n, dtype=np.float32) + 1000 * left), (skind, rkind, n)
                assert (got[n:] == -1).all()
    # b) a derived send type from host memory into a contiguous device receive, and the reverse
    nblk = 700
    desc, used, tsize, lb, ub = opal_vector(nblk, 256, 512)
    vdt = m.derived(desc, used, tsize, lb, ub)
    full = np.arange(nblk * 128, dtype=np.float32) + rank
    hp, _, kh = mk("host", full)
    dp, dread, kd = mk("dev", np.zeros(nblk * 64))
    rq, sq = ctypes.c_void_p(), ctypes.c_void_p()
    assert L.mini_irecv(dp, nblk * 64, fdt, left, 31, comm, ctypes.byref(rq)) == 0
    assert L.mini_isend(hp, 1, vdt, right, 31, comm, ctypes.byref(sq)) == 0
    assert L.mini_wait(ctypes.byref(rq)) == 0 and L.mini_wait(ctypes.byref(sq)) == 0
    assert np.array_equal(dread(), (np.arange(nblk * 128, dtype=np.float32) + left).reshape(nblk, 128)[:, :64].ravel())
    back, bread, kb = mk("host", np.full(nblk * 128, -5.0))
    flat, _, kf = mk("dev", np.arange(nblk * 64) * 2.0 + rank)
    assert L.mini_irecv(back, 1, vdt, left, 32, comm, ctypes.byref(rq)) == 0
    assert L.mini_isend(flat, nblk * 64, fdt, right, 32, comm, ctypes.byref(sq)) == 0
    assert L.mini_wait(ctypes.byref(rq)) == 0 and L.mini_wait(ctypes.byref(sq)) == 0
    b = bread().reshape(nblk, 128)
    assert np.array_equal(b[:, :64].ravel(), np.arange(nblk * 64, dtype=np.float32) * 2 + left) and (b[:, 64:] == -5).all()
    L.mini_datatype_destroy(vdt)
    # c) same-tag order across kinds and sizes between one pair; ANY_SOURCE over both kinds
    sizes = [3, 2000, 64, 262_144, 1024, 5000, 1]
    if rank == 0:
        keep = []
        for i, n in enumerate(sizes):
            p_, _, k_ = mk("dev" if i % 2 else "host", np.full(n, float(i)))
            keep.append(k_)
            q = ctypes.c_void_p()
            assert L.mini_isend(p_, n, fdt, 1, 33, comm, ctypes.byref(q)) == 0
            keep.append(q)
        for q in keep[1::2]:
            assert L.mini_wait(ctypes.byref(q)) == 0
    elif rank == 1:
        for i, n in enumerate(sizes):
            p_, read, k_ = mk("host" if i % 3 else "dev", np.zeros(262_144))
            assert L.mini_recv(p_, 262_144, fdt, 0, 33, comm, ctypes.byref(st)) == 0
            assert st._ucount == 4 * n and (read()[:n] == i).all(), ("order across kinds", i)
    if rank != 0:
        p_, _, k_ = mk("host" if rank % 2 else "dev", np.full(50 + rank, float(rank)))
        assert L.mini_send(p_, 50 + rank, fdt, 0, 34, comm) == 0
    else:
        seen = set()
        for i in range(1, size):
            p_, read, k_ = mk("dev" if i % 2 else "host", np.zeros(64))
            assert L.mini_recv(p_, 64, fdt, ANY, 34, comm, ctypes.byref(st)) == 0
            r = st.MPI_SOURCE
            assert r not in seen and st._ucount == 4 * (50 + r) and (read()[:50 + r] == r).all()
            seen.add(r)
        assert seen == set(range(1, size))
    # d) MPI_Bsend from device memory into a device receive; the unsafe small exchange
    bp, _, kbp = mk("dev", np.full(100_000, 3.0 + rank))
    assert L.mini_send_mode(bp, 100_000, fdt, right, 35, BSEND, comm) == 0   # completes at once
    kbp.fill_(0)  # the caller may reuse a buffered send's buffer immediately
    rp, read, kr = mk("dev", np.zeros(100_000))
    assert L.mini_recv(rp, 100_000, fdt, left, 35, comm, None) == 0
    assert (read() == 3.0 + left).all(), "bsend payload"
    sp, _, ks = mk("dev", np.full(512, 1.0 + rank))
    hp, read, kh = mk("host", np.zeros(512))
    assert L.mini_send(sp, 512, fdt, right, 36, comm) == 0    # eager: returns before the peer receives
    assert L.mini_recv(hp, 512, fdt, left, 36, comm, None) == 0
    assert (read() == 1.0 + left).all()
    # e) persistent requests: 3 rounds of MPI_Start on one send / receive pair (host send buffer,
    #    device receive buffer); the buffers are re-read at every start
    sbuf = np.zeros(2048, dtype=np.float32)
    rp, read, kr = mk("dev", np.zeros(2048))
    ps, pr = ctypes.c_void_p(), ctypes.c_void_p()
    assert L.mini_send_init(sbuf.ctypes.data, 2048, fdt, right, 37, STANDARD, comm, ctypes.byref(ps)) == 0
    assert L.mini_recv_init(rp, 2048, fdt, left, 37, comm, ctypes.byref(pr)) == 0
    for it in range(3):
        sbuf[:] = 100 * it + rank
        assert L.mini_start(ctypes.byref(pr)) == 0 and L.mini_start(ctypes.byref(ps)) == 0
        assert L.mini_wait_status(ctypes.byref(pr), ctypes.byref(st)) == 0 and st.MPI_SOURCE == left
        assert L.mini_wait(ctypes.byref(ps)) == 0
        assert not L.mini_request_is_null(ps) and not L.mini_request_is_null(pr), "persistent requests stay"
        assert (read() == 100 * it + left).all(), ("persistent round", it)
    assert L.mini_request_free(ctypes.byref(ps)) == 0 and L.mini_request_free(ctypes.byref(pr)) == 0
    assert L.mini_request_is_null(ps) and L.mini_request_is_null(pr)
    # f) matched probe: MPI_Mprobe + MPI_Mrecv (host), MPI_Improbe + MPI_Imrecv (device); the probed
    #    message can no longer be matched by a wildcard receive
    sp1, _, k1 = mk("dev", np.full(300, 11.0 + rank))
    sp2, _, k2 = mk("host", np.full(300, 22.0 + rank))
    q1, q2 = ctypes.c_void_p(), ctypes.c_void_p()
    assert L.mini_isend(sp1, 300, fdt, right, 38, comm, ctypes.byref(q1)) == 0
    assert L.mini_isend(sp2, 300, fdt, right, 38, comm, ctypes.byref(q2)) == 0
    msg = ctypes.c_void_p()
    assert L.mini_mprobe(left, 38, comm, ctypes.byref(msg), ctypes.byref(st)) == 0
    assert (st.MPI_SOURCE, st.MPI_TAG, st._ucount) == (left, 38, 1200) and not L.mini_message_is_null(msg)
    other, oread, ko = mk("host", np.zeros(300))
    assert L.mini_recv(other, 300, fdt, ANY, ANY, comm, None) == 0
    assert (oread() == 22.0 + left).all(), "a wildcard receive took the probed message"
    mine, mread, km = mk("host", np.zeros(300))
    assert L.mini_mrecv(mine, 300, fdt, ctypes.byref(msg), ctypes.byref(st)) == 0 and L.mini_message_is_null(msg)
    assert (mread() == 11.0 + left).all() and st._ucount == 1200
    assert L.mini_wait(ctypes.byref(q1)) == 0 and L.mini_wait(ctypes.byref(q2)) == 0
    sp3, _, k3 = mk("host", np.full(10, 7.0 + rank))
    assert L.mini_isend(sp3, 10, fdt, right, 39, comm, ctypes.byref(q1)) == 0
    flag = ctypes.c_int(0)
    t0 = time.time()
    while not flag.value:
        assert L.mini_improbe(ANY, 39, comm, ctypes.byref(flag), ctypes.byref(msg), ctypes.byref(st)) == 0
        assert time.time() - t0 < 30, "improbe never matched"
    dv, dread, kdv = mk("dev", np.zeros(10))
    rq = ctypes.c_void_p()
    assert L.mini_imrecv(dv, 10, fdt, ctypes.byref(msg), ctypes.byref(rq)) == 0 and L.mini_message_is_null(msg)
    assert L.mini_wait_status(ctypes.byref(rq), ctypes.byref(st)) == 0 and st.MPI_SOURCE == left
    assert (dread() == 7.0 + left).all()
    assert L.mini_wait(ctypes.byref(q1)) == 0
    # g) MPI_Cancel of a receive nothing will match; MPI_Probe (blocking) sees a host message
    cq = ctypes.c_void_p()
    cb = np.zeros(4, dtype=np.float32)
    assert L.mini_irecv(cb.ctypes.data, 4, fdt, left, 999, comm, ctypes.byref(cq)) == 0
    assert L.mini_cancel(cq) == 0
    assert L.mini_wait_status(ctypes.byref(cq), ctypes.byref(st)) == 0 and st._cancelled == 1
    pb, _, kpb = mk("host", np.full(6, 1.5))
    assert L.mini_isend(pb, 6, fdt, right, 40, comm, ctypes.byref(q1)) == 0
    assert L.mini_probe(left, 40, comm, ctypes.byref(st)) == 0 and st._ucount == 24
    assert L.mini_recv(cb.ctypes.data, 4, fdt, left, 40, comm, ctypes.byref(st)) == 15   # truncated
    assert st._ucount == 24 and (cb == 1.5).all()
    assert L.mini_wait(ctypes.byref(q1)) == 0


def pml_main():
    """MPI_Send / MPI_Ssend / MPI_Recv / MPI_Isend / MPI_Irecv / MPI_Iprobe (and the persistent and
    matched-probe calls) through the PML slot (`mca_pml`, the table the MPI layer calls, e.g.
    ompi/mpi/c/send.c:67) once coll/mi355x's init_query has hooked it: every call on the engine
    communicator -- device or host buffer -- goes to the engine's one matching queue, nothing reaches
    the saved (stub) PML, and closing the component restores the table"""
    rank, size = int(sys.argv[1]), int(sys.argv[2])
    import torch
    torch.cuda.set_device(rank % torch.cuda.device_count())
    m = mini()
    L, pkg = m.lib, m.pkg
    oracle = load_oracle()
    m.install_oracle_base(oracle)
    comp = m.component_ptr(m.coll, "mca_coll_mi355x_component")
    stub_send = L.mini_pml_fn(1)
    assert L.mini_coll_init(comp) == 0
    hooked = [L.mini_pml_fn(w) for w in range(13)]
    names = ["isend", "send", "irecv", "recv", "iprobe", "probe", "isend_init", "irecv_init", "start", "improbe",
             "mprobe", "imrecv", "mrecv"]
    for w, nm in enumerate(names):
        assert hooked[w] == m.addr(m.coll, f"mca_coll_mi355x_pml_{nm}"), f"pml_{nm} not hooked"
    comm = L.mini_comm_create(rank, size, 42)
    L.mini_comm_set_channel(comm, sys.argv[3].encode())
    L.mini_comm_install(comm, L.mini_stub_module())
    assert L.mini_coll_select(comm, comp) == 90
    fdt = m.dtype_for_slot(pkg.T["FLOAT"])
    ANY = -1
    st = Status()
    n = 1 << 20
    # 1. MPI_Send from rank 0 to every rank, MPI_Recv(MPI_ANY_SOURCE) with the status
    if rank == 0:
        for q in range(1, size):
            x = torch.arange(n, dtype=torch.float32, device="cuda") + 1000 * q
            torch.cuda.synchronize()
            assert L.mini_send(x.data_ptr(), n, fdt, q, 11, comm) == 0
    else:
        y = torch.zeros(n, device="cuda")
        assert L.mini_recv(y.data_ptr(), n, fdt, ANY, 11, comm, ctypes.byref(st)) == 0
        assert torch.equal(y, torch.arange(n, dtype=torch.float32, device="cuda") + 1000 * rank), "send/recv data"
        assert (st.MPI_SOURCE, st.MPI_TAG, st.MPI_ERROR, st._ucount) == (0, 11, 0, 4 * n), \
            (st.MPI_SOURCE, st.MPI_TAG, st.MPI_ERROR, st._ucount)
    # 2. MPI_Ssend back to rank 0, received by source in rank order, MPI_STATUS_IGNORE
    if rank == 0:
        for q in range(1, size):
            y = torch.zeros(777, dtype=torch.int32, device="cuda")
            assert L.mini_recv(y.data_ptr(), 777, m.dtype_for_slot(pkg.T["INT32"]), q, ANY, comm, None) == 0
            assert torch.equal(y, torch.full((777,), 7 * q, dtype=torch.int32, device="cuda")), "ssend data"
    else:
        x = torch.full((777,), 7 * rank, dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()
        assert L.mini_ssend(x.data_ptr(), 777, m.dtype_for_slot(pkg.T["INT32"]), 0, 12, comm) == 0
    # 3. ring of MPI_Irecv + MPI_Isend (receive posted first), MPI_Wait with status
    nr = 3_000_001
    src = torch.full((nr,), float(rank + 1), device="cuda")
    dst = torch.zeros(nr, device="cuda")
    torch.cuda.synchronize()
    rq, sq = ctypes.c_void_p(), ctypes.c_void_p()
    left, right = (rank - 1) % size, (rank + 1) % size
    assert L.mini_irecv(dst.data_ptr(), nr, fdt, left, 13, comm, ctypes.byref(rq)) == 0
    assert L.mini_isend(src.data_ptr(), nr, fdt, right, 13, comm, ctypes.byref(sq)) == 0
    assert L.mini_wait_status(ctypes.byref(sq), None) == 0
    assert L.mini_wait_status(ctypes.byref(rq), ctypes.byref(st)) == 0
    assert L.mini_request_is_null(rq) and L.mini_request_is_null(sq)
    assert (st.MPI_SOURCE, st.MPI_TAG, st._ucount) == (left, 13, 4 * nr)
    assert bool((dst == left + 1).all()), "isend/irecv ring"
    # 4. a derived send type (vector(1000, 64, 128, MPI_FLOAT)) into a contiguous receive
    if size >= 2 and rank in (0, 1):
        nblk = 1000
        desc, used, tsize, lb, ub = opal_vector(nblk, 256, 512)
        vdt = m.derived(desc, used, tsize, lb, ub)
        if rank == 0:
            full = torch.arange(nblk * 128, dtype=torch.float32, device="cuda")
            torch.cuda.synchronize()
            assert L.mini_send(full.data_ptr(), 1, vdt, 1, 14, comm) == 0
        else:
            got = torch.zeros(nblk * 64, device="cuda")
            assert L.mini_recv(got.data_ptr(), nblk * 64, fdt, 0, 14, comm, ctypes.byref(st)) == 0
            want = torch.arange(nblk * 128, dtype=torch.float32).view(nblk, 128)[:, :64].reshape(-1)
            assert torch.equal(got.cpu(), want), "derived send -> contiguous recv"
            assert st._ucount == tsize
        L.mini_datatype_destroy(vdt)
    # 5. MPI_Iprobe sees the envelope before the receive; truncation reports MPI_ERR_TRUNCATE
    if rank == 0:
        x = torch.ones(1000, device="cuda")
        torch.cuda.synchronize()
        q = ctypes.c_void_p()
        assert L.mini_isend(x.data_ptr(), 1000, fdt, size - 1, 15, comm, ctypes.byref(q)) == 0
        assert L.mini_wait_status(ctypes.byref(q), None) == 0
    elif rank == size - 1:
        flag = ctypes.c_int(0)
        t0 = time.time()
        while not flag.value:
            assert L.mini_iprobe(0, 15, comm, ctypes.byref(flag), ctypes.byref(st)) == 0
            assert time.time() - t0 < 30, "iprobe never matched"
        assert (st.MPI_SOURCE, st.MPI_TAG, st._ucount) == (0, 15, 4000)
        y = torch.zeros(500, device="cuda")
        rc = L.mini_recv(y.data_ptr(), 500, fdt, 0, 15, comm, ctypes.byref(st))
        assert rc == 15 and st.MPI_ERROR == 15, (rc, st.MPI_ERROR)  # MPI_ERR_TRUNCATE
        assert bool((y == 1).all())
    # 6. edge cases: zero-count messages, MPI_PROC_NULL, MPI_ANY_TAG, a derived receive type, many
    #    outstanding nonblocking messages between the same pair (ob1's per-pair ordering)
    z = torch.zeros(4, device="cuda")
    if rank == 0:
        assert L.mini_send(z.data_ptr(), 0, fdt, 1, 20, comm) == 0
    elif rank == 1:
        assert L.mini_recv(z.data_ptr(), 0, fdt, 0, 20, comm, ctypes.byref(st)) == 0
        assert (st.MPI_SOURCE, st.MPI_TAG, st._ucount) == (0, 20, 0)
    PROC_NULL = -2
    assert L.mini_send(z.data_ptr(), 4, fdt, PROC_NULL, 21, comm) == 0
    assert L.mini_recv(z.data_ptr(), 4, fdt, PROC_NULL, 21, comm, ctypes.byref(st)) == 0
    assert st.MPI_SOURCE == PROC_NULL and st._ucount == 0, (st.MPI_SOURCE, st._ucount)
    if rank in (0, 1):
        nblk = 300
        desc, used, tsize, lb, ub = opal_vector(nblk, 256, 512)
        vdt = m.derived(desc, used, tsize, lb, ub)
        if rank == 1:
            flat = torch.arange(nblk * 64, dtype=torch.float32, device="cuda") * 3
            torch.cuda.synchronize()
            assert L.mini_send(flat.data_ptr(), nblk * 64, fdt, 0, 22, comm) == 0
        else:
            strided = torch.full((nblk * 128,), -1.0, device="cuda")
            assert L.mini_recv(strided.data_ptr(), 1, vdt, 1, ANY, comm, ctypes.byref(st)) == 0
            got = strided.view(nblk, 128)
            assert torch.equal(got[:, :64].reshape(-1), torch.arange(nblk * 64, dtype=torch.float32, device="cuda") * 3)
            assert bool((got[:, 64:] == -1).all()), "gaps of the receive type untouched"
            assert st.MPI_TAG == 22
        L.mini_datatype_destroy(vdt)
        nmsg, cnt = 24, 5000
        bufs = [torch.full((cnt,), float(100 * rank + i), device="cuda") for i in range(nmsg)]
        torch.cuda.synchronize()
        reqs = [ctypes.c_void_p() for _ in range(nmsg)]
        for i in range(nmsg):  # same tag: the messages must match in sending order
            if rank == 0:
                assert L.mini_isend(bufs[i].data_ptr(), cnt, fdt, 1, 23, comm, ctypes.byref(reqs[i])) == 0
            else:
                assert L.mini_irecv(bufs[i].data_ptr(), cnt, fdt, 0, 23, comm, ctypes.byref(reqs[i])) == 0
        for i in range(nmsg):
            assert L.mini_wait_status(ctypes.byref(reqs[i]), None) == 0
        if rank == 1:
            for i in range(nmsg):
                assert bool((bufs[i] == float(i)).all()), ("ordering", i, float(bufs[i][0]))
    # 7. one matching queue for every buffer kind (ob1: pml_ob1_cuda.c:52-100 / pml_ob1_recvreq.c:647-663)
    pml_mixed(m, comm, rank, size, torch, fdt)
    # nothing of the above reached the saved (stub) PML: every call on an engine communicator is the engine's
    assert [L.mini_pml_stub_calls(w) for w in range(13)] == [0] * 13, [L.mini_pml_stub_calls(w) for w in range(13)]
    L.mini_comm_destroy(comm)
    assert L.mini_coll_close(comp) == 0
    assert L.mini_pml_fn(1) == stub_send, "component close restores the PML table"
    print(f"rank {rank} pml OK", flush=True)


def tuned_vars_main():
    """coll/tuned's variables read through the MCA variable system (no OMPI_MCA_coll_tuned_* in the
    environment): forced allreduce algorithm 3 (recursive doubling) on one communicator, then a
    rules file naming algorithm 2 (nonoverlapping) for every size on the next"""
    rank, size = int(sys.argv[1]), int(sys.argv[2])
    import torch
    torch.cuda.set_device(rank % torch.cuda.device_count())
    m = mini()
    L, pkg = m.lib, m.pkg
    oracle = load_oracle()
    m.install_oracle_base(oracle)
    L.mini_tuned_register.argtypes = [ctypes.c_int] * 5 + [ctypes.c_char_p]
    comp = m.component_ptr(m.coll, "mca_coll_mi355x_component")
    ptrs = lambda arrs: (ctypes.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])
    ty, code = pkg.T["FLOAT"], pkg.OP["SUM"]
    fdt = m.dtype_for_slot(ty)
    op = m.select_op(code)
    count = 300_001
    xs = [opdata.make("FLOAT", count, 900 + r) for r in range(size)]
    want = {}
    for alg in (0, 2, 3):
        outs = [np.zeros_like(xs[0]) for _ in range(size)]
        oracle.oracle_allreduce(alg, size, count, ty, code, 0, ptrs(xs), ptrs(outs))
        want[alg] = outs[rank]
    assert not np.array_equal(want[3], want[0]) and not np.array_equal(want[2], want[0]), "orders must differ"
    rules = pathlib.Path(f"/tmp/mi355x_rules_{sys.argv[3]}_{rank}.conf")
    rules.write_text(f"1\n2\n1\n{size} 1\n0 2 0 0\n")
    for step, (args, alg) in enumerate((((1, 3, 0, 0, 0, None), 3), ((1, 0, 0, 0, 0, str(rules).encode()), 2))):
        assert L.mini_tuned_register(*args) == 0
        comm = L.mini_comm_create(rank, size, 42 + step)
        L.mini_comm_set_channel(comm, f"{sys.argv[3]}_{step}".encode())
        L.mini_comm_install(comm, L.mini_stub_module())
        assert L.mini_coll_select(comm, comp) == 90
        dx = torch.from_numpy(xs[rank].view(np.uint8).copy()).cuda()
        dr = torch.zeros_like(dx)
        torch.cuda.synchronize()
        assert L.mini_allreduce(comm, dx.data_ptr(), dr.data_ptr(), count, fdt, op) == 0
        opdata.assert_same("FLOAT", "SUM", dr.cpu().numpy().view(np.float32), want[alg], f"tuned variables step {step}")
        L.mini_comm_destroy(comm)
    rules.unlink()
    L.mini_op_destroy(op)
    print(f"rank {rank} tuned_vars OK", flush=True)


def _linear(oracle, code, slot, xs):
    """coll/basic's linear reduction order (coll_basic_reduce.c:215-250): acc = x[n-1], then
    acc = x[i] op acc for i = n-2..0, through the oracle's 2-buff loop"""
    acc = xs[-1].copy()
    for x in reversed(xs[:-1]):
        assert oracle.oracle_op_2buff(code, slot, x.ctypes.data, acc.ctypes.data, len(acc)) == 0
    return acc


def staging_main():
    """coll/cuda's host staging (coll_cuda_allreduce.c:43-75 & siblings) for the reductions the engine
    declines, over a lower-priority module that really reduces on the CPU (the harness's host module:
    coll/basic's orders through the host channel) and fails any call that hands it device memory:
      * a non-commutative user MPI_Op (a op b = 3a + b on MPI_INT) on device buffers, rank 0 on host
        buffers: allreduce (also in place), reduce, reduce_scatter_block, reduce_scatter, scan, exscan,
        iallreduce, ireduce, ireduce_scatter_block;
      * MPI_SUM / MPI_PROD over MPI_LONG_DOUBLE and C_LONG_DOUBLE_COMPLEX served by the engine (the x87
        add / multiply on the GPU), bit-exact with the oracle's schedule on the host's x87;
      * MAXLOC / MINLOC over MPI_LONG_DOUBLE_INT served by the engine's gather-then-fold form
        (allreduce, reduce, reduce_scatter_block, reduce_scatter, scan) in coll/tuned's order for the
        decision and for forced algorithms, on NaN-bearing pairs, nothing staged;
      * MAXLOC / MINLOC over the other five pair types (built as libmpi builds them: OPAL-predefined
        flag cleared, DOUBLE_INT 12 bytes in 16) and MAX / MIN over MPI_LONG_DOUBLE on device
        buffers are served by the engine, bit-exact with the oracle, with nothing staged;
      * host buffers on every rank reach the host module and come back reduced.
    The host module never saw a device pointer."""
    rank, size = int(sys.argv[1]), int(sys.argv[2])
    import torch
    torch.cuda.set_device(rank % torch.cuda.device_count())
    m = mini()
    L, pkg = m.lib, m.pkg
    oracle = load_oracle()
    m.install_oracle_base(oracle)
    vp = ctypes.c_void_p
    L.mini_host_module.restype = vp
    L.mini_op_create_user.restype = vp
    L.mini_op_create_user.argtypes = [vp, ctypes.c_int]
    comm = L.mini_comm_create(rank, size, 42)
    assert L.mini_comm_set_channel(comm, sys.argv[3].encode()) == 0
    L.mini_comm_install(comm, L.mini_host_module())
    assert L.mini_coll_select(comm, m.component_ptr(m.coll, "mca_coll_mi355x_component")) == 90
    staged = ctypes.c_ulong.in_dll(m.coll, "mca_coll_mi355x_staged_calls")
    ptrs = lambda arrs: (ctypes.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])
    host = rank == 0

    def put(a, on_host=False):
        if on_host:
            h = np.ascontiguousarray(a).copy()
            return h, h.ctypes.data, (lambda: h.copy())
        d = torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).copy()).cuda()
        return d, d.data_ptr(), (lambda: d.cpu().numpy().view(a.dtype).copy())

    say = lambda what: print(f"rank {rank} staging: {what}", flush=True)
    say("selected")
    # ---- 1. a non-commutative user op: inout = 3 * in + inout (int32, wrapping)
    USER = ctypes.CFUNCTYPE(None, vp, vp, ctypes.POINTER(ctypes.c_int), vp)

    @USER
    def user_fn(invec, inoutvec, lenp, dtp):
        n = lenp[0]
        a = np.ctypeslib.as_array(ctypes.cast(invec, ctypes.POINTER(ctypes.c_int32)), (n,))
        b = np.ctypeslib.as_array(ctypes.cast(inoutvec, ctypes.POINTER(ctypes.c_int32)), (n,))
        b[:] = a * np.int32(3) + b

    uop = L.mini_op_create_user(ctypes.cast(user_fn, vp).value, 0)
    idt = m.dtype_for_slot(pkg.T["INT32"])
    f = lambda a, b: (a * np.int32(3) + b).astype(np.int32)   # a op b, a = in, b = inout
    count = 70_003   # several host-channel slots
    xs = [(np.arange(count, dtype=np.int32) * (r + 2) + 11 * r).astype(np.int32) for r in range(size)]
    lin = xs[-1].copy()
    for x in reversed(xs[:-1]):
        lin = f(x, lin)
    before = staged.value
    sk, sp, _ = put(xs[rank], host)   # (keep the buffer alive)
    rb, rp, rread = put(np.zeros(count, np.int32), host)
    torch.cuda.synchronize()
    assert L.mini_allreduce(comm, sp, rp, count, idt, uop) == 0
    assert np.array_equal(rread(), lin), "user-op allreduce"
    ib, ip, iread = put(xs[rank], host)
    torch.cuda.synchronize()
    assert L.mini_allreduce(comm, 1, ip, count, idt, uop) == 0      # MPI_IN_PLACE
    assert np.array_equal(iread(), lin), "user-op allreduce in place"
    root = size - 1
    rb2, rp2, rread2 = put(np.zeros(count, np.int32), host)
    torch.cuda.synchronize()
    assert L.mini_reduce(comm, sp, rp2 if rank == root else None, count, idt, uop, root) == 0
    if rank == root:
        assert np.array_equal(rread2(), lin), "user-op reduce"
    rc = 3001
    ys = [(np.arange(rc * size, dtype=np.int32) - 77 * r).astype(np.int32) for r in range(size)]
    ylin = ys[-1].copy()
    for y in reversed(ys[:-1]):
        ylin = f(y, ylin)
    yk, ysp, _ = put(ys[rank], host)
    ob, op_, oread = put(np.zeros(rc, np.int32), host)
    torch.cuda.synchronize()
    assert L.mini_reduce_scatter_block(comm, ysp, op_, rc, idt, uop) == 0
    assert np.array_equal(oread(), ylin[rank * rc:(rank + 1) * rc]), "user-op reduce_scatter_block"
    counts = [rc - 5 * q for q in range(size)]
    tot = sum(counts)
    lo = sum(counts[:rank])
    vk, vsp, _ = put(ys[rank][:tot], host)
    wb, wp, wread = put(np.zeros(counts[rank], np.int32), host)
    torch.cuda.synchronize()
    assert L.mini_reduce_scatter(comm, vsp, wp, (ctypes.c_int * size)(*counts), idt, uop) == 0
    assert np.array_equal(wread(), ylin[:tot][lo:lo + counts[rank]]), "user-op reduce_scatter"
    chain = [xs[0].copy()]
    for x in xs[1:]:
        chain.append(f(chain[-1], x))
    for exclusive in (0, 1):
        sentinel = np.full(count, -9, np.int32)
        cb, cp, cread = put(sentinel, host)
        torch.cuda.synchronize()
        fn = L.mini_exscan if exclusive else L.mini_scan
        assert fn(comm, sp, cp, count, idt, uop) == 0
        want = (chain[rank - 1] if rank else sentinel) if exclusive else chain[rank]
        assert np.array_equal(cread(), want), ("user-op scan", exclusive)
    say("blocking user-op calls done")
    # nonblocking forms: staged at initiation, copied back when the host request completes
    reqs = [ctypes.c_void_p() for _ in range(3)]
    nb1, np1, nread1 = put(np.zeros(count, np.int32), host)
    nb2, np2, nread2 = put(np.zeros(count, np.int32), host)
    nb3, np3, nread3 = put(np.zeros(rc, np.int32), host)
    torch.cuda.synchronize()
    assert L.mini_iallreduce(comm, sp, np1, count, idt, uop, ctypes.byref(reqs[0])) == 0
    assert L.mini_ireduce(comm, sp, np2 if rank == 0 else None, count, idt, uop, 0, ctypes.byref(reqs[1])) == 0
    assert L.mini_ireduce_scatter_block(comm, ysp, np3, rc, idt, uop, ctypes.byref(reqs[2])) == 0
    for q in reqs:
        assert L.mini_wait(ctypes.byref(q)) == 0
    assert np.array_equal(nread1(), lin), "user-op iallreduce"
    if rank == 0:
        assert np.array_equal(nread2(), lin), "user-op ireduce"
    assert np.array_equal(nread3(), ylin[rank * rc:(rank + 1) * rc]), "user-op ireduce_scatter_block"
    # ten calls, each staged once on a rank with device buffers (rank 0's host buffers need none)
    assert staged.value - before == (0 if host else 10), staged.value - before
    L.mini_op_destroy(uop)

    say("user op done")
    # ---- 2. x87 arithmetic slots: SUM / PROD over LONG_DOUBLE (16 B, the engine's fold families)
    #         and C_LONG_DOUBLE_COMPLEX (32 B, gather-then-fold) -- the x87 add / multiply on the GPU
    #         (f80_arith.hpp), engine-served in the reference schedule's order, nothing staged
    for opname, tname in (("SUM", "LONG_DOUBLE"), ("PROD", "LONG_DOUBLE"), ("SUM", "C_LONG_DOUBLE_COMPLEX"),
                          ("PROD", "C_LONG_DOUBLE_COMPLEX")):
        code, slot = pkg.OP[opname], pkg.T[tname]
        assert pkg.rt().mi355x_comm_op_supported(code, slot)
        op = m.select_op(code)
        dt = m.dtype_for_slot(slot)
        for n in (3, 20_001):
            xs2 = [opdata.make(tname, n, 40 + r) for r in range(size)]
            outs = [np.zeros_like(xs2[0]) for _ in range(size)]
            oracle.oracle_allreduce(0, size, n, slot, code, 0, ptrs(xs2), ptrs(outs))
            before = staged.value
            d, dp, read = put(xs2[rank])
            o, opp, oread2 = put(np.zeros_like(xs2[0]))
            torch.cuda.synchronize()
            assert L.mini_allreduce(comm, dp, opp, n, dt, op) == 0
            opdata.assert_same(tname, opname, oread2(), outs[rank], f"engine x87 {opname} allreduce n={n}")
            assert staged.value == before, "an x87 SUM / PROD call was staged"
        L.mini_op_destroy(op)
    # MAXLOC / MINLOC over MPI_LONG_DOUBLE_INT (32-byte pairs): served by the engine's gather-then-
    # fold form in the per-element order of the algorithm coll/tuned runs -- the fixed decision, then
    # forced algorithms (allreduce 3 / 4 / 5, reduce 2 / 5, reduce_scatter 1 / 2 / 3) on communicators
    # created after coll_tuned_use_dynamic_rules is set -- on pairs holding NaN and -0.0 values
    # (opdata.make), where the operand roles decide the result (op_base_functions.c:96-101), against
    # the oracle's simulations of those schedules; nothing staged
    L.mini_tuned_register.argtypes = [ctypes.c_int] * 5 + [ctypes.c_char_p]
    tname = "LONG_DOUBLE_INT"
    slot = pkg.T[tname]
    dt = m.dtype_for_slot(slot)
    n, rc_ = 20_001, 3001
    counts = [rc_ - 5 * q for q in range(size)]
    tot = sum(counts)
    lo = sum(counts[:rank])
    legs = [(comm, 0, 0, 0)]
    for step, (ar, red, rs) in enumerate(((3, 0, 1), (4, 2, 2), (5, 5, 3))):
        assert L.mini_tuned_register(1, ar, red, 0, rs, None) == 0
        cm = L.mini_comm_create(rank, size, 142 + step)
        assert L.mini_comm_set_channel(cm, f"{sys.argv[3]}_ldi{step}".encode()) == 0
        L.mini_comm_install(cm, L.mini_host_module())
        assert L.mini_coll_select(cm, m.component_ptr(m.coll, "mca_coll_mi355x_component")) == 90
        legs.append((cm, ar, red, rs))
    assert L.mini_tuned_register(0, 0, 0, 0, 0, None) == 0
    differs = 0
    for leg, (cm, ar, red, rs) in enumerate(legs):
        # the forced legs gather in 64 KiB windows (10 windows per allreduce; in place included)
        os.environ["MI355X_GFOLD_WINDOW_KIB"] = "64" if leg else "0"
        for opname in ("MAXLOC", "MINLOC"):
            code = pkg.OP[opname]
            assert pkg.rt().mi355x_comm_op_supported(code, slot)
            op = m.select_op(code)
            xs2 = [opdata.make(tname, n, 40 + r) for r in range(size)]
            before = staged.value
            what = f"LDI {opname} ar={ar} red={red} rs={rs}"
            outs = [np.zeros_like(xs2[0]) for _ in range(size)]
            oracle.oracle_allreduce(ar, size, n, slot, code, 0, ptrs(xs2), ptrs(outs))
            differs += int(len(opdata.mismatches(tname, opname, outs[rank], _linear(oracle, code, slot, xs2))) > 0)
            d, dp, read = put(xs2[rank])
            o, opp, oread2 = put(np.zeros_like(xs2[0]))
            torch.cuda.synchronize()
            assert L.mini_allreduce(cm, dp, opp, n, dt, op) == 0
            opdata.assert_same(tname, opname, oread2(), outs[rank], what + " allreduce")
            ip_, ipp, iread = put(xs2[rank])
            torch.cuda.synchronize()
            assert L.mini_allreduce(cm, 1, ipp, n, dt, op) == 0      # MPI_IN_PLACE
            opdata.assert_same(tname, opname, iread(), outs[rank], what + " allreduce in place")
            root = size - 1
            want = np.zeros_like(xs2[0])
            oracle.oracle_reduce(red, size, root, n, slot, code, 0, ptrs(xs2), want.ctypes.data)
            o3, opp3, oread3 = put(np.zeros_like(xs2[0]))
            torch.cuda.synchronize()
            assert L.mini_reduce(cm, dp, opp3 if rank == root else None, n, dt, op, root) == 0
            if rank == root:
                opdata.assert_same(tname, opname, oread3(), want, what + " reduce")
            ys2 = [opdata.make(tname, rc_ * size, 70 + r) for r in range(size)]
            if red == 0:
                youts = [np.zeros(rc_, dtype=ys2[0].dtype) for _ in range(size)]
                oracle.oracle_reduce_scatter_block(size, rc_, slot, code, ptrs(ys2), ptrs(youts))
                ywant = youts[rank]
            else:  # coll/basic: the (forced) reduce to 0, then the scatter
                yall = np.zeros_like(ys2[0])
                oracle.oracle_reduce(red, size, 0, rc_ * size, slot, code, 0, ptrs(ys2), yall.ctypes.data)
                ywant = yall[rank * rc_:(rank + 1) * rc_]
            yd, ydp, _ = put(ys2[rank])
            yo, yop, yread = put(np.zeros(rc_, dtype=ys2[0].dtype))
            torch.cuda.synchronize()
            assert L.mini_reduce_scatter_block(cm, ydp, yop, rc_, dt, op) == 0
            opdata.assert_same(tname, opname, yread(), ywant, what + " reduce_scatter_block")
            yi, yip, yiread = put(ys2[rank])
            torch.cuda.synchronize()
            assert L.mini_reduce_scatter_block(cm, 1, yip, rc_, dt, op) == 0   # MPI_IN_PLACE
            opdata.assert_same(tname, opname, yiread()[:rc_], ywant, what + " reduce_scatter_block in place")
            vouts = [np.zeros(counts[q], dtype=ys2[0].dtype) for q in range(size)]
            vin = [y[:tot].copy() for y in ys2]
            oracle.oracle_reduce_scatter_alg(rs, size, (ctypes.c_int * size)(*counts), slot, code, ptrs(vin), ptrs(vouts))
            vd, vdp, _ = put(vin[rank])
            vo, vop, vread = put(np.zeros(counts[rank], dtype=ys2[0].dtype))
            torch.cuda.synchronize()
            assert L.mini_reduce_scatter(cm, vdp, vop, (ctypes.c_int * size)(*counts), dt, op) == 0
            opdata.assert_same(tname, opname, vread(), vouts[rank], what + " reduce_scatter")
            if cm == comm:
                swant = [np.zeros_like(xs2[0]) for _ in range(size)]
                oracle.oracle_scan(0, size, n, slot, code, ptrs(xs2), ptrs(swant))
                so, sop, sread = put(np.zeros_like(xs2[0]))
                torch.cuda.synchronize()
                assert L.mini_scan(cm, dp, sop, n, dt, op) == 0
                opdata.assert_same(tname, opname, sread(), swant[rank], what + " scan")
            assert staged.value == before, "MPI_LONG_DOUBLE_INT was staged, not served by the engine"
            L.mini_op_destroy(op)
        if cm != comm:
            L.mini_comm_destroy(cm)
    os.environ.pop("MI355X_GFOLD_WINDOW_KIB", None)
    # the data discriminates: coll/basic's linear order gives other bits than the orders checked
    assert differs > 0, "the LDI test data does not separate the schedule orders"
    say("staged x87 done")
    # ---- 3. engine-served: MAXLOC / MINLOC over the five other pair types, MAX / MIN over LONG_DOUBLE
    for opname in ("MAXLOC", "MINLOC"):
        for tname in ("FLOAT_INT", "DOUBLE_INT", "LONG_INT", "2INT", "SHORT_INT"):
            code, slot = pkg.OP[opname], pkg.T[tname]
            dt = m.dtype_for_slot(slot)
            fn = m.coll.mca_coll_mi355x_reducible_type
            fn.argtypes = [ctypes.c_void_p]
            assert fn(dt) == slot, tname
            op = m.select_op(code)
            for n in (1, 4001, 100_003):
                xs3 = [opdata.make(tname, n, 60 + r) for r in range(size)]
                outs = [np.zeros_like(xs3[0]) for _ in range(size)]
                oracle.oracle_allreduce(0, size, n, slot, code, 0, ptrs(xs3), ptrs(outs))
                before = staged.value
                d, dp, read = put(xs3[rank])
                o, opp, oread3 = put(np.zeros_like(xs3[0]))
                torch.cuda.synchronize()
                assert L.mini_allreduce(comm, dp, opp, n, dt, op) == 0
                opdata.assert_same(tname, opname, oread3(), outs[rank], f"engine pair allreduce n={n}")
                assert staged.value == before, f"{opname}/{tname} was staged, not served by the engine"
                # MPI_Reduce to the last rank
                want = np.zeros_like(xs3[0])
                oracle.oracle_reduce(0, size, size - 1, n, slot, code, 0, ptrs(xs3), want.ctypes.data)
                r2, rp3, rread3 = put(np.zeros_like(xs3[0]))
                torch.cuda.synchronize()
                assert L.mini_reduce(comm, dp, rp3 if rank == size - 1 else None, n, dt, op, size - 1) == 0
                if rank == size - 1:
                    opdata.assert_same(tname, opname, rread3(), want, f"engine pair reduce n={n}")
            L.mini_op_destroy(op)
    for opname in ("MAX", "MIN"):
        code, slot = pkg.OP[opname], pkg.T["LONG_DOUBLE"]
        assert pkg.rt().mi355x_comm_op_supported(code, slot)
        op = m.select_op(code)
        dt = m.dtype_for_slot(slot)
        n = 30_007
        xs4 = [opdata.make("LONG_DOUBLE", n, 80 + r) for r in range(size)]
        outs = [np.zeros_like(xs4[0]) for _ in range(size)]
        oracle.oracle_allreduce(0, size, n, slot, code, 0, ptrs(xs4), ptrs(outs))
        before = staged.value
        d, dp, read = put(xs4[rank])
        o, opp, oread4 = put(np.zeros_like(xs4[0]))
        torch.cuda.synchronize()
        assert L.mini_allreduce(comm, dp, opp, n, dt, op) == 0
        opdata.assert_same("LONG_DOUBLE", opname, oread4(), outs[rank], "engine x87 allreduce")
        assert staged.value == before
        L.mini_op_destroy(op)

    say("engine pairs done")
    # ---- 4. host buffers on every rank: the host module reduces them (coll/basic's linear order)
    op = m.select_op(pkg.OP["SUM"])
    fdt = m.dtype_for_slot(pkg.T["FLOAT"])
    xs5 = [opdata.make("FLOAT", 50_000, 90 + r) for r in range(size)]
    want = _linear(oracle, pkg.OP["SUM"], pkg.T["FLOAT"], xs5)
    h = xs5[rank].copy()
    out = np.zeros_like(h)
    assert L.mini_allreduce(comm, h.ctypes.data, out.ctypes.data, 50_000, fdt, op) == 0
    opdata.assert_same("FLOAT", "SUM", out, want, "host-buffer allreduce through the host module")
    L.mini_op_destroy(op)
    vote_windows(m, oracle, rank, size, torch, staged, put)
    assert L.mini_device_hits() == 0, "a device pointer reached the host module"
    L.mini_comm_destroy(comm)
    print(f"rank {rank} staging OK", flush=True)


def vote_windows(m, oracle, rank, size, torch, staged, put):
    """the buffer-kind vote's windows (mi355x_comm_vote, 32 calls each): after a window of host-only
    calls the device ranks wait and the host ranks only publish, so a mixed call runs in the host
    component with the device ranks staging their buffers (coll/cuda's way, coll_cuda_allreduce.c:
    43-75) -- allreduce, reduce, bcast, allgather, gather, alltoall -- while an all-device call still
    runs in the engine; after a window with device calls the host ranks wait again and a mixed call
    runs in the engine.  Every result exact; no device pointer reaches the host module."""
    L, pkg = m.lib, m.pkg
    comm = L.mini_comm_create(rank, size, 77)
    assert L.mini_comm_set_channel(comm, (sys.argv[3] + "_votes").encode()) == 0
    L.mini_comm_install(comm, L.mini_host_module())
    assert L.mini_coll_select(comm, m.component_ptr(m.coll, "mca_coll_mi355x_component")) == 90
    idt = m.dtype_for_slot(pkg.T["INT32"])
    op = m.select_op(pkg.OP["SUM"])
    calls = [0]
    n = 4099
    xs = [(np.arange(n, dtype=np.int32) * (r + 3) - 5 * r).astype(np.int32) for r in range(size)]
    total = sum(xs)

    def allreduce(host_rank0, all_host=False):
        on_host = all_host or (host_rank0 and rank == 0)
        x, px, _ = put(xs[rank], on_host)
        y, py, rd = put(np.zeros(n, np.int32), on_host)
        torch.cuda.synchronize()
        assert L.mini_allreduce(comm, px, py, n, idt, op) == 0
        calls[0] += 1
        assert np.array_equal(rd(), total), ("vote window allreduce", calls[0])

    def fill_to_checkpoint():
        while calls[0] % 32:
            allreduce(False, all_host=True)

    say = lambda what: print(f"rank {rank} vote windows: {what}", flush=True)
    # window 1: host calls only -> window 2: device ranks wait
    fill_to_checkpoint() if calls[0] else [allreduce(False, all_host=True) for _ in range(32)]
    say("host window done")
    dev_rank = rank != 0
    before = staged.value
    allreduce(True)                                           # mixed: on the host, device ranks staged
    assert staged.value - before == (1 if dev_rank else 0), ("mixed call not staged to the host", staged.value - before)
    mixed = lambda a: put(a, rank == 0)
    say("mixed allreduce staged")
    # reduce to a device root
    root = size - 1
    x, px, _ = mixed(xs[rank])
    r_, pr, rr = mixed(np.zeros(n, np.int32))
    torch.cuda.synchronize()
    assert L.mini_reduce(comm, px, pr if rank == root else None, n, idt, op, root) == 0
    calls[0] += 1
    if rank == root:
        assert np.array_equal(rr(), total), "vote window mixed reduce"
    # bcast from the host rank
    b, pb, rb = mixed(np.full(n, 11 if rank == 0 else -1, np.int32))
    torch.cuda.synchronize()
    assert L.mini_bcast(comm, pb, n, idt, 0) == 0
    calls[0] += 1
    assert (rb() == 11).all(), "vote window mixed bcast"
    # allgather, gather, alltoall
    g, pg, rg = mixed(np.full(n * size, -1, np.int32))
    torch.cuda.synchronize()
    assert L.mini_allgather(comm, px, n, idt, pg, n, idt) == 0
    calls[0] += 1
    assert np.array_equal(rg(), np.concatenate(xs)), "vote window mixed allgather"
    g2, pg2, rg2 = mixed(np.full(n * size, -1, np.int32))
    torch.cuda.synchronize()
    assert L.mini_gather(comm, px, n, idt, pg2 if rank == root else None, n, idt, root) == 0
    calls[0] += 1
    if rank == root:
        assert np.array_equal(rg2(), np.concatenate(xs)), "vote window mixed gather"
    k = 100
    piece = lambda r, q: np.arange(k, dtype=np.int32) + 1000 * q + 100000 * r
    sa, psa, _ = mixed(np.concatenate([piece(rank, q) for q in range(size)]))
    ra, pra, rra = mixed(np.full(k * size, -1, np.int32))
    torch.cuda.synchronize()
    assert L.mini_alltoall(comm, psa, k, idt, pra, k, idt) == 0
    calls[0] += 1
    assert np.array_equal(rra(), np.concatenate([piece(q, rank) for q in range(size)])), "vote window mixed alltoall"
    say("mixed movement on the host")
    staged_mid = staged.value
    allreduce(False)                                          # all device: still the engine
    assert staged.value == staged_mid, "an all-device call was staged"
    fill_to_checkpoint()                                      # window 2 had device calls ->
    before = staged.value                                     # window 3: host ranks wait
    allreduce(True)                                           # mixed: in the engine, nothing staged
    assert staged.value == before, "a mixed call after device use was staged to the host"
    L.mini_op_destroy(op)
    L.mini_comm_destroy(comm)


def mca_vars_main():
    """the engine's crossovers as coll_mi355x_* MCA variables (registered through the harness's
    variable system, which reads OMPI_MCA_<name> like libopen-pal's environment source): with
    pipe_min_ranks = 2 and the service limits svc_max / svc_pull_max / svc_copy_max = 0 a 2-rank communicator runs a large allreduce through the
    pipelined flow (PIPE_CALLS) and keeps small calls off the resident service; re-registered with
    the defaults, the next communicator does neither -- both exact vs the oracle"""
    import os
    rank, size = int(sys.argv[1]), int(sys.argv[2])
    import torch
    torch.cuda.set_device(rank % torch.cuda.device_count())
    m = mini()
    L, pkg = m.lib, m.pkg
    oracle = load_oracle()
    m.install_oracle_base(oracle)
    comp = m.component_ptr(m.coll, "mca_coll_mi355x_component")
    m.coll.mca_coll_mi355x_engine_of.restype = ctypes.c_void_p
    m.coll.mca_coll_mi355x_engine_of.argtypes = [ctypes.c_void_p]
    rt = pkg.rt()
    ptrs = lambda arrs: (ctypes.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])

    def knob(eng, name):
        v = ctypes.c_long(0)
        assert rt.mi355x_comm_get(ctypes.c_void_p(eng), pkg.KNOB[name], ctypes.byref(v)) == 0
        return v.value

    fdt = m.dtype_for_slot(pkg.T["FLOAT"])
    op = m.select_op(pkg.OP["SUM"])
    count = 1 << 20
    xs = [opdata.make("FLOAT", count, 300 + r) for r in range(size)]
    outs = [np.zeros_like(xs[0]) for _ in range(size)]
    oracle.oracle_allreduce(0, size, count, pkg.T["FLOAT"], pkg.OP["SUM"], 0, ptrs(xs), ptrs(outs))
    names = ("pipe_min_ranks", "svc_max", "svc_pull_max", "svc_copy_max")
    off = {"pipe_min_ranks": "2", "svc_max": "0", "svc_pull_max": "0", "svc_copy_max": "0"}
    # (a registration takes the storage's current value as its default, as mca_base_var does, so the
    # second step names the shipped defaults instead of relying on a re-registration to reset them)
    dflt = {"pipe_min_ranks": "4", "svc_max": str(32 << 10), "svc_pull_max": str(128 << 10), "svc_copy_max": str(1 << 20)}
    for step, (env, pipe, svc) in enumerate(((off, 1, 0), (dflt, 0, 32 << 10))):
        for k in names:
            os.environ.pop("OMPI_MCA_coll_mi355x_" + k, None)
        for k, v in env.items():
            os.environ["OMPI_MCA_coll_mi355x_" + k] = v
        assert L.mini_component_register(comp) == 0
        comm = L.mini_comm_create(rank, size, 50 + step)
        assert L.mini_comm_set_channel(comm, f"{sys.argv[3]}_{step}".encode()) == 0
        L.mini_comm_install(comm, L.mini_stub_module())
        assert L.mini_coll_select(comm, comp) == 90
        eng = m.coll.mca_coll_mi355x_engine_of(comm)
        assert eng
        assert knob(eng, "PIPE") == pipe, ("PIPE", knob(eng, "PIPE"))
        assert knob(eng, "DEV_SETUP") == 0
        dx = torch.from_numpy(xs[rank].view(np.uint8).copy()).cuda()
        dr = torch.zeros_like(dx)
        torch.cuda.synchronize()
        assert L.mini_allreduce(comm, dx.data_ptr(), dr.data_ptr(), count, fdt, op) == 0
        opdata.assert_same("FLOAT", "SUM", dr.cpu().numpy().view(np.float32), outs[rank], f"mca vars step {step}")
        assert knob(eng, "PIPE_CALLS") == pipe, ("PIPE_CALLS", knob(eng, "PIPE_CALLS"))
        if svc == 0:
            assert knob(eng, "SVC_MAX_BYTES") == 0
            calls0 = knob(eng, "SVC_CALLS")
            x = torch.ones(256, device="cuda")
            y = torch.empty_like(x)
            torch.cuda.synchronize()
            for _ in range(40):
                assert L.mini_allreduce(comm, x.data_ptr(), y.data_ptr(), 256, fdt, op) == 0
            assert bool(torch.all(y == size).item())
            assert knob(eng, "SVC_CALLS") == calls0, "svc_max = 0, yet the service served"
        L.mini_comm_destroy(comm)
    for k in names:
        os.environ.pop("OMPI_MCA_coll_mi355x_" + k, None)
    assert L.mini_component_register(comp) == 0
    L.mini_op_destroy(op)
    print(f"rank {rank} mca_vars OK", flush=True)


def host8_main():
    """(measurement, not a test) an 8-byte host-buffer MPI_Allreduce through the harness: the host
    module alone (what the reference runs: coll/tuned over ob1/sm, here coll/basic's order over the
    channel), with coll/mi355x selected on top (the call votes its buffer kind, then reaches the host
    module, whose ompi_op_reduce dispatches through op/hip's slot), and with coll_mi355x_mixed_buffers
    = 0 (no vote).  One JSON line per variant from rank 0: microseconds per call (median of 15
    interleaved batches of 1000, Python's ctypes call included in every variant alike)."""
    import json
    import os
    import time
    rank, size = int(sys.argv[1]), int(sys.argv[2])
    import torch
    torch.cuda.set_device(rank % torch.cuda.device_count())
    m = mini()
    L, pkg = m.lib, m.pkg
    oracle = load_oracle()
    m.install_oracle_base(oracle)
    L.mini_host_module.restype = ctypes.c_void_p
    comp = m.component_ptr(m.coll, "mca_coll_mi355x_component")
    fdt = m.dtype_for_slot(pkg.T["DOUBLE"])
    # the three set-ups side by side (one communicator each), their batches interleaved so that
    # drift over the run touches every variant alike: 15 rounds x 3 variants x 1000 calls
    variants = (("host_module", False, 1), ("host_module_op_hip", True, 1), ("coll_mi355x", True, 1),
                ("coll_mi355x_no_vote", True, 0))
    setups = []
    for step, (variant, with_hip, mixed) in enumerate(variants):
        os.environ["OMPI_MCA_coll_mi355x_mixed_buffers"] = str(mixed)
        assert L.mini_component_register(comp) == 0
        op = m.select_op(pkg.OP["SUM"], with_hip=with_hip)
        comm = L.mini_comm_create(rank, size, 60 + step)
        assert L.mini_comm_set_channel(comm, f"{sys.argv[3]}_{step}".encode()) == 0
        L.mini_comm_install(comm, L.mini_host_module())
        if variant.startswith("coll_mi355x"):
            assert L.mini_coll_select(comm, comp) == 90
        setups.append((variant, comm, op))
    x = np.full(1, float(rank + 1))
    y = np.zeros(1)
    px, py = x.ctypes.data, y.ctypes.data
    times = {v: [] for v, _, _ in setups}
    for variant, comm, op in setups:
        for _ in range(200):
            assert L.mini_allreduce(comm, px, py, 1, fdt, op) == 0
    for _ in range(15):
        for variant, comm, op in setups:
            t0 = time.perf_counter()
            for _ in range(1000):
                L.mini_allreduce(comm, px, py, 1, fdt, op)
            times[variant].append((time.perf_counter() - t0) / 1000 * 1e6)
            assert y[0] == size * (size + 1) / 2
    rows = [{"variant": v, "n": size, "bytes": 8, "us_per_call": round(sorted(t)[len(t) // 2], 3),
             "us_min_batch": round(min(t), 3)} for v, t in times.items()]
    for variant, comm, op in setups:
        L.mini_comm_destroy(comm)
        L.mini_op_destroy(op)
    os.environ.pop("OMPI_MCA_coll_mi355x_mixed_buffers", None)
    assert L.mini_component_register(comp) == 0
    if rank == 0:
        for r in rows:
            print(json.dumps(r), flush=True)
    print(f"rank {rank} host8 OK", flush=True)


def main():
    if len(sys.argv) > 4 and sys.argv[4] == "split":
        return split_main()
    if len(sys.argv) > 4 and sys.argv[4] == "pml":
        return pml_main()
    if len(sys.argv) > 4 and sys.argv[4] == "tuned_vars":
        return tuned_vars_main()
    if len(sys.argv) > 4 and sys.argv[4] == "staging":
        return staging_main()
    if len(sys.argv) > 4 and sys.argv[4] == "mca_vars":
        return mca_vars_main()
    if len(sys.argv) > 4 and sys.argv[4] == "host8":
        return host8_main()
    rank, size = int(sys.argv[1]), int(sys.argv[2])
    import torch
    ndev = torch.cuda.device_count()
    torch.cuda.set_device(rank % ndev)
    m = mini()
    oracle = load_oracle()
    m.install_oracle_base(oracle)
    comm = m.lib.mini_comm_create(rank, size, 42)
    m.lib.mini_comm_set_channel(comm, sys.argv[3].encode())
    m.lib.mini_comm_install(comm, m.lib.mini_stub_module())
    prio = m.lib.mini_coll_select(comm, m.component_ptr(m.coll, "mca_coll_mi355x_component"))
    assert prio == 90, prio
    ptrs = lambda arrs: (ctypes.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])
    pkg = m.pkg
    for opname, tname in [("SUM", "FLOAT"), ("MAXLOC", "DOUBLE_INT"), ("PROD", "C_DOUBLE_COMPLEX"), ("BXOR", "INT32")]:
        code, slot = pkg.OP[opname], pkg.T[tname]
        dt = m.dtype_for_slot(slot)
        op = m.select_op(code)
        for count in (3, 4001, 200_003):
            xs = [opdata.make(tname, count, 500 + r) for r in range(size)]
            outs = [np.zeros_like(xs[0]) for _ in range(size)]
            oracle.oracle_allreduce(0, size, count, slot, code, 0, ptrs(xs), ptrs(outs))
            dx = torch.from_numpy(xs[rank].view(np.uint8).copy()).cuda()
            dr = torch.zeros_like(dx)
            torch.cuda.synchronize()
            assert m.lib.mini_allreduce(comm, dx.data_ptr(), dr.data_ptr(), count, dt, op) == 0
            opdata.assert_same(tname, opname, dr.cpu().numpy().view(xs[0].dtype), outs[rank], "component allreduce")
        # reduce to the last rank
        count, root = 3001, size - 1
        xs = [opdata.make(tname, count, 650 + r) for r in range(size)]
        want = np.zeros_like(xs[0])
        oracle.oracle_reduce.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_size_t, ctypes.c_int,
                                         ctypes.c_int, ctypes.c_uint32, ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p]
        oracle.oracle_reduce(0, size, root, count, slot, code, 0, ptrs(xs), want.ctypes.data)
        dx = torch.from_numpy(xs[rank].view(np.uint8).copy()).cuda()
        dr = torch.zeros_like(dx)
        torch.cuda.synchronize()
        assert m.lib.mini_reduce(comm, dx.data_ptr(), dr.data_ptr() if rank == root else None, count, dt, op, root) == 0
        if rank == root:
            opdata.assert_same(tname, opname, dr.cpu().numpy().view(xs[0].dtype), want, "component reduce")
        # reduce_scatter_block
        rcount = 1001
        xs = [opdata.make(tname, rcount * size, 600 + r) for r in range(size)]
        outs = [np.zeros(rcount, dtype=xs[0].dtype) for _ in range(size)]
        oracle.oracle_reduce_scatter_block(size, rcount, slot, code, ptrs(xs), ptrs(outs))
        dx = torch.from_numpy(xs[rank].view(np.uint8).copy()).cuda()
        dr = torch.zeros(rcount * xs[0].dtype.itemsize, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        assert m.lib.mini_reduce_scatter_block(comm, dx.data_ptr(), dr.data_ptr(), rcount, dt, op) == 0
        opdata.assert_same(tname, opname, dr.cpu().numpy().view(xs[0].dtype), outs[rank], "component rsb")
        m.lib.mini_op_destroy(op)
    # allgather + bcast (MPI_FLOAT)
    fdt = m.dtype_for_slot(pkg.T["FLOAT"])
    n = 12345
    src = torch.full((n,), float(rank + 1), device="cuda")
    dst = torch.zeros(n * size, device="cuda")
    torch.cuda.synchronize()
    assert m.lib.mini_allgather(comm, src.data_ptr(), n, fdt, dst.data_ptr(), n, fdt) == 0
    for r in range(size):
        assert bool((dst[r * n:(r + 1) * n] == r + 1).all())
    buf = torch.full((n,), float(rank), device="cuda")
    torch.cuda.synchronize()
    assert m.lib.mini_bcast(comm, buf.data_ptr(), n, fdt, size - 1) == 0
    assert bool((buf == size - 1).all())
    # nonblocking slots: MPI_Iallreduce / Ireduce / Ireduce_scatter_block / Iallgather / Ibcast posted
    # together, then MPI_Wait on each (requests progressed by the component's opal_progress callback)
    nonblocking(m, comm, oracle, rank, size, torch, ptrs)
    nonblocking_mixed_layouts(m, comm, oracle, rank, size, torch)
    mixed_buffers(m, comm, oracle, rank, size, torch)
    mixed_more(m, comm, oracle, rank, size, torch, ptrs)
    # derived datatypes through the GPU convertor: bcast of a vector type ...
    derived_bcast(m, comm, oracle, rank, size, torch)
    derived_allgather(m, comm, oracle, rank, size, torch)
    movement(m, comm, oracle, rank, size, torch, ptrs)
    # host buffers -> the lower-priority (stub) module
    h = np.zeros(16, dtype=np.float32)
    op = m.select_op(pkg.OP["SUM"])
    assert m.lib.mini_allreduce(comm, h.ctypes.data, h.ctypes.data, 16, fdt, op) == m.lib.mini_stub_marker()
    assert m.lib.mini_stub_calls(0) == 1
    m.lib.mini_comm_destroy(comm)
    print(f"rank {rank} OK", flush=True)


if __name__ == "__main__":
    main()
