"""Point-to-point (mi355x_isend / irecv / send / recv / sendrecv / iprobe / improbe / imrecv) on a loopback
communicator (one process, one rank per comm object).  The semantics checked are ob1's
(ompi/mca/pml/ob1/pml_ob1_recvfrag.c matching, pml_ob1_recvreq.h:172-180 truncation): messages
from one source are received in send order, posted receives are matched in posting order,
MPI_ANY_SOURCE / MPI_ANY_TAG wildcards, MPI_PROC_NULL, zero-byte messages, truncation keeps the
first bytes and reports the message size; host and device buffers share the queue.  Bytes moved through derived datatypes must equal the
oracle's unpack(pack(...)) (the convertor restatement under oracle/)."""
from __future__ import annotations

import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture()
def comms(gpu, pkg):
    cs = pkg.Comm.loopback(4, 0)
    yield cs
    for c in cs:
        c.destroy()


def _bytes(torch, n, seed):
    g = np.random.default_rng(seed)
    return torch.from_numpy(g.integers(0, 256, n, dtype=np.uint8)).cuda()


def _wait_all(reqs):
    return [r.wait() for r in reqs]


@pytest.mark.parametrize("nbytes", [1, 4096, 1 << 20, 3 * (1 << 20) + 7])
def test_ring_exchange(gpu, pkg, comms, nbytes):
    torch = gpu
    n = len(comms)
    src = [_bytes(torch, nbytes, r) for r in range(n)]
    dst = [torch.zeros(nbytes, dtype=torch.uint8, device="cuda") for _ in range(n)]
    reqs = []
    for r, c in enumerate(comms):
        reqs.append(c.irecv(dst[r].data_ptr(), nbytes, (r - 1) % n, 11))
    sends = [c.isend(src[r].data_ptr(), nbytes, (r + 1) % n, 11) for r, c in enumerate(comms)]
    st = _wait_all(reqs)
    _wait_all(sends)
    for r in range(n):
        assert torch.equal(dst[r], src[(r - 1) % n])
        assert st[r] == ((r - 1) % n, 11, 0, nbytes)


def test_order_and_tags(gpu, pkg, comms):
    """non-overtaking per source; a tag-specific receive skips earlier messages of other tags"""
    torch = gpu
    a, b = comms[0], comms[1]
    msgs = [(5, 100), (7, 200), (5, 300), (9, 0)]
    bufs = [_bytes(torch, ln, i) if ln else torch.zeros(1, dtype=torch.uint8, device="cuda")
            for i, (_, ln) in enumerate(msgs)]
    sends = [a.isend(bufs[i].data_ptr(), ln, 1, tag) for i, (tag, ln) in enumerate(msgs)]
    out = [torch.zeros(512, dtype=torch.uint8, device="cuda") for _ in range(4)]
    r7 = b.irecv(out[0].data_ptr(), 512, 0, 7)
    r_any1 = b.irecv(out[1].data_ptr(), 512, pkg.ANY_SOURCE, pkg.ANY_TAG)
    r_any2 = b.irecv(out[2].data_ptr(), 512, 0, pkg.ANY_TAG)
    r9 = b.irecv(out[3].data_ptr(), 512, 0, 9)
    assert r7.wait() == (0, 7, 0, 200)
    assert r_any1.wait() == (0, 5, 0, 100)
    assert r_any2.wait() == (0, 5, 0, 300)
    assert r9.wait() == (0, 9, 0, 0)
    _wait_all(sends)
    assert torch.equal(out[0][:200], bufs[1])
    assert torch.equal(out[1][:100], bufs[0])
    assert torch.equal(out[2][:300], bufs[2])


def test_any_source(gpu, pkg, comms):
    torch = gpu
    n = len(comms)
    src = [_bytes(torch, 64 + r, 40 + r) for r in range(n)]
    sends = [comms[r].isend(src[r].data_ptr(), 64 + r, 0, 3) for r in range(1, n)]
    out = [torch.zeros(128, dtype=torch.uint8, device="cuda") for _ in range(n - 1)]
    sts = _wait_all([comms[0].irecv(o.data_ptr(), 128, pkg.ANY_SOURCE, 3) for o in out])
    _wait_all(sends)
    assert sorted(s[0] for s in sts) == list(range(1, n))
    for s, o in zip(sts, out):
        assert s[1] == 3 and s[3] == 64 + s[0]
        assert torch.equal(o[:s[3]], src[s[0]])


def test_truncate(gpu, pkg, comms):
    torch = gpu
    src = _bytes(torch, 100, 1)
    dst = torch.zeros(64, dtype=torch.uint8, device="cuda")
    s = comms[2].isend(src.data_ptr(), 100, 3, 1)
    r = comms[3].irecv(dst.data_ptr(), 64, 2, 1)
    with pytest.raises(pkg.TruncateError) as ei:
        r.wait()
    assert ei.value.status == (2, 1, pkg.ERR_TRUNCATE, 100)
    s.wait()
    assert torch.equal(dst, src[:64])


def test_proc_null_and_self(gpu, pkg, comms):
    torch = gpu
    c = comms[1]
    c.send(None, 0, pkg.PROC_NULL, 4)
    assert c.recv(None, 10, pkg.PROC_NULL, 4) == (pkg.PROC_NULL, pkg.ANY_TAG, 0, 0)
    src = _bytes(torch, 777, 2)
    dst = torch.zeros(777, dtype=torch.uint8, device="cuda")
    s = c.isend(src.data_ptr(), 777, 1, 8)       # to itself
    assert c.recv(dst.data_ptr(), 777, 1, 8) == (1, 8, 0, 777)
    s.wait()
    assert torch.equal(dst, src)


@pytest.mark.parametrize("mode", ["STANDARD", "SYNCHRONOUS"])
def test_ring_wraps(gpu, pkg, comms, mode):
    """more messages in flight than envelopes per pair (32): later sends queue, order is kept.  Small
    standard sends complete for the caller at once (eager: the engine keeps the queued envelope);
    synchronous ones only once received"""
    torch = gpu
    k = 100
    src = _bytes(torch, k * 16, 5)
    sends = [comms[0].isend(src[i * 16:(i + 1) * 16].data_ptr(), 16, 1, i % 3, mode=mode) for i in range(k)]
    assert sends[-1].test() == (mode == "STANDARD")
    dst = torch.zeros(k * 16, dtype=torch.uint8, device="cuda")
    for i in range(k):
        r = comms[1].irecv(dst[i * 16:(i + 1) * 16].data_ptr(), 16, 0, pkg.ANY_TAG)
        while not r.test():
            comms[0].progress()   # the sender announces its queued messages as envelopes free up
        assert r.wait() == (0, i % 3, 0, 16)
    _wait_all(sends)
    assert torch.equal(dst, src)


def test_iprobe(gpu, pkg, comms):
    torch = gpu
    assert comms[0].iprobe(pkg.ANY_SOURCE, pkg.ANY_TAG) is None
    src = _bytes(torch, 50, 3)
    s = comms[2].isend(src.data_ptr(), 50, 0, 21)
    assert comms[0].iprobe(pkg.ANY_SOURCE, 22) is None
    assert comms[0].iprobe(2, 21) == (2, 21, 0, 50)
    dst = torch.zeros(50, dtype=torch.uint8, device="cuda")
    comms[0].recv(dst.data_ptr(), 50, 2, 21)
    s.wait()
    assert comms[0].iprobe(pkg.ANY_SOURCE, pkg.ANY_TAG) is None


def test_sendrecv_threads(gpu, pkg, comms):
    """blocking sendrecv ring, one thread per rank (as MPI ranks would be)"""
    torch = gpu
    n = len(comms)
    nbytes = 1 << 16
    src = [_bytes(torch, nbytes, 60 + r) for r in range(n)]
    dst = [torch.zeros(nbytes, dtype=torch.uint8, device="cuda") for _ in range(n)]
    sts, errs = [None] * n, []

    def run(r):
        try:
            torch.cuda.set_device(0)
            sts[r] = comms[r].sendrecv(src[r].data_ptr(), nbytes, (r + 1) % n, 2,
                                       dst[r].data_ptr(), nbytes, (r - 1) % n, 2)
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    ts = [threading.Thread(target=run, args=(r,)) for r in range(n)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(60)
    assert not errs, errs
    for r in range(n):
        assert sts[r] == ((r - 1) % n, 2, 0, nbytes)
        assert torch.equal(dst[r], src[(r - 1) % n])


def _oracle_move(oracle, sd, scount, src, rd, rcount, init):
    """expected receive buffer: oracle unpack(rd) of oracle pack(sd)"""
    total = scount * oracle.oracle_ddt_size(sd)
    packed = np.zeros(max(total, 1), dtype=np.uint8)
    oracle.oracle_ddt_pack(sd, scount, src.ctypes.data, 0, packed.ctypes.data, total)
    out = init.copy()
    oracle.oracle_ddt_unpack(rd, rcount, out.ctypes.data, 0, packed.ctypes.data, total)
    return out


@pytest.mark.parametrize("case", ["vec_to_contig", "contig_to_vec", "vec_to_indexed", "vec_to_vec"])
def test_datatypes(gpu, pkg, oracle, comms, case):
    """MPI_Type_vector(stride 2, block 64) from BASELINE config 5 and an indexed type, sent and
    received through the GPU convertor; bytes equal the oracle convertor's"""
    torch = gpu
    nvec, blk, stride = 96, 64, 128          # 96 blocks of 64 floats, every other block
    vec_elems = nvec * stride
    blocklens = [3, 64, 1, 200, 5000, 900]
    disps = [0, 10, 80, 100, 400, 5500]
    idx_bytes = sum(blocklens) * 4           # 6168 floats: larger than the vector's 6144
    ov = oracle.oracle_ddt_vector(nvec, blk, stride, 4)
    dv = pkg.Ddt.vector(nvec, blk, stride, 4)
    msg = nvec * blk * 4
    import ctypes
    oc = oracle.oracle_ddt_contiguous(msg, 1)
    bl = (ctypes.c_int * len(blocklens))(*blocklens)
    ds = (ctypes.c_int * len(disps))(*disps)
    oi = oracle.oracle_ddt_indexed(len(blocklens), bl, ds, 4)
    di = pkg.Ddt.indexed(blocklens, disps, 4)
    g = np.random.default_rng(7)
    if case == "vec_to_contig":
        sd, od_s, scount, sbytes = dv, ov, 1, vec_elems * 4
        rd, od_r, rcount, rbytes = None, oc, 1, msg
    elif case == "contig_to_vec":
        sd, od_s, scount, sbytes = None, oc, 1, msg
        rd, od_r, rcount, rbytes = dv, ov, 1, vec_elems * 4
    elif case == "vec_to_indexed":
        sd, od_s, scount, sbytes = dv, ov, 1, vec_elems * 4
        rd, od_r, rcount, rbytes = di, oi, 1, (disps[-1] + blocklens[-1]) * 4
    else:
        sd, od_s, scount, sbytes = dv, ov, 2, 2 * vec_elems * 4
        rd, od_r, rcount, rbytes = dv, ov, 2, 2 * vec_elems * 4
        msg = 2 * msg
    src = g.integers(0, 256, sbytes, dtype=np.uint8)
    init = np.full(rbytes, 0xA5, dtype=np.uint8)
    dsrc = torch.from_numpy(src).cuda()
    ddst = torch.from_numpy(init).cuda()
    s = comms[0].isend(dsrc.data_ptr(), scount if sd else msg, 1, 0, ddt=sd)
    st = None
    try:
        st = comms[1].irecv(ddst.data_ptr(), rcount if rd else msg, 0, 0, ddt=rd).wait()
    except pkg.TruncateError as e:   # the indexed type is larger than the vector: not truncated
        raise AssertionError(e)
    s.wait()
    assert st == (0, 0, 0, msg)
    want = _oracle_move(oracle, od_s, scount, src, od_r, rcount, init)
    assert np.array_equal(ddst.cpu().numpy(), want)
    for o in {id(x): x for x in (ov, oc, oi)}.values():
        oracle.oracle_ddt_free(o)
    dv.destroy()
    di.destroy()


def test_errors(gpu, pkg, comms):
    torch = gpu
    buf = torch.zeros(16, dtype=torch.uint8, device="cuda")
    with pytest.raises(pkg.MI355XError, match="bad destination"):
        comms[0].isend(buf.data_ptr(), 16, 9, 0)
    with pytest.raises(pkg.MI355XError, match="MPI_ANY_TAG"):
        comms[0].isend(buf.data_ptr(), 16, 1, pkg.ANY_TAG)
    with pytest.raises(pkg.MI355XError, match="bad send mode"):
        rt = pkg.rt()
        import ctypes
        h = ctypes.c_void_p()
        pkg.check(rt.mi355x_isend_mode(comms[0].h, buf.data_ptr(), 16, None, 1, 0, 9, None, ctypes.byref(h)), "isend_mode")


# ---- one matching queue for host and device buffers (ob1: pml_ob1_cuda.c:52-100 decides the
#      convertor per request on the send side, pml_ob1_recvreq.c:647-663 on the receive side; the
#      match itself never looks at the buffer kind)
def _buf(torch, kind, data: np.ndarray):
    """a host (numpy) or device (torch) buffer holding `data` (uint8); returns (ptr, reader, keep)"""
    if kind == "host":
        h = np.ascontiguousarray(data).copy()
        return h.ctypes.data, (lambda: h.copy()), h
    d = torch.from_numpy(np.ascontiguousarray(data).copy()).cuda()
    torch.cuda.synchronize()
    return d.data_ptr(), (lambda: d.cpu().numpy()), d


KINDS = [("dev", "dev"), ("dev", "host"), ("host", "dev"), ("host", "host")]


@pytest.mark.parametrize("skind,rkind", KINDS)
@pytest.mark.parametrize("nbytes", [0, 17, 4096, 4097, (1 << 20) + 3])
def test_host_device_pairs(gpu, pkg, comms, skind, rkind, nbytes):
    """every pairing of buffer kinds meets in one queue, sizes either side of the 4 KiB eager limit"""
    torch = gpu
    data = np.random.default_rng(nbytes + 7).integers(0, 256, max(nbytes, 1), dtype=np.uint8)
    sp, _, keep_s = _buf(torch, skind, data)
    rp, read, keep_r = _buf(torch, rkind, np.zeros(max(nbytes, 1) + 5, dtype=np.uint8))
    rq = comms[1].irecv(rp, nbytes + 5, 0, 4)
    sq = comms[0].isend(sp, nbytes, 1, 4)
    assert rq.wait() == (0, 4, 0, nbytes)
    sq.wait()
    got = read()
    assert np.array_equal(got[:nbytes], data[:nbytes]) and not got[nbytes:].any()


def test_any_source_and_order_across_kinds(gpu, pkg, comms):
    """MPI_ANY_SOURCE sees senders of both kinds; between one pair, same-tag messages of alternating
    kinds and sizes (eager and rendezvous) match in send order into alternating receive kinds"""
    torch = gpu
    n = len(comms)
    g = np.random.default_rng(11)
    # non-overtaking across kinds: 12 messages 0 -> 1 on one tag
    sizes = [3, 5000, 64, 1 << 20, 4096, 9000, 1, 70000, 4097, 12, 2 << 20, 100]
    payload = [g.integers(0, 256, ln, dtype=np.uint8) for ln in sizes]
    sends = [_buf(torch, "dev" if i % 2 else "host", payload[i]) for i in range(len(sizes))]
    sq = [comms[0].isend(sends[i][0], sizes[i], 1, 21) for i in range(len(sizes))]
    recvs = [_buf(torch, "host" if i % 3 else "dev", np.zeros(2 << 20, dtype=np.uint8)) for i in range(len(sizes))]
    rq = [comms[1].irecv(recvs[i][0], 2 << 20, 0, 21) for i in range(len(sizes))]
    for i, q in enumerate(rq):
        assert q.wait() == (0, 21, 0, sizes[i]), i
        assert np.array_equal(recvs[i][1]()[:sizes[i]], payload[i]), ("order", i)
    for q in sq:
        q.wait()
    # ANY_SOURCE: ranks 1..n-1 send (odd ranks from host memory), rank 0 receives into host and device
    src = {r: _buf(torch, "host" if r % 2 else "dev", np.full(40 + r, r, dtype=np.uint8)) for r in range(1, n)}
    sq = [comms[r].isend(src[r][0], 40 + r, 0, 5) for r in range(1, n)]
    seen = set()
    for i in range(1, n):
        rb = _buf(torch, "dev" if i % 2 else "host", np.zeros(64, dtype=np.uint8))
        st = comms[0].recv(rb[0], 64, pkg.ANY_SOURCE, 5)
        r = st[0]
        assert st == (r, 5, 0, 40 + r) and r not in seen
        assert np.array_equal(rb[1]()[:40 + r], np.full(40 + r, r, dtype=np.uint8))
        seen.add(r)
    assert seen == set(range(1, n))
    for q in sq:
        q.wait()


def test_send_completion_modes(gpu, pkg, comms):
    """ob1's completion rules: a standard send of <= 4 KiB completes before any receive is posted
    (eager), a synchronous one does not; a buffered send of any size completes at once and the
    receiver gets the bytes as they were at the send"""
    torch = gpu
    a, b = comms[0], comms[1]
    small = _buf(torch, "dev", np.full(4096, 7, dtype=np.uint8))
    q_std = a.isend(small[0], 4096, 1, 1)
    assert q_std.test(), "standard 4 KiB send is eager"
    q_sync = a.isend(small[0], 4096, 1, 2, mode="SYNCHRONOUS")
    for _ in range(50):
        assert not q_sync.test(), "a synchronous send completed before its receive was posted"
    big = torch.full((3 << 20,), 9, dtype=torch.uint8, device="cuda")
    hbig = np.full(3 << 20, 5, dtype=np.uint8)
    torch.cuda.synchronize()
    q_buf = a.isend(big.data_ptr(), 3 << 20, 1, 3, mode="BUFFERED")
    q_hbuf = a.isend(hbig.ctypes.data, 3 << 20, 1, 4, mode="BUFFERED")
    assert q_buf.test() and q_hbuf.test(), "buffered sends complete at once"
    big.fill_(0)
    hbig[:] = 0
    torch.cuda.synchronize()
    q_big = a.isend(big.data_ptr(), 3 << 20, 1, 5)
    assert not q_big.test(), "a 3 MiB standard send is rendezvous"
    out = [np.zeros(3 << 20, dtype=np.uint8) for _ in range(5)]
    for tag, o in zip((1, 2, 3, 4, 5), out):
        b.recv(o.ctypes.data, 3 << 20, 0, tag)
    for q in (q_std, q_sync, q_buf, q_hbuf, q_big):
        q.wait()
    assert (out[0][:4096] == 7).all() and (out[1][:4096] == 7).all()
    assert (out[2] == 9).all() and (out[3] == 5).all(), "buffered payload changed after completion"
    assert not out[4].any()


def test_unsafe_exchange_small(gpu, pkg, comms):
    """both ranks MPI_Send before MPI_Recv: legal to deadlock in MPI, but ob1's eager protocol lets
    it through for small messages -- and so must this engine (threads, blocking calls)"""
    torch = gpu
    bufs = {r: (_buf(torch, "dev", np.full(1000, r + 1, dtype=np.uint8)), np.zeros(1000, dtype=np.uint8))
            for r in (0, 1)}
    errs = []

    def run(r):
        try:
            torch.cuda.set_device(0)
            comms[r].send(bufs[r][0][0], 1000, 1 - r, 8)
            comms[r].recv(bufs[r][1].ctypes.data, 1000, 1 - r, 8)
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    ts = [threading.Thread(target=run, args=(r,)) for r in (0, 1)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(60)
    assert not errs, errs
    assert (bufs[0][1] == 2).all() and (bufs[1][1] == 1).all()


def test_matched_probe_and_cancel(gpu, pkg, comms):
    """MPI_Improbe takes the message out of the queue (a later wildcard receive gets the NEXT one),
    MPI_Imrecv receives exactly it, into host memory; MPI_Cancel of an unmatched receive; negative
    (system) tags travel but MPI_ANY_TAG never matches them (pml_ob1_recvfrag.c:487)"""
    torch = gpu
    a, b = comms[2], comms[3]
    m1 = _buf(torch, "dev", np.arange(100, dtype=np.uint8))
    m2 = _buf(torch, "host", np.arange(100, 200, dtype=np.uint8))
    s1 = a.isend(m1[0], 100, 3, 6)
    s2 = a.isend(m2[0], 100, 3, 6)
    hit = None
    while hit is None:
        hit = b.improbe(2, 6)
    msg, st = hit
    assert st == (2, 6, 0, 100)
    other = np.zeros(100, dtype=np.uint8)
    assert b.recv(other.ctypes.data, 100, pkg.ANY_SOURCE, pkg.ANY_TAG) == (2, 6, 0, 100)
    assert np.array_equal(other, np.arange(100, 200, dtype=np.uint8)), "the probed message was stolen"
    mine = np.zeros(100, dtype=np.uint8)
    assert b.imrecv(mine.ctypes.data, 100, msg).wait() == (2, 6, 0, 100)
    assert np.array_equal(mine, np.arange(100, dtype=np.uint8))
    s1.wait()
    s2.wait()
    # cancel
    dummy = np.zeros(8, dtype=np.uint8)
    q = b.irecv(dummy.ctypes.data, 8, 2, 77)
    q.cancel()
    assert q.test() and q.cancelled()
    q.wait()
    # system tags
    neg = _buf(torch, "host", np.full(8, 3, dtype=np.uint8))
    sq = a.isend(neg[0], 8, 3, -17)
    anyq = b.irecv(dummy.ctypes.data, 8, 2, pkg.ANY_TAG)
    for _ in range(20):
        assert not anyq.test(), "MPI_ANY_TAG matched a system tag"
    got = np.zeros(8, dtype=np.uint8)
    assert b.recv(got.ctypes.data, 8, 2, -17) == (2, -17, 0, 8) and (got == 3).all()
    sq.wait()
    anyq.cancel()
    anyq.wait()


@pytest.mark.parametrize("skind,rkind", KINDS)
def test_host_device_datatypes(gpu, pkg, oracle, comms, skind, rkind):
    """derived layouts on either side, either kind: host layouts go through the host convertor
    (mi355x_pack_host / unpack_host), device layouts through the GPU convertor; vector -> indexed"""
    torch = gpu
    nblk = 3000
    dv = pkg.Ddt.vector(nblk, 3, 5, 4)              # 3 floats every 5: 12-B runs, 36000 B packed
    di = pkg.Ddt.indexed([5, 2, 8, 9], [0, 7, 11, 30], 4)  # 24 floats = 96 B per instance
    assert dv.size == 36000 and di.size == 96
    g = np.random.default_rng(3)
    src = g.integers(0, 256, dv.extent, dtype=np.uint8)
    inst = 36000 // 96
    dst0 = np.full(di.extent * inst + 64, 0xAB, dtype=np.uint8)
    sp, _, ks = _buf(torch, skind, src)
    rp, read, kr = _buf(torch, rkind, dst0)
    rq = comms[1].irecv(rp, inst, 0, 2, ddt=di)
    sq = comms[0].isend(sp, 1, 1, 2, ddt=dv)
    assert rq.wait() == (0, 2, 0, 36000)
    sq.wait()
    packed = np.zeros(36000, dtype=np.uint8)
    dv.pack_host(1, src.ctypes.data, 0, packed.ctypes.data, 36000)
    want = dst0.copy()
    di.unpack_host(inst, want.ctypes.data, 0, packed.ctypes.data, 36000)
    assert np.array_equal(read(), want)
    dv.destroy()
    di.destroy()


@pytest.mark.parametrize("rkind", ["host", "dev"])
@pytest.mark.parametrize("layout", ["contig", "vector_send", "vector_recv"])
def test_streamed_host_payloads(gpu, pkg, comms, rkind, layout):
    """host payloads of >= 1 MiB are announced first and copied into the sender's arena in 256-KiB
    fragments the receiver copies out as they land (the sm BTL's fragment pipeline): contiguous,
    a packed host layout, a host / device receive layout, and a truncating receive"""
    torch = gpu
    g = np.random.default_rng(41)
    nblk = 70000                                     # 64 floats every 128: 17.9 MB packed
    dv = pkg.Ddt.vector(nblk, 64, 128, 4)
    packed_bytes = dv.size
    if layout == "vector_send":
        src = g.integers(0, 256, dv.extent, dtype=np.uint8)
        sq_args = (1, dv)
    else:
        src = g.integers(0, 256, packed_bytes, dtype=np.uint8)
        sq_args = (packed_bytes, None)
    want_packed = np.zeros(packed_bytes, dtype=np.uint8)
    if layout == "vector_send":
        dv.pack_host(1, src.ctypes.data, 0, want_packed.ctypes.data, packed_bytes)
    else:
        want_packed[:] = src
    if layout == "vector_recv":
        dst0 = np.full(dv.extent, 0xAB, dtype=np.uint8)
        want = dst0.copy()
        dv.unpack_host(1, want.ctypes.data, 0, want_packed.ctypes.data, packed_bytes)
        rcount, rddt = 1, dv
    else:
        dst0 = np.zeros(packed_bytes + 64, dtype=np.uint8)
        want = dst0.copy()
        want[:packed_bytes] = want_packed
        rcount, rddt = packed_bytes + 64, None
    rp, read, kr = _buf(torch, rkind, dst0)
    rq = comms[1].irecv(rp, rcount, 0, 12, ddt=rddt)
    sq = comms[0].isend(src.ctypes.data, sq_args[0], 1, 12, ddt=sq_args[1])
    assert rq.wait() == (0, 12, 0, packed_bytes)
    sq.wait()
    assert np.array_equal(read(), want)
    # truncation: the receive takes what its buffer holds, the status the whole size
    small = np.zeros((3 << 20) + 1, dtype=np.uint8)
    sq = comms[0].isend(src.ctypes.data, sq_args[0], 1, 13, ddt=sq_args[1])
    with pytest.raises(pkg.MI355XError, match="truncated"):
        comms[1].recv(small.ctypes.data, small.size, 0, 13)
    sq.wait()
    assert np.array_equal(small, want_packed[:small.size])
    dv.destroy()


def test_streamed_host_payload_overlap(gpu, pkg, comms):
    """a receiver already waiting (its own thread) copies a 48 MiB host message out while the sender
    still copies it in; both directions at once"""
    torch = gpu
    n = (48 << 20) + 5
    data = {r: np.random.default_rng(60 + r).integers(0, 256, n, dtype=np.uint8) for r in (0, 1)}
    out = {r: np.zeros(n, dtype=np.uint8) for r in (0, 1)}
    errs = []

    def run(r):
        try:
            torch.cuda.set_device(0)
            rq = comms[r].irecv(out[r].ctypes.data, n, 1 - r, 14)
            comms[r].send(data[r].ctypes.data, n, 1 - r, 14)
            assert rq.wait() == (1 - r, 14, 0, n)
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    ts = [threading.Thread(target=run, args=(r,)) for r in (0, 1)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(120)
    assert not errs, errs
    assert np.array_equal(out[0], data[1]) and np.array_equal(out[1], data[0])


def _ob1_match_model(arrived, recvs):
    """ob1's matching restated (pml_ob1_recvfrag.c: posted receives in posting order, each takes the
    first message in arrival order whose source and tag match; wildcards -1).  `arrived` is the
    arrival order; for messages already queued this engine drains sources in rank order (MPI
    leaves the interleaving of sources unspecified, per-source order is what it guarantees)."""
    pending = list(arrived)
    out = []
    for src, tag in recvs:
        for i, (s, t, ident) in enumerate(pending):
            if (src == -1 or src == s) and (tag == -1 or tag == t):
                out.append(pending.pop(i))
                break
        else:
            out.append(None)
    return out


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_matching_random(gpu, pkg, comms, seed):
    """random tags / sources / wildcards vs the ob1 matching model, payload ids checked"""
    torch = gpu
    g = np.random.default_rng(seed)
    n = len(comms)
    msgs = {s: [] for s in range(1, n)}
    ident = 0
    for _ in range(80):
        s = int(g.integers(1, n))
        if len(msgs[s]) >= 30:          # stay inside one envelope ring per pair
            continue
        msgs[s].append((s, int(g.integers(0, 4)), ident))
        ident += 1
    payload = {m[2]: torch.full((2,), m[2], dtype=torch.int32, device="cuda") for s in msgs for m in msgs[s]}
    sends = [comms[s].isend(payload[m[2]].data_ptr(), 8, 0, m[1]) for s in msgs for m in msgs[s]]
    comms[0].progress()                 # every envelope drained: arrival order is source-major
    arrived = [m for s in range(1, n) for m in msgs[s]]
    model_pending = list(arrived)
    recvs = []
    for _ in range(len(arrived)):
        src = -1 if g.random() < 0.4 else int(g.integers(1, n))
        tag = -1 if g.random() < 0.4 else int(g.integers(0, 4))
        if _ob1_match_model(model_pending, [(src, tag)])[0] is None:
            src, tag = -1, -1
        hit = _ob1_match_model(model_pending, [(src, tag)])[0]
        model_pending.remove(hit)
        recvs.append((src, tag))
    want = _ob1_match_model(arrived, recvs)
    bufs = [torch.zeros(2, dtype=torch.int32, device="cuda") for _ in recvs]
    reqs = [comms[0].irecv(b.data_ptr(), 8, s, t) for b, (s, t) in zip(bufs, recvs)]
    sts = [r.wait() for r in reqs]
    for r in sends:
        r.wait()
    for st, b, w in zip(sts, bufs, want):
        assert st[:2] == (w[0], w[1]), (st, w)
        assert int(b[0]) == w[2], (int(b[0]), w)


def test_p2p_beside_nonblocking_collective(gpu, pkg, comms):
    """point-to-point on the caller's thread while a posted iallreduce runs on the progress thread
    (both use the communicator's registration cache)"""
    torch = gpu
    n = len(comms)
    count = 1 << 20
    xs = [torch.full((count,), float(r + 1), device="cuda") for r in range(n)]
    ys = [torch.empty_like(x) for x in xs]
    src = [_bytes(torch, 1 << 20, 80 + r) for r in range(n)]
    dst = [torch.zeros(1 << 20, dtype=torch.uint8, device="cuda") for _ in range(n)]
    torch.cuda.synchronize()
    errs = []

    def run(r):
        try:
            torch.cuda.set_device(0)
            q = comms[r].iallreduce(xs[r].data_ptr(), ys[r].data_ptr(), count, pkg.T["FLOAT"], pkg.OP["SUM"])
            for _ in range(3):
                comms[r].sendrecv(src[r].data_ptr(), 1 << 20, (r + 1) % n, 9, dst[r].data_ptr(), 1 << 20,
                                  (r - 1) % n, 9)
            q.wait()
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    ts = [threading.Thread(target=run, args=(r,)) for r in range(n)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(120)
    assert not errs, errs
    want = float(n * (n + 1) // 2)
    for r in range(n):
        assert bool(torch.all(ys[r] == want))
        assert torch.equal(dst[r], src[(r - 1) % n])
