"""GPU convertor (mi355x_pack / mi355x_unpack) vs the oracle, with the reference's datatype
known-answer tests restated on device buffers (test/datatype/position_noncontig.c,
position.c, checksum.c), random windows over vector / indexed / struct layouts, and the
BASELINE config-5 shape (MPI_Type_vector(2^22, 64, 128, MPI_FLOAT): 1 GiB packed) checked against
torch's strided view."""
from __future__ import annotations

import ctypes

import numpy as np
import pytest

from ddtcases import LDI, ldi_struct, segments, shuffle

pytestmark = pytest.mark.gpu


def _dev(torch, a):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1).copy()).cuda()


def test_position_noncontig_gpu(gpu, pkg, oracle):
    torch = gpu
    nelt = 300
    od = oracle.oracle_ddt_vector(nelt // 2, 1, 2, 4)
    d = pkg.Ddt.vector(nelt // 2, 1, 2, 4)
    send = np.arange(nelt, dtype=np.int32)
    dsend = _dev(torch, send)
    drecv = _dev(torch, np.full(nelt, 0xdeadbeef, dtype=np.uint32))
    segs = shuffle(segments(oracle, od, 1, 113))
    bufs = []
    for pos, size in segs:
        b = torch.zeros(128, dtype=torch.uint8, device="cuda")
        d.pack(1, dsend.data_ptr(), pos, b.data_ptr(), size)
        want = np.zeros(size, dtype=np.uint8)
        oracle.oracle_ddt_pack(od, 1, send.ctypes.data, pos, want.ctypes.data, size)
        assert np.array_equal(b[:size].cpu().numpy(), want), (pos, size)
        bufs.append(b)
    for (pos, size), b in zip(segs, bufs):
        d.unpack(1, drecv.data_ptr(), pos, b.data_ptr(), size)
    got = drecv.cpu().numpy().view(np.int32)
    want = np.where(np.arange(nelt) % 2 == 1, np.int32(-559038737), np.arange(nelt, dtype=np.int32))
    assert np.array_equal(got, want)


def test_position_long_double_int_gpu(gpu, pkg, oracle):
    torch = gpu
    n = 2048
    od = ldi_struct(oracle)
    d = pkg.Ddt.runs([0, 16], [16, 4], extent=32)
    send = np.zeros(n, dtype=LDI)
    send["ld"] = np.arange(n, dtype=np.longdouble) + np.arange(n, dtype=np.longdouble) / 100000.0
    send["i"] = np.arange(n)
    dsend, drecv = _dev(torch, send), torch.zeros(n * 32, dtype=torch.uint8, device="cuda")
    segs = shuffle(segments(oracle, od, n, 113))
    for pos, size in segs:
        b = torch.zeros(128, dtype=torch.uint8, device="cuda")
        d.pack(n, dsend.data_ptr(), pos, b.data_ptr(), size)
        d.unpack(n, drecv.data_ptr(), pos, b.data_ptr(), size)
    recv = drecv.cpu().numpy().view(LDI)
    assert np.array_equal(recv["ld"], send["ld"]) and np.array_equal(recv["i"], send["i"])


def test_checksum_gpu(gpu, pkg, oracle):
    torch = gpu
    size = 1024
    d = pkg.Ddt.vector(size, 1, 2, 4)
    od = oracle.oracle_ddt_vector(size, 1, 2, 4)
    rng = np.random.default_rng(11)
    data = np.zeros(2 * size, dtype=np.int32)
    data[0::2] = rng.integers(0, 2**31 - 1, size)
    packed = np.zeros(size, dtype=np.int32)
    want = oracle.oracle_ddt_pack_checksum(od, 1, data.ctypes.data, packed.ctypes.data)
    dd = _dev(torch, data)
    dp = torch.zeros(size * 4, dtype=torch.uint8, device="cuda")
    cs = d.pack(1, dd.data_ptr(), 0, dp.data_ptr(), size * 4, checksum=True)
    assert cs == want
    assert np.array_equal(dp.cpu().numpy().view(np.int32), packed)
    out = torch.zeros(2 * size * 4, dtype=torch.uint8, device="cuda")
    half = size * 2
    c1 = d.unpack(1, out.data_ptr(), 0, dp.data_ptr(), half, checksum=True)
    c2 = d.unpack(1, out.data_ptr(), half, dp.data_ptr() + half, size * 4 - half, checksum=True)
    assert (c1 + c2) & 0xFFFFFFFF == want
    # odd window splits: the per-window sums still add up to the message checksum
    parts = [0, 3, 101, 2047, 4093, size * 4]
    tot = 0
    for a, b in zip(parts[:-1], parts[1:]):
        tot += d.pack(1, dd.data_ptr(), a, dp.data_ptr(), b - a, checksum=True)
    assert tot & 0xFFFFFFFF == want


KINDS = ["vector", "indexed", "struct", "vector_odd", "vector_rows", "gapped_rows"]


@pytest.mark.parametrize("kind", KINDS)
def test_random_windows(gpu, pkg, oracle, kind):
    """random fragment windows; the *_rows kinds keep every window 16-B aligned so the row
    kernel (one run per block) takes them, the others exercise the general kernel"""
    torch = gpu
    rng = np.random.default_rng(KINDS.index(kind) + 5)
    align = 16 if kind.endswith("rows") else 1
    if kind == "vector_rows":
        count, args = 3, (1001, 32, 48, 4)
        d, od = pkg.Ddt.vector(*args), oracle.oracle_ddt_vector(*args)
    elif kind == "gapped_rows":  # one run of 48 B at disp 16 in a 96-B extent, count 700
        count = 700
        d = pkg.Ddt.runs([16], [48], extent=96)
        i64 = ctypes.c_int64 * 1
        od = oracle.oracle_ddt_struct(1, i64(16), i64(48), i64(8), 96)
    elif kind == "vector":
        count, args = 3, (97, 64, 128, 4)
        d, od = pkg.Ddt.vector(*args), oracle.oracle_ddt_vector(*args)
    elif kind == "vector_odd":
        count, args = 5, (33, 3, 7, 2)
        d, od = pkg.Ddt.vector(*args), oracle.oracle_ddt_vector(*args)
    elif kind == "indexed":
        bl = [int(x) for x in rng.integers(0, 9, 40)]
        dp = list(np.cumsum(rng.integers(0, 12, 40)))
        dp = [int(x) for x in dp]
        count = 4
        d = pkg.Ddt.indexed(bl, dp, 8)
        od = oracle.oracle_ddt_indexed(40, (ctypes.c_int * 40)(*bl), (ctypes.c_int * 40)(*dp), 8)
    else:
        count = 50
        d = pkg.Ddt.runs([0, 16], [16, 4], extent=32)
        od = ldi_struct(oracle)
    total = count * oracle.oracle_ddt_size(od)
    assert d.size * count == total
    span = (count - 1) * oracle.oracle_ddt_extent(od) + 4096 + oracle.oracle_ddt_extent(od)
    base = rng.integers(0, 256, span, dtype=np.uint8)
    dbase = _dev(torch, base)
    full = np.zeros(total, dtype=np.uint8)
    oracle.oracle_ddt_pack(od, count, base.ctypes.data, 0, full.ctypes.data, total)
    cuts = sorted(set([0, total] + [int(x) // align * align for x in rng.integers(0, total, 9)]))
    out = torch.zeros(total + 64, dtype=torch.uint8, device="cuda")
    for a, b in zip(cuts[:-1], cuts[1:]):
        d.pack(count, dbase.data_ptr(), a, out.data_ptr() + a, b - a)
    assert np.array_equal(out[:total].cpu().numpy(), full)
    # unpack into zeros reproduces exactly the type map's bytes
    z = torch.zeros(span, dtype=torch.uint8, device="cuda")
    for a, b in zip(cuts[:-1], cuts[1:]):
        d.unpack(count, z.data_ptr(), a, out.data_ptr() + a, b - a)
    want = np.zeros(span, dtype=np.uint8)
    oracle.oracle_ddt_unpack(od, count, want.ctypes.data, 0, full.ctypes.data, total)
    assert np.array_equal(z.cpu().numpy(), want)


def test_row_kernel_checksum(gpu, pkg, oracle):
    torch = gpu
    args = (5000, 64, 128, 4)
    d, od = pkg.Ddt.vector(*args), oracle.oracle_ddt_vector(*args)
    data = np.random.default_rng(8).integers(0, 2**32, 5000 * 128, dtype=np.uint32)
    packed = np.zeros(5000 * 64, dtype=np.uint32)
    want = oracle.oracle_ddt_pack_checksum(od, 1, data.ctypes.data, packed.ctypes.data)
    dd = _dev(torch, data)
    dp = torch.zeros(d.size, dtype=torch.uint8, device="cuda")
    assert d.pack(1, dd.data_ptr(), 0, dp.data_ptr(), d.size, checksum=True) == want
    assert np.array_equal(dp.cpu().numpy().view(np.uint32), packed)
    out = torch.zeros_like(dd)
    assert d.unpack(1, out.data_ptr(), 0, dp.data_ptr(), d.size, checksum=True) == want


def test_config5_vector_1gib(gpu, pkg):
    """MPI_Type_vector(2^22, 64, 128, MPI_FLOAT) over a 2 GiB-extent buffer: pack == the strided
    view's blocks, unpack into zeros restores them and leaves the gaps untouched"""
    torch = gpu
    nblk = 1 << 22
    d = pkg.Ddt.vector(nblk, 64, 128, 4)
    x = torch.randn(nblk, 128, device="cuda")
    packed = torch.empty(nblk, 64, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    d.pack(1, x.data_ptr(), 0, packed.data_ptr(), d.size, s)
    torch.cuda.synchronize()
    assert torch.equal(packed, x[:, :64])
    y = torch.zeros_like(x)
    d.unpack(1, y.data_ptr(), 0, packed.data_ptr(), d.size, s)
    torch.cuda.synchronize()
    assert torch.equal(y[:, :64], x[:, :64]) and int(torch.count_nonzero(y[:, 64:])) == 0
    del x, y, packed
    torch.cuda.empty_cache()


# ---- opal_datatype_test.c's convertor dances replayed on the GPU convertor, each type compiled
#      from the description records the reference would hold (oracle/opal_types.py) through
#      mi355x_ddt_from_opal -- the call coll/mi355x makes for a derived MPI datatype
from ddtcases import CONVERTOR_CASES, c_oracle, expected_copy, fill_pattern, ot, span_of, windows  # noqa: E402


def _gpu_convertor_copy(torch, pkg, oracle, t, count, chunk, recv=None):
    recv = recv or t
    sizes = ot.basic_sizes()
    ds = pkg.Ddt.from_opal(t.desc_bytes(), len(t.desc), t.extent, sizes)
    dr = pkg.Ddt.from_opal(recv.desc_bytes(), len(recv.desc), recv.extent, sizes)
    ods = c_oracle(oracle, t)
    n, origin = span_of(t, count)
    nr, origin_r = span_of(recv, count)
    src = fill_pattern(n)
    dsrc = torch.from_numpy(src).cuda()
    ddst = torch.zeros(nr, dtype=torch.uint8, device="cuda")
    total = count * t.size
    packed = torch.zeros(total + 16, dtype=torch.uint8, device="cuda")
    for pos, size in windows(oracle, ods, count, chunk):
        tmp = packed[pos:]  # each window lands at its stream offset so the whole stream can be checked
        ds.pack(count, dsrc.data_ptr() + origin, pos, tmp.data_ptr(), size)
        dr.unpack(count, ddst.data_ptr() + origin_r, pos, tmp.data_ptr(), size)
    want_stream = np.zeros(total, dtype=np.uint8)
    oracle.oracle_ddt_pack(ods, count, src.ctypes.data + origin, 0, want_stream.ctypes.data, total)
    oracle.oracle_ddt_free(ods)
    ds.destroy()
    dr.destroy()
    return src, ddst.cpu().numpy(), origin, packed[:total].cpu().numpy(), want_stream


@pytest.mark.parametrize("case", [c[0] for c in CONVERTOR_CASES])
def test_convertor_cases_gpu(gpu, pkg, oracle, case):
    """local_copy_with_convertor(pdt, count, chunk) for every case of opal_datatype_test.c main()
    (upper_matrix(100) in 48-byte chunks, vector(450, 10, 11) in 12/82/6000/36000, blacs in
    956/16K/64K, ...): the packed stream equals the oracle's, the destination holds exactly the
    type map's bytes"""
    torch = gpu
    name, build, count, chunks = next(c for c in CONVERTOR_CASES if c[0] == case)
    t = build()
    for chunk in chunks:
        src, dst, origin, stream, want_stream = _gpu_convertor_copy(torch, pkg, oracle, t, count, chunk)
        assert np.array_equal(stream, want_stream), (case, chunk, "packed stream")
        assert np.array_equal(dst, expected_copy(t, count, src, origin)), (case, chunk, "unpacked")


def test_convertor_two_datatypes_blacs_gpu(gpu, pkg, oracle):
    """local_copy_with_convertor_2datatypes(blacs1, 1, blacs2, 1, 100) (opal_datatype_test.c:533-538)"""
    src, dst, _, _, _ = _gpu_convertor_copy(gpu, pkg, oracle, ot.blacs1(), 1, 100, recv=ot.blacs2())
    assert np.array_equal(dst[:52].view(np.int32)[0::2], src[:76].view(np.int32)[0::3])
    assert not dst[:52].view(np.int32)[1::2].any()


def test_upper_500_gpu(gpu, pkg):
    """test_upper(500) (opal_datatype_test.c:46-115) on device memory: the packed upper triangle
    unpacked in (length + 1) * 8-byte chunks into a zeroed matrix, then check_diag_matrix"""
    torch = gpu
    n = 500
    t = ot.upper_matrix(n)
    d = pkg.Ddt.from_opal(t.desc_bytes(), len(t.desc), t.extent, ot.basic_sizes())
    mat1 = torch.zeros(n, n, dtype=torch.float64)
    iu = torch.triu_indices(n, n)
    mat1[iu[0], iu[1]] = torch.from_numpy(np.random.default_rng(5).integers(0, 2**31, iu.shape[1]).astype(np.float64))
    inbuf = mat1[iu[0], iu[1]].contiguous().cuda()
    mat2 = torch.zeros(n, n, dtype=torch.float64, device="cuda")
    chunk, pos, nbytes = (n + 1) * 8, 0, inbuf.numel() * 8
    while pos < nbytes:
        size = min(chunk, nbytes - pos)
        d.unpack(1, mat2.data_ptr(), pos, inbuf.data_ptr() + pos, size)
        pos += size
    assert torch.equal(mat2.cpu(), mat1), "check_diag_matrix"
    # and the other direction: pack the matrix back into the triangle stream
    out = torch.zeros_like(inbuf)
    d.pack(1, mat2.data_ptr(), 0, out.data_ptr(), nbytes)
    assert torch.equal(out, inbuf)
    d.destroy()


NARROW = [  # (vector args, count): the widest slot every address allows
    ((5001, 1, 3, 8), 2),    # a column of doubles: 8-B runs, 24-B stride -> 8-B slots
    ((1001, 2, 3, 8), 3),    # 16-B runs at a 24-B stride -> 8-B slots
    ((3001, 3, 5, 4), 2),    # 3-float blocks -> 4-B slots
    ((2001, 3, 4, 2), 3),    # 6-B runs -> 2-B slots
    ((1001, 5, 7, 1), 3),    # 5-B runs -> 1-B slots
]


@pytest.mark.parametrize("case", range(len(NARROW)))
def test_narrow_row_slots(gpu, pkg, oracle, case):
    """the row kernel with 8/4/2/1-byte slots (mode 2) against the oracle: packed stream, unpacked
    bytes and the per-window checksums (additive to the whole message's), windows cut at multiples
    of the element size and at odd bytes; modes 1 (16-B slots only) and 0 (general kernel) give
    the same bytes"""
    torch = gpu
    args, count = NARROW[case]
    d, od = pkg.Ddt.vector(*args), oracle.oracle_ddt_vector(*args)
    total = count * oracle.oracle_ddt_size(od)
    span = (count - 1) * oracle.oracle_ddt_extent(od) + oracle.oracle_ddt_extent(od) + 64
    rng = np.random.default_rng(40 + case)
    base = rng.integers(0, 256, span, dtype=np.uint8)
    dbase = _dev(torch, base)
    full = np.zeros(total, dtype=np.uint8)
    want_cs = oracle.oracle_ddt_pack_checksum(od, count, base.ctypes.data, full.ctypes.data)
    want_mem = np.zeros(span, dtype=np.uint8)
    oracle.oracle_ddt_unpack(od, count, want_mem.ctypes.data, 0, full.ctypes.data, total)
    esz = args[3]
    cuts = sorted(set([0, total] + [int(x) // esz * esz for x in rng.integers(0, total, 6)] +
                      [int(x) for x in rng.integers(0, total, 2)]))
    try:
        for mode in (2, 1, 0):
            pkg.ddt_tune_rows(mode)
            out = torch.zeros(total + 64, dtype=torch.uint8, device="cuda")
            cs = 0
            for a, b in zip(cuts[:-1], cuts[1:]):
                # packed windows at their stream offset (alignment = the window's own)
                cs += d.pack(count, dbase.data_ptr(), a, out.data_ptr() + a, b - a, checksum=True)
            assert np.array_equal(out[:total].cpu().numpy(), full), mode
            assert cs % 2**32 == want_cs, (mode, cs, want_cs)
            z = torch.zeros(span, dtype=torch.uint8, device="cuda")
            cs = 0
            for a, b in zip(cuts[:-1], cuts[1:]):
                cs += d.unpack(count, z.data_ptr(), a, out.data_ptr() + a, b - a, checksum=True)
            assert np.array_equal(z.cpu().numpy(), want_mem), mode
            assert cs % 2**32 == want_cs, mode
    finally:
        pkg.ddt_tune_rows(2)


UNIT_CASES = [  # run lists (several runs per block): (blocklens, disps, elem size, count)
    ([int(100 - i) for i in range(100)], [int(101 * i) for i in range(100)], 8, 2),  # upper triangle of 100x100 doubles
    ([1, 3, 2, 7, 1, 1, 4], [0, 2, 9, 13, 25, 27, 40], 4, 300),
    ([3, 1, 5, 2], [1, 6, 9, 17], 2, 500),
    ([2, 5, 1], [0, 4, 13], 1, 900),
    ([37, 50, 23], [1, 41, 97], 4, 400),  # long runs of floats at odd float offsets: wide slots, W = 4
]


@pytest.mark.parametrize("case", range(len(UNIT_CASES)))
def test_unit_kernel(gpu, pkg, oracle, case):
    """the unit kernel (run tables staged in LDS; 16-B packed slots over 8/4-B aligned runs where
    the window allows, else W-byte units) against the oracle for indexed run lists, windows at
    element multiples, at 16-B multiples and at odd bytes, with checksums; mode 3 (W-byte units
    only) and mode 0 (the general kernel) give the same bytes"""
    torch = gpu
    bl, dp, esz, count = UNIT_CASES[case]
    n = len(bl)
    d = pkg.Ddt.indexed(bl, dp, esz)
    od = oracle.oracle_ddt_indexed(n, (ctypes.c_int * n)(*bl), (ctypes.c_int * n)(*dp), esz)
    total = count * oracle.oracle_ddt_size(od)
    assert d.size * count == total
    span = count * oracle.oracle_ddt_extent(od) + 64
    rng = np.random.default_rng(60 + case)
    base = rng.integers(0, 256, span, dtype=np.uint8)
    dbase = _dev(torch, base)
    full = np.zeros(total, dtype=np.uint8)
    want_cs = oracle.oracle_ddt_pack_checksum(od, count, base.ctypes.data, full.ctypes.data)
    want_mem = np.zeros(span, dtype=np.uint8)
    oracle.oracle_ddt_unpack(od, count, want_mem.ctypes.data, 0, full.ctypes.data, total)
    cuts = sorted(set([0, total] + [int(x) // esz * esz for x in rng.integers(0, total, 6)] +
                      [int(x) // 16 * 16 for x in rng.integers(0, total, 6)] +
                      [int(x) for x in rng.integers(0, total, 2)]))
    try:
        for mode in (2, 3, 0):
            pkg.ddt_tune_rows(mode)
            out = torch.zeros(total + 64, dtype=torch.uint8, device="cuda")
            cs = sum(d.pack(count, dbase.data_ptr(), a, out.data_ptr() + a, b - a, checksum=True)
                     for a, b in zip(cuts[:-1], cuts[1:]))
            assert np.array_equal(out[:total].cpu().numpy(), full), mode
            assert cs % 2**32 == want_cs, mode
            z = torch.zeros(span, dtype=torch.uint8, device="cuda")
            cs = sum(d.unpack(count, z.data_ptr(), a, out.data_ptr() + a, b - a, checksum=True)
                     for a, b in zip(cuts[:-1], cuts[1:]))
            assert np.array_equal(z.cpu().numpy(), want_mem), mode
            assert cs % 2**32 == want_cs, mode
    finally:
        pkg.ddt_tune_rows(2)


# ---- ddt_raw.c / ddt_test.c on the GPU convertor
from ddtcases import COPY_CASES, RAW_CASES  # noqa: E402


def _compiled(pkg, t):
    return pkg.Ddt.from_opal(t.desc_bytes(), len(t.desc), t.extent, ot.basic_sizes())


@pytest.mark.parametrize("case", [c[0] for c in RAW_CASES])
def test_raw_pieces_are_the_packed_stream_gpu(gpu, pkg, case):
    """the memory pieces mi355x_ddt_raw describes, read in order, are exactly the stream the GPU
    pack kernel produces (opal_convertor_raw vs opal_convertor_pack on one convertor)"""
    torch = gpu
    _, build, count = next(c for c in RAW_CASES if c[0] == case)
    t = build()
    n, origin = span_of(t, count)
    src = fill_pattern(n)
    d = _compiled(pkg, t)
    pieces = [p for c in d.raw(count, 5) for p in c]
    want = np.concatenate([src[origin + off:origin + off + ln] for off, ln in pieces])
    dsrc = torch.from_numpy(src).cuda()
    out = torch.zeros(count * t.size, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    d.pack(count, dsrc.data_ptr() + origin, 0, out.data_ptr(), count * t.size)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), want)
    d.destroy()


@pytest.mark.parametrize("case", [c[0] for c in COPY_CASES])
def test_local_copy_ddt_count_gpu(gpu, pkg, case):
    """ompi_datatype_copy_content_same_ddt (ddt_test.c:141-170) on device memory: pack + unpack
    kernels leave exactly the type map's bytes in a zeroed destination, and agree with the host
    convertor"""
    torch = gpu
    _, build, count = next(c for c in COPY_CASES if c[0] == case)
    t = build()
    n, origin = span_of(t, count)
    src = fill_pattern(n)
    total = count * t.size
    d = _compiled(pkg, t)
    dsrc = torch.from_numpy(src).cuda()
    ddst = torch.zeros(n, dtype=torch.uint8, device="cuda")
    tmp = torch.zeros(total, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    d.pack(count, dsrc.data_ptr() + origin, 0, tmp.data_ptr(), total)
    d.unpack(count, ddst.data_ptr() + origin, 0, tmp.data_ptr(), total)
    torch.cuda.synchronize()
    assert np.array_equal(ddst.cpu().numpy(), expected_copy(t, count, src, origin))
    hp = np.zeros(total, dtype=np.uint8)
    d.pack_host(count, src.ctypes.data + origin, 0, hp.ctypes.data, total)
    assert np.array_equal(tmp.cpu().numpy(), hp)
    d.destroy()


def test_zero_count_contiguous_types_gpu(gpu, pkg):
    """ddt_test.c:401-411 types (pdt1 with long double elements) packed on the GPU == host convertor"""
    torch = gpu
    for t in ot.ddt_test_zero_count_types():
        d = _compiled(pkg, t)
        n, origin = span_of(t, 5)
        src = fill_pattern(n)
        dsrc = torch.from_numpy(src).cuda()
        out = torch.zeros(5 * t.size, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        d.pack(5, dsrc.data_ptr() + origin, 0, out.data_ptr(), 5 * t.size)
        torch.cuda.synchronize()
        hp = np.zeros(5 * t.size, dtype=np.uint8)
        d.pack_host(5, src.ctypes.data + origin, 0, hp.ctypes.data, hp.size)
        assert np.array_equal(out.cpu().numpy(), hp)
        d.destroy()


RUNS_CASES = [  # (disps, lens, nblk, stride, extent, count): long 8- / 4-B aligned runs (>= 512 B on
    # average) with unaligned heads / tails, 16-B multiple extents
    ([int(i * 257 * 8) for i in range(256)], [int((256 - i) * 8) for i in range(256)], 1, 0, 256 * 256 * 8, 2),  # triangle
    ([4, 2052, 6000], [1000, 3000, 604], 1, 0, 8192, 60),          # floats, W = 4: 12-B heads and tails
    ([8, 40, 1000], [8, 24, 9000], 1, 0, 10016, 40),               # doubles: a run inside its head; a run over 3 chunks
    ([16, 1032], [1000, 1000], 50, 2048, 50 * 2048, 12),           # blocks: 2 runs per block, 50 blocks
]


@pytest.mark.parametrize("case", range(len(RUNS_CASES)))
def test_long_run_unpack(gpu, pkg, case):
    """unpack of long W-aligned runs (the triangle of the unpack ceiling probe, floats with 12-B heads
    and tails, runs spanning several 4-KiB spans, two runs per block), whole messages under both row
    modes of the unit kernel and random convertor windows (the wave-per-run kernel clips the first and
    last run): the bytes equal the host convertor's, gaps untouched"""
    torch = gpu
    disps, lens, nblk, stride, extent, count = RUNS_CASES[case]
    d = pkg.Ddt.runs(disps, lens, nblk, stride, extent)
    total = count * d.size
    span = count * extent + 64
    rng = np.random.default_rng(90 + case)
    packed = rng.integers(0, 256, total, dtype=np.uint8)
    init = rng.integers(0, 256, span, dtype=np.uint8)
    want = init.copy()
    d.unpack_host(count, want.ctypes.data, 0, packed.ctypes.data, total)
    dp = _dev(torch, packed)
    try:
        for mode in (2, 3):
            pkg.ddt_tune_rows(mode)
            z = _dev(torch, init)
            d.unpack(count, z.data_ptr(), 0, dp.data_ptr(), total)
            torch.cuda.synchronize()
            assert np.array_equal(z.cpu().numpy(), want), (case, mode)
        # the same through convertor windows (set_position fragments): W-aligned cut points, windows
        # starting and ending inside runs, inside heads / tails and on run edges
        W = 4 if case == 1 else 8
        for trial in range(3):
            cuts = sorted(set([0, total] + [int(c) * W for c in rng.integers(1, total // W, 2 + 3 * trial)]))
            z = _dev(torch, init)
            for lo, hi in zip(cuts[:-1], cuts[1:]):
                d.unpack(count, z.data_ptr(), lo, dp.data_ptr() + lo, hi - lo)
            torch.cuda.synchronize()
            assert np.array_equal(z.cpu().numpy(), want), (case, "windows", cuts)
    finally:
        pkg.ddt_tune_rows(2)
    d.destroy()
