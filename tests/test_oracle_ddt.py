"""The convertor oracle checked with the reference's own known-answer tests, restated:

* test/datatype/position_noncontig.c:189-253 -- vector(NELT/2, 1, 2, MPI_INT), NELT = 300,
  fragments of 113 bytes, shuffled, packed and unpacked segment by segment;
* test/datatype/position.c:220-286 -- 2048 MPI_LONG_DOUBLE_INT, same segment dance;
* test/datatype/checksum.c:29-154 -- vector(1024, 1, 2, MPI_INT): the checksum of packing the
  sparse data, of packing the packed ints as a contiguous type, of unpacking through two iovecs,
  and OPAL_CSUM_PARTIAL over the packed buffer must all agree.
Plus the constructors' size/extent/run-merging rules (ompi_datatype_create_vector.c:36-65,
ompi_datatype_create_indexed.c:32-66)."""
from __future__ import annotations

import ctypes

import numpy as np

from ddtcases import LDI, ldi_struct, segments, shuffle


def test_position_noncontig(oracle):
    nelt = 300
    od = oracle.oracle_ddt_vector(nelt // 2, 1, 2, 4)
    send = np.arange(nelt, dtype=np.int32)
    recv = np.full(nelt, 0xdeadbeef, dtype=np.uint32).view(np.int32)
    segs = shuffle(segments(oracle, od, 1, 113))
    bufs = []
    for pos, size in segs:
        b = np.zeros(113, dtype=np.uint8)
        assert oracle.oracle_ddt_pack(od, 1, send.ctypes.data, pos, b.ctypes.data, size) == 0
        bufs.append(b)
    for (pos, size), b in zip(segs, bufs):
        assert oracle.oracle_ddt_unpack(od, 1, recv.ctypes.data, pos, b.ctypes.data, size) == 0
    want = np.where(np.arange(nelt) % 2 == 1, np.int32(-559038737), np.arange(nelt, dtype=np.int32))
    assert np.array_equal(recv, want)
    # every segment ends on an int boundary (set_position semantics)
    assert all(p % 4 == 0 for p, _ in segs)


def test_position_long_double_int(oracle):
    n = 2048
    od = ldi_struct(oracle)
    assert oracle.oracle_ddt_size(od) == 20 and oracle.oracle_ddt_extent(od) == 32
    send = np.zeros(n, dtype=LDI)
    send["ld"] = np.arange(n, dtype=np.longdouble) + np.arange(n, dtype=np.longdouble) / 100000.0
    send["i"] = np.arange(n)
    recv = np.zeros(n, dtype=LDI)
    segs = shuffle(segments(oracle, od, n, 113))
    bufs = []
    for pos, size in segs:
        b = np.zeros(113, dtype=np.uint8)
        oracle.oracle_ddt_pack(od, n, send.ctypes.data, pos, b.ctypes.data, size)
        bufs.append(b)
    for (pos, size), b in zip(segs, bufs):
        oracle.oracle_ddt_unpack(od, n, recv.ctypes.data, pos, b.ctypes.data, size)
    assert np.array_equal(recv["ld"], send["ld"]) and np.array_equal(recv["i"], send["i"])


def test_checksum_kat(oracle):
    size = 1024
    sparse = oracle.oracle_ddt_vector(size, 1, 2, 4)
    contig = oracle.oracle_ddt_contiguous(size, 4)
    rng = np.random.default_rng(7)
    data = np.zeros(2 * size, dtype=np.int32)
    data[0::2] = rng.integers(0, 2**31 - 1, size)
    packed = np.zeros(size, dtype=np.int32)
    pack_cs = oracle.oracle_ddt_pack_checksum(sparse, 1, data.ctypes.data, packed.ctypes.data)
    array = np.zeros(size, dtype=np.int32)
    contig_cs = oracle.oracle_ddt_pack_checksum(contig, 1, packed.ctypes.data, array.ctypes.data)
    # unpack through two iovecs (checksum.c:101-117): two windows of the same stream
    sparse_out = np.zeros(2 * size, dtype=np.int32)
    half = size * 4 // 2
    oracle.oracle_ddt_unpack(sparse, 1, sparse_out.ctypes.data, 0, array.ctypes.data, half)
    oracle.oracle_ddt_unpack(sparse, 1, sparse_out.ctypes.data, half, array.ctypes.data + half, size * 4 - half)
    ui1, ui2 = ctypes.c_uint(0), ctypes.c_size_t(0)
    unpack_cs = 0
    for off, ln in ((0, half), (half, size * 4 - half)):
        unpack_cs = (unpack_cs + oracle.oracle_uicsum_partial(array.ctypes.data + off, ln, ctypes.byref(ui1),
                                                              ctypes.byref(ui2))) & 0xFFFFFFFF
    ui1, ui2 = ctypes.c_uint(0), ctypes.c_size_t(0)
    manual = oracle.oracle_uicsum_partial(packed.ctypes.data, size * 4, ctypes.byref(ui1), ctypes.byref(ui2)) & 0xFFFFFFFF
    assert pack_cs == contig_cs == unpack_cs == manual
    assert np.array_equal(sparse_out[0::2], data[0::2])
    assert manual == int(packed.view(np.uint32).sum(dtype=np.uint64) & 0xFFFFFFFF)


def test_checksum_partial_any_split(oracle):
    """opal_uicsum_partial carried across arbitrary splits == the one-shot word sum"""
    rng = np.random.default_rng(3)
    buf = rng.integers(0, 256, 1003, dtype=np.uint8)
    want = int(np.frombuffer(np.concatenate([buf, np.zeros(1, np.uint8)]).tobytes(), dtype=np.uint32).sum(dtype=np.uint64)
               & 0xFFFFFFFF)
    for cuts in ([1, 2, 3, 500], [7, 11, 13], [999], [4, 8, 12]):
        ui1, ui2 = ctypes.c_uint(0), ctypes.c_size_t(0)
        tot, prev = 0, 0
        for c in cuts + [len(buf)]:
            tot += oracle.oracle_uicsum_partial(buf.ctypes.data + prev, c - prev, ctypes.byref(ui1), ctypes.byref(ui2))
            prev = c
        assert tot & 0xFFFFFFFF == want


def test_constructor_rules(oracle):
    v = oracle.oracle_ddt_vector(4, 64, 128, 4)            # config 5 shape, 4 blocks
    assert oracle.oracle_ddt_size(v) == 4 * 256 and oracle.oracle_ddt_extent(v) == (3 * 128 + 64) * 4
    c = oracle.oracle_ddt_vector(4, 64, 64, 4)             # stride == blocklen -> contiguous
    assert oracle.oracle_ddt_size(c) == oracle.oracle_ddt_extent(c) == 1024
    bl = (ctypes.c_int * 3)(2, 3, 1)
    dp = (ctypes.c_int * 3)(0, 2, 10)                       # first two blocks are adjacent -> merged
    ix = oracle.oracle_ddt_indexed(3, bl, dp, 8)
    assert oracle.oracle_ddt_size(ix) == 48 and oracle.oracle_ddt_extent(ix) == 88


# ---- test/datatype/opal_datatype_test.c:366-383 and opal_ddt_lib.c:478-850, restated through
#      oracle/opal_types.py (opal_datatype_add's bounds rules + the test library's constructors)
from ddtcases import CONVERTOR_CASES, c_oracle, expected_copy, fill_pattern, ot, span_of  # noqa: E402

import pytest  # noqa: E402


def _bounds(t):
    return t.lb, t.ub, t.extent, t.size


def test_mpich_typeub():
    """mpich_typeub (opal_ddt_lib.c:619-679): a UB marker sets the extent, and a smaller UB marker
    added later does not shrink it (MPIF semantics: 16, not 4)"""
    t1, t2, t3 = ot.typeub()
    assert t1.extent == 5 * 4 and t2.extent == 16 and t3.extent == 16


def test_mpich_typeub2():
    """Example 3.26 of MPI-1 (opal_ddt_lib.c:681-758): {LB -3, int 0, UB 6}, its contiguous(2) and
    the same as a struct of two instances"""
    dt1, dt2, dt3 = ot.typeub2()
    assert (dt1.lb, dt1.ub, dt1.extent) == (-3, 6, 9)
    assert (dt2.lb, dt2.ub, dt2.extent) == (-3, 15, 18)
    assert (dt3.lb, dt3.ub, dt3.extent) == (-3, 15, 18)
    assert dt1.size == 4 and dt2.size == dt3.size == 8


def test_mpich_typeub3():
    """hindexed / indexed / hvector / vector of the explicit-bounds type (opal_ddt_lib.c:760-850)"""
    hi, ix, hv, ve = ot.typeub3()
    assert (hi.lb, hi.ub, hi.extent) == (-7, 13, 20)
    assert (ix.lb, ix.ub, ix.extent) == (-39, 69, 108)
    assert (hv.lb, hv.ub, hv.extent) == (-3, 20, 23)
    assert (ve.lb, ve.ub, ve.extent) == (-3, 132, 135)


def test_constructed_bounds():
    """upper_matrix(100): 5050 doubles over a 100x100 extent; test_struct / test_contiguous
    (alignment epsilon), the resized strange type, matrix borders"""
    u = ot.upper_matrix(100)
    assert _bounds(u) == (0, 80000, 80000, 5050 * 8) and (u.true_lb, u.true_ub) == (0, 80000)
    s = ot.test_struct()
    assert _bounds(s) == (0, 32, 32, 20) and (s.true_lb, s.true_ub) == (0, 29)
    c = ot.contiguous_alignment()  # {double, char} -> extent 16 by alignment, x4 x2
    assert _bounds(c) == (0, 128, 128, 72)
    st = ot.strange_dt()  # {double, char} resized to 12, x10
    assert _bounds(st) == (0, 120, 120, 90)
    assert ot.struct_char_double().extent == 16 and ot.twice_two_doubles().extent == 7 * 8


@pytest.mark.parametrize("case", [c[0] for c in CONVERTOR_CASES])
def test_desc_walk_is_the_type_map(case):
    """the description records opal_datatype_add writes, walked the way the convertor walks them,
    visit exactly the type map (for every convertor case type)"""
    t = dict((c[0], c[1]) for c in CONVERTOR_CASES)[case]()
    assert ot.walk_desc(t, 2) == [(d + k * t.extent, s) for k in range(2) for d, s in t.tmap]


def _convertor_copy(oracle, t, count, chunk, recv=None):
    """local_copy_with_convertor(_2datatypes) (opal_datatype_test.c:163-329) on the oracle: pack
    `chunk`-byte windows (ending on element boundaries, as the convertor stops) and unpack each"""
    from ddtcases import windows
    recv = recv or t
    ods, odr = c_oracle(oracle, t), c_oracle(oracle, recv)
    n, origin = span_of(t, count)
    nr, origin_r = span_of(recv, count)
    src = fill_pattern(n)
    dst = np.zeros(nr, dtype=np.uint8)
    tmp = np.zeros(chunk + 16, dtype=np.uint8)
    total = 0
    for pos, size in windows(oracle, ods, count, chunk):
        assert oracle.oracle_ddt_pack(ods, count, src.ctypes.data + origin, pos, tmp.ctypes.data, size) == 0
        assert oracle.oracle_ddt_unpack(odr, count, dst.ctypes.data + origin_r, pos, tmp.ctypes.data, size) == 0
        total += size
    oracle.oracle_ddt_free(ods)
    oracle.oracle_ddt_free(odr)
    return src, dst, origin, total


@pytest.mark.parametrize("case", [c[0] for c in CONVERTOR_CASES])
def test_convertor_copy_cases(oracle, case):
    name, build, count, chunks = next(c for c in CONVERTOR_CASES if c[0] == case)
    t = build()
    for chunk in chunks[:2]:
        src, dst, origin, total = _convertor_copy(oracle, t, count, chunk)
        assert total == count * t.size
        assert np.array_equal(dst, expected_copy(t, count, src, origin)), (case, chunk)


def test_convertor_two_datatypes_blacs(oracle):
    """local_copy_with_convertor_2datatypes(blacs1, 1, blacs2, 1, 100) (opal_datatype_test.c:533-538):
    vector(7, 1, 3, int) packed, unpacked as vector(7, 1, 2, int)"""
    t1, t2 = ot.blacs1(), ot.blacs2()
    src, dst, _, total = _convertor_copy(oracle, t1, 1, 100, recv=t2)
    assert total == 28
    assert np.array_equal(dst[:52].view(np.int32)[0::2], src[:76].view(np.int32)[0::3])


def test_upper_500(oracle):
    """test_upper(500) (opal_datatype_test.c:46-115): the packed upper triangle unpacked through a
    recv convertor in (length + 1) * 8-byte chunks, then check_diag_matrix"""
    n = 500
    t = ot.upper_matrix(n)
    od = c_oracle(oracle, t)
    mat1 = np.zeros((n, n))
    iu = np.triu_indices(n)
    mat1[iu] = np.random.default_rng(5).integers(0, 2**31, len(iu[0])).astype(np.float64)
    inbuf = np.ascontiguousarray(mat1[iu])  # row by row from the diagonal, as the test fills it
    assert inbuf.nbytes == n * (n + 1) * 4
    mat2 = np.zeros((n, n))
    chunk, pos = (n + 1) * 8, 0
    while pos < inbuf.nbytes:
        size = min(chunk, inbuf.nbytes - pos)
        assert oracle.oracle_ddt_unpack(od, 1, mat2.ctypes.data, pos, inbuf.ctypes.data + pos, size) == 0
        assert mat2[0, 0] == inbuf[0]
        pos += size
    assert np.array_equal(mat2[iu], mat1[iu]) and not mat2[np.tril_indices(n, -1)].any()
    oracle.oracle_ddt_free(od)


def test_from_opal_matches_restated_types(pkg):
    """the GPU convertor compiles each restated type's description records (the records the
    coll/mi355x component hands to mi355x_ddt_from_opal) to the same size and extent"""
    sizes = ot.basic_sizes()
    types = [c[1]() for c in CONVERTOR_CASES] + list(ot.typeub2()) + [ot.blacs1(), ot.blacs2()]
    for t in types:
        d = pkg.Ddt.from_opal(t.desc_bytes(), len(t.desc), t.extent, sizes)
        assert (d.size, d.extent) == (t.size, t.extent)
        assert d.nruns <= len(t.runs())
        d.destroy()


def test_ddt_pack_c_types():
    """the types test/datatype/ddt_pack.c:70-101 builds: hindexed(2, {10, 10}, {0, 160 B},
    MPI_DOUBLE) = 160 B of data over a 240-B extent; struct {11 x MPI_INT at 0, 2 x the hindexed at
    64} = 44 + 320 B over [0, 544)"""
    from ddtcases import _ddt_pack_hindexed
    h = _ddt_pack_hindexed()
    assert (h.size, h.lb, h.ub) == (160, 0, 240)
    s = ot.struct_([11, 2], [0, 64], [ot.OpalType.basic("INT4"), h]).commit()
    assert (s.size, s.lb, s.ub) == (364, 0, 544)
    elems = ot.walk_desc(s)  # the convertor's visit order: 11 ints, then 2 x (10 + 10) doubles
    assert sum(n for _, n in elems) == 364 and [a for a, _ in elems[:12]] == [4 * i for i in range(11)] + [64]


# ---- test/datatype/ddt_raw.c and ddt_test.c, restated (VERDICT r2 missing #4)
from ddtcases import COPY_CASES, RAW_CASES  # noqa: E402


def _compiled(pkg, t):
    """the engine's layout of a restated type: its description records through mi355x_ddt_from_opal
    (what coll/mi355x hands the engine for a committed derived datatype)"""
    return pkg.Ddt.from_opal(t.desc_bytes(), len(t.desc), t.extent, ot.basic_sizes())


@pytest.mark.parametrize("case", [c[0] for c in RAW_CASES])
def test_raw_walk_kat(pkg, case):
    """opal_convertor_raw's walk: calls of at most 5 iovecs that together describe every byte
    (ddt_raw.c:118-131 -- the reference's check is `remaining_length == 0`) in type-map order, on the
    restated convertor walk and on the engine's mi355x_ddt_raw (no GPU)"""
    _, build, count = next(c for c in RAW_CASES if c[0] == case)
    t = build()
    tmap = ot.merge_pieces([(d + k * t.extent, s) for k in range(count) for d, s in t.tmap])
    calls = ot.convertor_raw(t, count, 5)
    assert all(len(c) <= 5 for c in calls) and all(len(c) == 5 for c in calls[:-1])
    assert sum(n for c in calls for _, n in c) == count * t.size
    assert ot.merge_pieces([p for c in calls for p in c]) == tmap
    d = _compiled(pkg, t)
    ecalls = d.raw(count, 5)
    assert all(len(c) <= 5 for c in ecalls) and all(len(c) == 5 for c in ecalls[:-1])
    assert sum(n for c in ecalls for _, n in c) == count * t.size
    assert ot.merge_pieces([p for c in ecalls for p in c]) == tmap
    # resuming at any packed position describes the rest (opal_convertor_raw restarts from its stack)
    for cut in (1, 7, count * t.size // 3):
        pos = ctypes.c_size_t(cut)
        got = []
        while True:
            disp = (ctypes.c_int64 * 5)()
            lens = (ctypes.c_size_t * 5)()
            cnt, mx = ctypes.c_uint32(5), ctypes.c_size_t()
            rc = pkg.rt().mi355x_ddt_raw(d.h, count, ctypes.byref(pos), disp, lens, ctypes.byref(cnt), ctypes.byref(mx))
            got += [(disp[i], lens[i]) for i in range(cnt.value)]
            if rc == 1:
                break
        assert sum(n for _, n in got) == count * t.size - cut
    d.destroy()


@pytest.mark.parametrize("case", [c[0] for c in COPY_CASES])
def test_local_copy_ddt_count_host(pkg, oracle, case):
    """ompi_datatype_copy_content_same_ddt(pdt, count, dst, src) (ddt_test.c:141-170) through the
    engine's host convertor (pack then unpack, the bytes a same-type copy moves): the destination
    holds exactly the type map's bytes of the source; the packed stream equals the oracle's"""
    _, build, count = next(c for c in COPY_CASES if c[0] == case)
    t = build()
    n, origin = span_of(t, count)
    src = fill_pattern(n)
    dst = np.zeros(n, dtype=np.uint8)
    total = count * t.size
    d = _compiled(pkg, t)
    packed = np.zeros(total, dtype=np.uint8)
    d.pack_host(count, src.ctypes.data + origin, 0, packed.ctypes.data, total)
    d.unpack_host(count, dst.ctypes.data + origin, 0, packed.ctypes.data, total)
    assert np.array_equal(dst, expected_copy(t, count, src, origin))
    od = c_oracle(oracle, t)
    want = np.zeros(total, dtype=np.uint8)
    assert oracle.oracle_ddt_pack(od, count, src.ctypes.data + origin, 0, want.ctypes.data, total) == 0
    assert np.array_equal(packed, want)
    # and in arbitrary windows (the convertor's fragments): 956-byte chunks as ddt_test.c:353
    dst2 = np.zeros(n, dtype=np.uint8)
    for pos in range(0, total, 956):
        sz = min(956, total - pos)
        d.unpack_host(count, dst2.ctypes.data + origin, pos, packed.ctypes.data + pos, sz)
    assert np.array_equal(dst2, dst)
    oracle.oracle_ddt_free(od)
    d.destroy()


def test_zero_count_contiguous_types(pkg, oracle):
    """ddt_test.c:401-411: types grown from contiguous(0, MPI_DATATYPE_NULL) by ompi_datatype_add --
    sizes / extents by opal_datatype_add's rules (long double's 16-byte alignment pads pdt1's extent
    to 80), compiled by the engine to the same layout, packed like the oracle"""
    p1, p2, p3 = ot.ddt_test_zero_count_types()
    assert [(t.size, t.extent) for t in (p1, p2, p3)] == [(72, 80), (184, 184), (60, 60)]
    for t in (p1, p2, p3):
        d = _compiled(pkg, t)
        assert (d.size, d.extent) == (t.size, t.extent)
        n, origin = span_of(t, 3)
        src = fill_pattern(n)
        got = np.zeros(3 * t.size, dtype=np.uint8)
        d.pack_host(3, src.ctypes.data + origin, 0, got.ctypes.data, got.size)
        od = c_oracle(oracle, t)
        want = np.zeros_like(got)
        assert oracle.oracle_ddt_pack(od, 3, src.ctypes.data + origin, 0, want.ctypes.data, want.size) == 0
        assert np.array_equal(got, want)
        oracle.oracle_ddt_free(od)
        d.destroy()
