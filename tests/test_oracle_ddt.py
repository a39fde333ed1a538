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
