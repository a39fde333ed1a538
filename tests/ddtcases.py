"""Datatype cases shared by the CPU (oracle) and GPU convertor tests, restated from the
reference's own known-answer tests in test/datatype/."""
from __future__ import annotations

import ctypes

import numpy as np


def segments(oracle, od, count, fragment):
    """create_segments() of test/datatype/position.c:43-90: fragment-sized windows whose ends are
    moved back to element boundaries by opal_convertor_set_position; one more segment until the
    windows cover the message."""
    total = count * oracle.oracle_ddt_size(od)
    nseg = total // fragment + (1 if total % fragment else 0)
    while True:
        segs, pos, cover = [], 0, 0
        for _ in range(nseg):
            start = pos
            pos = oracle.oracle_ddt_round_position(od, count, min(pos + fragment, total))
            segs.append((start, pos - start))
            cover += pos - start
        if cover == total:
            return segs
        nseg += 1


def shuffle(segs):
    """shuffle_segments() of position.c: swap i and n-1-i for even i < n/2"""
    segs = list(segs)
    n = len(segs)
    for i in range(0, n // 2, 2):
        segs[i], segs[n - i - 1] = segs[n - i - 1], segs[i]
    return segs


def ldi_struct(oracle):
    """MPI_LONG_DOUBLE_INT: {long double (16 B) at 0, int at 16}, extent 32"""
    i64 = ctypes.c_int64 * 2
    return oracle.oracle_ddt_struct(2, i64(0, 16), i64(16, 4), i64(16, 4), 32)


LDI = np.dtype([("ld", np.longdouble), ("i", "<i4")], align=True)


# ---- opal description records (dt_elem_desc_t, 32 bytes each; opal_datatype_internal.h:148-188)
import struct  # noqa: E402

OPAL_UINT1, OPAL_INT4, OPAL_FLOAT4 = 9, 6, 15


def rec_loop(loops, items, extent):
    return struct.pack("<HHII4xQq", 0, 0, loops, items, 0, extent)


def rec_elem(typ, count, extent, disp):
    return struct.pack("<HHII4xqq", 0x0100, typ, count, 1, extent, disp)


def rec_end(items, size, first):
    return struct.pack("<HHII4xQq", 0, 1, items, 0, size, first)


def opal_vector(nblk, block_bytes, stride_bytes):
    """optimized description of a vector of byte-granular blocks: LOOP nblk x {UINT1 x block}
    extent stride (what opal_datatype_optimize_short leaves for vector(n, 64, 128, MPI_FLOAT),
    SURVEY.md §0).  Returns (desc, used, size, lb, ub)."""
    desc = rec_loop(nblk, 2, stride_bytes) + rec_elem(OPAL_UINT1, block_bytes, 1, 0) + rec_end(2, block_bytes, 0)
    return desc, 3, nblk * block_bytes, 0, (nblk - 1) * stride_bytes + block_bytes


def opal_strided_elems(n, elem_type, elem_size, stride_bytes, disp=0):
    """one ELEM record of n strided basic elements (extent != size): e.g. vector(n, 1, 2, MPI_FLOAT)"""
    desc = rec_elem(elem_type, n, stride_bytes, disp)
    return desc, 1, n * elem_size, disp, disp + (n - 1) * stride_bytes + elem_size


# ---- the datatype tests of test/datatype/opal_datatype_test.c:338-541, on types restated by
#      oracle/opal_types.py (opal_datatype_add + the test library's constructors)
import pathlib  # noqa: E402
import sys  # noqa: E402

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parent.parent / "oracle"))
import opal_types as ot  # noqa: E402


def _f8():
    return ot.OpalType.basic("FLOAT8")


def _ddt_pack_hindexed():
    return ot.hindexed([10, 10], [0, 20 * 8], _f8()).commit()


# (name, builder, count, chunks): every local_copy_with_convertor(pdt, count, chunk) of main()
CONVERTOR_CASES = [
    ("contig_int1x10", lambda: ot.contiguous(10, ot.OpalType.basic("INT1")).commit(), 100, [956]),   # :350-354
    ("strange", ot.strange_dt, 1, [956]),                                                          # :358-362
    ("upper_matrix_100", lambda: ot.upper_matrix(100), 1, [48]),                                   # :367-371
    ("float8", _f8, 4500, [12]),                                                                   # :433-436
    ("contig_f8_4500", lambda: ot.contiguous(4500, _f8()).commit(), 1, [12]),                      # :443-447
    ("contig_f8_450", lambda: ot.contiguous(450, _f8()).commit(), 10, [12]),
    ("contig_f8_45", lambda: ot.contiguous(45, _f8()).commit(), 100, [12]),
    ("contig_f8_100", lambda: ot.contiguous(100, _f8()).commit(), 45, [12]),
    ("contig_f8_10", lambda: ot.contiguous(10, _f8()).commit(), 450, [12]),
    ("contig_f8_1", lambda: ot.contiguous(1, _f8()).commit(), 4500, [12]),
    ("vector_450_10_11", lambda: ot.vector(450, 10, 11, _f8()).commit(), 1, [12, 82, 6000, 36000]),  # :482-493
    ("struct_char_double", ot.struct_char_double, 4500, [12]),                                     # :499-503
    ("twice_two_doubles", ot.twice_two_doubles, 4500, [12]),                                       # :509-513
    ("blacs", ot.blacs, 4500, [956, 16 * 1024, 64 * 1024]),                                        # :519-528
    ("typeub_hindexed", lambda: ot.typeub3()[0], 7, [5]),  # the LB/UB types moved as data too
    ("typeub_indexed", lambda: ot.typeub3()[1], 7, [6]),
    ("typeub_vector", lambda: ot.typeub3()[3], 5, [4]),
    ("test_struct", ot.test_struct, 33, [7]),
    # test/datatype/ddt_pack.c:70-101: hindexed(2, {10, 10}, {0, 20 * sizeof(double)}, MPI_DOUBLE)
    # and struct {11 x MPI_INT at 0, 2 x that hindexed at 64} -- the types whose descriptions it
    # packs, moved here as data
    ("ddt_pack_hindexed", lambda: _ddt_pack_hindexed(), 7, [12, 100, 956]),
    ("ddt_pack_struct", lambda: ot.struct_([11, 2], [0, 64], [ot.OpalType.basic("INT4"), _ddt_pack_hindexed()]).commit(),
     5, [12, 100, 956]),
]


def windows(oracle, od, count, chunk):
    """the successive (pos, size) of a convertor driven with `chunk`-byte iovecs: each stops at the
    last basic-element boundary that fits (opal_generic_simple_pack packs whole elements)"""
    total = count * oracle.oracle_ddt_size(od)
    pos, out = 0, []
    while pos < total:
        nxt = oracle.oracle_ddt_round_position(od, count, min(pos + chunk, total))
        if nxt <= pos:  # an element larger than the chunk: split it (contiguous fast path)
            nxt = min(pos + chunk, total)
        out.append((pos, nxt - pos))
        pos = nxt
    return out


def c_oracle(oracle, t):
    """the byte-level oracle (oracle/ddt_oracle.c) of a restated type: its merged runs + extent"""
    runs = t.runs()
    n = len(runs)
    a = ctypes.c_int64 * n
    return oracle.oracle_ddt_struct(n, a(*[r[0] for r in runs]), a(*[r[1] for r in runs]), a(*[r[2] for r in runs]),
                                    t.extent)


def span_of(t, count):
    """(bytes, origin): a buffer holding `count` instances whose first instance starts at origin"""
    lo = min(0, t.true_lb, t.lb)
    hi = max((count - 1) * t.extent + t.true_ub, (count - 1) * t.extent + t.ub)
    return hi - lo, -lo


def fill_pattern(n):
    """psrc[i] = i % 128 + 32 (opal_datatype_test.c:269-272)"""
    return (np.arange(n) % 128 + 32).astype(np.uint8)


def expected_copy(t, count, src, origin):
    """what a send/recv convertor pair leaves in a zeroed destination: the type map's bytes"""
    one = np.concatenate([np.arange(d, d + n) for d, n, _ in t.runs()])
    idx = (origin + np.arange(count, dtype=np.int64)[:, None] * t.extent + one[None, :]).reshape(-1)
    want = np.zeros_like(src)
    want[idx] = src[idx]
    return want


RAW_CASES = [  # ddt_raw.c:150-177 (local_copy_ddt_raw with iov_num = 5) and test_upper(500) (:45-80)
    ("inversed_vector_int_10", lambda: ot.inversed_vector(10), 100),
    ("strange_dt", ot.strange_dt, 1),
    ("upper_matrix_100", lambda: ot.upper_matrix(100), 1),
    ("upper_matrix_500", lambda: ot.upper_matrix(500), 1),
    ("mpi_double", lambda: ot.OpalType.basic("FLOAT8"), 4500),                              # :232-235
    ("contig_4500x1", lambda: ot.contiguous(4500, ot.OpalType.basic("FLOAT8")).commit(), 1),  # :238-263
    ("contig_450x10", lambda: ot.contiguous(450, ot.OpalType.basic("FLOAT8")).commit(), 10),
    ("contig_45x100", lambda: ot.contiguous(45, ot.OpalType.basic("FLOAT8")).commit(), 100),
    ("contig_100x45", lambda: ot.contiguous(100, ot.OpalType.basic("FLOAT8")).commit(), 45),
    ("contig_10x450", lambda: ot.contiguous(10, ot.OpalType.basic("FLOAT8")).commit(), 450),
    ("contig_1x4500", lambda: ot.contiguous(1, ot.OpalType.basic("FLOAT8")).commit(), 4500),
    ("vector_450_10_11", lambda: ot.vector(450, 10, 11, ot.OpalType.basic("FLOAT8")).commit(), 1),  # :268-277
    ("struct_char_double", ot.struct_char_double, 4500),                                    # :279-285
    ("twice_two_doubles", ot.twice_two_doubles, 4500),                                      # :287-293
    ("blacs", ot.blacs, 4500),                                                              # :295-304
    ("blacs1_int", ot.blacs1, 1),                                                           # :306-311
    ("ddt_test_pdt1", lambda: ot.ddt_test_zero_count_types()[0], 1),
]


COPY_CASES = [  # ddt_test.c:350-372, 433-524: local_copy_ddt_count(pdt, count)
    ("inversed_vector_int_10", lambda: ot.inversed_vector(10), 100),
    ("strange_dt", ot.strange_dt, 1),
    ("upper_matrix_100", lambda: ot.upper_matrix(100), 1),
    ("mpi_double", lambda: ot.OpalType.basic("FLOAT8"), 4500),
    ("contig_4500x1", lambda: ot.contiguous(4500, ot.OpalType.basic("FLOAT8")).commit(), 1),  # :442-477
    ("contig_450x10", lambda: ot.contiguous(450, ot.OpalType.basic("FLOAT8")).commit(), 10),
    ("contig_45x100", lambda: ot.contiguous(45, ot.OpalType.basic("FLOAT8")).commit(), 100),
    ("contig_100x45", lambda: ot.contiguous(100, ot.OpalType.basic("FLOAT8")).commit(), 45),
    ("contig_10x450", lambda: ot.contiguous(10, ot.OpalType.basic("FLOAT8")).commit(), 450),
    ("contig_1x4500", lambda: ot.contiguous(1, ot.OpalType.basic("FLOAT8")).commit(), 4500),
    ("vector_450_10_11", lambda: ot.vector(450, 10, 11, ot.OpalType.basic("FLOAT8")).commit(), 1),  # :482-486
    ("struct_char_double", ot.struct_char_double, 4500),                                    # :498-505
    ("twice_two_doubles", ot.twice_two_doubles, 4500),                                      # :508-515
    ("blacs_2", ot.blacs, 2),                                                               # :518-524
    ("blacs_4500", ot.blacs, 4500),
]
