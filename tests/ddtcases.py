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
