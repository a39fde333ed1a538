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
