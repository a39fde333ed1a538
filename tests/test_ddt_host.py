"""GPU-convertor datatype layouts built on the host (no GPU): sizes/extents agree with the oracle's
restatement of the MPI constructors, and an opal description (opt_desc records, restated from
opal_datatype_internal.h:148-188) compiles to the same layout as the constructor."""
from __future__ import annotations

import ctypes

import pytest

from ddtcases import rec_elem, rec_end, rec_loop


@pytest.mark.parametrize("count,blocklen,stride,elem", [(4, 64, 128, 4), (150, 1, 2, 4), (7, 3, 3, 8), (1, 5, 9, 2),
                                                        (1 << 22, 64, 128, 4)])
def test_vector_matches_oracle(pkg, oracle, count, blocklen, stride, elem):
    d = pkg.Ddt.vector(count, blocklen, stride, elem)
    od = oracle.oracle_ddt_vector(count, blocklen, stride, elem)
    assert d.size == oracle.oracle_ddt_size(od)
    assert d.extent == oracle.oracle_ddt_extent(od)
    assert d.nruns == 1
    d.destroy()


def test_indexed_merges_adjacent(pkg, oracle):
    bl, dp = [2, 3, 1, 4], [0, 2, 10, 11]
    d = pkg.Ddt.indexed(bl, dp, 8)
    od = oracle.oracle_ddt_indexed(4, (ctypes.c_int * 4)(*bl), (ctypes.c_int * 4)(*dp), 8)
    assert d.size == oracle.oracle_ddt_size(od) and d.extent == oracle.oracle_ddt_extent(od)
    assert d.nruns == 2


def test_from_opal_vector_description(pkg):
    """'LOOP n x {UINT1 count 256} extent 512' -- the optimized description of
    vector(n, 64, 128, MPI_FLOAT)"""
    n = 4
    desc = rec_loop(n, 2, 512) + rec_elem(9, 256, 1, 0) + rec_end(2, 256, 0)
    sizes = [0] * 32
    sizes[9] = 1  # OPAL_DATATYPE_UINT1
    d = pkg.Ddt.from_opal(desc, 3, (n - 1) * 512 + 256, sizes)
    assert d.size == n * 256 and d.nruns == 1
    # a strided element (extent != size) unrolls into one run per element
    desc2 = rec_elem(6, 5, 8, 4)  # INT4 x5 every 8 bytes starting at 4
    sizes[6] = 4
    d2 = pkg.Ddt.from_opal(desc2, 1, 40, sizes)
    assert d2.size == 20 and d2.nruns == 5
