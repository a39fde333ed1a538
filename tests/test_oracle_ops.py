"""CPU tests of the op oracle (test infrastructure) against known answers.

The known answers in tests/golden/op_specials.json were recorded from the reference's own
compiled op loops during the survey (SURVEY.md §0, row "Special-value semantics of the compiled
reference ops"); the rest follow directly from the C expressions of op_base_functions.c.
"""
from __future__ import annotations

import json
import pathlib
import struct

import numpy as np
import pytest

import opdata

GOLD = pathlib.Path(__file__).parent / "golden" / "op_specials.json"


def _run2(oracle, pkg, op, ty, out_vals, in_vals, dt):
    o = np.array(out_vals, dtype=dt)
    i = np.array(in_vals, dtype=dt)
    assert oracle.oracle_op_2buff(pkg.OP[op], pkg.T[ty], i.ctypes.data, o.ctypes.data, len(o)) == 0
    return o


def _run3(oracle, pkg, op, ty, a_vals, b_vals, dt):
    a = np.array(a_vals, dtype=dt)
    b = np.array(b_vals, dtype=dt)
    o = np.zeros_like(a)
    assert oracle.oracle_op_3buff(pkg.OP[op], pkg.T[ty], a.ctypes.data, b.ctypes.data, o.ctypes.data, len(a)) == 0
    return o


def _bits(x):
    return [struct.pack("<d", float(v)).hex() for v in x]


def test_slot_count(oracle, pkg):
    """116 non-NULL (op,type) slots with Fortran disabled (op_base_functions.c:1373-1543)"""
    n = sum(oracle.oracle_has_op(op, ty) for op in range(15) for ty in range(39))
    assert n == 116


def test_golden_specials(oracle, pkg):
    cases = json.loads(GOLD.read_text())["cases"]
    assert len(cases) >= 10
    for c in cases:
        dt = {"FLOAT": np.float32, "DOUBLE": np.float64, "INT8": np.int8, "INT32": np.int32}[c["type"]]
        vals = [float.fromhex(v) if isinstance(v, str) else v for v in c["args"]]
        if c["form"] == "2buff":
            got = _run2(oracle, pkg, c["op"], c["type"], [vals[0]], [vals[1]], dt)[0]
        else:
            got = _run3(oracle, pkg, c["op"], c["type"], [vals[0]], [vals[1]], dt)[0]
        want = c["want"]
        if want == "nan":
            assert np.isnan(got), c
        elif isinstance(want, str):
            w = float.fromhex(want)
            assert got == w and np.signbit(got) == np.signbit(w), (c, got)
        else:
            assert got == want, (c, got)


def test_maxloc_tie_asymmetry(oracle, pkg):
    """2-buff keeps out.v on ties, 3-buff takes in1.v (op_base_functions.c:96-101 vs :672-681)"""
    dt = opdata.dtype_of("FLOAT_INT")
    out = np.array([(-0.0, 5)], dtype=dt)
    inn = np.array([(0.0, 3)], dtype=dt)
    assert oracle.oracle_op_2buff(pkg.OP["MAXLOC"], pkg.T["FLOAT_INT"], inn.ctypes.data, out.ctypes.data, 1) == 0
    assert np.signbit(out["v"][0]) and out["k"][0] == 3
    a = np.array([(0.0, 7)], dtype=dt)
    b = np.array([(-0.0, 2)], dtype=dt)
    o = np.zeros(1, dtype=dt)
    assert oracle.oracle_op_3buff(pkg.OP["MAXLOC"], pkg.T["FLOAT_INT"], a.ctypes.data, b.ctypes.data, o.ctypes.data, 1) == 0
    assert not np.signbit(o["v"][0]) and o["k"][0] == 2


@pytest.mark.parametrize("tname", ["INT8", "UINT16", "INT32", "INT64", "FLOAT", "DOUBLE"])
def test_sum_prod_match_numpy(oracle, pkg, tname):
    """integer SUM/PROD wrap like two's complement (numpy wraps identically); fp matches IEEE"""
    a = opdata.make(tname, 4096, 5)
    b = opdata.make(tname, 4096, 6)
    with np.errstate(all="ignore"):
        for op, fn in (("SUM", np.add), ("PROD", np.multiply)):
            got = _run3(oracle, pkg, op, tname, a, b, a.dtype)
            want = fn(a, b).astype(a.dtype)
            opdata.assert_same(tname, op, got, want, "numpy")


def test_complex_prod_annex_g(oracle, pkg):
    """(inf + i nan) * (1 + i0) recovers an infinity (C99 G.5.1 via libgcc __mulsc3)"""
    a = np.array([complex(np.inf, np.nan)], dtype=np.complex64)
    b = np.array([complex(1.0, 0.0)], dtype=np.complex64)
    o = _run3(oracle, pkg, "PROD", "C_FLOAT_COMPLEX", a, b, np.complex64)
    assert np.isinf(o.real[0]) or np.isinf(o.imag[0])


def test_mt_equals_st(oracle, pkg):
    a = opdata.make("DOUBLE", 100_003, 1)
    b = opdata.make("DOUBLE", 100_003, 2)
    o1 = np.zeros_like(a)
    o2 = np.zeros_like(a)
    oracle.oracle_op_3buff(pkg.OP["SUM"], pkg.T["DOUBLE"], a.ctypes.data, b.ctypes.data, o1.ctypes.data, len(a))
    oracle.oracle_op_3buff_mt(pkg.OP["SUM"], pkg.T["DOUBLE"], a.ctypes.data, b.ctypes.data, o2.ctypes.data, len(a), 4)
    assert o1.tobytes() == o2.tobytes()


def test_comparator_every_slot(oracle, pkg):
    """the GPU-test comparator accepts identical results for every slot (guards the test itself)"""
    for op in range(1, 13):
        for ty in range(39):
            if not oracle.oracle_has_op(op, ty):
                continue
            tname, opname = pkg.TYPES[ty], pkg.OPS[op]
            a = opdata.make(tname, 257, 1)
            b = opdata.make(tname, 257, 2)
            o1 = np.zeros_like(a)
            o2 = np.zeros_like(a)
            with np.errstate(all="ignore"):
                oracle.oracle_op_3buff(op, ty, a.ctypes.data, b.ctypes.data, o1.ctypes.data, 257)
                oracle.oracle_op_3buff(op, ty, a.ctypes.data, b.ctypes.data, o2.ctypes.data, 257)
            opdata.assert_same(tname, opname, o1, o2, "self")
            c = b.copy()
            oracle.oracle_op_2buff(op, ty, a.ctypes.data, c.ctypes.data, 257)
            assert len(opdata.mismatches(tname, opname, c, c.copy())) == 0
