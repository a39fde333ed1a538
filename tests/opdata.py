"""Adversarial inputs and comparison rules for the op/hip parity tests.

Inputs per element type (numpy, host memory, x86-64 C layouts):
  * integers: full-range random bits (exercise two's-complement wrap of SUM/PROD), plus the
    extremes INT_MIN/INT_MAX/-1/0/1 at the head;
  * float/double: N(0,1) with injected specials at 1/16 density -- quiet NaN (two payloads),
    +-Inf, +-0, +-denormals, +-max -- so MAX/MIN operand order, NaN propagation and denormal
    handling are all exercised;
  * complex: the same per component (PROD then reaches the C99 Annex G recovery branches);
  * bool: 0/1 bytes (C _Bool values); byte: random;
  * MAXLOC pairs: values drawn from a small set so ~1/4 of the pairs tie, random indices.
Comparison (`assert_same`): bit-exact for everything, with two documented relaxations:
  * SUM/PROD on float/double/complex: an element where both results are NaN matches whatever
    the NaN payloads (x86 SSE and CDNA propagate different payloads; MPI defines none);
  * pair types: only the `v` and `k` members are compared (3-buff never writes the padding in
    the reference, op_base_functions.c:661-683).
"""
from __future__ import annotations

import numpy as np

SEED = 0x5EED

_INT = {"INT8": np.int8, "UINT8": np.uint8, "INT16": np.int16, "UINT16": np.uint16,
        "INT32": np.int32, "UINT32": np.uint32, "INT64": np.int64, "UINT64": np.uint64}
_FP = {"FLOAT": np.float32, "DOUBLE": np.float64, "LONG_DOUBLE": np.longdouble}
_CPLX = {"C_FLOAT_COMPLEX": np.complex64, "C_DOUBLE_COMPLEX": np.complex128,
         "C_LONG_DOUBLE_COMPLEX": np.clongdouble}
_PAIR = {
    "FLOAT_INT": np.dtype([("v", "<f4"), ("k", "<i4")], align=True),
    "DOUBLE_INT": np.dtype([("v", "<f8"), ("k", "<i4")], align=True),
    "LONG_INT": np.dtype([("v", "<i8"), ("k", "<i4")], align=True),
    "2INT": np.dtype([("v", "<i4"), ("k", "<i4")], align=True),
    "SHORT_INT": np.dtype([("v", "<i2"), ("k", "<i4")], align=True),
    "LONG_DOUBLE_INT": np.dtype([("v", np.longdouble), ("k", "<i4")], align=True),
}

FLOAT_OPS = {"SUM", "PROD"}


def dtype_of(tname: str) -> np.dtype:
    if tname in _INT:
        return np.dtype(_INT[tname])
    if tname in _FP:
        return np.dtype(_FP[tname])
    if tname in _CPLX:
        return np.dtype(_CPLX[tname])
    if tname in _PAIR:
        return _PAIR[tname]
    if tname == "BOOL":
        return np.dtype(np.uint8)
    if tname == "BYTE":
        return np.dtype(np.int8)
    raise KeyError(tname)


def _fp_values(rng, n, dt):
    x = rng.standard_normal(n).astype(dt)
    fi = np.finfo(dt)
    specials = np.array([np.nan, -np.nan, np.inf, -np.inf, 0.0, -0.0, fi.tiny / 4, -fi.tiny / 4,
                         fi.max, -fi.max, 1.0, -1.0], dtype=dt)
    mask = rng.random(n) < 1.0 / 16
    x[mask] = rng.choice(specials, int(mask.sum()))
    # a second NaN payload
    if dt in (np.float32, np.float64):
        bits = x.view(np.uint32 if dt == np.float32 else np.uint64)
        pay = rng.random(n) < 1.0 / 64
        bits[pay] = np.uint32(0x7FC00123) if dt == np.float32 else np.uint64(0x7FF8000000000123)
    return x


def make(tname: str, n: int, salt: int = 0) -> np.ndarray:
    rng = np.random.default_rng(SEED + salt * 7919 + sum(tname.encode()))
    dt = dtype_of(tname)
    if tname in _INT or tname == "BYTE":
        raw = rng.integers(0, 256, size=n * dt.itemsize, dtype=np.uint8)
        x = raw.view(dt).copy()
        info = np.iinfo(dt)
        head = np.array([info.min, info.max, -1 if info.min < 0 else 0, 0, 1], dtype=dt)
        m = min(n, len(head))
        x[:m] = np.roll(head, salt)[:m]
        return x
    if tname == "BOOL":
        return rng.integers(0, 2, size=n, dtype=np.uint8)
    if tname in _FP:
        return _fp_values(rng, n, _FP[tname])
    if tname in _CPLX:
        base = np.float32 if tname == "C_FLOAT_COMPLEX" else (np.float64 if tname == "C_DOUBLE_COMPLEX" else np.longdouble)
        x = np.empty(n, dtype=dt)
        x.real = _fp_values(rng, n, base)
        x.imag = _fp_values(rng, n, base)
        return x
    if tname in _PAIR:
        x = np.zeros(n, dtype=dt)
        vals = np.array([-2, -1, 0, 1, 2, 3, 5, 7], dtype=dt["v"])
        x["v"] = rng.choice(vals, n)
        if dt["v"].kind == "f":
            sp = rng.random(n) < 1.0 / 32
            x["v"][sp] = np.array([np.nan, -0.0], dtype=dt["v"])[rng.integers(0, 2, int(sp.sum()))]
        x["k"] = rng.integers(-1000, 1000, n, dtype=np.int32)
        return x
    raise KeyError(tname)


def _bytes_equal(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    a = np.ascontiguousarray(a)
    b = np.ascontiguousarray(b)
    nb = 10 if a.dtype == np.longdouble else a.dtype.itemsize  # x87: 10 significant bytes
    isz = a.dtype.itemsize
    return (a.view(np.uint8).reshape(len(a), isz)[:, :nb] == b.view(np.uint8).reshape(len(b), isz)[:, :nb]).all(1)


def _nan_equal_fp(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    return _bytes_equal(a, b) | (np.isnan(a) & np.isnan(b))


def mismatches(tname: str, opname: str, got: np.ndarray, want: np.ndarray) -> np.ndarray:
    """indices where got != want under the comparison rules above"""
    if tname in _PAIR:
        gv = np.ascontiguousarray(got["v"])
        wv = np.ascontiguousarray(want["v"])
        nb = 10 if gv.dtype == np.longdouble else gv.dtype.itemsize  # x87: 10 significant bytes
        ok = (got["k"] == want["k"]) & (
            gv.view(np.uint8).reshape(len(gv), gv.dtype.itemsize)[:, :nb]
            == wv.view(np.uint8).reshape(len(wv), wv.dtype.itemsize)[:, :nb]).all(1)
        return np.nonzero(~ok)[0]
    if opname in FLOAT_OPS and tname in _FP:
        return np.nonzero(~_nan_equal_fp(got, want))[0]
    if opname in FLOAT_OPS and tname in _CPLX:
        ok = _nan_equal_fp(got.real.copy(), want.real.copy()) & _nan_equal_fp(got.imag.copy(), want.imag.copy())
        return np.nonzero(~ok)[0]
    if tname in _CPLX:
        ok = _bytes_equal(got.real.copy(), want.real.copy()) & _bytes_equal(got.imag.copy(), want.imag.copy())
        return np.nonzero(~ok)[0]
    return np.nonzero(~_bytes_equal(got, want))[0]


def assert_same(tname: str, opname: str, got: np.ndarray, want: np.ndarray, what: str = "") -> None:
    bad = mismatches(tname, opname, got, want)
    if len(bad):
        i = int(bad[0])
        raise AssertionError(f"{what} {opname}/{tname}: {len(bad)} mismatches, first at {i}: "
                             f"got {got[i]!r} want {want[i]!r}")
