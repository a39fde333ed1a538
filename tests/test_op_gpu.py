"""op/hip kernels (libmi355x_rt.so, C ABI) vs the CPU oracle: every (op, type) slot, 2-buff and
3-buff, aligned / co-misaligned / mutually misaligned operands, odd sizes, empty input.

Reference semantics: ompi/mca/op/base/op_base_functions.c:39-103 (2-buff), :606-683 (3-buff).
Bar: bit-exact (opdata.assert_same documents the two relaxations: NaN payloads of float
SUM/PROD, padding bytes of MAXLOC pairs).
"""
from __future__ import annotations

import ctypes

import numpy as np
import pytest

import opdata

pytestmark = pytest.mark.gpu

N = 50_021  # odd: exercises head/tail handling around the 16-B vector body


def _slots(pkg, oracle):
    out = []
    for op in range(1, 13):
        for ty in range(len(pkg.TYPES)):
            if oracle.oracle_has_op(op, ty) and pkg.op_supported(op, ty):
                out.append((pkg.OPS[op], pkg.TYPES[ty]))
    return out


def _dev(torch, arr: np.ndarray, off_bytes: int = 0):
    raw = arr.view(np.uint8).reshape(-1)
    t = torch.zeros(raw.size + 64, dtype=torch.uint8, device="cuda")
    t[off_bytes:off_bytes + raw.size].copy_(torch.from_numpy(raw.copy()))
    return t, t.data_ptr() + off_bytes


def _host(t, off_bytes, like: np.ndarray) -> np.ndarray:
    nb = like.view(np.uint8).size
    return t[off_bytes:off_bytes + nb].cpu().numpy().view(like.dtype).copy()


def test_slot_coverage(gpu, pkg, oracle):
    """every reference slot has a GPU kernel (116 of 116): the x87 long double slots too -- MAX/MIN
    and MAXLOC/MINLOC compare and select on the 80-bit encoding, SUM/PROD (real and complex) run the
    x87 add / multiply restated in integer arithmetic (f80_arith.hpp)"""
    have, missing = 0, []
    for op in range(15):
        for ty in range(len(pkg.TYPES)):
            if oracle.oracle_has_op(op, ty):
                if pkg.op_supported(op, ty):
                    have += 1
                else:
                    missing.append((pkg.OPS[op], pkg.TYPES[ty]))
    assert not missing, missing
    assert have == 116


def _x87(m, se):
    """an 80-bit x87 value in 16 bytes of storage (padding bytes set to 0xA5: never compared)"""
    b = bytearray(16)
    b[0:8] = int(m).to_bytes(8, "little")
    b[8:10] = int(se).to_bytes(2, "little")
    b[10:16] = b"\xa5" * 6
    return bytes(b)


def x87_adversarial():
    """every class of the 80-bit encoding, both signs: zeros, denormals, pseudo-denormals (equal to
    the normal of the same significand), normals, the largest finite, infinities, quiet and
    signalling NaNs, and the invalid operands of the 387 -- pseudo-NaN / pseudo-infinity and
    unnormals (integer bit clear), which compare unordered"""
    I = 1 << 63
    vals = [(0, 0), (1, 0), (0x7FFFFFFFFFFFFFFF, 0), (I, 0), (I | 5, 0), (I, 1), (I | 5, 1), (I, 0x3FFF),
            (I | 1, 0x3FFF), (I | (1 << 62), 0x3FFF), (0xFFFFFFFFFFFFFFFF, 0x7FFE), (I, 0x7FFF),
            (I | (1 << 62), 0x7FFF), (I | 1, 0x7FFF), (1 << 62, 0x7FFF), (0, 0x7FFF), (5, 0x3FFF), (0, 0x4000)]
    out = []
    for mant, exp in vals:
        for sign in (0, 0x8000):
            out.append(_x87(mant, exp | sign))
    return out


@pytest.mark.parametrize("tname", ["LONG_DOUBLE", "LONG_DOUBLE_INT"])
def test_x87_compare_slots(gpu, pkg, oracle, tname):
    """MAX/MIN (LONG_DOUBLE) and MAXLOC/MINLOC (LONG_DOUBLE_INT) on the GPU against the oracle's C
    loops, which run on this host's x87 unit (op_base_functions.c:110, :170, :576, :598): every
    ordered pair of the adversarial encodings, 2-buff and 3-buff, bit-exact in the 10 value bytes"""
    torch = gpu
    enc = x87_adversarial()
    pairs = [(x, y) for x in enc for y in enc]
    dt = opdata.dtype_of(tname)
    a = np.zeros(len(pairs), dtype=dt)
    b = np.zeros(len(pairs), dtype=dt)
    av = a.view(np.uint8).reshape(len(pairs), dt.itemsize)
    bv = b.view(np.uint8).reshape(len(pairs), dt.itemsize)
    for i, (x, y) in enumerate(pairs):
        av[i, :16] = np.frombuffer(x, np.uint8)
        bv[i, :16] = np.frombuffer(y, np.uint8)
    if tname == "LONG_DOUBLE_INT":
        a["k"] = np.arange(len(pairs)) % 7
        b["k"] = np.arange(len(pairs)) % 5
    ops = ("MAX", "MIN") if tname == "LONG_DOUBLE" else ("MAXLOC", "MINLOC")
    s = torch.cuda.current_stream().cuda_stream
    for opname in ops:
        op, ty = pkg.OP[opname], pkg.T[tname]
        assert pkg.op_supported(op, ty)
        ta, pa = _dev(torch, a)
        tb, pb = _dev(torch, b)
        to, po = _dev(torch, np.zeros_like(a))
        pkg.op_reduce_3buff(op, ty, pa, pb, po, len(pairs), s)
        pkg.op_reduce(op, ty, pa, pb, len(pairs), s)
        torch.cuda.synchronize()
        want3 = np.zeros_like(a)
        assert oracle.oracle_op_3buff(op, ty, a.ctypes.data, b.ctypes.data, want3.ctypes.data, len(pairs)) == 0
        want2 = b.copy()
        assert oracle.oracle_op_2buff(op, ty, a.ctypes.data, want2.ctypes.data, len(pairs)) == 0
        opdata.assert_same(tname, opname, _host(to, 0, a), want3, "x87 3buff")
        opdata.assert_same(tname, opname, _host(tb, 0, a), want2, "x87 2buff")


def _x87_random(n, seed):
    """n random 80-bit values over the whole exponent range (normals, denormals, values near
    overflow and underflow), both signs, in 16 bytes of storage"""
    rng = np.random.default_rng(seed)
    out = np.zeros((n, 16), dtype=np.uint8)
    m = rng.integers(0, 2**63, n, dtype=np.uint64) | (np.uint64(1) << np.uint64(63))
    mode = rng.integers(0, 4, n)
    e = np.where(mode == 0, rng.integers(0, 0x7fff, n), np.where(mode == 1, rng.integers(0, 140, n),
                 np.where(mode == 2, 0x7ffe - rng.integers(0, 140, n), 0x3fff + rng.integers(-65, 65, n))))
    m = np.where(e == 0, m & np.uint64(2**63 - 1), m)
    se = (e | (rng.integers(0, 2, n) << 15)).astype(np.uint16)
    out[:, :8] = m.view(np.uint8).reshape(n, 8)
    out[:, 8:10] = se.view(np.uint8).reshape(n, 2)
    return out


@pytest.mark.parametrize("tname", ["LONG_DOUBLE", "C_LONG_DOUBLE_COMPLEX"])
def test_x87_arith_slots(gpu, pkg, oracle, tname):
    """SUM / PROD on x87 long double (real and complex) on the GPU against the oracle's C loops,
    which run on this host's x87 unit (op_base_functions.c:110-170; complex PROD through GCC's
    inline multiply + libgcc __mulxc3): every ordered pair of the adversarial encodings (NaNs of
    equal significands and both signs, invalid encodings, infinities, denormals) and 200k random
    pairs over the whole exponent range (complex: also every combination of 11 specials in the four
    parts), 2-buff and 3-buff, bit-exact in the 10 value bytes"""
    torch = gpu
    enc = [np.frombuffer(x, np.uint8) for x in x87_adversarial()]
    pairs = np.array([(x, y) for x in enc for y in enc], dtype=np.uint8)   # (P, 2, 16)
    ra, rb = _x87_random(200_000, 1), _x87_random(200_000, 2)
    A = np.concatenate([pairs[:, 0], ra])
    B = np.concatenate([pairs[:, 1], rb])
    dt = opdata.dtype_of(tname)
    if tname == "C_LONG_DOUBLE_COMPLEX":  # re from one list, im from the other, both roles
        # plus every (a.re, a.im, b.re, b.im) over a set of specials, so each branch of the Annex G
        # recovery (an infinite operand part, an infinite product, NaN parts) meets every other
        I = 1 << 63
        spec = [np.frombuffer(_x87(m, e), np.uint8) for m, e in
                [(0, 0), (0, 0x8000), (I, 0x3FFF), (I, 0xBFFF), (I, 0x7FFF), (I, 0xFFFF), (I | (1 << 62), 0x7FFF),
                 (I | 1, 0xFFFF), (0xFFFFFFFFFFFFFFFF, 0x7FFE), (5, 0), (5, 0x3FFF)]]
        k = len(spec)
        idx = np.indices((k, k, k, k)).reshape(4, -1)
        S = np.array(spec, dtype=np.uint8)
        n0 = len(A) // 2
        n = n0 + idx.shape[1]
        a = np.zeros(n, dtype=dt)
        b = np.zeros(n, dtype=dt)
        av, bv = a.view(np.uint8).reshape(n, 32), b.view(np.uint8).reshape(n, 32)
        av[:n0, :16], av[:n0, 16:] = A[:n0], B[n0:2 * n0]
        bv[:n0, :16], bv[:n0, 16:] = B[:n0], A[n0:2 * n0]
        av[n0:, :16], av[n0:, 16:], bv[n0:, :16], bv[n0:, 16:] = S[idx[0]], S[idx[1]], S[idx[2]], S[idx[3]]
    else:
        n = len(A)
        a = np.zeros(n, dtype=dt)
        b = np.zeros(n, dtype=dt)
        a.view(np.uint8).reshape(n, 16)[:] = A
        b.view(np.uint8).reshape(n, 16)[:] = B
    s = torch.cuda.current_stream().cuda_stream
    for opname in ("SUM", "PROD"):
        op, ty = pkg.OP[opname], pkg.T[tname]
        assert pkg.op_supported(op, ty)
        ta, pa = _dev(torch, a)
        tb, pb = _dev(torch, b)
        to, po = _dev(torch, np.zeros_like(a))
        pkg.op_reduce_3buff(op, ty, pa, pb, po, n, s)
        pkg.op_reduce(op, ty, pa, pb, n, s)
        torch.cuda.synchronize()
        want3 = np.zeros_like(a)
        assert oracle.oracle_op_3buff(op, ty, a.ctypes.data, b.ctypes.data, want3.ctypes.data, n) == 0
        want2 = b.copy()
        assert oracle.oracle_op_2buff(op, ty, a.ctypes.data, want2.ctypes.data, n) == 0
        nb = 10
        for got, want, form in ((_host(to, 0, a), want3, "3buff"), (_host(tb, 0, a), want2, "2buff")):
            g = got.view(np.uint8).reshape(n, -1)
            w = want.view(np.uint8).reshape(n, -1)
            cols = list(range(nb)) + ([16 + i for i in range(nb)] if tname == "C_LONG_DOUBLE_COMPLEX" else [])
            bad = np.nonzero((g[:, cols] != w[:, cols]).any(1))[0]
            assert len(bad) == 0, (f"{opname} {form}: {len(bad)} of {n} differ; first", bad[:4].tolist(),
                                   g[bad[:2]].tolist(), w[bad[:2]].tolist())


@pytest.mark.parametrize("offs", [(0, 0, 0), (1, 1, 1), (1, 0, 2)], ids=["aligned", "comisaligned", "misaligned"])
def test_all_slots(gpu, pkg, oracle, offs):
    torch = gpu
    bad = []
    for opname, tname in _slots(pkg, oracle):
        op, ty = pkg.OP[opname], pkg.T[tname]
        esz = pkg.type_size(ty)
        assert esz == oracle.oracle_type_size(ty)
        a = opdata.make(tname, N, 1)
        b = opdata.make(tname, N, 2)
        o1, o2, o3 = (x * esz for x in offs)
        # 3-buff
        ta, pa = _dev(torch, a, o1)
        tb, pb = _dev(torch, b, o2)
        to, po = _dev(torch, np.zeros_like(a), o3)
        pkg.op_reduce_3buff(op, ty, pa, pb, po, N, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        want = np.zeros_like(a)
        assert oracle.oracle_op_3buff(op, ty, a.ctypes.data, b.ctypes.data, want.ctypes.data, N) == 0
        try:
            opdata.assert_same(tname, opname, _host(to, o3, want), want, "3buff")
        except AssertionError as e:
            bad.append(str(e))
        # 2-buff: inout = b, in = a
        tio, pio = _dev(torch, b, o2)
        pkg.op_reduce(op, ty, pa, pio, N, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        want2 = b.copy()
        assert oracle.oracle_op_2buff(op, ty, a.ctypes.data, want2.ctypes.data, N) == 0
        try:
            opdata.assert_same(tname, opname, _host(tio, o2, want2), want2, "2buff")
        except AssertionError as e:
            bad.append(str(e))
    assert not bad, "\n".join(bad[:20])


@pytest.mark.parametrize("offs", [(0, 0, 0), (32, 48, 16), (8, 8, 8), (0, 8, 0)],
                         ids=["halves", "halves_offset", "wide_8", "wide_mixed"])
@pytest.mark.parametrize("n", [1, 2, 3, 1023, 1024, 1025, 50_021])
def test_long_double_int_kernels(gpu, pkg, oracle, offs, n):
    """the two 32-byte kernels: 16-B aligned operands take k_wide_halves (one half per lane, the
    partner's half by a DPP swap), any 8-B misalignment the element-per-lane k_wide; both bit-exact
    vs the oracle (op_base_functions.c:576-598, :661-683), on counts around the 1024-lane block"""
    torch = gpu
    tname = "LONG_DOUBLE_INT"
    for opname in ("MAXLOC", "MINLOC"):
        op, ty = pkg.OP[opname], pkg.T[tname]
        a = opdata.make(tname, n, 5)
        b = opdata.make(tname, n, 6)
        o1, o2, o3 = offs
        ta, pa = _dev(torch, a, o1)
        tb, pb = _dev(torch, b, o2)
        to, po = _dev(torch, np.zeros_like(a), o3)
        s = torch.cuda.current_stream().cuda_stream
        pkg.op_reduce_3buff(op, ty, pa, pb, po, n, s)
        pkg.op_reduce(op, ty, pa, pb, n, s)
        torch.cuda.synchronize()
        want3 = np.zeros_like(a)
        assert oracle.oracle_op_3buff(op, ty, a.ctypes.data, b.ctypes.data, want3.ctypes.data, n) == 0
        want2 = b.copy()
        assert oracle.oracle_op_2buff(op, ty, a.ctypes.data, want2.ctypes.data, n) == 0
        opdata.assert_same(tname, opname, _host(to, o3, a), want3, f"3buff {offs} n={n}")
        opdata.assert_same(tname, opname, _host(tb, o2, a), want2, f"2buff {offs} n={n}")
        # nothing written past the last element
        assert not to[o3 + a.nbytes:].cpu().numpy().any()


def test_small_counts(gpu, pkg, oracle):
    """count = 0, 1, 2, 15, 16, 17 (all of the body empty or one vector)"""
    torch = gpu
    for n in (0, 1, 2, 15, 16, 17, 33):
        for opname, tname in [("SUM", "FLOAT"), ("MAXLOC", "DOUBLE_INT"), ("BXOR", "INT8"), ("PROD", "C_DOUBLE_COMPLEX")]:
            op, ty = pkg.OP[opname], pkg.T[tname]
            a = opdata.make(tname, max(n, 1), 3)[:n]
            b = opdata.make(tname, max(n, 1), 4)[:n]
            ta, pa = _dev(torch, a)
            tb, pb = _dev(torch, b)
            pkg.op_reduce(op, ty, pa, pb, n, torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            want = b.copy()
            oracle.oracle_op_2buff(op, ty, a.ctypes.data, want.ctypes.data, n)
            opdata.assert_same(tname, opname, _host(tb, 0, want), want, f"n={n}")


def test_golden_specials_on_device(gpu, pkg):
    """every case of tests/golden/op_specials.json (outputs of the reference's compiled op loops:
    MAX/MIN NaN and signed-zero operand order, int8/int32 wrap) through the HIP kernels, 2-buff as
    (out, in) and 3-buff as (in1, in2), each case also embedded in a vector body (lane 37 of 4099)
    so the 16-B vector path sees it as well as the scalar path"""
    import json
    import pathlib
    torch = gpu
    cases = json.loads((pathlib.Path(__file__).parent / "golden" / "op_specials.json").read_text())["cases"]
    assert len(cases) >= 10
    dts = {"FLOAT": np.float32, "DOUBLE": np.float64, "INT8": np.int8, "INT32": np.int32}
    stream = torch.cuda.current_stream().cuda_stream
    for c in cases:
        dt = dts[c["type"]]
        op, ty = pkg.OP[c["op"]], pkg.T[c["type"]]
        vals = [float.fromhex(v) if isinstance(v, str) and v != "nan" else (float("nan") if v == "nan" else v)
                for v in c["args"]]
        for n, at in ((1, 0), (4099, 37)):
            first = np.ones(n, dtype=dt)
            second = np.ones(n, dtype=dt)
            first[at], second[at] = vals[0], vals[1]
            t1, p1 = _dev(torch, first)
            t2, p2 = _dev(torch, second)
            if c["form"] == "2buff":   # args = (out, in): inout holds the first
                pkg.op_reduce(op, ty, p2, p1, n, stream)
                torch.cuda.synchronize()
                got = _host(t1, 0, first)[at]
            else:                      # args = (in1, in2)
                to, po = _dev(torch, np.zeros(n, dtype=dt))
                pkg.op_reduce_3buff(op, ty, p1, p2, po, n, stream)
                torch.cuda.synchronize()
                got = _host(to, 0, first)[at]
            want = c["want"]
            if want == "nan":
                assert np.isnan(got), (c, n, got)
            elif isinstance(want, str):
                w = float.fromhex(want)
                assert got == w and np.signbit(got) == np.signbit(w), (c, n, got)
            else:
                assert got == want, (c, n, got)


def test_large_fp32_sum_property(gpu, pkg):
    """1 GiB-class buffer (BASELINE config 2 size): out = in1 + in2 on exactly-representable
    values, checked on device against torch's own add (a size-independent property: the sum of
    small integers is exact in any order)."""
    torch = gpu
    n = 1 << 28  # 268,435,456 fp32 = 1 GiB per operand
    a = torch.randint(-1000, 1000, (n,), device="cuda", dtype=torch.int32).float()
    b = torch.randint(-1000, 1000, (n,), device="cuda", dtype=torch.int32).float()
    o = torch.empty_like(a)
    pkg.op_reduce_3buff(pkg.OP["SUM"], pkg.T["FLOAT"], a.data_ptr(), b.data_ptr(), o.data_ptr(), n,
                        torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert torch.equal(o, a + b)
    del a, b, o
    torch.cuda.empty_cache()


def test_tune_variants_same_result(gpu, pkg):
    torch = gpu
    n = 3_000_017
    a = torch.randn(n, device="cuda")
    b = torch.randn(n, device="cuda")
    ref = a + b
    saved, mode = pkg.get_tune(), pkg.get_mode()
    try:
        for m in (0, 1):
            pkg.set_mode(m)
            for u in (1, 2, 4, 8):
                for nt in (0, 1, 2, 3):
                    for tpb in (256, 1024):
                        pkg.set_threads(tpb)
                        pkg.tune(u, 4, nt)
                        o = torch.empty_like(a)
                        pkg.op_reduce_3buff(pkg.OP["SUM"], pkg.T["FLOAT"], a.data_ptr(), b.data_ptr(), o.data_ptr(), n,
                                            torch.cuda.current_stream().cuda_stream)
                        torch.cuda.synchronize()
                        assert torch.equal(o, ref), (m, u, nt, tpb)
    finally:
        pkg.tune(*saved)
        pkg.set_mode(mode)
        pkg.set_threads(1024)


def test_max_mpi_count(gpu, pkg):
    """The largest count an MPI call can pass (INT_MAX elements, `int *count` in op.h:253-266):
    int8 SUM (wraps, 2 GiB - 1 byte per operand: byte offsets past 2^31) and fp32 SUM (8 GiB per
    operand: offsets past 2^32), 3-buff and 2-buff, against torch's own wrapping / exact add."""
    torch = gpu
    n = 2**31 - 1
    s = torch.cuda.current_stream().cuda_stream
    a = torch.randint(-128, 128, (n,), device="cuda", dtype=torch.int8)
    b = torch.randint(-128, 128, (n,), device="cuda", dtype=torch.int8)
    o = torch.empty_like(a)
    pkg.op_reduce_3buff(pkg.OP["SUM"], pkg.T["INT8"], a.data_ptr(), b.data_ptr(), o.data_ptr(), n, s)
    torch.cuda.synchronize()
    assert torch.equal(o, a + b)
    pkg.op_reduce(pkg.OP["SUM"], pkg.T["INT8"], a.data_ptr(), b.data_ptr(), n, s)  # b = b + a
    torch.cuda.synchronize()
    assert torch.equal(o, b)
    del a, b, o
    torch.cuda.empty_cache()
    a = torch.randint(-1000, 1000, (n,), device="cuda", dtype=torch.int16).float()
    b = torch.randint(-1000, 1000, (n,), device="cuda", dtype=torch.int16).float()
    o = torch.empty_like(a)
    pkg.op_reduce_3buff(pkg.OP["SUM"], pkg.T["FLOAT"], a.data_ptr(), b.data_ptr(), o.data_ptr(), n, s)
    torch.cuda.synchronize()
    assert torch.equal(o, a + b)
    del a, b, o
    torch.cuda.empty_cache()
