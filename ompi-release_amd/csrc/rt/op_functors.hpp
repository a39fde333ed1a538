// op_functors.hpp -- device-side element rules for every (MPI_Op, element type) slot that
// op/hip computes on the GPU.
//
// Each functor F provides
//     using T;                               the element (a C type or a MAXLOC pair struct)
//     static T op2(T out, T in);             2-buff rule: new inout value      (op_base_functions.c:39-103)
//     static T op3(T in1, T in2);            3-buff rule: out value            (op_base_functions.c:606-683)
// Operand roles follow the reference exactly (see oracle/op_oracle.c for the CPU restatement):
// MAX/MIN are selects `(o > a) ? o : a`, never v_max/v_min (NaN and signed-zero results depend
// on which operand is first); integer SUM/PROD wrap in the element width; complex PROD follows
// the C99 Annex G multiply that GCC emits for `_Complex *=` (inline fast path + libgcc
// __mulsc3/__muldc3 recovery, libgcc from GCC 11.4 -- the compiler the reference build uses on
// this host); MAXLOC/MINLOC keep the 2-buff / 3-buff asymmetry on ties.
// Compiled with -ffp-contract=off: no FMA contraction anywhere (the reference x86-64 build
// has none), denormals preserved (gfx950 default f32/f64 denormal mode is IEEE).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "../../../include/mi355x_types.h"
#include "f80_arith.hpp"

namespace mi355x {

// ------------------------------------------------------------------ element types
struct cf32 { float re, im; };
struct cf64 { double re, im; };
// MAXLOC/MINLOC pairs, byte-identical to the C structs of op_base_functions.c:539-555 on
// x86-64 (gfx950 uses the same sizes and alignments for these members).
struct p_float_int { float v; int k; };
struct p_double_int { double v; int k; };
struct p_long_int { long v; int k; };
struct p_2int { int v; int k; };
struct p_short_int { short v; int k; };
static_assert(sizeof(p_float_int) == 8, "float_int");
static_assert(sizeof(p_double_int) == 16, "double_int");
static_assert(sizeof(p_long_int) == 16, "long_int");
static_assert(sizeof(p_2int) == 8, "2int");
static_assert(sizeof(p_short_int) == 8, "short_int");
static_assert(sizeof(cf32) == 8 && sizeof(cf64) == 16, "complex");

// x86-64 `long double`: the x87 80-bit extended format (64-bit significand with an explicit
// integer bit, 15-bit exponent, sign) in 16 bytes of storage aligned to 16.  The GPU has no
// arithmetic for it, but MAX/MIN/MAXLOC/MINLOC only compare and select, and an x87 compare is
// exact integer work on the encoding:
//   * NaNs, and the encodings the 387 rejects as invalid operands (pseudo-NaN / pseudo-infinity:
//     exponent 0x7fff with the integer bit clear; unnormals: exponent 1..0x7ffe with the integer
//     bit clear), compare unordered -- every relation false, as FCOMI/FUCOMI report them;
//   * zero, denormals and pseudo-denormals (exponent 0) take effective exponent 1, so a
//     pseudo-denormal equals the normal of the same significand and +0 == -0;
//   * ordered values compare by sign, then (effective exponent, significand) lexicographically.
// A selected operand keeps its bits (FLD / FSTP of an m80 operand copy them unchanged).
struct alignas(16) f80 {
    uint64_t m;
    uint16_t se;
    uint16_t pad[3];
};
static_assert(sizeof(f80) == 16, "x86-64 long double storage");

#define MI_DEV __device__ __forceinline__
// -1 / 0 / +1, or 2 when unordered
MI_DEV int x87_cmp(const f80 &a, const f80 &b)
{
    uint32_t ea = a.se & 0x7fffu, eb = b.se & 0x7fffu;
    const bool ia = (a.m >> 63) != 0, ib = (b.m >> 63) != 0;
    const bool oka = ea == 0x7fffu ? (ia && (a.m << 1) == 0) : (ea == 0 || ia);
    const bool okb = eb == 0x7fffu ? (ib && (b.m << 1) == 0) : (eb == 0 || ib);
    if (!oka || !okb) return 2;
    if (ea == 0) ea = 1;
    if (eb == 0) eb = 1;
    if (a.m == 0 && b.m == 0) return 0;  // +-0 (an ordered nonzero value has a nonzero significand)
    const bool na = (a.se >> 15) != 0, nb = (b.se >> 15) != 0;
    if (na != nb) return na ? -1 : 1;
    const int mag = ea != eb ? (ea < eb ? -1 : 1) : (a.m != b.m ? (a.m < b.m ? -1 : 1) : 0);
    return na ? -mag : mag;
}
MI_DEV bool operator>(const f80 &a, const f80 &b) { return x87_cmp(a, b) == 1; }
MI_DEV bool operator<(const f80 &a, const f80 &b) { return x87_cmp(a, b) == -1; }
MI_DEV bool operator==(const f80 &a, const f80 &b) { return x87_cmp(a, b) == 0; }
MI_DEV bool operator!=(const f80 &a, const f80 &b) { return x87_cmp(a, b) != 0; }
// SUM / PROD: the x87 unit's add / multiply restated in integer arithmetic (f80_arith.hpp; checked
// bit for bit against the host's x87 by tools/f80_check.cpp); a selected or computed value's pad
// bytes are zero (never compared: the reference stores 10 bytes)
MI_DEV x87::Bits f80_bits(const f80 &x) { return x87::Bits{x.m, x.se}; }
MI_DEV f80 f80_of(x87::Bits b)
{
    f80 r;
    r.m = b.m;
    r.se = b.se;
    r.pad[0] = r.pad[1] = r.pad[2] = 0;
    return r;
}
MI_DEV f80 operator+(const f80 &a, const f80 &b) { return f80_of(x87::add(f80_bits(a), f80_bits(b), false)); }
MI_DEV f80 operator-(const f80 &a, const f80 &b) { return f80_of(x87::add(f80_bits(a), f80_bits(b), true)); }
MI_DEV f80 operator*(const f80 &a, const f80 &b) { return f80_of(x87::mul(f80_bits(a), f80_bits(b))); }
#undef MI_DEV

// MPI_LONG_DOUBLE_INT: {long double v; int k;} -- 32 bytes (LOC_STRUCT, op_base_functions.c:554)
struct alignas(16) p_ldouble_int {
    f80 v;
    int k;
};
static_assert(sizeof(p_ldouble_int) == 32, "long_double_int");

// unsigned twin used for wrap-around integer arithmetic (signed overflow is UB in C++; the
// reference relies on gcc's two's-complement code generation, which this reproduces)
template <typename T> struct uns { using type = T; };
template <> struct uns<int8_t> { using type = uint8_t; };
template <> struct uns<int16_t> { using type = uint16_t; };
template <> struct uns<int32_t> { using type = uint32_t; };
template <> struct uns<int64_t> { using type = uint64_t; };

// ------------------------------------------------------------------ elementwise rules
#define MI_DEV __device__ __forceinline__

template <typename E> struct OpMax {
    using T = E;
    static MI_DEV T op2(T o, T a) { return (o > a) ? o : a; }
    static MI_DEV T op3(T o, T a) { return (o > a) ? o : a; }
};
template <typename E> struct OpMin {
    using T = E;
    static MI_DEV T op2(T o, T a) { return (o < a) ? o : a; }
    static MI_DEV T op3(T o, T a) { return (o < a) ? o : a; }
};

template <typename E, bool IS_INT> struct SumImpl;
template <typename E> struct SumImpl<E, true> {
    static MI_DEV E f(E o, E a)
    {
        using U = typename uns<E>::type;
        return (E)(U)((U)o + (U)a);
    }
};
template <typename E> struct SumImpl<E, false> {
    static MI_DEV E f(E o, E a) { return o + a; }
};
template <typename E> struct OpSum {
    using T = E;
    static MI_DEV T op2(T o, T a) { return SumImpl<E, __is_integral(E)>::f(o, a); }
    static MI_DEV T op3(T o, T a) { return SumImpl<E, __is_integral(E)>::f(o, a); }
};

template <typename E, bool IS_INT> struct ProdImpl;
template <typename E> struct ProdImpl<E, true> {
    static MI_DEV E f(E o, E a)
    {
        // C promotes 8/16-bit operands to int; the low bits of the product are the same as the
        // low bits of an unsigned 32-bit product, so compute there and truncate.
        using W = typename std::conditional<(sizeof(E) <= 4), uint32_t, uint64_t>::type;
        return (E)(W)((W)(typename uns<E>::type)o * (W)(typename uns<E>::type)a);
    }
};
template <typename E> struct ProdImpl<E, false> {
    static MI_DEV E f(E o, E a) { return o * a; }
};
template <typename E> struct OpProd {
    using T = E;
    static MI_DEV T op2(T o, T a) { return ProdImpl<E, __is_integral(E)>::f(o, a); }
    static MI_DEV T op3(T o, T a) { return ProdImpl<E, __is_integral(E)>::f(o, a); }
};

// Logical ops on 1- and 2-byte elements also have a whole-word form (`swar`): the streaming
// kernels apply `word` to each 32-bit word of a 16-B vector instead of testing every element.
// nz(x) leaves the top bit of each element set iff the element is nonzero (the low bits are
// cleared first, so the add never carries across elements); the result is 1 / 0 per element,
// what the element form returns.
template <typename E> struct Swar {
    static constexpr bool on = sizeof(E) <= 2;
    static constexpr uint32_t lo = sizeof(E) == 1 ? 0x7f7f7f7fu : 0x7fff7fffu;
    static constexpr int top = 8 * sizeof(E) - 1;
    static MI_DEV uint32_t nz(uint32_t x) { return (((x & lo) + lo) | x) & ~lo; }
    static MI_DEV uint32_t ones(uint32_t m) { return m >> top; }
};
template <typename E> struct OpLand {
    using T = E;
    static constexpr bool swar = Swar<E>::on;
    static MI_DEV T op2(T o, T a) { return (T)((o != 0) && (a != 0)); }
    static MI_DEV T op3(T o, T a) { return (T)((o != 0) && (a != 0)); }
    static MI_DEV uint32_t word(uint32_t o, uint32_t a) { return Swar<E>::ones(Swar<E>::nz(o) & Swar<E>::nz(a)); }
};
template <typename E> struct OpLor {
    using T = E;
    static constexpr bool swar = Swar<E>::on;
    static MI_DEV T op2(T o, T a) { return (T)((o != 0) || (a != 0)); }
    static MI_DEV T op3(T o, T a) { return (T)((o != 0) || (a != 0)); }
    static MI_DEV uint32_t word(uint32_t o, uint32_t a) { return Swar<E>::ones(Swar<E>::nz(o) | Swar<E>::nz(a)); }
};
template <typename E> struct OpLxor {
    using T = E;
    static constexpr bool swar = Swar<E>::on;
    static MI_DEV T op2(T o, T a) { return (T)((o != 0 ? 1 : 0) ^ (a != 0 ? 1 : 0)); }
    static MI_DEV T op3(T o, T a) { return (T)((o != 0 ? 1 : 0) ^ (a != 0 ? 1 : 0)); }
    static MI_DEV uint32_t word(uint32_t o, uint32_t a) { return Swar<E>::ones(Swar<E>::nz(o) ^ Swar<E>::nz(a)); }
};
template <typename E> struct OpBand {
    using T = E;
    static MI_DEV T op2(T o, T a) { return (T)(o & a); }
    static MI_DEV T op3(T o, T a) { return (T)(o & a); }
};
template <typename E> struct OpBor {
    using T = E;
    static MI_DEV T op2(T o, T a) { return (T)(o | a); }
    static MI_DEV T op3(T o, T a) { return (T)(o | a); }
};
template <typename E> struct OpBxor {
    using T = E;
    static MI_DEV T op2(T o, T a) { return (T)(o ^ a); }
    static MI_DEV T op3(T o, T a) { return (T)(o ^ a); }
};

// ------------------------------------------------------------------ complex
// x86-64 `long double _Complex`: two 16-byte x87 values (C_LONG_DOUBLE_COMPLEX, 32 bytes)
struct alignas(16) cf80 {
    f80 re, im;
};
static_assert(sizeof(cf80) == 32, "long double complex");

template <typename R> struct CplxOf;
template <> struct CplxOf<float> { using type = cf32; };
template <> struct CplxOf<double> { using type = cf64; };
template <> struct CplxOf<f80> { using type = cf80; };

template <typename R> MI_DEV bool is_nan(R x) { return x != x; }
template <typename R> MI_DEV bool is_inf(R x) { return __builtin_isinf(x); }
template <typename R> MI_DEV R copysgn(R m, R s) { return __builtin_copysign(m, s); }
template <typename R> MI_DEV R cst(double v) { return (R)v; }
// x87: isnan is an unordered self-compare (NaNs and the invalid encodings: kind 3 and 4), isinf exact infinity,
// copysign the sign bit
template <> MI_DEV bool is_nan<f80>(f80 x) { return x87::kind(f80_bits(x)) >= 3; }  // == x87_cmp(x, x) == 2
template <> MI_DEV bool is_inf<f80>(f80 x) { return x87::kind(f80_bits(x)) == 2; }
template <> MI_DEV f80 copysgn<f80>(f80 m, f80 s)
{
    m.se = (uint16_t)((m.se & 0x7fffu) | (s.se & 0x8000u));
    return m;
}
template <> MI_DEV f80 cst<f80>(double v) { return f80_of(x87::from_double(v)); }

// (a + ib) * (c + id) as GCC evaluates `_Complex` multiplication without -ffast-math:
// x = ac - bd, y = ad + bc; if both are NaN, libgcc's __mul?c3 recovery rules (C99 G.5.1).
template <typename R> MI_DEV typename CplxOf<R>::type cmul(R a, R b, R c, R d)
{
    R ac = a * c, bd = b * d, ad = a * d, bc = b * c;
    R x = ac - bd, y = ad + bc;
    if (is_nan(x) && is_nan(y)) {
        bool recalc = false;
        if (is_inf(a) || is_inf(b)) {
            a = copysgn(is_inf(a) ? cst<R>(1) : cst<R>(0), a);
            b = copysgn(is_inf(b) ? cst<R>(1) : cst<R>(0), b);
            if (is_nan(c)) c = copysgn(cst<R>(0), c);
            if (is_nan(d)) d = copysgn(cst<R>(0), d);
            recalc = true;
        }
        if (is_inf(c) || is_inf(d)) {
            c = copysgn(is_inf(c) ? cst<R>(1) : cst<R>(0), c);
            d = copysgn(is_inf(d) ? cst<R>(1) : cst<R>(0), d);
            if (is_nan(a)) a = copysgn(cst<R>(0), a);
            if (is_nan(b)) b = copysgn(cst<R>(0), b);
            recalc = true;
        }
        if (!recalc && (is_inf(ac) || is_inf(bd) || is_inf(ad) || is_inf(bc))) {
            if (is_nan(a)) a = copysgn(cst<R>(0), a);
            if (is_nan(b)) b = copysgn(cst<R>(0), b);
            if (is_nan(c)) c = copysgn(cst<R>(0), c);
            if (is_nan(d)) d = copysgn(cst<R>(0), d);
            recalc = true;
        }
        if (recalc) {
            x = cst<R>(__builtin_inf()) * (a * c - b * d);
            y = cst<R>(__builtin_inf()) * (a * d + b * c);
        }
    }
    typename CplxOf<R>::type r;
    r.re = x;
    r.im = y;
    return r;
}

template <typename C> struct RealOf;
template <> struct RealOf<cf32> { using type = float; };
template <> struct RealOf<cf64> { using type = double; };
template <> struct RealOf<cf80> { using type = f80; };

template <typename C> struct OpCsum {
    using T = C;
    static MI_DEV T op2(T o, T a) { T r; r.re = o.re + a.re; r.im = o.im + a.im; return r; }
    static MI_DEV T op3(T o, T a) { return op2(o, a); }
};
template <typename C> struct OpCprod {
    using T = C;
    using R = typename RealOf<C>::type;
    static MI_DEV T op2(T o, T a) { return cmul<R>(o.re, o.im, a.re, a.im); }
    static MI_DEV T op3(T o, T a) { return cmul<R>(o.re, o.im, a.re, a.im); }
};

// ------------------------------------------------------------------ MAXLOC / MINLOC
// CMP(x, y) is x > y (maxloc) or x < y (minloc).
template <typename P, bool MAX> struct OpLoc {
    using T = P;
    static MI_DEV bool cmp(decltype(P::v) x, decltype(P::v) y) { return MAX ? (x > y) : (x < y); }
    // 2-buff (op_base_functions.c:87-103): o is inout, a is in
    static MI_DEV T op2(T o, T a)
    {
        if (cmp(a.v, o.v)) {
            o.v = a.v;
            o.k = a.k;
        } else if (a.v == o.v) {
            o.k = (o.k < a.k) ? o.k : a.k;
        }
        return o;
    }
    // 3-buff (op_base_functions.c:661-683): o is in1, a is in2
    static MI_DEV T op3(T o, T a)
    {
        if (cmp(o.v, a.v)) return o;
        if (o.v == a.v) {
            o.k = (a.k < o.k) ? a.k : o.k;
            return o;
        }
        return a;
    }
};

#undef MI_DEV
} // namespace mi355x
