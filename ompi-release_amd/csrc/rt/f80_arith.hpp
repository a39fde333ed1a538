// f80_arith.hpp -- x87 extended-precision (80-bit) addition, subtraction and multiplication in
// integer arithmetic, bit-exact with what the x86-64 reference build's `long double` SUM / PROD
// loops compute on the x87 unit (op_base_functions.c's `*(out) += *(in)` / `*= ` on long double,
// :110-170; precision control extended, round to nearest even, every exception masked).
//
// Operands are the 80-bit encoding in 16 bytes of storage (f80, op_functors.hpp): 64-bit
// significand with an explicit integer bit, 15-bit exponent, sign.  The x87 rules restated:
//   * the encodings the 387 rejects -- pseudo-NaN / pseudo-infinity (exponent 0x7fff, integer bit
//     clear) and unnormals (exponent 1..0x7ffe, integer bit clear) -- are invalid operands: the
//     result is the real indefinite (sign 1, exponent 0x7fff, significand 0xC000000000000000);
//   * NaNs: a signalling NaN is quieted (significand bit 62 set); with one NaN operand the result is
//     that NaN quieted; with two, a quiet one beats a signalling one, else the larger significand,
//     and on equal significands the positive one (measured on the host's x87, tools/f80_check.cpp);
//   * inf - inf and 0 x inf are invalid (real indefinite);
//   * denormals and pseudo-denormals (exponent 0) are operands of effective exponent 1; results
//     underflow gradually (denormal results, one rounding at the denormal grid) and overflow to
//     infinity; an exact zero sum of opposite signs is +0.
// Host and device compile this header (the CPU check, tools/f80_check.cpp, runs it against the
// host's x87 unit), so it uses no HIP API.
#pragma once

#include <stdint.h>

#ifndef MI_HD
#define MI_HD __host__ __device__ inline
#endif

namespace mi355x {
namespace x87 {

typedef unsigned __int128 u128;

struct Bits {
    uint64_t m;
    uint16_t se;
};

constexpr uint64_t kInt = 1ull << 63;  // the explicit integer bit
constexpr uint64_t kQuiet = 1ull << 62;

MI_HD Bits indefinite() { return Bits{0xC000000000000000ull, 0xffff}; }

// 0 zero, 1 finite nonzero (normal, denormal, pseudo-denormal), 2 infinity, 3 NaN, 4 invalid encoding
MI_HD int kind(Bits x)
{
    const uint32_t e = x.se & 0x7fffu;
    if (e == 0x7fffu) {
        if (!(x.m & kInt)) return 4;
        return (x.m << 1) ? 3 : 2;
    }
    if (e == 0) return x.m ? 1 : 0;
    return (x.m & kInt) ? 1 : 4;
}

MI_HD Bits quiet(Bits x) { return Bits{x.m | kQuiet, x.se}; }

// NaN operands (at least one NaN, none invalid): the x87 choice (Intel SDM vol. 1, Table 4-7)
MI_HD Bits nan_result(Bits a, Bits b, int ka, int kb)
{
    if (ka == 3 && kb == 3) {
        const bool qa = (a.m & kQuiet) != 0, qb = (b.m & kQuiet) != 0;
        if (qa != qb) return qa ? a : b;
        const uint64_t ma = a.m & ~kQuiet, mb = b.m & ~kQuiet;
        if (ma == mb) return quiet((a.se & 0x8000) ? b : a);  // equal significands: the positive one
        return quiet(mb > ma ? b : a);
    }
    return quiet(ka == 3 ? a : b);
}

MI_HD int clz128(u128 x)
{
    const uint64_t hi = (uint64_t)(x >> 64), lo = (uint64_t)x;
    return hi ? __builtin_clzll(hi) : (lo ? 64 + __builtin_clzll(lo) : 128);
}

// x >> s with every shifted-out bit ORed into bit 0 (sticky), for any s >= 0
MI_HD u128 shr_sticky(u128 x, int s)
{
    if (s <= 0) return x;
    if (s >= 128) return x != 0 ? 1 : 0;
    const u128 out = x >> s;
    return out | (u128)((x << (128 - s)) != 0 ? 1 : 0);
}

// round sig x 2^(E - 16383 - 127) (sig != 0, any E) to the 80-bit format
MI_HD Bits round_pack(uint32_t sign, int32_t E, u128 sig)
{
    // normalise: leading one to bit 127, but not below the denormal exponent 1
    int lz = clz128(sig);
    if (lz > 0) {
        int sh = lz;
        if (E - sh < 1) sh = E - 1 > 0 ? E - 1 : 0;
        sig <<= sh;
        E -= sh;
    }
    if (E < 1) {  // below the denormal grid: shift right, keeping the bits shifted out sticky
        sig = shr_sticky(sig, 1 - E);
        E = 1;
    }
    uint64_t hi = (uint64_t)(sig >> 64);
    const uint64_t lo = (uint64_t)sig;
    const bool rnd = (lo >> 63) != 0, sticky = (lo << 1) != 0;
    if (rnd && (sticky || (hi & 1))) {
        hi += 1;
        if (hi == 0) {  // carried out of the significand: 1.000... one exponent up
            hi = kInt;
            E += 1;
        }
    }
    if (E >= 0x7fff) return Bits{kInt, (uint16_t)((sign << 15) | 0x7fffu)};  // overflow: infinity
    if (!(hi & kInt)) return Bits{hi, (uint16_t)(sign << 15)};                // denormal (or zero)
    return Bits{hi, (uint16_t)((sign << 15) | (uint32_t)E)};
}

MI_HD int32_t eff_exp(Bits x)
{
    const int32_t e = x.se & 0x7fff;
    return e ? e : 1;
}

// both operands normal (exponent 1..0x7ffe, integer bit set): the fast paths' precondition
MI_HD bool both_normal(Bits a, Bits b)
{
    return ((a.m & b.m) >> 63) != 0 && (uint32_t)(a.se & 0x7fff) - 1u < 0x7ffeu &&
           (uint32_t)(b.se & 0x7fff) - 1u < 0x7ffeu;
}

// round a significand whose leading one is at bit 127 (hi:lo) with exponent field E to nearest even,
// when the result is certainly normal and finite (1 <= E < 0x7ffe; a carry out of the significand
// then still leaves E <= 0x7ffe) -- round_pack's normal case, without its normalise / denormal /
// overflow steps
MI_HD Bits round_normal(uint32_t sign, int32_t E, uint64_t hi, uint64_t lo)
{
    if ((lo >> 63) && ((lo << 1) != 0 || (hi & 1))) {
        hi += 1;
        if (hi == 0) {
            hi = kInt;
            E += 1;
        }
    }
    return Bits{hi, (uint16_t)((sign << 15) | (uint32_t)E)};
}

// a + b (b's sign flipped first when sub: the NaN and invalid rules look at the operands as given)
MI_HD Bits add(Bits a, Bits b, bool sub)
{
    if (both_normal(a, b)) {  // the common case: no specials, normal result unless it says otherwise
        const uint32_t sa = a.se >> 15, sb = (uint32_t)((b.se >> 15) ^ (sub ? 1 : 0));
        const int32_t ea = a.se & 0x7fff, eb = b.se & 0x7fff;
        const bool bl = eb > ea || (eb == ea && b.m > a.m);  // |b| > |a|: b leads
        const uint64_t ma = bl ? b.m : a.m, mb = bl ? a.m : b.m;
        const uint32_t d = (uint32_t)(bl ? eb - ea : ea - eb);
        // the trailing significand aligned: (mb << 64) >> d as bh:blo, shifted-out bits sticky in
        // bit 0 (64-bit halves: the operands' low halves are zero, so half the u128 work is known)
        uint64_t bh, blo;
        if (d < 64) {
            bh = mb >> d;
            blo = d ? mb << (64 - d) : 0;
        } else if (d < 128) {
            bh = 0;
            blo = (mb >> (d - 64)) | (d > 64 && (mb << (128 - d)) != 0 ? 1 : 0);
        } else {
            bh = 0;
            blo = 1;  // (mb != 0: a normal significand)
        }
        uint64_t hi, lo;
        int32_t E = bl ? eb : ea;
        if (sa == sb) {
            hi = ma + bh;
            lo = blo;
            if (hi < ma) {  // carry out of bit 127: one place right, the bit shifted out sticky
                lo = (lo >> 1) | (hi << 63) | (lo & 1);
                hi = (hi >> 1) | kInt;
                E += 1;
            }
        } else {
            lo = 0 - blo;
            hi = ma - bh - (blo != 0 ? 1 : 0);
            if ((hi | lo) == 0) return Bits{0, 0};
            const int lz = hi ? __builtin_clzll(hi) : 64 + __builtin_clzll(lo);  // exact when lz > 1
            if (lz >= 64) {
                hi = lo << (lz - 64);
                lo = 0;
            } else if (lz > 0) {
                hi = (hi << lz) | (lo >> (64 - lz));
                lo <<= lz;
            }
            E -= lz;
        }
        if (E >= 1 && E < 0x7ffe) return round_normal(bl ? sb : sa, E, hi, lo);
    }
    const int ka = kind(a), kb = kind(b);
    if (ka == 4 || kb == 4) return indefinite();
    if (ka == 3 || kb == 3) return nan_result(a, b, ka, kb);
    if (sub) b.se ^= 0x8000;
    const uint32_t sa = a.se >> 15, sb = b.se >> 15;
    if (ka == 2 || kb == 2) {
        if (ka == 2 && kb == 2) return sa == sb ? a : indefinite();
        return ka == 2 ? a : b;
    }
    if (ka == 0 && kb == 0) return Bits{0, (uint16_t)((sa & sb) << 15)};
    int32_t Ea = eff_exp(a), Eb = eff_exp(b);
    u128 A = (u128)a.m << 64, B = (u128)b.m << 64;
    uint32_t sign = sa;
    if (Eb > Ea || (Eb == Ea && B > A)) {  // |b| > |a|: b leads
        u128 t = A;
        A = B;
        B = t;
        int32_t te = Ea;
        Ea = Eb;
        Eb = te;
        sign = sb;
    }
    B = shr_sticky(B, Ea - Eb);
    u128 S;
    int32_t E = Ea;
    if (sa == sb) {
        S = A + B;
        if (S < A) {  // carry out of bit 127
            S = shr_sticky(S, 1) | ((u128)1 << 127);
            E += 1;
        }
    } else {
        S = A - B;  // |A| >= |B|
        if (S == 0) return Bits{0, 0};  // exact cancellation: +0 (round to nearest)
    }
    return round_pack(sign, E, S);
}

MI_HD Bits mul(Bits a, Bits b)
{
    if (both_normal(a, b)) {  // product of two normal significands: leading one at bit 127 or 126
        const u128 P = (u128)a.m * (u128)b.m;
        uint64_t hi = (uint64_t)(P >> 64), lo = (uint64_t)P;
        int32_t E = (int32_t)(a.se & 0x7fff) + (int32_t)(b.se & 0x7fff) - 16383 + 1;
        if (!(hi >> 63)) {
            hi = (hi << 1) | (lo >> 63);
            lo <<= 1;
            E -= 1;
        }
        if (E >= 1 && E < 0x7ffe) return round_normal((uint32_t)((a.se ^ b.se) >> 15), E, hi, lo);
    }
    const int ka = kind(a), kb = kind(b);
    if (ka == 4 || kb == 4) return indefinite();
    if (ka == 3 || kb == 3) return nan_result(a, b, ka, kb);
    const uint32_t sign = (a.se >> 15) ^ (b.se >> 15);
    if (ka == 2 || kb == 2) {
        if (ka == 0 || kb == 0) return indefinite();  // 0 x inf
        return Bits{kInt, (uint16_t)((sign << 15) | 0x7fffu)};
    }
    if (ka == 0 || kb == 0) return Bits{0, (uint16_t)(sign << 15)};
    const u128 P = (u128)a.m * (u128)b.m;
    return round_pack(sign, eff_exp(a) + eff_exp(b) - 16383 + 1, P);
}

// exact conversion of a double (the constants of the complex multiply's recovery)
MI_HD Bits from_double(double v)
{
    uint64_t d;
    __builtin_memcpy(&d, &v, 8);
    const uint32_t sign = (uint32_t)(d >> 63);
    const uint32_t e = (uint32_t)(d >> 52) & 0x7ff;
    const uint64_t f = d & ((1ull << 52) - 1);
    if (e == 0x7ff) return Bits{f ? (kInt | kQuiet | (f << 11)) : kInt, (uint16_t)((sign << 15) | 0x7fffu)};
    if (e == 0) {
        if (!f) return Bits{0, (uint16_t)(sign << 15)};
        const int lz = __builtin_clzll(f) - 11;  // normalise the denormal double
        return Bits{(f << (11 + lz)) | 0, (uint16_t)((sign << 15) | (uint32_t)(16383 - 1022 - lz))};
    }
    return Bits{kInt | (f << 11), (uint16_t)((sign << 15) | (e - 1023 + 16383))};
}

} // namespace x87
} // namespace mi355x
