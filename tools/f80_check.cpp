// f80_check.cpp -- (check, host only) ompi-release_amd/csrc/rt/f80_arith.hpp against this host's x87
// unit: `long double` +, - and * on adversarial encodings (every class, both signs) and on random
// operands over the whole exponent range (overflow, gradual underflow, cancellation), bit-exact in
// the 10 value bytes.  Prints one JSON line; exit status 1 on any mismatch.
//   g++ -O2 -o tools/build/f80_check tools/f80_check.cpp && tools/build/f80_check [random pairs]
#define MI_HD inline
#include "../ompi-release_amd/csrc/rt/f80_arith.hpp"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

using mi355x::x87::Bits;

static Bits bits_of(long double x)
{
    unsigned char b[16] = {0};
    std::memcpy(b, &x, 10);
    Bits r;
    std::memcpy(&r.m, b, 8);
    std::memcpy(&r.se, b + 8, 2);
    return r;
}

static long double ld_of(Bits x)
{
    unsigned char b[16] = {0};
    std::memcpy(b, &x.m, 8);
    std::memcpy(b + 8, &x.se, 2);
    long double r;
    std::memcpy(&r, b, sizeof(r));
    return r;
}

static bool same(Bits a, Bits b) { return a.m == b.m && a.se == b.se; }

int main(int argc, char **argv)
{
    const long nrand = argc > 1 ? atol(argv[1]) : 2000000;
    std::vector<Bits> enc;
    const uint64_t I = 1ull << 63;
    const uint64_t ms[] = {0, 1, 0x7FFFFFFFFFFFFFFFull, I, I | 5, I | 1, I | (1ull << 62), 0xFFFFFFFFFFFFFFFFull,
                           1ull << 62, 5, I | 0x123456789ull, 0xC000000000000000ull};
    const uint16_t es[] = {0, 1, 2, 63, 64, 65, 0x3FFF, 0x4000, 0x7FFD, 0x7FFE, 0x7FFF};
    for (uint64_t m : ms)
        for (uint16_t e : es)
            for (uint16_t s : {0, 0x8000}) enc.push_back(Bits{m, (uint16_t)(e | s)});
    long checked = 0, bad = 0;
    auto check = [&](Bits a, Bits b) {
        volatile long double x = ld_of(a), y = ld_of(b);
        const long double rs = x + y, rd = x - y, rm = x * y;
        const Bits gs = mi355x::x87::add(a, b, false), gd = mi355x::x87::add(a, b, true), gm = mi355x::x87::mul(a, b);
        const Bits ws = bits_of(rs), wd = bits_of(rd), wm = bits_of(rm);
        checked += 3;
        const struct { const char *op; Bits g, w; } r[3] = {{"+", gs, ws}, {"-", gd, wd}, {"*", gm, wm}};
        for (const auto &t : r)
            if (!same(t.g, t.w)) {
                if (bad < 20)
                    fprintf(stderr, "%016llx:%04x %s %016llx:%04x = %016llx:%04x (x87) vs %016llx:%04x\n",
                            (unsigned long long)a.m, a.se, t.op, (unsigned long long)b.m, b.se, (unsigned long long)t.w.m,
                            t.w.se, (unsigned long long)t.g.m, t.g.se);
                bad++;
            }
    };
    for (Bits a : enc)
        for (Bits b : enc) check(a, b);
    std::mt19937_64 rng(20261018);
    for (long i = 0; i < nrand; ++i) {
        Bits a, b;
        const int mode = (int)(rng() % 4);
        auto pick = [&](Bits &x) {
            x.m = rng() | (rng() % 8 ? I : 0);  // mostly normal significands
            uint32_t e;
            switch (mode) {
            case 0: e = (uint32_t)(rng() % 0x7fff); break;                          // anywhere
            case 1: e = (uint32_t)(rng() % 140); break;                              // near underflow
            case 2: e = 0x7fff - 1 - (uint32_t)(rng() % 140); break;                 // near overflow
            default: e = 0x3fff + (uint32_t)(rng() % 130) - 65; break;               // moderate
            }
            if (e == 0 && rng() % 2) x.m &= ~I;                                      // denormal
            x.se = (uint16_t)(e | (rng() % 2 ? 0x8000 : 0));
        };
        pick(a);
        pick(b);
        if (mode == 3 && rng() % 4 == 0) {  // near-cancellation: b close to -a
            b = a;
            b.se ^= 0x8000;
            b.m ^= rng() % 1024;
            if (!(b.m & I) && (b.se & 0x7fff)) b.m |= I;
        }
        check(a, b);
    }
    printf("{\"checked\": %ld, \"mismatches\": %ld, \"adversarial_pairs\": %zu, \"random_pairs\": %ld}\n", checked, bad,
           enc.size() * enc.size(), nrand);
    return bad ? 1 : 0;
}
