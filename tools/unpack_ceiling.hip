// unpack_ceiling.hip -- standalone probe of the partial-write ceiling under the GPU convertor's
// unpack: how fast can ANY kernel scatter a packed stream into a layout whose
// runs leave gaps that must stay untouched?
//
// Three layouts, 256 MiB packed each, timed with HIP events on one MI355X (algorithmic bytes =
// 2 x packed, as the convertor legs count them):
//   F7  MPI_Type_indexed 7 runs of FLOAT {1,3,2,7,1,1,4} at {0,2,9,13,25,27,40} (19 of 44 floats,
//       176-B extent; tools/bench_legs.py leg_ddt_runs) -- unpack and pack
//   TRI upper triangle of a 256 x 256 double matrix (256 runs of 8..2048 B per instance, the
//       long-run case) -- unpack and pack; specialised form: one wave per row moving 16-B ALIGNED
//       memory slots (odd rows start mid-slot), 8-B head / tail
//   COL vector(2^25, 1, 2, DOUBLE): a column of doubles, 8-B runs at a 16-B stride
// Kernels per layout, every one a hand-specialised form of the same scatter (compile-time run
// tables, no run search, nothing the general engine has to do):
//   unit   one 4-B (F7) / 8-B (COL) unit per lane, 4 units per lane 256 apart -- the shape of the
//          engine's unit / row kernels without their index math
//   inst   F7 only: one instance per lane, each run written with the widest aligned stores it
//          allows (dwordx4 / x2 / x1) -- fewest store instructions
//   lds    F7 only: a workgroup gathers its instances' units into an LDS image of the destination
//          span and writes the image back run by run with wide stores (LDS write-combining)
//   dense  writes EVERY byte of the destination span (gaps too: not a valid unpack) -- the
//          full-sector write rate the gaps cost us
// and, in the same process on the same buffers, the engine's own mi355x_unpack (libmi355x_rt).
// Every valid variant's destination is compared with the engine's.  Output: one JSON line per
// kernel.  Build (tools/build.sh unpack_ceiling): hipcc --offload-arch=gfx950 -O3 -o
// tools/build/unpack_ceiling tools/unpack_ceiling.hip -I include -L ompi-release_amd/lib -lmi355x_rt
// -Wl,-rpath,'$ORIGIN/../../ompi-release_amd/lib'
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "mi355x_rt.h"

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));           \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)
#define CKM(x)                                                                                  \
    do {                                                                                        \
        int r_ = (x);                                                                           \
        if (r_) {                                                                               \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, mi355x_last_error());             \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)

// ---- F7: 19 units (floats) per 44-float instance
constexpr int F7_UNITS = 19, F7_EXT = 44;
__constant__ int f7_off[F7_UNITS] = {0, 2, 3, 4, 9, 10, 13, 14, 15, 16, 17, 18, 19, 25, 27, 40, 41, 42, 43};

__global__ __launch_bounds__(256) void k_f7_unit(const float *__restrict__ p, float *__restrict__ d, uint64_t units)
{
    const uint64_t base = (uint64_t)blockIdx.x * 1024 + threadIdx.x;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint64_t u = base + 256 * k;
        if (u >= units) return;
        const uint64_t inst = u / F7_UNITS;
        const int j = (int)(u - inst * F7_UNITS);
        d[inst * F7_EXT + f7_off[j]] = __builtin_nontemporal_load(p + u);
    }
}

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x3 __attribute__((ext_vector_type(3)));

// one instance per lane; runs (floats): [0,1) [2,5) [9,11) [13,20) [25,26) [27,28) [40,44);
// byte addresses of an instance are 16-B aligned (176 = 11 x 16), so 40..43 is one dwordx4 and
// 16..19 another
__global__ __launch_bounds__(256) void k_f7_inst(const float *__restrict__ p, float *__restrict__ d, uint64_t ninst)
{
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= ninst) return;
    const float *s = p + i * F7_UNITS;
    float *o = d + i * F7_EXT;
    float v[F7_UNITS];
#pragma unroll
    for (int k = 0; k < F7_UNITS; ++k) v[k] = s[k];
    o[0] = v[0];
    o[2] = v[1];
    *(f32x2 *)(o + 3) = f32x2{v[2], v[3]};       // 12 B
    *(f32x2 *)(o + 9) = f32x2{v[4], v[5]};       // 36 B (8-B aligned)
    o[13] = v[6];
    o[14] = v[7];
    o[15] = v[8];
    *(f32x4 *)(o + 16) = f32x4{v[9], v[10], v[11], v[12]};
    o[25] = v[13];
    o[27] = v[14];
    *(f32x4 *)(o + 40) = f32x4{v[15], v[16], v[17], v[18]};
}

// LDS write-combining: a workgroup owns 256 consecutive instances; lanes gather the packed units
// (coalesced reads) into an LDS image of the 256 x 176-B destination span, then each lane writes one
// instance's runs back with the widest stores (as k_f7_inst) -- reads coalesced like the unit kernel,
// stores as wide as the layout allows
__global__ __launch_bounds__(256) void k_f7_lds(const float *__restrict__ p, float *__restrict__ d, uint64_t ninst)
{
    __shared__ float img[256 * F7_EXT];   // 44 KiB
    const uint64_t i0 = (uint64_t)blockIdx.x * 256;
    const uint64_t n = ninst - i0 < 256 ? ninst - i0 : 256;
    const float *s = p + i0 * F7_UNITS;
    for (uint64_t u = threadIdx.x; u < n * F7_UNITS; u += 256) {
        const uint64_t li = u / F7_UNITS;
        img[li * F7_EXT + f7_off[u - li * F7_UNITS]] = __builtin_nontemporal_load(s + u);
    }
    __syncthreads();
    if (threadIdx.x >= n) return;
    const float *v = img + threadIdx.x * F7_EXT;
    float *o = d + (i0 + threadIdx.x) * F7_EXT;
    o[0] = v[0];
    o[2] = v[2];
    *(f32x2 *)(o + 3) = f32x2{v[3], v[4]};
    *(f32x2 *)(o + 9) = f32x2{v[9], v[10]};
    o[13] = v[13];
    o[14] = v[14];
    o[15] = v[15];
    *(f32x4 *)(o + 16) = *(const f32x4 *)(v + 16);
    o[25] = v[25];
    o[27] = v[27];
    *(f32x4 *)(o + 40) = *(const f32x4 *)(v + 40);
}

// every byte of the span (not a valid unpack: the gaps are overwritten) -- one 16-B vector per lane
__global__ __launch_bounds__(256) void k_dense(const f32x4 *__restrict__ p, f32x4 *__restrict__ d, uint64_t nvec,
                                                uint64_t pvec)
{
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= nvec) return;
    __builtin_nontemporal_store(__builtin_nontemporal_load(p + (i % pvec)), d + i);
}

// ---- COL: vector(2^25, 1, 2, DOUBLE)
__global__ __launch_bounds__(256) void k_col_unit(const double *__restrict__ p, double *__restrict__ d, uint64_t units)
{
    const uint64_t base = (uint64_t)blockIdx.x * 2048 + threadIdx.x;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const uint64_t u = base + 256 * k;
        if (u >= units) return;
        d[2 * u] = __builtin_nontemporal_load(p + u);
    }
}

// ---- F7 pack: one 4-B unit per lane (the gather mirror of k_f7_unit)
__global__ __launch_bounds__(256) void k_f7_pack_unit(const float *__restrict__ m, float *__restrict__ p, uint64_t units)
{
    const uint64_t base = (uint64_t)blockIdx.x * 1024 + threadIdx.x;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint64_t u = base + 256 * k;
        if (u >= units) return;
        const uint64_t inst = u / F7_UNITS;
        const int j = (int)(u - inst * F7_UNITS);
        __builtin_nontemporal_store(m[inst * F7_EXT + f7_off[j]], p + u);
    }
}

// ---- TRI: upper triangle of a 256 x 256 double matrix (indexed, row i = (256 - i) doubles at
// (257 i) doubles), the convertor's long-run case.  One wave per row; the memory side moves in
// 16-B ALIGNED slots (row starts are 8-B aligned: odd rows begin mid-slot), the packed side in
// 8-B aligned 16-B accesses, the row's 8-B head and tail with one 8-B access each.
constexpr int TRI_N = 256;
typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
typedef unsigned long long u64x2a8 __attribute__((ext_vector_type(2), aligned(8)));

template <bool PACK>
__global__ __launch_bounds__(256) void k_tri_rows(char *__restrict__ mem, char *__restrict__ packed, uint64_t rows)
{
    const uint64_t row = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= rows) return;
    const int lane = threadIdx.x & 63;
    const uint64_t inst = row / TRI_N;
    const int i = (int)(row - inst * TRI_N);
    const uint64_t len = (uint64_t)(TRI_N - i) * 8;
    const uint64_t pfx = (uint64_t)i * TRI_N * 8 - (uint64_t)i * (i - 1) / 2 * 8;   // sum_{k<i} (256-k) * 8
    char *m = mem + inst * (uint64_t)TRI_N * TRI_N * 8 + (uint64_t)i * (TRI_N + 1) * 8;
    char *pk = packed + inst * ((uint64_t)TRI_N * (TRI_N + 1) / 2 * 8) + pfx;
    const uint64_t head = ((uintptr_t)m & 15) ? 8 : 0;
    const uint64_t body = (len - head) & ~(uint64_t)15;
    if (lane == 0 && head) {
        if (PACK) *(uint64_t *)pk = *(const uint64_t *)m;
        else *(uint64_t *)m = *(const uint64_t *)pk;
    }
    for (uint64_t o = head + (uint64_t)lane * 16; o < head + body; o += 64 * 16) {
        if (PACK) *(u64x2a8 *)(pk + o) = *(const u64x2 *)(m + o);
        else *(u64x2 *)(m + o) = *(const u64x2a8 *)(pk + o);
    }
    if (lane == 63 && head + body < len) {
        const uint64_t o = head + body;
        if (PACK) *(uint64_t *)(pk + o) = *(const uint64_t *)(m + o);
        else *(uint64_t *)(m + o) = *(const uint64_t *)(pk + o);
    }
}

static float time_ms(void (*launch)(void *), void *ctx, int reps)
{
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    launch(ctx);
    launch(ctx);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a, nullptr));
    for (int r = 0; r < reps; ++r) launch(ctx);
    CK(hipEventRecord(b, nullptr));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return ms / reps;
}

struct Ctx {
    void *p, *d;
    uint64_t n, m;
    mi355x_ddt_t *ddt;
    size_t count, bytes;
};

static void emit(const char *layout, const char *kernel, double alg, double ms, const char *note)
{
    printf("{\"leg\": \"unpack_ceiling\", \"layout\": \"%s\", \"kernel\": \"%s\", \"alg_bytes\": %.0f, "
           "\"kernel_avg_ms\": %.5f, \"achieved_GBs\": %.1f, \"frac\": %.4f%s%s}\n",
           layout, kernel, alg, ms, alg / (ms * 1e-3) / 1e9, alg / (ms * 1e-3) / 1e9 / 8000.0, note ? ", " : "",
           note ? note : "");
    fflush(stdout);
}

static bool same(const void *a, const void *b, size_t n)
{
    std::vector<unsigned char> x(n), y(n);
    CK(hipMemcpy(x.data(), a, n, hipMemcpyDeviceToHost));
    CK(hipMemcpy(y.data(), b, n, hipMemcpyDeviceToHost));
    return memcmp(x.data(), y.data(), n) == 0;
}

int main(int argc, char **argv)
{
    const int reps = argc > 1 ? atoi(argv[1]) : 20;
    // ---------------- F7
    {
        int bl[7] = {1, 3, 2, 7, 1, 1, 4}, dp[7] = {0, 2, 9, 13, 25, 27, 40};
        mi355x_ddt_t *ddt = nullptr;
        CKM(mi355x_ddt_create_indexed(7, bl, dp, 4, &ddt));
        const size_t inst_bytes = mi355x_ddt_size(ddt);   // 76
        const size_t count = ((size_t)256 << 20) / inst_bytes;
        const size_t packed = count * inst_bytes, span = count * F7_EXT * 4;
        float *p, *d_eng, *d;
        CK(hipMalloc(&p, packed));
        CK(hipMalloc(&d_eng, span));
        CK(hipMalloc(&d, span));
        std::vector<float> hp(packed / 4);
        for (size_t i = 0; i < hp.size(); ++i) hp[i] = (float)(i % 1000003);
        CK(hipMemcpy(p, hp.data(), packed, hipMemcpyHostToDevice));
        CK(hipMemset(d_eng, 0x5a, span));
        const double alg = 2.0 * (double)packed;
        Ctx c{p, d_eng, 0, 0, ddt, count, packed};
        float ms = time_ms([](void *x) {
            Ctx *c = (Ctx *)x;
            CKM(mi355x_unpack(c->ddt, c->count, c->d, 0, c->p, c->bytes, nullptr, nullptr));
        }, &c, reps);
        emit("F7", "engine mi355x_unpack", alg, ms, nullptr);
        const uint64_t units = packed / 4;
        struct V { const char *name; void (*fn)(void *); } vs[] = {
            {"unit (4-B units, constexpr table)", [](void *x) {
                 Ctx *c = (Ctx *)x;
                 const uint64_t units = c->bytes / 4;
                 k_f7_unit<<<(unsigned)((units + 1023) / 1024), 256>>>((const float *)c->p, (float *)c->d, units);
             }},
            {"inst (one instance per lane, widest stores)", [](void *x) {
                 Ctx *c = (Ctx *)x;
                 k_f7_inst<<<(unsigned)((c->count + 255) / 256), 256>>>((const float *)c->p, (float *)c->d, c->count);
             }},
            {"lds (LDS image of the span, wide stores)", [](void *x) {
                 Ctx *c = (Ctx *)x;
                 k_f7_lds<<<(unsigned)((c->count + 255) / 256), 256>>>((const float *)c->p, (float *)c->d, c->count);
             }},
        };
        (void)units;
        for (auto &v : vs) {
            CK(hipMemset(d, 0x5a, span));
            Ctx cv{p, d, 0, 0, ddt, count, packed};
            ms = time_ms(v.fn, &cv, reps);
            const bool ok = same(d, d_eng, span);
            char note[96];
            snprintf(note, sizeof(note), "\"equals_engine\": %s", ok ? "true" : "false");
            emit("F7", v.name, alg, ms, note);
        }
        Ctx cd{p, d, span / 16, packed / 16, ddt, count, packed};
        ms = time_ms([](void *x) {
            Ctx *c = (Ctx *)x;
            k_dense<<<(unsigned)((c->n + 255) / 256), 256>>>((const f32x4 *)c->p, (f32x4 *)c->d, c->n, c->m);
        }, &cd, reps);
        char note[160];
        snprintf(note, sizeof(note), "\"note\": \"writes all %zu span bytes (gaps too: not a valid unpack); "
                 "span GB/s %.1f\"", span, ((double)span + packed) / (ms * 1e-3) / 1e9);
        emit("F7", "dense (full-sector writes of the span)", alg, ms, note);
        // pack direction: gather the span into the packed stream
        float *p2;
        CK(hipMalloc(&p2, packed));
        Ctx cpk{d_eng, p, 0, 0, ddt, count, packed};
        ms = time_ms([](void *x) {
            Ctx *c = (Ctx *)x;
            CKM(mi355x_pack(c->ddt, c->count, c->p, 0, c->d, c->bytes, nullptr, nullptr));
        }, &cpk, reps);
        emit("F7", "PACK engine mi355x_pack", alg, ms, nullptr);
        Ctx cpu2{d_eng, p2, 0, 0, ddt, count, packed};
        ms = time_ms([](void *x) {
            Ctx *c = (Ctx *)x;
            const uint64_t units = c->bytes / 4;
            k_f7_pack_unit<<<(unsigned)((units + 1023) / 1024), 256>>>((const float *)c->p, (float *)c->d, units);
        }, &cpu2, reps);
        snprintf(note, sizeof(note), "\"equals_engine\": %s", same(p, p2, packed) ? "true" : "false");
        emit("F7", "PACK unit (4-B units, constexpr table)", alg, ms, note);
        CK(hipFree(p2));
        CK(hipFree(p));
        CK(hipFree(d));
        CK(hipFree(d_eng));
        mi355x_ddt_destroy(ddt);
    }
    // ---------------- TRI
    {
        std::vector<int> bl(TRI_N), dp(TRI_N);
        for (int i = 0; i < TRI_N; ++i) {
            bl[i] = TRI_N - i;
            dp[i] = i * (TRI_N + 1);
        }
        mi355x_ddt_t *ddt = nullptr;
        CKM(mi355x_ddt_create_indexed(TRI_N, bl.data(), dp.data(), 8, &ddt));
        const size_t inst_bytes = mi355x_ddt_size(ddt);   // 263168
        const size_t count = ((size_t)256 << 20) / inst_bytes;
        const size_t packed = count * inst_bytes, span = count * (size_t)TRI_N * TRI_N * 8;
        char *p, *d_eng, *d, *p2;
        CK(hipMalloc(&p, packed));
        CK(hipMalloc(&p2, packed));
        CK(hipMalloc(&d_eng, span));
        CK(hipMalloc(&d, span));
        std::vector<uint64_t> hp(packed / 8);
        for (size_t i = 0; i < hp.size(); ++i) hp[i] = i * 0x9e3779b97f4a7c15ull;
        CK(hipMemcpy(p, hp.data(), packed, hipMemcpyHostToDevice));
        CK(hipMemset(d_eng, 0x5a, span));
        CK(hipMemset(d, 0x5a, span));
        const double alg = 2.0 * (double)packed;
        Ctx c{p, d_eng, 0, 0, ddt, count, packed};
        float ms = time_ms([](void *x) {
            Ctx *c = (Ctx *)x;
            CKM(mi355x_unpack(c->ddt, c->count, c->d, 0, c->p, c->bytes, nullptr, nullptr));
        }, &c, reps);
        emit("TRI", "engine mi355x_unpack", alg, ms, nullptr);
        Ctx cr{p, d, count * TRI_N, 0, ddt, count, packed};
        ms = time_ms([](void *x) {
            Ctx *c = (Ctx *)x;
            k_tri_rows<false><<<(unsigned)((c->n + 3) / 4), 256>>>((char *)c->d, (char *)c->p, c->n);
        }, &cr, reps);
        char note[96];
        snprintf(note, sizeof(note), "\"equals_engine\": %s", same(d, d_eng, span) ? "true" : "false");
        emit("TRI", "rows (wave per row, 16-B aligned memory slots)", alg, ms, note);
        Ctx cpk{d_eng, p2, 0, 0, ddt, count, packed};
        ms = time_ms([](void *x) {
            Ctx *c = (Ctx *)x;
            CKM(mi355x_pack(c->ddt, c->count, c->p, 0, c->d, c->bytes, nullptr, nullptr));
        }, &cpk, reps);
        snprintf(note, sizeof(note), "\"equals_input\": %s", same(p, p2, packed) ? "true" : "false");
        emit("TRI", "PACK engine mi355x_pack", alg, ms, note);
        CK(hipMemset(p2, 0, packed));
        Ctx crp{p2, d_eng, count * TRI_N, 0, ddt, count, packed};
        ms = time_ms([](void *x) {
            Ctx *c = (Ctx *)x;
            k_tri_rows<true><<<(unsigned)((c->n + 3) / 4), 256>>>((char *)c->d, (char *)c->p, c->n);
        }, &crp, reps);
        snprintf(note, sizeof(note), "\"equals_input\": %s", same(p, p2, packed) ? "true" : "false");
        emit("TRI", "PACK rows (wave per row, 16-B aligned memory slots)", alg, ms, note);
        CK(hipFree(p));
        CK(hipFree(p2));
        CK(hipFree(d));
        CK(hipFree(d_eng));
        mi355x_ddt_destroy(ddt);
    }
    // ---------------- COL
    {
        mi355x_ddt_t *ddt = nullptr;
        const size_t count = (size_t)1 << 25;
        CKM(mi355x_ddt_create_vector(count, 1, 2, 8, &ddt));
        const size_t packed = count * 8, span = count * 16;
        double *p, *d_eng, *d;
        CK(hipMalloc(&p, packed));
        CK(hipMalloc(&d_eng, span));
        CK(hipMalloc(&d, span));
        std::vector<double> hp(count);
        for (size_t i = 0; i < count; ++i) hp[i] = (double)i;
        CK(hipMemcpy(p, hp.data(), packed, hipMemcpyHostToDevice));
        CK(hipMemset(d_eng, 0x5a, span));
        const double alg = 2.0 * (double)packed;
        Ctx c{p, d_eng, 0, 0, ddt, 1, packed};
        float ms = time_ms([](void *x) {
            Ctx *c = (Ctx *)x;
            CKM(mi355x_unpack(c->ddt, c->count, c->d, 0, c->p, c->bytes, nullptr, nullptr));
        }, &c, reps);
        emit("COL", "engine mi355x_unpack", alg, ms, nullptr);
        CK(hipMemset(d, 0x5a, span));
        Ctx cu{p, d, count, 0, ddt, 1, packed};
        ms = time_ms([](void *x) {
            Ctx *c = (Ctx *)x;
            k_col_unit<<<(unsigned)((c->n + 2047) / 2048), 256>>>((const double *)c->p, (double *)c->d, c->n);
        }, &cu, reps);
        char note[96];
        snprintf(note, sizeof(note), "\"equals_engine\": %s", same(d, d_eng, span) ? "true" : "false");
        emit("COL", "unit (8-B units, 8 per lane)", alg, ms, note);
        Ctx cd{p, d, span / 16, packed / 16, ddt, 1, packed};
        ms = time_ms([](void *x) {
            Ctx *c = (Ctx *)x;
            k_dense<<<(unsigned)((c->n + 255) / 256), 256>>>((const f32x4 *)c->p, (f32x4 *)c->d, c->n, c->m);
        }, &cd, reps);
        char note2[160];
        snprintf(note2, sizeof(note2), "\"note\": \"writes all %zu span bytes (gaps too: not a valid unpack)\"", span);
        emit("COL", "dense (full-sector writes of the span)", alg, ms, note2);
        CK(hipFree(p));
        CK(hipFree(d));
        CK(hipFree(d_eng));
        mi355x_ddt_destroy(ddt);
    }
    return 0;
}
