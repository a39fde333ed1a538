// op_kernels.hip -- op/hip streaming reduction kernels for gfx950 (MI355X).
//
// One kernel template serves every (MPI_Op, type) slot, 2-buff and 3-buff:
//   * 16-byte accesses per lane (global_load/store_dwordx4): 1 KiB per wave-instruction, full
//     128-B lines, for every element size (1..16 B); MAXLOC pairs are decoded in registers from
//     the same 16-byte vectors (no LDS round trip: each pair is consumed by the lane that loads
//     it, so staging would only add LDS traffic).
//   * default launch: one-shot grid, one 16-B vector per operand per lane, non-temporal loads
//     and stores when the three streams exceed the 256 MiB Infinity Cache (measured best on
//     MI355X, profiles/r01_op_tune.json); a persistent grid-stride form (U vectors in flight
//     per lane, blocks_per_cu x CUs) serves misaligned operands and tuning.
//   * scalar head/tail so any alignment works: when all three operands share the same
//     misalignment mod 16 the head peels to a 16-B boundary; otherwise the whole range takes
//     the element-wise path (still coalesced, one element per lane).
//   * no MFMA, no LDS: the work is 2 reads + 1 write per element -> HBM bound.
// Algorithmic bytes per call = 3 x count x sizeof(T) (2-buff: read in, read+write inout;
// 3-buff: read in1, in2, write out).
#include "op_functors.hpp"
#include "rt_internal.hpp"

#include <type_traits>

namespace mi355x {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <typename T> struct alignas(16) Vec16 {
    T e[16 / sizeof(T)];
};

struct StreamArgs {
    const void *a;    // 2-buff: in (source)          3-buff: in1
    const void *b;    // 2-buff: inout (target)       3-buff: in2
    void *out;        // 2-buff: == b                 3-buff: out
    size_t head;      // scalar elements before the 16-B aligned body
    size_t nvec;      // 16-B vectors in the body
    size_t n;         // total elements
};

template <class F, bool THREE>
__device__ __forceinline__ typename F::T apply(const typename F::T &xa, const typename F::T &xb)
{
    // 2-buff: new inout = op2(out = inout (b), in = source (a)); 3-buff: op3(in1 (a), in2 (b))
    if constexpr (THREE)
        return F::op3(xa, xb);
    else
        return F::op2(xb, xa);
}

// the functor has a whole-word form for its element size (op_functors.hpp, Swar)
template <class F, class = void> struct HasWord : std::false_type {};
template <class F> struct HasWord<F, std::enable_if_t<F::swar>> : std::true_type {};

// one 16-B vector of results from the raw operand vectors (word form when the functor has one)
template <class F, bool THREE>
__device__ __forceinline__ u32x4 apply_vec(const u32x4 &ra, const u32x4 &rb)
{
    u32x4 out;
    if constexpr (HasWord<F>::value) {
#pragma unroll
        for (int k = 0; k < 4; ++k) out[k] = F::word(ra[k], rb[k]);
    } else {
        using T = typename F::T;
        Vec16<T> xa, xb, r;
        __builtin_memcpy(&xa, &ra, 16);
        __builtin_memcpy(&xb, &rb, 16);
#pragma unroll
        for (int j = 0; j < (int)(16 / sizeof(T)); ++j) r.e[j] = apply<F, THREE>(xa.e[j], xb.e[j]);
        __builtin_memcpy(&out, &r, 16);
    }
    return out;
}

template <bool NT, typename V> __device__ __forceinline__ V vload(const V *p)
{
    u32x4 raw;
    if constexpr (NT)
        raw = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
    else
        raw = *reinterpret_cast<const u32x4 *>(p);
    V v;
    __builtin_memcpy(&v, &raw, 16);
    return v;
}

template <bool NT, typename V> __device__ __forceinline__ void vstore(V *p, const V &v)
{
    u32x4 raw;
    __builtin_memcpy(&raw, &v, 16);
    if constexpr (NT)
        __builtin_nontemporal_store(raw, reinterpret_cast<u32x4 *>(p));
    else
        *reinterpret_cast<u32x4 *>(p) = raw;
}

// NTM bit 0: non-temporal loads, bit 1: non-temporal stores (streams larger than the 256 MiB
// Infinity Cache gain ~9 % from not allocating in L2/MALL; small, re-read operands lose)
template <class F, bool THREE, int U, int NTM>
__global__ __launch_bounds__(256) void k_stream(StreamArgs args)
{
    using T = typename F::T;
    using V = Vec16<T>;
    constexpr int EPV = 16 / sizeof(T);
    const T *a = static_cast<const T *>(args.a);
    const T *b = static_cast<const T *>(args.b);
    T *o = static_cast<T *>(args.out);
    const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t nthr = (size_t)gridDim.x * blockDim.x;

    for (size_t i = tid; i < args.head; i += nthr) o[i] = apply<F, THREE>(a[i], b[i]);

    const V *av = reinterpret_cast<const V *>(a + args.head);
    const V *bv = reinterpret_cast<const V *>(b + args.head);
    V *ov = reinterpret_cast<V *>(o + args.head);
    const size_t nvec = args.nvec;
    for (size_t base = tid; base < nvec; base += nthr * U) {
        V xa[U], xb[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t i = base + (size_t)u * nthr;
            if (i < nvec) {
                xa[u] = vload<(NTM & 1) != 0>(av + i);
                xb[u] = vload<(NTM & 1) != 0>(bv + i);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t i = base + (size_t)u * nthr;
            if (i < nvec) {
                u32x4 ra, rb;
                __builtin_memcpy(&ra, &xa[u], 16);
                __builtin_memcpy(&rb, &xb[u], 16);
                const u32x4 r = apply_vec<F, THREE>(ra, rb);
                if constexpr ((NTM & 2) != 0)
                    __builtin_nontemporal_store(r, reinterpret_cast<u32x4 *>(ov + i));
                else
                    *reinterpret_cast<u32x4 *>(ov + i) = r;
            }
        }
    }

    const size_t t0 = args.head + nvec * EPV;
    for (size_t i = t0 + tid; i < args.n; i += nthr) o[i] = apply<F, THREE>(a[i], b[i]);
}

// One-shot variant: no grid-stride loop.  Block b owns the contiguous run of 256*U vectors
// starting at b*256*U; lane t touches vectors t, t+256, ... (each wave-instruction reads 1 KiB
// contiguous).  Grid = ceil(nvec / (256*U)) blocks -- the hardware dispatcher, not a loop,
// balances the 8 XCDs.  Head/tail elements are handled by block 0 / the last block.
template <class F, bool THREE, int U, int NTM>
__global__ __launch_bounds__(1024) void k_chunk(StreamArgs args)
{
    using T = typename F::T;
    using V = Vec16<T>;
    constexpr int EPV = 16 / sizeof(T);
    const T *a = static_cast<const T *>(args.a);
    const T *b = static_cast<const T *>(args.b);
    T *o = static_cast<T *>(args.out);
    const V *av = reinterpret_cast<const V *>(a + args.head);
    const V *bv = reinterpret_cast<const V *>(b + args.head);
    V *ov = reinterpret_cast<V *>(o + args.head);
    const size_t nvec = args.nvec;
    const size_t tpb = blockDim.x;
    const size_t base = (size_t)blockIdx.x * (tpb * U) + threadIdx.x;
    u32x4 ra[U], rb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const size_t i = base + (size_t)u * tpb;
        if (i < nvec) {
            if constexpr ((NTM & 1) != 0) {
                ra[u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(av + i));
                rb[u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(bv + i));
            } else {
                ra[u] = *reinterpret_cast<const u32x4 *>(av + i);
                rb[u] = *reinterpret_cast<const u32x4 *>(bv + i);
            }
        }
    }
    // Pin the loaded dwordx4 values (after all loads are issued): without it the byte-element
    // kernels get their loads re-typed to <16 x i8> and the non-temporal hint is dropped.
    if constexpr ((NTM & 1) != 0 && sizeof(T) == 1) {
#pragma unroll
        for (int u = 0; u < U; ++u) asm volatile("" : "+v"(ra[u]), "+v"(rb[u]));
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const size_t i = base + (size_t)u * tpb;
        if (i < nvec) {
            const u32x4 r = apply_vec<F, THREE>(ra[u], rb[u]);
            if constexpr ((NTM & 2) != 0)
                __builtin_nontemporal_store(r, reinterpret_cast<u32x4 *>(ov + i));
            else
                *reinterpret_cast<u32x4 *>(ov + i) = r;
        }
    }
    if (blockIdx.x == 0) {
        for (size_t i = threadIdx.x; i < args.head; i += tpb) o[i] = apply<F, THREE>(a[i], b[i]);
    }
    if (blockIdx.x == gridDim.x - 1) {
        for (size_t i = args.head + nvec * EPV + threadIdx.x; i < args.n; i += tpb)
            o[i] = apply<F, THREE>(a[i], b[i]);
    }
}

// only the bench-critical functors get every launch-shape variant; the rest use the default
constexpr int kDefaultUnroll = 1;
template <class F> struct Tunable : std::false_type {};
template <> struct Tunable<OpSum<float>> : std::true_type {};
template <> struct Tunable<OpSum<double>> : std::true_type {};

template <class F, bool THREE, int U, int NTM>
static int launch_shape(const StreamArgs &args, hipStream_t s)
{
    using T = typename F::T;
    constexpr int EPV = 16 / sizeof(T);
    const StreamTune &t = stream_tune();
    const size_t threads = 256;
    const size_t scalar = args.head + (args.n - args.head - args.nvec * EPV);
    if (t.mode == 1 && args.nvec > 0 && scalar <= 64) {
        // one-shot chunked grid (head/tail < 16 elements are handled by the edge blocks)
        const size_t tpb = (size_t)t.threads;
        size_t blocks = (args.nvec + tpb * U - 1) / (tpb * U);
        if (blocks > 0x7fffffffu) return set_error(MI355X_ERR_ARG, "count too large for one launch");
        hipLaunchKernelGGL((k_chunk<F, THREE, U, NTM>), dim3((unsigned)blocks), dim3((unsigned)tpb), 0, s, args);
        MI_HIP(hipGetLastError());
        return MI355X_SUCCESS;
    }
    size_t work = args.nvec ? (args.nvec + (size_t)U - 1) / U : 0;
    if (scalar > work) work = scalar;
    size_t blocks = (work + threads - 1) / threads;
    const size_t cap = (size_t)t.blocks_per_cu * (size_t)device_cu_count();
    if (blocks > cap) blocks = cap;
    if (blocks == 0) blocks = 1;
    hipLaunchKernelGGL((k_stream<F, THREE, U, NTM>), dim3((unsigned)blocks), dim3(threads), 0, s,
                       args);
    MI_HIP(hipGetLastError());
    return MI355X_SUCCESS;
}

// elements wider than one 16-B vector (MPI_LONG_DOUBLE_INT, 32 B), operands not 16-B aligned:
// one element per lane (the pair is consumed whole by the lane that loads it)
template <class F, bool THREE>
__global__ __launch_bounds__(256) void k_wide(const typename F::T *a, const typename F::T *b, typename F::T *o, size_t n)
{
    const size_t nthr = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += nthr) o[i] = apply<F, THREE>(a[i], b[i]);
}

// 32-B elements on 16-B aligned operands: one 16-B half per lane, so every wave instruction
// moves 1 KiB contiguous (the one-element-per-lane form strides 32 B per lane: two half-used
// instructions per operand, 0.80 of the 2R+1W ceiling, profiles/r06_bench_sweep.json).  The two
// lanes of an element swap halves with one DPP quad permute per dword (no LDS), both evaluate the
// element, each stores its own half.  One-shot grid, non-temporal beyond the Infinity Cache, as
// k_chunk.
// The complex x87 slots evaluate one component per lane instead of the whole element twice: the
// lane holding the real halves computes the real part, its partner the imaginary part.  CSUM needs
// nothing from the partner; CPROD reads the partner's halves for the cross products and, when both
// parts come out NaN (the pair agrees on that through one more DPP swap), both lanes redo the whole
// product under the recovery rules of cmul.  The integer x87 arithmetic makes these two slots
// VALU-bound, so halving the work per lane is what moves them toward the memory ceiling.
template <class F> struct PerComponent : std::false_type {};
template <> struct PerComponent<OpCsum<cf80>> : std::true_type {};
template <> struct PerComponent<OpCprod<cf80>> : std::true_type {};

__device__ __forceinline__ f80 f80_of_vec(u32x4 v)
{
    f80 x;
    __builtin_memcpy(&x, &v, 16);
    return x;
}

__device__ __forceinline__ u32x4 vec_of_f80(f80 x)
{
    u32x4 v;
    __builtin_memcpy(&v, &x, 16);
    return v;
}

__device__ __forceinline__ u32x4 dpp_swap(u32x4 v)  // lanes 2k <-> 2k+1 (quad_perm [1,0,3,2])
{
    u32x4 p;
#pragma unroll
    for (int k = 0; k < 4; ++k) p[k] = (unsigned)__builtin_amdgcn_update_dpp(0, (int)v[k], 0xB1, 0xF, 0xF, false);
    return p;
}

template <class F, bool THREE>
__device__ __forceinline__ u32x4 component(u32x4 ra, u32x4 rb, bool hi)
{
    // operand roles as apply(): 2-buff op2(inout = b, in = a), 3-buff op3(in1 = a, in2 = b)
    const u32x4 vo = THREE ? ra : rb, va = THREE ? rb : ra;
    const f80 om = f80_of_vec(vo), am = f80_of_vec(va);
    if constexpr (std::is_same<F, OpCsum<cf80>>::value) {
        return vec_of_f80(om + am);  // (o.re + a.re) or (o.im + a.im)
    } else {
        const u32x4 po = dpp_swap(vo), pa = dpp_swap(va);
        const f80 op = f80_of_vec(po), ap = f80_of_vec(pa);
        // cmul(a, b, c, d) with a = o.re, b = o.im, c = a.re, d = a.im: x = ac - bd, y = ad + bc
        // one instruction stream for both lanes of the pair (the wave alternates lo / hi lanes, so
        // a branch on hi would run both paths): operands selected, subtract flag per lane
        const f80 m1 = (hi ? op : om) * am, m2 = (hi ? om : op) * ap;
        const f80 r = f80_of(x87::add(f80_bits(m1), f80_bits(m2), !hi));
        // cmul changes the result only when both parts are NaN and an operand or one of the four
        // products is infinite (it recomputes then); the pair shares "NaN" and "a product of mine
        // is infinite" in one swapped word
        int mine = 0;
        if (is_nan(r)) mine = 1 | (is_inf(m1) || is_inf(m2) ? 2 : 0);  // (never taken on finite data)
        const int partner = __builtin_amdgcn_update_dpp(0, mine, 0xB1, 0xF, 0xF, false);
        if ((mine & partner & 1) &&
            (((mine | partner) & 2) || is_inf(om) || is_inf(op) || is_inf(am) || is_inf(ap))) {
            const cf80 w = hi ? cmul<f80>(op, om, ap, am) : cmul<f80>(om, op, am, ap);
            return vec_of_f80(hi ? w.im : w.re);
        }
        return vec_of_f80(r);
    }
}

template <class F, bool THREE, int NTM>
__global__ __launch_bounds__(1024) void k_wide_halves(const u32x4 *a, const u32x4 *b, u32x4 *o, size_t nhalf)
{
    using T = typename F::T;
    static_assert(sizeof(T) == 32, "two halves per element");
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool live = i < nhalf;  // nhalf is even and pairs start at even i: both lanes or neither
    u32x4 ra = {0, 0, 0, 0}, rb = {0, 0, 0, 0};
    if (live) {
        if constexpr ((NTM & 1) != 0) {
            ra = __builtin_nontemporal_load(a + i);
            rb = __builtin_nontemporal_load(b + i);
        } else {
            ra = a[i];
            rb = b[i];
        }
    }
    const bool hi = (i & 1) != 0;
    if constexpr (PerComponent<F>::value) {
        const u32x4 mine = component<F, THREE>(ra, rb, hi);  // (every lane: the DPP swaps inside)
        if (!live) return;
        if constexpr ((NTM & 2) != 0)
            __builtin_nontemporal_store(mine, o + i);
        else
            o[i] = mine;
        return;
    }
    const u32x4 pa = dpp_swap(ra), pb = dpp_swap(rb);  // the partner lane's halves
    if (!live) return;
    u32x4 ea[2] = {hi ? pa : ra, hi ? ra : pa};
    u32x4 eb[2] = {hi ? pb : rb, hi ? rb : pb};
    T xa, xb;
    __builtin_memcpy(&xa, ea, 32);
    __builtin_memcpy(&xb, eb, 32);
    const T r = apply<F, THREE>(xa, xb);
    u32x4 er[2];
    __builtin_memcpy(er, &r, 32);
    const u32x4 mine = hi ? er[1] : er[0];
    if constexpr ((NTM & 2) != 0)
        __builtin_nontemporal_store(mine, o + i);
    else
        o[i] = mine;
}

template <class F, bool THREE>
static int launch(const void *a, const void *b, void *out, size_t n, hipStream_t s)
{
    using T = typename F::T;
    if (n == 0) return MI355X_SUCCESS;
    if constexpr (sizeof(T) > 16) {
        if ((((uintptr_t)a | (uintptr_t)b | (uintptr_t)out) & 15) == 0 && n < ((size_t)1 << 40)) {
            const size_t nhalf = 2 * n;
            const size_t blocks = (nhalf + 1023) / 1024;
            const bool nt = 3 * n * sizeof(T) > ((size_t)256 << 20);
            const u32x4 *ha = static_cast<const u32x4 *>(a), *hb = static_cast<const u32x4 *>(b);
            u32x4 *ho = static_cast<u32x4 *>(out);
            if (nt)
                hipLaunchKernelGGL((k_wide_halves<F, THREE, 3>), dim3((unsigned)blocks), dim3(1024), 0, s, ha, hb, ho, nhalf);
            else
                hipLaunchKernelGGL((k_wide_halves<F, THREE, 0>), dim3((unsigned)blocks), dim3(1024), 0, s, ha, hb, ho, nhalf);
            MI_HIP(hipGetLastError());
            return MI355X_SUCCESS;
        }
        size_t blocks = (n + 255) / 256;
        const size_t cap = (size_t)stream_tune().blocks_per_cu * (size_t)device_cu_count();
        if (blocks > cap) blocks = cap;
        hipLaunchKernelGGL((k_wide<F, THREE>), dim3((unsigned)blocks), dim3(256), 0, s, static_cast<const T *>(a),
                           static_cast<const T *>(b), static_cast<T *>(out), n);
        MI_HIP(hipGetLastError());
        return MI355X_SUCCESS;
    } else {
    constexpr size_t EPV = 16 / sizeof(T);
    StreamArgs args;
    args.a = a;
    args.b = b;
    args.out = out;
    args.n = n;
    const uintptr_t ma = (uintptr_t)a & 15, mb = (uintptr_t)b & 15, mo = (uintptr_t)out & 15;
    if (ma == mb && mb == mo && (ma % sizeof(T)) == 0) {
        size_t head = ma ? (16 - ma) / sizeof(T) : 0;
        if (head > n) head = n;
        args.head = head;
        args.nvec = (n - head) / EPV;
    } else {
        args.head = n; // element-wise path
        args.nvec = 0;
    }
    const StreamTune &t = stream_tune();
    // non-temporal policy: explicit 0..3, or auto (-1): streams beyond the Infinity Cache
    int ntm = t.nontemporal;
    if (ntm < 0) ntm = (3 * n * sizeof(T) > ((size_t)256 << 20)) ? 3 : 0;
    if constexpr (Tunable<F>::value) {
#define MI_NT(U_)                                                              \
    switch (ntm) {                                                             \
    case 1: return launch_shape<F, THREE, U_, 1>(args, s);                     \
    case 2: return launch_shape<F, THREE, U_, 2>(args, s);                     \
    case 3: return launch_shape<F, THREE, U_, 3>(args, s);                     \
    default: return launch_shape<F, THREE, U_, 0>(args, s);                    \
    }
        switch (t.unroll) {
        case 2: MI_NT(2)
        case 4: MI_NT(4)
        case 8: MI_NT(8)
        default: MI_NT(1)
        }
#undef MI_NT
    } else {
        return ntm ? launch_shape<F, THREE, kDefaultUnroll, 3>(args, s)
                   : launch_shape<F, THREE, kDefaultUnroll, 0>(args, s);
    }
    }
}

// ------------------------------------------------------------------ dispatch table
typedef int (*launch_fn)(const void *, const void *, void *, size_t, hipStream_t);

struct Slot {
    launch_fn two = nullptr;
    launch_fn three = nullptr;
};

template <class F> static void put(Slot (&tab)[MI355X_OP_MAX_][MI355X_T_MAX], int op, int ty)
{
    tab[op][ty].two = &launch<F, false>;
    tab[op][ty].three = &launch<F, true>;
}

template <template <typename> class OP>
static void put_ints(Slot (&tab)[MI355X_OP_MAX_][MI355X_T_MAX], int op)
{
    put<OP<int8_t>>(tab, op, MI355X_T_INT8);
    put<OP<uint8_t>>(tab, op, MI355X_T_UINT8);
    put<OP<int16_t>>(tab, op, MI355X_T_INT16);
    put<OP<uint16_t>>(tab, op, MI355X_T_UINT16);
    put<OP<int32_t>>(tab, op, MI355X_T_INT32);
    put<OP<uint32_t>>(tab, op, MI355X_T_UINT32);
    put<OP<int64_t>>(tab, op, MI355X_T_INT64);
    put<OP<uint64_t>>(tab, op, MI355X_T_UINT64);
}

struct Table {
    Slot s[MI355X_OP_MAX_][MI355X_T_MAX];
    Table()
    {
        // groups as in op_base_functions.c:1373-1457 (Fortran types disabled)
        put_ints<OpMax>(s, MI355X_OP_MAX);
        put<OpMax<float>>(s, MI355X_OP_MAX, MI355X_T_FLOAT);
        put<OpMax<double>>(s, MI355X_OP_MAX, MI355X_T_DOUBLE);
        put_ints<OpMin>(s, MI355X_OP_MIN);
        put<OpMin<float>>(s, MI355X_OP_MIN, MI355X_T_FLOAT);
        put<OpMin<double>>(s, MI355X_OP_MIN, MI355X_T_DOUBLE);
        put_ints<OpSum>(s, MI355X_OP_SUM);
        put<OpSum<float>>(s, MI355X_OP_SUM, MI355X_T_FLOAT);
        put<OpSum<double>>(s, MI355X_OP_SUM, MI355X_T_DOUBLE);
        put<OpCsum<cf32>>(s, MI355X_OP_SUM, MI355X_T_C_FLOAT_COMPLEX);
        put<OpCsum<cf64>>(s, MI355X_OP_SUM, MI355X_T_C_DOUBLE_COMPLEX);
        put_ints<OpProd>(s, MI355X_OP_PROD);
        put<OpProd<float>>(s, MI355X_OP_PROD, MI355X_T_FLOAT);
        put<OpProd<double>>(s, MI355X_OP_PROD, MI355X_T_DOUBLE);
        put<OpCprod<cf32>>(s, MI355X_OP_PROD, MI355X_T_C_FLOAT_COMPLEX);
        put<OpCprod<cf64>>(s, MI355X_OP_PROD, MI355X_T_C_DOUBLE_COMPLEX);
        put_ints<OpLand>(s, MI355X_OP_LAND);
        put<OpLand<uint8_t>>(s, MI355X_OP_LAND, MI355X_T_BOOL);
        put_ints<OpLor>(s, MI355X_OP_LOR);
        put<OpLor<uint8_t>>(s, MI355X_OP_LOR, MI355X_T_BOOL);
        put_ints<OpLxor>(s, MI355X_OP_LXOR);
        put<OpLxor<uint8_t>>(s, MI355X_OP_LXOR, MI355X_T_BOOL);
        put_ints<OpBand>(s, MI355X_OP_BAND);
        put<OpBand<int8_t>>(s, MI355X_OP_BAND, MI355X_T_BYTE);
        put_ints<OpBor>(s, MI355X_OP_BOR);
        put<OpBor<int8_t>>(s, MI355X_OP_BOR, MI355X_T_BYTE);
        put_ints<OpBxor>(s, MI355X_OP_BXOR);
        put<OpBxor<int8_t>>(s, MI355X_OP_BXOR, MI355X_T_BYTE);
        put<OpLoc<p_float_int, true>>(s, MI355X_OP_MAXLOC, MI355X_T_FLOAT_INT);
        put<OpLoc<p_double_int, true>>(s, MI355X_OP_MAXLOC, MI355X_T_DOUBLE_INT);
        put<OpLoc<p_long_int, true>>(s, MI355X_OP_MAXLOC, MI355X_T_LONG_INT);
        put<OpLoc<p_2int, true>>(s, MI355X_OP_MAXLOC, MI355X_T_2INT);
        put<OpLoc<p_short_int, true>>(s, MI355X_OP_MAXLOC, MI355X_T_SHORT_INT);
        put<OpLoc<p_float_int, false>>(s, MI355X_OP_MINLOC, MI355X_T_FLOAT_INT);
        put<OpLoc<p_double_int, false>>(s, MI355X_OP_MINLOC, MI355X_T_DOUBLE_INT);
        put<OpLoc<p_long_int, false>>(s, MI355X_OP_MINLOC, MI355X_T_LONG_INT);
        put<OpLoc<p_2int, false>>(s, MI355X_OP_MINLOC, MI355X_T_2INT);
        put<OpLoc<p_short_int, false>>(s, MI355X_OP_MINLOC, MI355X_T_SHORT_INT);
        // x87 long double: compare-and-select (MAX/MIN) and the x87 add / multiply restated in
        // integer arithmetic (SUM/PROD, f80_arith.hpp), real and complex
        put<OpMax<f80>>(s, MI355X_OP_MAX, MI355X_T_LONG_DOUBLE);
        put<OpMin<f80>>(s, MI355X_OP_MIN, MI355X_T_LONG_DOUBLE);
        put<OpSum<f80>>(s, MI355X_OP_SUM, MI355X_T_LONG_DOUBLE);
        put<OpProd<f80>>(s, MI355X_OP_PROD, MI355X_T_LONG_DOUBLE);
        put<OpCsum<cf80>>(s, MI355X_OP_SUM, MI355X_T_C_LONG_DOUBLE_COMPLEX);
        put<OpCprod<cf80>>(s, MI355X_OP_PROD, MI355X_T_C_LONG_DOUBLE_COMPLEX);
        put<OpLoc<p_ldouble_int, true>>(s, MI355X_OP_MAXLOC, MI355X_T_LONG_DOUBLE_INT);
        put<OpLoc<p_ldouble_int, false>>(s, MI355X_OP_MINLOC, MI355X_T_LONG_DOUBLE_INT);
    }
};

static const Table &table()
{
    static const Table t;
    return t;
}

static const Slot *slot_of(int op, int type)
{
    if (op < 0 || op >= MI355X_OP_MAX_ || type < 0 || type >= MI355X_T_MAX) return nullptr;
    const Slot *sl = &table().s[op][type];
    return sl->two ? sl : nullptr;
}

} // namespace mi355x

using namespace mi355x;

extern "C" {

int mi355x_op_supported(int op, int type) { return slot_of(op, type) ? 1 : 0; }

size_t mi355x_type_size(int type)
{
    switch (type) {
    case MI355X_T_INT8: case MI355X_T_UINT8: case MI355X_T_BOOL: case MI355X_T_BYTE: return 1;
    case MI355X_T_INT16: case MI355X_T_UINT16: return 2;
    case MI355X_T_INT32: case MI355X_T_UINT32: case MI355X_T_FLOAT: return 4;
    case MI355X_T_INT64: case MI355X_T_UINT64: case MI355X_T_DOUBLE: return 8;
    case MI355X_T_LONG_DOUBLE: return 16;            /* x86-64 long double storage */
    case MI355X_T_C_FLOAT_COMPLEX: return 8;
    case MI355X_T_C_DOUBLE_COMPLEX: return 16;
    case MI355X_T_C_LONG_DOUBLE_COMPLEX: return 32;
    case MI355X_T_FLOAT_INT: case MI355X_T_2INT: case MI355X_T_SHORT_INT: return 8;
    case MI355X_T_DOUBLE_INT: case MI355X_T_LONG_INT: return 16;
    case MI355X_T_LONG_DOUBLE_INT: return 32;
    default: return 0;
    }
}

int mi355x_op_reduce(int op, int type, const void *in, void *inout, size_t count, void *stream)
{
    const Slot *sl = slot_of(op, type);
    if (!sl) return set_error(MI355X_ERR_UNSUPPORTED, "no GPU kernel for op %d type %d", op, type);
    if (count && (!in || !inout)) return set_error(MI355X_ERR_ARG, "NULL buffer");
    return sl->two(in, inout, inout, count, resolve_stream(stream));
}

int mi355x_op_reduce_3buff(int op, int type, const void *in1, const void *in2, void *out,
                           size_t count, void *stream)
{
    const Slot *sl = slot_of(op, type);
    if (!sl) return set_error(MI355X_ERR_UNSUPPORTED, "no GPU kernel for op %d type %d", op, type);
    if (count && (!in1 || !in2 || !out)) return set_error(MI355X_ERR_ARG, "NULL buffer");
    return sl->three(in1, in2, out, count, resolve_stream(stream));
}

} // extern "C"
