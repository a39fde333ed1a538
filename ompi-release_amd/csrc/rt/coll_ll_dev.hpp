// coll_ll_dev.hpp -- device side of the low-latency protocol (tagged 8-byte granules, see
// coll_ll.hip), shared by the per-call LL kernels and the resident service kernel (coll_svc.hip).
#pragma once

#include <type_traits>

#include "coll_internal.hpp"
#include "op_functors.hpp"
#include "rt_internal.hpp"

namespace mi355x {

typedef unsigned int u32x4l __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint64_t ll_load(const uint64_t *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void ll_store(uint64_t *p, uint64_t v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// SYS (the resident service, which has no kernel boundary between calls): the caller's input is
// read and the result written with the system-coherent cache policy (sc0 sc1, raw buffer ops) --
// loads skip this CU's L1, which may still hold the lines of an earlier call's input, and stores
// go through the XCD's L2 to memory, so the call's results need no L2 write-back fence.
// A buffer resource lives in scalar registers: it is built from a workgroup-uniform base (made
// scalar with readfirstlane -- the service keeps its arguments in LDS, where the compiler cannot
// see they are uniform; a per-lane base would compile to a loop over the wave's distinct values)
// and each lane passes its own byte offset.
constexpr int kLLSysCoherent = 1 | 16;  // gfx950 cache-policy bits: sc0 (1) | sc1 (16)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t ll_rsrc(const void *uniform_base)
{
    const uint64_t u = (uint64_t)(uintptr_t)uniform_base;
    const uint64_t s = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(u >> 32)) << 32) |
                       (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)u);
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(s), 0, 0x7fffffff, 0x00020000);
}

// up to 16 bytes at base + off (len valid bytes) as 4 little-endian words (zero padded); base is
// uniform across the workgroup
template <bool SYS = false>
__device__ __forceinline__ void ll_read16(const char *base, size_t off, size_t len, uint32_t w[4])
{
    const char *src = base + off;
    if constexpr (SYS) {
        const __amdgpu_buffer_rsrc_t rs = ll_rsrc(base);
        if (len == 16 && (((uintptr_t)src) & 15) == 0) {
            const u32x4l v = __builtin_amdgcn_raw_buffer_load_b128(rs, (unsigned)off, 0, kLLSysCoherent);
            w[0] = v.x, w[1] = v.y, w[2] = v.z, w[3] = v.w;
            return;
        }
        if ((((uintptr_t)src) & 3) == 0 && (len & 3) == 0) {  // whole words
#pragma unroll
            for (int i = 0; i < 4; ++i)
                w[i] = (size_t)(4 * i) < len ? __builtin_amdgcn_raw_buffer_load_b32(rs, (unsigned)(off + 4 * i), 0, kLLSysCoherent) : 0;
            return;
        }
        unsigned char b[16];
#pragma unroll
        for (int i = 0; i < 16; ++i)
            b[i] = (size_t)i < len ? __builtin_amdgcn_raw_buffer_load_b8(rs, (unsigned)(off + i), 0, kLLSysCoherent) : 0;
        __builtin_memcpy(w, b, 16);
        return;
    }
    if (len == 16 && (((uintptr_t)src) & 15) == 0) {
        const u32x4l v = *reinterpret_cast<const u32x4l *>(src);
        w[0] = v.x, w[1] = v.y, w[2] = v.z, w[3] = v.w;
        return;
    }
    unsigned char b[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) b[i] = (size_t)i < len ? (unsigned char)src[i] : 0;
    __builtin_memcpy(w, b, 16);
}
template <bool SYS = false>
__device__ __forceinline__ void ll_write16(char *base, size_t off, size_t len, const uint32_t w[4])
{
    char *dst = base + off;
    if constexpr (SYS) {
        const __amdgpu_buffer_rsrc_t rs = ll_rsrc(base);
        if (len == 16 && (((uintptr_t)dst) & 15) == 0) {
            u32x4l v;
            v.x = w[0], v.y = w[1], v.z = w[2], v.w = w[3];
            __builtin_amdgcn_raw_buffer_store_b128(v, rs, (unsigned)off, 0, kLLSysCoherent);
            return;
        }
        if ((((uintptr_t)dst) & 3) == 0 && (len & 3) == 0) {  // whole words (4- / 8-B elements)
            for (size_t i = 0; i < len / 4; ++i)
                __builtin_amdgcn_raw_buffer_store_b32(w[i], rs, (unsigned)(off + 4 * i), 0, kLLSysCoherent);
            return;
        }
        // (bytes taken from the words by shifts, unrolled: an indexed byte array would live in scratch)
#pragma unroll
        for (int i = 0; i < 16; ++i)
            if ((size_t)i < len)
                __builtin_amdgcn_raw_buffer_store_b8((unsigned char)(w[i >> 2] >> (8 * (i & 3))), rs, (unsigned)(off + i), 0,
                                                     kLLSysCoherent);
        return;
    }
    if (len == 16 && (((uintptr_t)dst) & 15) == 0) {
        u32x4l v;
        v.x = w[0], v.y = w[1], v.z = w[2], v.w = w[3];
        *reinterpret_cast<u32x4l *>(dst) = v;
        return;
    }
    unsigned char b[16];
    __builtin_memcpy(b, w, 16);
    for (size_t i = 0; i < len; ++i) dst[i] = (char)b[i];
}

struct LLBlock {
    size_t lo, off, len;   // block payload start; this thread's 16-B chunk offset / valid bytes
    int ngran;             // granules of this thread (0: past the end)
    uint32_t tag;
};

// thread `tid`'s 16 B of the 4 KiB slice `chunk` of the call (the per-call kernels: chunk =
// blockIdx.x, tid = threadIdx.x)
__device__ __forceinline__ LLBlock ll_block(const LLArgs &a, size_t chunk, unsigned tid = threadIdx.x)
{
    LLBlock k;
    k.lo = chunk * kLLChunk;
    k.off = k.lo + (size_t)tid * 16;
    k.len = k.off < a.nbytes ? (a.nbytes - k.off < 16 ? a.nbytes - k.off : 16) : 0;
    k.ngran = (int)((k.len + 3) / 4);
    k.tag = (uint32_t)a.seq;
    return k;
}

// step 1: every peer this rank pushes to has acknowledged the call two calls back; false on
// timeout (the error word is set).  Every thread of the workgroup calls it.
static __device__ bool ll_wait_acks(const LLArgs &a)
{
    __shared__ int timed_out;
    const int t = (int)threadIdx.x;
    if (t == 0) timed_out = 0;
    __syncthreads();
    if (a.src && t < a.n && t != a.me && ((a.push_mask >> t) & 1u) && a.seq > 2) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        unsigned spins = 0;
        while (ll_load(a.my_ack + t) + 2 < a.seq) {
            __builtin_amdgcn_s_sleep(1);
            if (__builtin_amdgcn_s_memrealtime() - t0 > a.timeout_ticks) {
                __hip_atomic_store(a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                timed_out = 1;
                break;
            }
            // the call failed elsewhere, or the host gave up on a peer that is gone (ll_err_set)
            if ((++spins & 255u) == 0 && __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) {
                timed_out = 1;
                break;
            }
        }
    }
    __syncthreads();
    return !timed_out;
}

// this thread's 16 B of slice k (read with ll_read16<SYS>)
template <bool SYS = false> __device__ __forceinline__ void ll_read_slice(const LLArgs &a, const LLBlock &k, uint32_t w[4])
{
    w[0] = w[1] = w[2] = w[3] = 0;
    if (a.src && k.ngran) ll_read16<SYS>(static_cast<const char *>(a.src), k.off, k.len, w);
}

// step 2: the 16 B as granules into slot (parity, me) of every peer in push_mask
__device__ __forceinline__ void ll_push_slice(const LLArgs &a, const LLBlock &k, const uint32_t w[4])
{
    if (!a.src || !k.ngran) return;  // (bcast: only the root has data to push)
    const size_t g0 = k.off / 4;
    for (int q = 0; q < a.n; ++q) {
        if (!((a.push_mask >> q) & 1u)) continue;
        uint64_t *d = a.peer_data[q] + g0;
        if (k.ngran == 4) {
            // two granules per 16-B store (32-B aligned: g0 is a multiple of 4); each 8-B half
            // carries its own tag, so a store seen half-landed is only partly accepted
            const __amdgpu_buffer_rsrc_t rs = ll_rsrc(a.peer_data[q]);
            const unsigned o = (unsigned)(g0 * 8);
            __builtin_amdgcn_raw_buffer_store_b128(u32x4l{w[0], k.tag, w[1], k.tag}, rs, o, 0, kLLSysCoherent);
            __builtin_amdgcn_raw_buffer_store_b128(u32x4l{w[2], k.tag, w[3], k.tag}, rs, o + 16, 0, kLLSysCoherent);
            continue;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (i < k.ngran) ll_store(d + i, ((uint64_t)k.tag << 32) | w[i]);
    }
}

// steps 1-2 for one slice (the input read is issued before the acknowledgement wait); false on timeout
template <bool SYS = false> static __device__ bool ll_push(const LLArgs &a, const LLBlock &k)
{
    uint32_t w[4];
    ll_read_slice<SYS>(a, k, w);
    if (!ll_wait_acks(a)) return false;
    ll_push_slice(a, k, w);
    return true;
}

// step 3 for the sources in qmask (<= 8 of them, slot index = rank): w[q] gets rank q's 16 B.
// Granules are read in pairs (16-B loads: {payload, tag, payload, tag}), each half checked.
static __device__ bool ll_recv(const LLArgs &a, const LLBlock &k, uint64_t qmask, uint32_t (&w)[8][4])
{
    if (!k.ngran) return true;
    const size_t g0 = k.off / 4;
    const int npair = (k.ngran + 1) / 2;  // pairs holding this thread's granules
    auto load_pair = [&](int q, int h) {
        // (a pair past ngran: the slot holds it, so the read stays inside the region)
        const u32x4l v = __builtin_amdgcn_raw_buffer_load_b128(ll_rsrc(a.my_data + (size_t)q * a.slot_gran),
                                                               (unsigned)(g0 * 8 + 16 * h), 0, kLLSysCoherent);
        w[q][2 * h] = v.x;
        w[q][2 * h + 1] = v.z;
        const bool lo = v.y == k.tag, hi = v.w == k.tag || 2 * h + 1 >= k.ngran;
        return lo && hi;
    };
    uint32_t pending = 0;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        if (!((qmask >> q) & 1u)) continue;
#pragma unroll
        for (int h = 0; h < 2; ++h)
            if (h < npair && !load_pair(q, h)) pending |= 1u << (q * 2 + h);
    }
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    unsigned spins = 0;
    while (pending) {
        __builtin_amdgcn_s_sleep(1);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
#pragma unroll
            for (int h = 0; h < 2; ++h)
                if (((pending >> (q * 2 + h)) & 1u) && load_pair(q, h)) pending &= ~(1u << (q * 2 + h));
        }
        if ((++spins & 255u) == 0) {
            if (__builtin_amdgcn_s_memrealtime() - t0 > a.timeout_ticks) {
                __hip_atomic_store(a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                return false;
            }
            if (__hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) return false;  // (as above)
        }
    }
    return true;
}

// step 5: after every thread of the block is done with its slots
static __device__ void ll_done(const LLArgs &a)
{
    __syncthreads();
    if (threadIdx.x != 0) return;
    const uint64_t old = __hip_atomic_fetch_add(a.ctr, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old + 1 != a.ctr_target) return;
    for (int q = 0; q < a.n; ++q)
        if (q != a.me) ll_store(a.peer_ack[q], a.seq);
}

template <typename T> struct alignas(16) LLVec {
    T e[16 / sizeof(T)];
};

// One element's value on every rank, indexed by rank at run time (tree programs, ring orders).
// An array here ends up a dynamically indexed stack slot -- the compiler folds the select chains
// back into indexed loads -- so every pick is a scratch round trip on the service's latency path
// (~1.6 us of an 8-B call).  Arithmetic types are kept in one vector register tuple instead,
// indexed in place; other element types (complex, value-index pairs) keep the array.
template <typename T, bool kVec = (std::is_integral<T>::value || std::is_floating_point<T>::value) &&
                                  !std::is_same<T, bool>::value>
struct RankRegs {
    T r[kLLMaxRanks];
    __device__ __forceinline__ T get(int k) const
    {
        T v = r[0];
#pragma unroll
        for (int s = 1; s < kLLMaxRanks; ++s)
            if (s == k) v = r[s];
        return v;
    }
    __device__ __forceinline__ void set(int k, T x)
    {
#pragma unroll
        for (int s = 0; s < kLLMaxRanks; ++s)
            if (s == k) r[s] = x;
    }
};
template <typename T> struct RankRegs<T, true> {
    typedef T V __attribute__((ext_vector_type(kLLMaxRanks)));
    V r;
    __device__ __forceinline__ T get(int k) const { return r[k]; }
    __device__ __forceinline__ void set(int k, T x) { r[k] = x; }
};

// per-element program (scalar); X = every rank's element i
template <class F> __device__ __forceinline__ typename F::T ll_eval(const LLArgs &a, size_t i, const RankRegs<typename F::T> &X)
{
    using T = typename F::T;
    if (a.prog == LL_TREE) {
        // (LL calls have <= kLLMaxRanks ranks: the program's registers are the ranks' values)
        RankRegs<T> R = X;
        for (int k = 0; k < a.nsteps; ++k) {
            const TreeStep st = a.steps[k];
            R.set(st.dst, F::op2(R.get(st.out), R.get(st.in)));
        }
        return R.get(a.result);
    }
    // left fold; LL_RING: the order starts at the element's ring block
    // (coll_tuned_allreduce.c:470-512: the partial is the `in` operand at every step)
    int b0 = 0;
    if (a.prog == LL_RING) {
        const uint64_t se = a.split * a.early;
        b0 = (i < se) ? (int)(i / a.early) : (int)(a.split + (i - se) / a.late);
    }
    auto rank_at = [&](int j) -> int {
        if (a.prog == LL_RING) {
            const int r = b0 + j;
            return r >= a.n ? r - a.n : r;
        }
        return a.order[j];
    };
    T acc = X.get(rank_at(0));
    for (int j = 1; j < a.n; ++j) {
        const T v = X.get(rank_at(j));
        acc = ((a.role_mask >> j) & 1u) ? F::op2(acc, v) : F::op2(v, acc);
    }
    return acc;
}

// allreduce / reduce: this thread's 16 B of the result from the n inputs held in registers
// (<= 8 ranks: ll_usable); w[q] = rank q's 16 B
template <class F, bool SYS = false>
__device__ __forceinline__ void ll_reduce_out(const LLArgs &a, const LLBlock &k, const uint32_t (&w)[8][4])
{
    using T = typename F::T;
    using V = LLVec<T>;
    constexpr int EPV = 16 / sizeof(T);
    V xv[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) __builtin_memcpy(&xv[q], w[q], 16);
    const size_t i0 = k.off / sizeof(T);
    const int ne = (int)(k.len / sizeof(T));
    V r;
#pragma unroll
    for (int e = 0; e < EPV; ++e) {
        if (e >= ne) continue;
        RankRegs<T> X;
#pragma unroll
        for (int q = 0; q < kLLMaxRanks; ++q) X.set(q, xv[q].e[e]);
        r.e[e] = ll_eval<F>(a, i0 + e, X);
    }
    uint32_t ow[4];
    __builtin_memcpy(ow, &r, 16);
    ll_write16<SYS>(static_cast<char *>(a.dst), k.off, k.len, ow);
}

// allgather (slot q -> dst + q*nbytes) and bcast (slot root -> dst, non-roots)
template <bool SYS = false>
__device__ __forceinline__ void ll_copy_out(const LLArgs &a, const LLBlock &k, const uint32_t (&w)[8][4])
{
    char *dst = static_cast<char *>(a.dst);
    if (a.mode == LL_BC) {
        uint32_t v[4];
#pragma unroll
        for (int q = 0; q < 8; ++q)
            if (q == a.root) __builtin_memcpy(v, w[q], 16);
        ll_write16<SYS>(dst, k.off, k.len, v);
    } else {
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            if (!((a.recv_mask >> q) & 1u)) continue;
            char *d = dst + (size_t)q * a.nbytes;
            if (q == a.me && static_cast<const char *>(a.src) == d) continue;  // in place
            ll_write16<SYS>(d, k.off, k.len, w[q]);
        }
    }
}

} // namespace mi355x
