// coll_ll.hip -- low-latency one-shot collectives for small messages (see coll_internal.hpp).
//
// One launch per rank per call, one 256-thread block per 4 KiB slice of the message, no host
// barrier: the reference's recursive-doubling / small-ring region (coll_tuned_decision_fixed.c:
// 42-85) is latency-bound, and a host round trip (stream sync + shm barrier, tens of µs) costs more
// than the data movement.  Block b of every rank:
//   1. pushes slice b of its data into slot (parity, me) of every peer named in push_mask
//      (16-B stores over xGMI into the peer's uncached LL region),
//   2. after a system-scope release, raises flag (parity, me, b) = seq in EVERY peer -- the flag
//      is also the acknowledgement that makes the parity reusable two calls later,
//   3. waits until flag (parity, q, b) = seq for every q in its own region (bounded spin: after
//      ~10 s it records a timeout in the host-visible error word and gives up),
//   4. finishes locally from the slots: the reference schedule's per-element program over the n
//      inputs (allreduce; reduce: the root only, the others push to the root alone), or copies
//      (allgather / bcast).
// Slices are independent, so blocks never wait on each other.  The LL region is allocated with
// hipDeviceMallocUncached: remote xGMI writes do not update the owner's L2, so the flags and
// data a rank polls must never be cached there.
#include "coll_internal.hpp"
#include "op_functors.hpp"
#include "rt_internal.hpp"
#include "slot_list.hpp"

namespace mi355x {

typedef unsigned int u32x4l __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint64_t ll_flag_load(const uint64_t *p)
{
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void ll_flag_store(uint64_t *p, uint64_t v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// copy bytes [lo, hi) of src to dst (slot bases are 16-B aligned; user buffers may not be)
__device__ __forceinline__ void ll_copy_slice(char *dst, const char *src, size_t lo, size_t hi)
{
    const size_t t = threadIdx.x;
    if ((((uintptr_t)src | (uintptr_t)dst) & 15) == 0) {
        const size_t nv = (hi - lo) / 16;
        for (size_t v = t; v < nv; v += blockDim.x)
            *reinterpret_cast<u32x4l *>(dst + lo + v * 16) = *reinterpret_cast<const u32x4l *>(src + lo + v * 16);
        for (size_t k = lo + nv * 16 + t; k < hi; k += blockDim.x) dst[k] = src[k];
    } else {
        for (size_t k = lo + t; k < hi; k += blockDim.x) dst[k] = src[k];
    }
}

// steps 1-3; returns false on timeout
__device__ bool ll_exchange(const LLArgs &a)
{
    const unsigned b = blockIdx.x;
    const size_t lo = (size_t)b * kLLChunk;
    const size_t hi = lo + kLLChunk < a.nbytes ? lo + kLLChunk : a.nbytes;
    if (a.src) {
        const char *src = static_cast<const char *>(a.src);
        const size_t t = threadIdx.x;
        if (((uintptr_t)src & 15) == 0) {
            const size_t nv = (hi - lo) / 16;  // <= blockDim.x: one vector per thread
            if (t < nv) {
                const u32x4l v = *reinterpret_cast<const u32x4l *>(src + lo + t * 16);
                for (int q = 0; q < a.n; ++q)
                    if ((a.push_mask >> q) & 1u) *reinterpret_cast<u32x4l *>(a.peer_data[q] + lo + t * 16) = v;
            }
            for (size_t k = lo + nv * 16 + t; k < hi; k += blockDim.x)
                for (int q = 0; q < a.n; ++q)
                    if ((a.push_mask >> q) & 1u) a.peer_data[q][k] = src[k];
        } else {
            for (size_t k = lo + t; k < hi; k += blockDim.x) {
                const char v = src[k];
                for (int q = 0; q < a.n; ++q)
                    if ((a.push_mask >> q) & 1u) a.peer_data[q][k] = v;
            }
        }
    }
    __threadfence_system();
    __syncthreads();
    const int t = (int)threadIdx.x;
    if (t < a.n) ll_flag_store(a.peer_flag[t] + b, a.seq);
    __shared__ int timed_out;
    if (t == 0) timed_out = 0;
    __syncthreads();
    if (t < a.n) {
        const uint64_t *f = a.my_flag + (size_t)t * a.kmax + b;
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while (ll_flag_load(f) != a.seq) {
            __builtin_amdgcn_s_sleep(2);
            if (__builtin_amdgcn_s_memrealtime() - t0 > a.timeout_ticks) {
                __hip_atomic_store(a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                timed_out = 1;
                break;
            }
        }
    }
    __syncthreads();
    __threadfence_system();
    return timed_out == 0;
}

template <class F> __device__ __forceinline__ typename F::T ll_pick(const typename F::T (&R)[kTreeMax], int k)
{
    typename F::T v = R[0];
#pragma unroll
    for (int s = 1; s < kTreeMax; ++s)
        if (s == k) v = R[s];
    return v;
}

template <typename T> struct alignas(16) LLVec {
    T e[16 / sizeof(T)];
};

// per-element program (scalar); x(q) = rank q's element i
template <class F, class X> __device__ __forceinline__ typename F::T ll_eval(const LLArgs &a, size_t i, X x)
{
    using T = typename F::T;
    if (a.prog == LL_TREE) {
        T R[kTreeMax];
#pragma unroll
        for (int s = 0; s < kTreeMax; ++s)
            if (s < a.n) R[s] = x(s);
        for (int k = 0; k < a.nsteps; ++k) {
            const TreeStep st = a.steps[k];
            const T r = F::op2(ll_pick<F>(R, st.out), ll_pick<F>(R, st.in));
#pragma unroll
            for (int s = 0; s < kTreeMax; ++s)
                if (s == st.dst) R[s] = r;
        }
        return ll_pick<F>(R, a.result);
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
    T acc = x(rank_at(0));
    for (int j0 = 1; j0 < a.n; j0 += 8) {
        T v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if (j0 + j < a.n) v[j] = x(rank_at(j0 + j));
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if (j0 + j < a.n) acc = ((a.role_mask >> (j0 + j)) & 1u) ? F::op2(acc, v[j]) : F::op2(v[j], acc);
    }
    return acc;
}

// allreduce: exchange, then this slice from the n slots.  Thread t owns the slice's t-th 16-B
// vector; it loads that vector from every slot with all loads in flight at once (the slots are
// uncached, so one round of latency per thread instead of one per element).  A vector whose
// elements straddle two ring blocks (at most n - 1 in a message) is evaluated element-wise.
template <class F> __global__ __launch_bounds__(256) void k_ll_allreduce(LLArgs a)
{
    using T = typename F::T;
    using V = LLVec<T>;
    constexpr int EPV = 16 / sizeof(T);
    if (!ll_exchange(a)) return;
    if (a.mode == LL_RED && a.me != a.root) return;  // reduce: only the root evaluates
    const size_t i0 = ((size_t)blockIdx.x * kLLChunk + (size_t)threadIdx.x * 16) / sizeof(T);
    if (i0 >= a.count) return;
    const int ne = (a.count - i0) < (size_t)EPV ? (int)(a.count - i0) : EPV;
    T *dst = static_cast<T *>(a.dst);
    auto slot = [&](int q) { return reinterpret_cast<const T *>(a.my_data + (size_t)q * a.slot_bytes); };
    bool uniform = (ne == EPV) && a.n <= 8;
    if (uniform && a.prog == LL_RING) {
        const uint64_t se = a.split * a.early;
        auto blk = [&](size_t i) { return (i < se) ? i / a.early : a.split + (i - se) / a.late; };
        uniform = blk(i0) == blk(i0 + EPV - 1);
    }
    if (uniform) {
        V xv[8];
#pragma unroll
        for (int q = 0; q < 8; ++q)
            if (q < a.n) xv[q] = *reinterpret_cast<const V *>(slot(q) + i0);
        V r;
#pragma unroll
        for (int e = 0; e < EPV; ++e)
            r.e[e] = ll_eval<F>(a, i0 + e, [&](int q) {
                T v = xv[0].e[e];  // register select (no dynamic indexing into xv)
#pragma unroll
                for (int s2 = 1; s2 < 8; ++s2)
                    if (s2 == q) v = xv[s2].e[e];
                return v;
            });
        if ((((uintptr_t)(dst + i0)) & 15) == 0) {
            *reinterpret_cast<V *>(dst + i0) = r;
        } else {
#pragma unroll
            for (int e = 0; e < EPV; ++e) dst[i0 + e] = r.e[e];
        }
        return;
    }
    for (int e = 0; e < ne; ++e) {
        const size_t i = i0 + e;
        dst[i] = ll_eval<F>(a, i, [&](int q) { return slot(q)[i]; });
    }
}

// allgather (slot q -> dst + q*nbytes) and bcast (slot root -> dst, non-roots)
__global__ __launch_bounds__(256) void k_ll_copy(LLArgs a)
{
    if (!ll_exchange(a)) return;
    const size_t lo = (size_t)blockIdx.x * kLLChunk;
    const size_t hi = lo + kLLChunk < a.nbytes ? lo + kLLChunk : a.nbytes;
    char *dst = static_cast<char *>(a.dst);
    if (a.mode == LL_BC) {
        if (a.me != a.root) ll_copy_slice(dst, a.my_data + (size_t)a.root * a.slot_bytes, lo, hi);
        return;
    }
    for (int q = 0; q < a.n; ++q) {
        char *d = dst + (size_t)q * a.nbytes;
        if (q == a.me && static_cast<const char *>(a.src) == d) continue;  // in place
        ll_copy_slice(d, a.my_data + (size_t)q * a.slot_bytes, lo, hi);
    }
}

static unsigned ll_grid(const LLArgs &a) { return (unsigned)((a.nbytes + kLLChunk - 1) / kLLChunk); }

template <class F> static int launch_ll(const LLArgs &a, hipStream_t s)
{
    hipLaunchKernelGGL((k_ll_allreduce<F>), dim3(ll_grid(a)), dim3(256), 0, s, a);
    MI_HIP(hipGetLastError());
    return MI355X_SUCCESS;
}

int launch_ll_copy(const LLArgs &a, hipStream_t s)
{
    hipLaunchKernelGGL(k_ll_copy, dim3(ll_grid(a)), dim3(256), 0, s, a);
    MI_HIP(hipGetLastError());
    return MI355X_SUCCESS;
}

struct LLTable {
    int (*f[MI355X_OP_MAX_][MI355X_T_MAX])(const LLArgs &, hipStream_t) = {};
    LLTable()
    {
        for_each_slot([&](auto tag, int op, int ty) {
            using F = typename decltype(tag)::type;
            f[op][ty] = &launch_ll<F>;
        });
    }
};

int launch_ll_slot(int op, int type, const LLArgs &a, hipStream_t s)
{
    static const LLTable t;
    if (op < 0 || op >= MI355X_OP_MAX_ || type < 0 || type >= MI355X_T_MAX || !t.f[op][type])
        return set_error(MI355X_ERR_UNSUPPORTED, "no LL kernel for op %d type %d", op, type);
    return t.f[op][type](a, s);
}

} // namespace mi355x
