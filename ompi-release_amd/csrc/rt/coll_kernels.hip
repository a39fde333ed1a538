// coll_kernels.hip -- device side of coll/mi355x: one launch per rank per collective step that
// reads the ranks' inputs directly from IPC-mapped peer HBM over xGMI, folds them in the exact
// operand order of the reference schedule, and writes (pushes) the result into every
// destination -- local rbuf and/or the peers' rbufs.
//
// Three kernel families, instantiated per (MPI_Op, type) slot through the op functors:
//   k_fold  : acc = x[order[0]]; for j >= 1: acc = role[j] ? op2(out=acc, in=x[order[j]])
//                                                        : op2(out=x[order[j]], in=acc)
//             -- the ring / segmented-ring allreduce order (coll_tuned_allreduce.c:470-512,
//             acc is `in`), the pipeline / chain / linear reduce order (coll_tuned_reduce.c:
//             177-222, 687-703, acc is `out`), the ring reduce_scatter order.
//             All NR <= 8 loads of a vector are issued before the first op (one 16-B load per
//             rank per vector, U vectors in flight); ranks beyond 8 are folded in chunks,
//             which keeps the left-fold order.
//   k_tree  : a register program R[dst] = op2(out=R[o], in=R[i]) over <= 16 rank inputs --
//             the recursive-doubling butterfly (:193-284), binomial / binary reduce trees.
//   k_copy  : no arithmetic (allgather, bcast slices): one source, many destinations.
// Source/destination pointers arrive in the kernarg segment (uniform, scalar-loaded), so the
// per-rank indirection costs no VGPRs.  Same alignment scheme as op_kernels.hip: if every
// pointer shares the misalignment mod 16 a scalar head peels to the 16-B body, else the whole
// range runs element-wise.
#include "coll_internal.hpp"
#include "op_functors.hpp"
#include "rt_internal.hpp"
#include "slot_list.hpp"

namespace mi355x {

typedef unsigned int u32x4c __attribute__((ext_vector_type(4)));

template <typename T> struct alignas(16) CVec {
    T e[16 / sizeof(T)];
};

template <typename V> __device__ __forceinline__ V cload(const void *p)
{
    u32x4c raw = *reinterpret_cast<const u32x4c *>(p);
    V v;
    __builtin_memcpy(&v, &raw, 16);
    return v;
}
template <typename V> __device__ __forceinline__ void cstore(void *p, const V &v)
{
    u32x4c raw;
    __builtin_memcpy(&raw, &v, 16);
    *reinterpret_cast<u32x4c *>(p) = raw;
}
// non-temporal forms: streams larger than the Infinity Cache (same policy as op_kernels.hip)
template <bool NT, typename V> __device__ __forceinline__ V cload_t(const void *p)
{
    if constexpr (!NT) return cload<V>(p);
    u32x4c raw = __builtin_nontemporal_load(reinterpret_cast<const u32x4c *>(p));
    V v;
    __builtin_memcpy(&v, &raw, 16);
    return v;
}
template <bool NT, typename V> __device__ __forceinline__ void cstore_t(void *p, const V &v)
{
    if constexpr (!NT) {
        cstore<V>(p, v);
    } else {
        u32x4c raw;
        __builtin_memcpy(&raw, &v, 16);
        __builtin_nontemporal_store(raw, reinterpret_cast<u32x4c *>(p));
    }
}

// ------------------------------------------------------------------ fold
template <class F>
__device__ __forceinline__ typename F::T fold_step(const typename F::T &acc, const typename F::T &x,
                                                   bool acc_is_out)
{
    return acc_is_out ? F::op2(acc, x) : F::op2(x, acc);
}

// fold of element i (scalar path)
template <class F>
__device__ __forceinline__ typename F::T fold_scalar(const FoldArgs &a, size_t i)
{
    using T = typename F::T;
    T acc = static_cast<const T *>(a.src[a.order[0]])[i];
    for (int j = 1; j < a.nr; ++j) {
        const T x = static_cast<const T *>(a.src[a.order[j]])[i];
        acc = fold_step<F>(acc, x, (a.role_mask >> j) & 1u);
    }
    return acc;
}

template <class F, int U, bool NT>
__global__ __launch_bounds__(256) void k_fold(FoldArgs a)
{
    using T = typename F::T;
    using V = CVec<T>;
    constexpr int EPV = 16 / sizeof(T);
    const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t nthr = (size_t)gridDim.x * blockDim.x;

    for (size_t i = tid; i < a.head; i += nthr) {
        const T r = fold_scalar<F>(a, i);
        for (int d = 0; d < a.nd; ++d) static_cast<T *>(a.dst[d])[i] = r;
    }

    const size_t nvec = a.nvec;
    const size_t hb = a.head * sizeof(T);
    for (size_t base = tid; base < nvec; base += nthr * U) {
        V acc[U];
        // first chunk of up to 8 ranks: issue every load, then fold
        {
            V x[kFoldChunk][U];
#pragma unroll
            for (int j = 0; j < kFoldChunk; ++j) {
                if (j < a.nr) {
                    const char *p = static_cast<const char *>(a.src[a.order[j]]) + hb;
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const size_t v = base + (size_t)u * nthr;
                        if (v < nvec) x[j][u] = cload_t<NT, V>(p + v * 16);
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) acc[u] = x[0][u];
#pragma unroll
            for (int j = 1; j < kFoldChunk; ++j) {
                if (j < a.nr) {
                    const bool ao = (a.role_mask >> j) & 1u;
#pragma unroll
                    for (int u = 0; u < U; ++u)
#pragma unroll
                        for (int e = 0; e < EPV; ++e) acc[u].e[e] = fold_step<F>(acc[u].e[e], x[j][u].e[e], ao);
                }
            }
        }
        // remaining ranks (communicators larger than 8), chunk by chunk, order preserved
        for (int j0 = kFoldChunk; j0 < a.nr; j0 += kFoldChunk) {
            V x[kFoldChunk][U];
#pragma unroll
            for (int j = 0; j < kFoldChunk; ++j) {
                if (j0 + j < a.nr) {
                    const char *p = static_cast<const char *>(a.src[a.order[j0 + j]]) + hb;
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const size_t v = base + (size_t)u * nthr;
                        if (v < nvec) x[j][u] = cload_t<NT, V>(p + v * 16);
                    }
                }
            }
#pragma unroll
            for (int j = 0; j < kFoldChunk; ++j) {
                if (j0 + j < a.nr) {
                    const bool ao = (a.role_mask >> (j0 + j)) & 1u;
#pragma unroll
                    for (int u = 0; u < U; ++u)
#pragma unroll
                        for (int e = 0; e < EPV; ++e) acc[u].e[e] = fold_step<F>(acc[u].e[e], x[j][u].e[e], ao);
                }
            }
        }
        for (int d = 0; d < a.nd; ++d) {
            char *q = static_cast<char *>(a.dst[d]) + hb;
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const size_t v = base + (size_t)u * nthr;
                if (v < nvec) cstore_t<NT, V>(q + v * 16, acc[u]);
            }
        }
    }

    const size_t t0 = a.head + nvec * EPV;
    for (size_t i = t0 + tid; i < a.n; i += nthr) {
        const T r = fold_scalar<F>(a, i);
        for (int d = 0; d < a.nd; ++d) static_cast<T *>(a.dst[d])[i] = r;
    }
}

// ------------------------------------------------------------------ ring order, whole vector
// Small ring-ordered messages: every rank evaluates every block (one element per lane, the n loads
// issued before the fold), so the allreduce needs one launch and one host barrier instead of two.
template <class F> __global__ __launch_bounds__(256) void k_ring_all(RingAllArgs a)
{
    using T = typename F::T;
    const uint32_t se = a.split * a.early;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < a.count; i += gridDim.x * blockDim.x) {
        const int b = (int)(i < se ? i / a.early : a.split + (i - se) / a.late);
        T acc{};
        for (int j0 = 0; j0 < a.n; j0 += kFoldChunk) {  // up to 8 loads in flight, then fold them
            T x[kFoldChunk];
#pragma unroll
            for (int j = 0; j < kFoldChunk; ++j) {
                const int jj = j0 + j, r = b + jj < a.n ? b + jj : b + jj - a.n;
                if (jj < a.n) x[j] = static_cast<const T *>(a.src[r])[i];
            }
#pragma unroll
            for (int j = 0; j < kFoldChunk; ++j) {
                if (j0 + j < a.n) acc = (j0 + j == 0) ? x[0] : F::op2(x[j], acc);
            }
        }
        static_cast<T *>(a.dst)[i] = acc;
    }
}

// ------------------------------------------------------------------ tree program
template <class F>
__device__ __forceinline__ typename F::T pick(const typename F::T (&R)[kTreeMax], int k)
{
    typename F::T v = R[0];
#pragma unroll
    for (int s = 1; s < kTreeMax; ++s)
        if (s == k) v = R[s];
    return v;
}

template <class F> __global__ __launch_bounds__(256) void k_tree(TreeArgs a)
{
    using T = typename F::T;
    const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t nthr = (size_t)gridDim.x * blockDim.x;
    for (size_t i = tid; i < a.n; i += nthr) {
        T R[kTreeMax];
#pragma unroll
        for (int s = 0; s < kTreeMax; ++s)
            if (s < a.nr) R[s] = static_cast<const T *>(a.src[s])[i];
        for (int k = 0; k < a.nsteps; ++k) {
            const TreeStep st = a.steps[k];
            const T r = F::op2(pick<F>(R, st.out), pick<F>(R, st.in));
#pragma unroll
            for (int s = 0; s < kTreeMax; ++s)
                if (s == st.dst) R[s] = r;
        }
        const T res = pick<F>(R, a.result);
        for (int d = 0; d < a.nd; ++d) static_cast<T *>(a.dst[d])[i] = res;
    }
}

// ------------------------------------------------------------------ copy (no arithmetic)
__global__ __launch_bounds__(256) void k_copy(CopyArgs a)
{
    const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t nthr = (size_t)gridDim.x * blockDim.x;
    const char *s = static_cast<const char *>(a.src);
    for (size_t i = tid; i < a.head; i += nthr)
        for (int d = 0; d < a.nd; ++d) static_cast<char *>(a.dst[d])[i] = s[i];
    const size_t nvec = a.nvec;
    constexpr int U = 4;
    for (size_t base = tid; base < nvec; base += nthr * U) {
        u32x4c x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t v = base + (size_t)u * nthr;
            if (v < nvec) x[u] = *reinterpret_cast<const u32x4c *>(s + a.head + v * 16);
        }
        for (int d = 0; d < a.nd; ++d) {
            char *q = static_cast<char *>(a.dst[d]) + a.head;
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const size_t v = base + (size_t)u * nthr;
                if (v < nvec) *reinterpret_cast<u32x4c *>(q + v * 16) = x[u];
            }
        }
    }
    for (size_t i = a.head + nvec * 16 + tid; i < a.n; i += nthr)
        for (int d = 0; d < a.nd; ++d) static_cast<char *>(a.dst[d])[i] = s[i];
}

// ------------------------------------------------------------------ multi-segment copy
template <bool NT> __global__ __launch_bounds__(256) void k_multicopy(MultiCopyArgs a)
{
    // find this block's segment (<= 64 segments, uniform per block)
    int sgi = 0;
    while (sgi + 1 < a.nseg && blockIdx.x >= a.first_block[sgi + 1]) ++sgi;
    const unsigned nb = a.first_block[sgi + 1] - a.first_block[sgi];
    const unsigned b = blockIdx.x - a.first_block[sgi];
    const char *s = static_cast<const char *>(a.src[sgi]);
    char *d = static_cast<char *>(a.dst[sgi]);
    const size_t n = a.len[sgi];
    const size_t tid = (size_t)b * blockDim.x + threadIdx.x;
    const size_t nthr = (size_t)nb * blockDim.x;
    const uintptr_t ms = (uintptr_t)s & 15, md = (uintptr_t)d & 15;
    size_t head = n, nvec = 0;
    if (ms == md) {
        head = ms ? 16 - ms : 0;
        if (head > n) head = n;
        nvec = (n - head) / 16;
    }
    for (size_t i = tid; i < head; i += nthr) d[i] = s[i];
    constexpr int U = 4;
    for (size_t base = tid; base < nvec; base += nthr * U) {
        u32x4c x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t v = base + (size_t)u * nthr;
            if (v < nvec) x[u] = cload_t<NT, u32x4c>(s + head + v * 16);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t v = base + (size_t)u * nthr;
            if (v < nvec) cstore_t<NT, u32x4c>(d + head + v * 16, x[u]);
        }
    }
    for (size_t i = head + nvec * 16 + tid; i < n; i += nthr) d[i] = s[i];
}

// ------------------------------------------------------------------ launchers
static size_t grid_for(size_t work, int blocks_per_cu)
{
    size_t blocks = (work + 255) / 256;
    const size_t cap = (size_t)blocks_per_cu * (size_t)device_cu_count();
    if (blocks > cap) blocks = cap;
    return blocks ? blocks : 1;
}

template <class F> static int launch_fold(FoldArgs a, hipStream_t s)
{
    using T = typename F::T;
    constexpr size_t EPV = 16 / sizeof(T);
    if (a.n == 0) return MI355X_SUCCESS;
    uintptr_t m = (uintptr_t)a.src[a.order[0]] & 15;
    bool co = (m % sizeof(T)) == 0;
    for (int j = 0; j < a.nr && co; ++j) co = (((uintptr_t)a.src[j]) & 15) == m;
    for (int d = 0; d < a.nd && co; ++d) co = (((uintptr_t)a.dst[d]) & 15) == m;
    if (co) {
        size_t head = m ? (16 - m) / sizeof(T) : 0;
        if (head > a.n) head = a.n;
        a.head = head;
        a.nvec = (a.n - head) / EPV;
    } else {
        a.head = a.n;
        a.nvec = 0;
    }
    constexpr int U = 2;
    size_t work = a.nvec ? (a.nvec + U - 1) / U : 0;
    const size_t scalar = a.n - a.nvec * EPV;
    if (scalar > work) work = scalar;
    const size_t blocks = grid_for(work, coll_tune().blocks_per_cu);
    if ((size_t)(a.nr + a.nd) * a.n * sizeof(T) > ((size_t)256 << 20))
        hipLaunchKernelGGL((k_fold<F, U, true>), dim3((unsigned)blocks), dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL((k_fold<F, U, false>), dim3((unsigned)blocks), dim3(256), 0, s, a);
    MI_HIP(hipGetLastError());
    return MI355X_SUCCESS;
}

template <class F> static int launch_ring_all(const RingAllArgs &a, hipStream_t s)
{
    if (a.count == 0) return MI355X_SUCCESS;
    hipLaunchKernelGGL((k_ring_all<F>), dim3((unsigned)grid_for(a.count, 8)), dim3(256), 0, s, a);
    MI_HIP(hipGetLastError());
    return MI355X_SUCCESS;
}

template <class F> static int launch_tree(const TreeArgs &a, hipStream_t s)
{
    if (a.n == 0) return MI355X_SUCCESS;
    const size_t blocks = grid_for(a.n, 4);
    hipLaunchKernelGGL((k_tree<F>), dim3((unsigned)blocks), dim3(256), 0, s, a);
    MI_HIP(hipGetLastError());
    return MI355X_SUCCESS;
}

int launch_copy(CopyArgs a, hipStream_t s)
{
    if (a.n == 0) return MI355X_SUCCESS;
    uintptr_t m = (uintptr_t)a.src & 15;
    bool co = true;
    for (int d = 0; d < a.nd && co; ++d) co = (((uintptr_t)a.dst[d]) & 15) == m;
    if (co) {
        size_t head = m ? 16 - m : 0;
        if (head > a.n) head = a.n;
        a.head = head;
        a.nvec = (a.n - head) / 16;
    } else {
        a.head = a.n;
        a.nvec = 0;
    }
    size_t work = a.nvec ? (a.nvec + 3) / 4 : a.n;
    const size_t blocks = grid_for(work, coll_tune().blocks_per_cu);
    hipLaunchKernelGGL(k_copy, dim3((unsigned)blocks), dim3(256), 0, s, a);
    MI_HIP(hipGetLastError());
    return MI355X_SUCCESS;
}

int launch_multicopy(MultiCopyArgs a, hipStream_t s)
{
    size_t total = 0;
    for (int i = 0; i < a.nseg; ++i) total += a.len[i];
    if (total == 0) return MI355X_SUCCESS;
    // copy_block_kib per block (default 4 KiB: one 16-B vector per lane); at most
    // blocks_per_cu x CUs blocks overall (beyond that the blocks loop)
    const size_t cap = (size_t)coll_tune().blocks_per_cu * (size_t)device_cu_count();
    unsigned next = 0;
    for (int i = 0; i < a.nseg; ++i) {
        a.first_block[i] = next;
        const size_t cb = (size_t)coll_tune().copy_block_kib << 10;
        size_t want = (a.len[i] + cb - 1) / cb;
        size_t share = total ? (cap * a.len[i] + total - 1) / total : 1;
        size_t nb = want < share ? want : share;
        if (a.len[i] && nb == 0) nb = 1;
        next += (unsigned)nb;
    }
    a.first_block[a.nseg] = next;
    if (next == 0) return MI355X_SUCCESS;
    if (2 * total > ((size_t)256 << 20))
        hipLaunchKernelGGL(k_multicopy<true>, dim3(next), dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL(k_multicopy<false>, dim3(next), dim3(256), 0, s, a);
    MI_HIP(hipGetLastError());
    return MI355X_SUCCESS;
}

// dispatch table (same slot set as op_kernels.hip)
struct CollSlot {
    int (*fold)(FoldArgs, hipStream_t) = nullptr;
    int (*tree)(const TreeArgs &, hipStream_t) = nullptr;
    int (*ring_all)(const RingAllArgs &, hipStream_t) = nullptr;
};

struct CollTable {
    CollSlot s[MI355X_OP_MAX_][MI355X_T_MAX];
    CollTable()
    {
        for_each_slot([&](auto tag, int op, int ty) {
            using F = typename decltype(tag)::type;
            s[op][ty].fold = &launch_fold<F>;
            s[op][ty].tree = &launch_tree<F>;
            s[op][ty].ring_all = &launch_ring_all<F>;
        });
    }
};

static const CollSlot *cslot(int op, int type)
{
    static const CollTable t;
    if (op < 0 || op >= MI355X_OP_MAX_ || type < 0 || type >= MI355X_T_MAX) return nullptr;
    const CollSlot *s = &t.s[op][type];
    return s->fold ? s : nullptr;
}

int launch_fold_slot(int op, int type, const FoldArgs &a, hipStream_t s)
{
    const CollSlot *sl = cslot(op, type);
    if (!sl) return set_error(MI355X_ERR_UNSUPPORTED, "no device fold for op %d type %d", op, type);
    return sl->fold(a, s);
}

int launch_ring_all_slot(int op, int type, const RingAllArgs &a, hipStream_t s)
{
    const CollSlot *sl = cslot(op, type);
    if (!sl) return set_error(MI355X_ERR_UNSUPPORTED, "no device ring fold for op %d type %d", op, type);
    return sl->ring_all(a, s);
}

int launch_tree_slot(int op, int type, const TreeArgs &a, hipStream_t s)
{
    const CollSlot *sl = cslot(op, type);
    if (!sl) return set_error(MI355X_ERR_UNSUPPORTED, "no device tree for op %d type %d", op, type);
    return sl->tree(a, s);
}

bool coll_slot_supported(int op, int type) { return cslot(op, type) != nullptr; }

} // namespace mi355x

// every op/hip slot: the fold families' (slot_list.hpp) directly, the others gather-then-fold (coll_gfold.cpp)
extern "C" int mi355x_comm_op_supported(int op, int type) { return mi355x_op_supported(op, type); }
