// coll_pipe.hip -- pipelined allreduce: the reduce (owner folds its ring block) and the copy
// (every rank pulls the other blocks) of one MPI_Allreduce in ONE launch per rank, overlapped
// chunk by chunk with device-side readiness flags instead of a host barrier between them.
//
// The reference overlaps the receive of segment k+1 with the reduction of segment k inside the
// segmented ring (coll_tuned_allreduce.c:721-831: irecv into inbuf[inbi ^ 1] while
// ompi_op_reduce runs on inbuf[inbi]).  MI355X-first the same overlap is a work queue:
//   * the owner-computes partition is the reference's ring block partition
//     (COLL_TUNED_COMPUTE_BLOCKCOUNT, coll_tuned.h:546-552): rank r folds block r from every
//     rank's input in the ring's per-element order (ring_block_program), so the bits equal the
//     reference's whichever chunking is used;
//   * every block is cut into C chunks; items 0..C-1 fold my block's chunks, items C..C*n-1 pull
//     chunk k of peer q's block out of q's rbuf (ordered by chunk, then peer).  Workgroups take
//     items from a device counter (one returning atomic per item), so a pull is only ever taken
//     after every fold item has been taken by a running workgroup: folds never wait, hence the
//     queue drains on every rank whatever the dispatch order or the number of co-resident
//     workgroups (no grid barrier, no residency assumption);
//   * a fold item publishes chunk k: every storing wave drains its stores (s_waitcnt vmcnt(0)),
//     workgroup barrier, one lane releases at SYSTEM scope (writes the XCD's L2 back to HBM: a
//     peer reading over xGMI does not probe our L2) and stores `seq` into flag (me, k) of every
//     peer's uncached flag region over xGMI;
//   * a pull item polls its own uncached flag (q, k) from one lane (s_sleep between polls,
//     bounded by a deadline: on timeout the host-visible error word is set and every later wait
//     gives up at once), acquires at system scope (drops stale lines of peer memory from this
//     XCD's caches), then the workgroup copies the chunk with 16-B vectors.
// Flags carry the call number and are compared with >=, so no reset between calls: a flag of
// call s+1 can only be raised after every rank left call s (host barrier at the end of a call).
#include "coll_internal.hpp"
#include "op_functors.hpp"
#include "rt_internal.hpp"
#include "slot_list.hpp"

namespace mi355x {

typedef unsigned int u32x4p __attribute__((ext_vector_type(4)));

template <typename T> struct alignas(16) PVec {
    T e[16 / sizeof(T)];
};

template <bool NT> __device__ __forceinline__ u32x4p pload(const void *p)
{
    if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const u32x4p *>(p));
    return *reinterpret_cast<const u32x4p *>(p);
}
template <bool NT> __device__ __forceinline__ void pstore(void *p, const u32x4p &v)
{
    if constexpr (NT) __builtin_nontemporal_store(v, reinterpret_cast<u32x4p *>(p));
    else *reinterpret_cast<u32x4p *>(p) = v;
}

// write-through publishing (MI355X_KNOB_PIPE_WT): fold results stored with the system-coherent
// cache policy (sc0 sc1: through the XCD's L2 to memory) and peers' results loaded the same way,
// so a chunk needs neither the producer's L2 write-back fence nor the consumer's invalidate --
// the hand-off form MI355X_MICROARCH.md measures faster for tens of KB per workgroup
// ("publish-large").  Raw buffer ops carry the policy bits; the resource covers <= 2 GiB from base.
constexpr int kSysCoherent = 1 | 16;  // gfx950 cache-policy bits: sc0 (1) | sc1 (16)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wt_rsrc(const void *base)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), 0, 0x7fffffff, 0x00020000);
}

template <class F>
__device__ __forceinline__ typename F::T pfold_step(const typename F::T &acc, const typename F::T &x, bool acc_is_out)
{
    return acc_is_out ? F::op2(acc, x) : F::op2(x, acc);
}

// element i (absolute index into the vector) folded in my block's order: scalar path
template <class F> __device__ __forceinline__ typename F::T pfold_scalar(const PipeArgs &a, size_t i)
{
    using T = typename F::T;
    T acc = static_cast<const T *>(a.src[a.order[0]])[i];
    for (int j = 1; j < a.n; ++j) acc = pfold_step<F>(acc, static_cast<const T *>(a.src[a.order[j]])[i], (a.role_mask >> j) & 1u);
    return acc;
}

// fold the vector body: U 16-B vectors per lane in flight per source, sources loaded FC at a time
template <class F, bool NT, int U, int FC>
__device__ __forceinline__ void fold_body(const PipeArgs &a, typename F::T *dst, size_t v0, size_t nvec, bool wt)
{
    using T = typename F::T;
    using V = PVec<T>;
    constexpr int EPV = 16 / sizeof(T);
    const size_t t = threadIdx.x, nt = blockDim.x;
    const __amdgpu_buffer_rsrc_t rs = wt_rsrc(dst + v0);
    for (size_t base = t; base < nvec; base += nt * U) {
        V acc[U];
        for (int j0 = 0; j0 < a.n; j0 += FC) {
            V x[FC][U];
#pragma unroll
            for (int j = 0; j < FC; ++j) {
                if (j0 + j < a.n) {
                    const T *p = static_cast<const T *>(a.src[a.order[j0 + j]]) + v0;
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const size_t v = base + (size_t)u * nt;
                        if (v < nvec) {
                            const u32x4p raw = pload<NT>(p + v * EPV);
                            __builtin_memcpy(&x[j][u], &raw, 16);
                        }
                    }
                }
            }
            if (j0 == 0) {
#pragma unroll
                for (int u = 0; u < U; ++u) acc[u] = x[0][u];
            }
#pragma unroll
            for (int j = 0; j < FC; ++j) {
                if (j0 + j > 0 && j0 + j < a.n) {
                    const bool ao = (a.role_mask >> (j0 + j)) & 1u;
#pragma unroll
                    for (int u = 0; u < U; ++u)
#pragma unroll
                        for (int e = 0; e < EPV; ++e) acc[u].e[e] = pfold_step<F>(acc[u].e[e], x[j][u].e[e], ao);
                }
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t v = base + (size_t)u * nt;
            if (v < nvec) {
                u32x4p raw;
                __builtin_memcpy(&raw, &acc[u], 16);
                if (wt) __builtin_amdgcn_raw_buffer_store_b128(raw, rs, (unsigned)(v * 16), 0, kSysCoherent);
                else pstore<NT>(dst + v0 + v * EPV, raw);
            }
        }
    }
}

// fold elements [lo, hi) (absolute) into dst.  Few ranks: 4 vectors per lane per source (a
// persistent grid of a few workgroups per CU needs that much in flight to stream HBM); many
// ranks: 2 per source, 8 sources per load group (the n loads already fill the queue).
template <class F, bool NT> __device__ void fold_range(const PipeArgs &a, size_t lo, size_t hi, bool wt)
{
    using T = typename F::T;
    constexpr int EPV = 16 / sizeof(T);
    T *dst = reinterpret_cast<T *>(a.dst);
    const size_t t = threadIdx.x, nt = blockDim.x;
    size_t head = hi - lo, nvec = 0;
    if (a.co_fold) {
        const uintptr_t mis = ((uintptr_t)(dst + lo)) & 15;
        head = mis ? (16 - mis) / sizeof(T) : 0;
        if (head > hi - lo) head = hi - lo;
        nvec = (hi - lo - head) / EPV;
    }
    for (size_t i = lo + t; i < lo + head; i += nt) dst[i] = pfold_scalar<F>(a, i);
    const size_t v0 = lo + head;  // first element of the vector body
    if (a.n <= 4)
        fold_body<F, NT, 4, 4>(a, dst, v0, nvec, wt);
    else
        fold_body<F, NT, 2, kFoldChunk>(a, dst, v0, nvec, wt);
    for (size_t i = v0 + nvec * EPV + t; i < hi; i += nt) dst[i] = pfold_scalar<F>(a, i);
}

// copy bytes [lo, hi) (absolute byte offsets) from src to dst
template <bool NT> __device__ void copy_range(char *dst, const char *src, size_t lo, size_t hi, bool co, bool wt)
{
    const size_t t = threadIdx.x, nt = blockDim.x;
    size_t head = hi - lo, nvec = 0;
    if (co) {
        const uintptr_t mis = ((uintptr_t)(dst + lo)) & 15;
        head = mis ? 16 - mis : 0;
        if (head > hi - lo) head = hi - lo;
        nvec = (hi - lo - head) / 16;
    }
    for (size_t i = lo + t; i < lo + head; i += nt) dst[i] = src[i];
    const size_t b0 = lo + head;
    constexpr int U = 8;
    const __amdgpu_buffer_rsrc_t rs = wt_rsrc(src + b0);
    for (size_t base = t; base < nvec; base += nt * U) {
        u32x4p x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t v = base + (size_t)u * nt;
            if (v < nvec)
                x[u] = wt ? __builtin_amdgcn_raw_buffer_load_b128(rs, (unsigned)(v * 16), 0, kSysCoherent)
                          : pload<NT>(src + b0 + v * 16);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t v = base + (size_t)u * nt;
            if (v < nvec) pstore<NT>(dst + b0 + v * 16, x[u]);
        }
    }
    for (size_t i = b0 + nvec * 16 + t; i < hi; i += nt) dst[i] = src[i];
}

__device__ __forceinline__ uint64_t flag_load(const uint64_t *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// a value every lane holds alike, made visibly uniform (scalar) for the compiler: the loop below
// has workgroup barriers, so every branch around them must be uniform, including the ones on
// values read back from LDS
__device__ __forceinline__ uint64_t uniform64(uint64_t v)
{
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ void dbg_store(const PipeArgs &a, int w, uint64_t v)
{
    if (a.dbg) __hip_atomic_store(a.dbg + 4 * blockIdx.x + w, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <class F, bool NT> __global__ __launch_bounds__(256) void k_pipe_allreduce(PipeArgs a)
{
    using T = typename F::T;
    constexpr size_t esz = sizeof(T);
    __shared__ uint64_t item_s;
    __shared__ uint32_t give_up_s;
    const uint64_t total = (uint64_t)a.nchunks * (uint64_t)a.n;
    for (;;) {
        if (threadIdx.x == 0) item_s = __hip_atomic_fetch_add(a.queue, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - a.qbase;
        __syncthreads();
        const uint64_t it = uniform64(item_s);
        if (threadIdx.x == 0) dbg_store(a, 0, it);
        if (it >= total) break;
        if (it < a.nchunks) {
            // ---- fold chunk `it` of my block, then publish it to every peer
            const uint64_t k = it;
            const size_t blen = a.blen[a.me], lo = k * a.chunk, hi = lo + a.chunk < blen ? lo + a.chunk : blen;
            // write-through needs every store of the chunk to be a vector one: no scalar edges
            const bool wt = a.wt && a.co_fold && ((uintptr_t)(a.dst + (a.boff[a.me] + lo) * esz) & 15) == 0 &&
                            (((hi - lo) * esz) & 15) == 0;
            if (lo < hi) fold_range<F, NT>(a, a.boff[a.me] + lo, a.boff[a.me] + hi, wt);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave: its stores done
            __syncthreads();
            if (threadIdx.x == 0) {
                if (!wt) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: L2 written back
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                for (int q = 0; q < a.n; ++q)
                    if (q != a.me) __hip_atomic_store(a.peer_flag[q] + k, a.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                dbg_store(a, 1, 2);
            }
        } else {
            // ---- pull chunk k of peer q's block
            const uint64_t j = it - a.nchunks;
            const uint64_t k = j / (uint64_t)(a.n - 1);
            const int q = (int)((a.me + 1 + (int)(j % (uint64_t)(a.n - 1))) % a.n);
            const size_t blen = a.blen[q], lo = k * a.chunk, hi = lo + a.chunk < blen ? lo + a.chunk : blen;
            const size_t b0 = (a.boff[q] + lo) * esz, b1 = (a.boff[q] + hi) * esz;
            const bool co = (a.co_pull >> q) & 1u;
            const bool wt = a.wt && co && ((uintptr_t)(a.dst + b0) & 15) == 0 && ((b1 - b0) & 15) == 0;
            if (threadIdx.x == 0) {
                uint32_t give_up = 0;
                const uint64_t *f = a.my_flag + (size_t)q * a.kmax + k;
                const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
                unsigned polls = 0;
                while (flag_load(f) < a.seq) {
                    __builtin_amdgcn_s_sleep(2);
                    if ((++polls & 1023u) == 0 &&
                        (__hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0 ||
                         __builtin_amdgcn_s_memrealtime() - t0 > a.timeout_ticks)) {
                        __hip_atomic_store(a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                        give_up = 1;
                        break;
                    }
                }
                if (!wt) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope: no stale peer lines
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                give_up_s = give_up;
                dbg_store(a, 1, give_up ? 8 : 4);
                dbg_store(a, 3, polls);
            }
            __syncthreads();
            const bool give_up = __builtin_amdgcn_readfirstlane(give_up_s) != 0;
            if (!give_up && lo < hi) copy_range<NT>(a.dst, a.peer_rbuf[q], b0, b1, co, wt);
        }
        __syncthreads();  // every lane is done with item_s / give_up_s before lane 0 rewrites them
    }
}

static bool pipe_nt(size_t bytes) { return 2 * bytes > ((size_t)256 << 20); }

template <class F> static int launch_pipe(const PipeArgs &a, unsigned grid, hipStream_t s)
{
    if (pipe_nt((size_t)a.count * sizeof(typename F::T)))
        hipLaunchKernelGGL((k_pipe_allreduce<F, true>), dim3(grid), dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL((k_pipe_allreduce<F, false>), dim3(grid), dim3(256), 0, s, a);
    MI_HIP(hipGetLastError());
    return MI355X_SUCCESS;
}

// workgroups of the kernel launch_pipe would pick that one CU holds at once
template <class F> static int occupancy_pipe(size_t count)
{
    int nb = 0;
    hipError_t e = pipe_nt(count * sizeof(typename F::T))
                       ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_pipe_allreduce<F, true>, 256, 0)
                       : hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_pipe_allreduce<F, false>, 256, 0);
    return e == hipSuccess && nb > 0 ? nb : 1;
}

struct PipeTable {
    int (*f[MI355X_OP_MAX_][MI355X_T_MAX])(const PipeArgs &, unsigned, hipStream_t) = {};
    int (*occ[MI355X_OP_MAX_][MI355X_T_MAX])(size_t) = {};
    PipeTable()
    {
        for_each_slot([&](auto tag, int op, int ty) {
            using F = typename decltype(tag)::type;
            f[op][ty] = &launch_pipe<F>;
            occ[op][ty] = &occupancy_pipe<F>;
        });
    }
};

static const PipeTable &pipe_table()
{
    static const PipeTable t;
    return t;
}

int launch_pipe_slot(int op, int type, const PipeArgs &a, unsigned grid, hipStream_t s)
{
    const PipeTable &t = pipe_table();
    if (op < 0 || op >= MI355X_OP_MAX_ || type < 0 || type >= MI355X_T_MAX || !t.f[op][type])
        return set_error(MI355X_ERR_UNSUPPORTED, "no pipelined allreduce for op %d type %d", op, type);
    return t.f[op][type](a, grid, s);
}

int pipe_blocks_per_cu(int op, int type, size_t count)
{
    const PipeTable &t = pipe_table();
    if (op < 0 || op >= MI355X_OP_MAX_ || type < 0 || type >= MI355X_T_MAX || !t.occ[op][type]) return 1;
    return t.occ[op][type](count);
}

} // namespace mi355x
