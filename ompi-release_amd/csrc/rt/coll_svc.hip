// coll_svc.hip -- the resident LL service: device-resident progress for small collectives.
//
// The host-synchronised small allreduce spends 11-12 of its 15-16 us in the platform's launch-
// to-completion round trip (profiles/r03_latency_probe.jsonl), and the per-call LL kernels
// (coll_ll.hip) pay the same launch.  Here the LL protocol (tagged 8-byte granules pushed into
// every peer's uncached LL region, coll_ll_dev.hpp) runs inside a kernel that stays resident
// between calls on a private HSA queue (svc_queue.cpp) and waits on a doorbell: a call is a host
// store and a device poll (3.8-3.9 us round trip measured for the doorbell alone,
// profiles/r03_svc_probe.jsonl), and the host observes completion by a word the kernel stores
// into host memory.
//
// Every workgroup runs the same loop:
//   1. workgroup 0 polls the doorbell until it carries the next call number (or kSvcQuit; or the
//      service has been idle for idle_ticks: the kernel leaves and the host relaunches it on the
//      next call) and publishes its verdict -- serve call k with p workgroups, or leave -- which
//      the other workgroups follow (one decision per call);
//   2. a workgroup the call needs copies the call's descriptor (SvcCall, in the doorbell page)
//      into LDS and expands it into LLArgs;
//   3. the workgroup serves slices wg, wg + nwg, ... of the call exactly as a per-call LL block
//      serves its slice (push, receive, evaluate the reference schedule's per-element program or
//      copy), reading the inputs with system-coherent loads and storing the results write-through
//      (no kernel boundary between calls does the cache maintenance for it);
//   4. it counts itself done once its stores have reached memory; the workgroup that completes
//      the count (or the only one, for a call of one slice) acknowledges the call to every peer
//      (the LL parity protocol) and stores the call number into the host's completion word.
// The pull forms (LL_PULL, the one-phase ring allreduce of 32-128 KiB; LL_PULL_AG / LL_PULL_BC,
// allgather and bcast to 1 MiB; LL_PULL_RS, reduce_scatter(_block) up to 128 KiB per block) replace
// step 3's granules by reads of the peers' mapped inputs, and step 4 waits until every peer has
// read this rank's.
// Every wait is bounded (timeout_ticks; the error word is set and the workgroup leaves) and leaves
// early once the error word is set -- by another workgroup, or by the host when a peer is gone.
#include "coll_ll_dev.hpp"
#include "slot_list.hpp"

namespace mi355x {

static_assert(sizeof(SvcCall) % 8 == 0, "the descriptor is copied in 8-byte words");
constexpr int kSvcCallWords = (int)(sizeof(SvcCall) / 8);
static_assert(kSvcCallWords <= kSvcThreads, "one word per thread");
constexpr int kSvcPass = 4;  // slices whose inputs one workgroup reads at once
constexpr int kSvcPullU = 4; // LL_PULL: 16-B vectors per lane per pass

// element i of ring block b folds x_b, x_{b+1}, ..., x_{b+n-1} with the partial as the `in`
// operand (coll_tuned_allreduce.c:470-512; the LL_RING program of ll_eval, without its tree form)
template <class F> __device__ __forceinline__ typename F::T svc_ring_fold(const LLArgs &a, uint64_t i,
                                                                        const RankRegs<typename F::T> &X)
{
    const uint64_t se = a.split * a.early;
    const int b0 = (i < se) ? (int)(i / a.early) : (int)(a.split + (i - se) / a.late);
    typename F::T acc = X.get(b0);
    for (int j = 1; j < a.n; ++j) {
        const int r = b0 + j >= a.n ? b0 + j - a.n : b0 + j;
        acc = F::op2(X.get(r), acc);
    }
    return acc;
}

// LL_PULL (one-phase ring-ordered allreduce from the mapped inputs, no granules): every element
// of this workgroup's 4-KiB slices folded from the n inputs in its ring block's order, the inputs
// read with system-coherent 16-B loads, the result stored write-through; the last partial vector's
// elements one by one
template <class F> static __device__ void svc_pull(const LLArgs &a, const SvcCall &sc, uint64_t stride)
{
    using T = typename F::T;
    using V = LLVec<T>;
    constexpr int EPV = 16 / sizeof(T);
    const uint64_t nvec = a.nbytes / 16;
    // kSvcPullU vectors per lane per pass, every source's loads of the pass issued before any
    // evaluation: the loads cross xGMI, so the pass is latency-bound, not bandwidth-bound
    const uint64_t step = stride * kSvcThreads;
    for (uint64_t v0 = (uint64_t)blockIdx.x * kSvcThreads + threadIdx.x; v0 < nvec; v0 += step * kSvcPullU) {
        V xv[kSvcPullU][kLLMaxRanks];
#pragma unroll
        for (int q = 0; q < kLLMaxRanks; ++q) {
            if (q >= a.n) continue;
            const __amdgpu_buffer_rsrc_t rs = ll_rsrc(sc.srcs[q]);
#pragma unroll
            for (int u = 0; u < kSvcPullU; ++u) {
                const uint64_t v = v0 + (uint64_t)u * step;
                if (v >= nvec) continue;
                const u32x4l raw = __builtin_amdgcn_raw_buffer_load_b128(rs, (unsigned)(v * 16), 0, kLLSysCoherent);
                __builtin_memcpy(&xv[u][q], &raw, 16);
            }
        }
#pragma unroll
        for (int u = 0; u < kSvcPullU; ++u) {
            const uint64_t v = v0 + (uint64_t)u * step;
            if (v >= nvec) continue;
            V r;
#pragma unroll
            for (int e = 0; e < EPV; ++e) {
                RankRegs<T> X;
#pragma unroll
                for (int q = 0; q < kLLMaxRanks; ++q) X.set(q, xv[u][q].e[e]);
                r.e[e] = svc_ring_fold<F>(a, v * EPV + e, X);
            }
            u32x4l out;
            __builtin_memcpy(&out, &r, 16);
            __builtin_amdgcn_raw_buffer_store_b128(out, ll_rsrc(a.dst), (unsigned)(v * 16), 0, kLLSysCoherent);
        }
    }
    const uint64_t i = nvec * EPV + threadIdx.x;  // the tail: fewer than EPV elements
    if (blockIdx.x == 0 && i < a.count) {
        T xs[kLLMaxRanks];
#pragma unroll
        for (int q = 0; q < kLLMaxRanks; ++q) {
            if (q >= a.n) continue;
            uint32_t w[4];
            ll_read16<true>(static_cast<const char *>(sc.srcs[q]), i * sizeof(T), sizeof(T), w);
            __builtin_memcpy(&xs[q], w, sizeof(T));
        }
        RankRegs<T> X;
#pragma unroll
        for (int q = 0; q < kLLMaxRanks; ++q) X.set(q, xs[q]);
        const T r = svc_ring_fold<F>(a, i, X);
        uint32_t w[4] = {0, 0, 0, 0};
        __builtin_memcpy(w, &r, sizeof(T));
        ll_write16<true>(static_cast<char *>(a.dst), i * sizeof(T), sizeof(T), w);
    }
}

// len bytes from src (a peer's mapped buffer) to dst (mine), this workgroup's share of the 16-B
// vectors (4 per lane in flight), or of the words / bytes when an end is not 16-B aligned; src and
// dst are the same for the whole workgroup
static __device__ void svc_copy_seg(const char *src, char *dst, uint64_t len, uint64_t stride)
{
    const __amdgpu_buffer_rsrc_t rs = ll_rsrc(src), rd = ll_rsrc(dst);
    const uint64_t step = stride * kSvcThreads;
    const uint64_t first = (uint64_t)blockIdx.x * kSvcThreads + threadIdx.x;
    if (((((uintptr_t)src) | ((uintptr_t)dst) | len) & 15) == 0) {
        const uint64_t nvec = len / 16;
        for (uint64_t v0 = first; v0 < nvec; v0 += step * kSvcPullU) {
            u32x4l x[kSvcPullU];
#pragma unroll
            for (int u = 0; u < kSvcPullU; ++u) {
                const uint64_t v = v0 + (uint64_t)u * step;
                if (v < nvec) x[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, (unsigned)(v * 16), 0, kLLSysCoherent);
            }
#pragma unroll
            for (int u = 0; u < kSvcPullU; ++u) {
                const uint64_t v = v0 + (uint64_t)u * step;
                if (v < nvec) __builtin_amdgcn_raw_buffer_store_b128(x[u], rd, (unsigned)(v * 16), 0, kLLSysCoherent);
            }
        }
        return;
    }
    if (((((uintptr_t)src) | ((uintptr_t)dst) | len) & 3) == 0) {
        for (uint64_t w = first; w < len / 4; w += step)
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_amdgcn_raw_buffer_load_b32(rs, (unsigned)(w * 4), 0, kLLSysCoherent),
                                                  rd, (unsigned)(w * 4), 0, kLLSysCoherent);
        return;
    }
    for (uint64_t b = first; b < len; b += step)
        __builtin_amdgcn_raw_buffer_store_b8(__builtin_amdgcn_raw_buffer_load_b8(rs, (unsigned)b, 0, kLLSysCoherent), rd,
                                             (unsigned)b, 0, kLLSysCoherent);
}

// LL_PULL_AG / LL_PULL_BC: allgather (block q from rank q's input, own block skipped in place) and
// bcast (the root's buffer) copied from the mapped peers
static __device__ void svc_pull_copy(const LLArgs &a, const SvcCall &sc, uint64_t stride)
{
    char *dst = static_cast<char *>(a.dst);
    if (a.mode == LL_PULL_BC) {
        if (a.me != a.root) svc_copy_seg(static_cast<const char *>(sc.srcs[a.root]), dst, a.nbytes, stride);
        return;
    }
    for (int q = 0; q < a.n; ++q) {
        char *d = dst + (uint64_t)q * a.nbytes;
        if (q == a.me && static_cast<const char *>(a.src) == d) continue;  // in place: already there
        svc_copy_seg(static_cast<const char *>(sc.srcs[q]), d, a.nbytes, stride);
    }
}

// Step 3's second half for every slice of this workgroup: receive the peers' granules (LL_PULL_RS:
// read the peers' blocks), then the reference program per element (or the copy); or the pull form.  One out-of-line function per
// (op, type) slot, entered once per call: the call's slot decides which (inlining every slot's
// evaluation into one body makes the compiler's register allocation take tens of minutes; the
// hot float / double SUM slots are inlined, svc_finish_call).  Returns 1 on a timeout.
template <class F>
static __device__ __forceinline__ int svc_finish_body(const LLArgs &a, const SvcCall &sc, uint64_t nchunks,
                                                      uint64_t stride, uint64_t *tr)
{
    if constexpr (F::kCopy) {
        if (a.mode == LL_PULL_AG || a.mode == LL_PULL_BC) {
            svc_pull_copy(a, sc, stride);
            return 0;
        }
    }
    if constexpr (!F::kCopy) {
        // (the pull form serves element types of 4 bytes and more -- svc_pull_usable -- so the
        // 16- and 8-element vectors of the 1- and 2-byte types never instantiate it)
        if constexpr (sizeof(typename F::T) >= 4) {
            if (a.mode == LL_PULL) {
                svc_pull<F>(a, sc, stride);
                return 0;
            }
        }
    }
    for (uint64_t c = blockIdx.x; c < nchunks; c += stride) {
        const LLBlock k = ll_block(a, c);
        uint32_t w[8][4];
        int bad = 0;
        if (k.ngran) {
            bool pulled = false;
            if constexpr (!F::kCopy) {
                if (a.mode == LL_PULL_RS) {  // this thread's 16 B of every rank's block, where they are
#pragma unroll
                    for (int q = 0; q < kLLMaxRanks; ++q) {
                        w[q][0] = w[q][1] = w[q][2] = w[q][3] = 0;
                        if (q < a.n) ll_read16<true>(static_cast<const char *>(sc.srcs[q]), k.off, k.len, w[q]);
                    }
                    pulled = true;
                }
            }
            if (!pulled) bad = !ll_recv(a, k, a.recv_mask, w);
            if (tr && threadIdx.x == 0 && c == blockIdx.x) tr[4] = __builtin_amdgcn_s_memrealtime();
            if (!bad) {
                if constexpr (F::kCopy)
                    ll_copy_out<true>(a, k, w);
                else
                    ll_reduce_out<F, true>(a, k, w);
            }
            if (tr && threadIdx.x == 0 && c == blockIdx.x) tr[8] = __builtin_amdgcn_s_memrealtime();
        }
        const int any_bad = __syncthreads_or(bad);
        if (tr && threadIdx.x == 0 && c == blockIdx.x) tr[9] = __builtin_amdgcn_s_memrealtime();
        if (any_bad) return 1;
    }
    return 0;
}

template <class F>
static __device__ __noinline__ int svc_finish(const LLArgs &a, const SvcCall &sc, uint64_t nchunks, uint64_t stride,
                                              uint64_t *tr)
{
    return svc_finish_body<F>(a, sc, nchunks, stride, tr);
}

struct SvcCopy {  // allgather / bcast: no evaluation
    static constexpr bool kCopy = true;
};
template <class F> struct SvcReduce : F {
    static constexpr bool kCopy = false;
};

// every other slot: one out-of-line function per slot behind one out-of-line dispatcher
static __device__ __noinline__ int svc_finish_call(int op, int type, const LLArgs &a, const SvcCall &sc,
                                                   uint64_t nchunks, uint64_t stride, uint64_t *tr)
{
    int rc = 0;
    for_each_slot([&](auto tag, int o, int t) {
        using F = typename decltype(tag)::type;
        if (o == op && t == type) rc = svc_finish<SvcReduce<F>>(a, sc, nchunks, stride, tr);
    });
    return rc;
}

// LL_PULL, the last participant: tell every peer its input has been read, then wait until every
// peer has read mine (the caller may reuse its input once the call completes); false on timeout
static __device__ bool svc_pull_handshake(const SvcArgs &g, uint64_t want)
{
    for (int q = 0; q < g.n; ++q)
        if (q != g.me) ll_store(reinterpret_cast<uint64_t *>(g.peer_ll[q]) + kSvcPullDoneWord + g.me, want);
    const uint64_t *mine = reinterpret_cast<const uint64_t *>(g.my_ll) + kSvcPullDoneWord;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    unsigned spins = 0;
    for (int q = 0; q < g.n; ++q) {
        if (q == g.me) continue;
        while (ll_load(mine + q) < want) {
            __builtin_amdgcn_s_sleep(1);
            if (__builtin_amdgcn_s_memrealtime() - t0 > g.timeout_ticks) {
                __hip_atomic_store(g.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                return false;
            }
            // the host gave up on a peer that is gone (svc_call)
            if ((++spins & 255u) == 0 && __hip_atomic_load(g.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) return false;
        }
    }
    return true;
}

} // namespace mi355x

using namespace mi355x;

extern "C" __global__ __launch_bounds__(kSvcThreads) void mi355x_k_svc(SvcArgs g)
{
    if (g.probe) return;
    __shared__ LLArgs a;
    __shared__ SvcCall sc;
    __shared__ uint64_t s_door;
    __shared__ int s_fail;
    __shared__ uint64_t s_tr[kSvcTraceCols];  // (MI355X_SVC_TRACE, workgroup 0) this call's stamps
    const int t = (int)threadIdx.x;
    SvcPage *page = const_cast<SvcPage *>(g.page);
    uint64_t want = g.first;
    uint64_t idle0 = __builtin_amdgcn_s_memrealtime();
    uint64_t nalive = (uint64_t)g.nwg;  // (workgroup 0, thread 0) workgroups still resident
    for (;;) {
        // 1. the doorbell: (call number << kSvcPartBits) | participating workgroups.  Workgroup 0
        // alone decides whether the next call is served or the service leaves (quit request, idle,
        // a number out of turn) and publishes the verdict in `go`; the others follow it --
        // workgroups deciding on their own could split over a call (some serving it, some gone),
        // and a call served in part never completes.  The verdict carries the participant count,
        // so a workgroup the call does not need never reads the descriptor (which the host may
        // already be rewriting for the next call once the participants are done).
        if (t == 0) {
            uint64_t v;
            if (blockIdx.x == 0) {
                for (;;) {
                    v = __hip_atomic_load(&page->door, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    if ((v >> kSvcPartBits) >= want) break;
                    __builtin_amdgcn_s_sleep(2);
                    const uint64_t idle = __builtin_amdgcn_s_memrealtime() - idle0;
                    if (idle > g.idle_ticks) {
                        v = kSvcQuit;
                        break;
                    }
                    // idle between calls (every participant of the last call is done): the other
                    // workgroups leave, so a service waiting through a compute phase holds one CU
                    // instead of nwg; it serves the small calls alone from then on
                    if (nalive > 1 && g.shrink_ticks && idle > g.shrink_ticks) {
                        nalive = 1;
                        __hip_atomic_store(&page->shrink, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                        __hip_atomic_store(g.shrunk, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    }
                }
                if ((v >> kSvcPartBits) != want) v = kSvcQuit;
                // the participants: as many as the host asked for, of those still resident
                if (v != kSvcQuit && (v & ((1u << kSvcPartBits) - 1)) > nalive)
                    v = (v & ~(uint64_t)((1u << kSvcPartBits) - 1)) | nalive;
                __hip_atomic_store(&page->go, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            } else {
                for (;;) {  // (bounded too: never longer than the leader's idle limit plus a timeout)
                    v = __hip_atomic_load(&page->go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    if ((v >> kSvcPartBits) >= want) break;
                    // told to leave while idle: workgroup 0 never again counts this one in (it sets
                    // `shrink` only between calls, and its later verdicts name itself alone)
                    if (__hip_atomic_load(&page->shrink, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) {
                        v = kSvcQuit;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(2);
                    if (__builtin_amdgcn_s_memrealtime() - idle0 > g.idle_ticks + g.timeout_ticks) {
                        v = kSvcQuit;
                        break;
                    }
                }
                // (a follower no call has needed since it last looked may find the verdict of a
                // later call: those calls completed without it; it joins this one)
            }
            s_door = v;
        }
        __syncthreads();
        if (s_door == kSvcQuit) break;
        want = s_door >> kSvcPartBits;
        const uint64_t part = s_door & ((1u << kSvcPartBits) - 1);
        if (blockIdx.x >= part) {  // not needed by this call: on to the next verdict
            ++want;
            idle0 = __builtin_amdgcn_s_memrealtime();
            // every wave has read s_door before thread 0 may write the next verdict into it (a
            // lagging wave would otherwise follow the next call's verdict to a different barrier)
            __syncthreads();
            continue;
        }
        uint64_t *tr = (g.trace && blockIdx.x == 0) ? s_tr : nullptr;
        if (tr && t == 0) {
            for (int k = 0; k < kSvcTraceCols; ++k) tr[k] = 0;
            tr[0] = want;
            tr[1] = __builtin_amdgcn_s_memrealtime();
        }
        // 2. the descriptor (stored before the doorbell; not rewritten before every participant
        // of this call is done) into LDS
        if (t < kSvcCallWords)
            reinterpret_cast<uint64_t *>(&sc)[t] = __hip_atomic_load(reinterpret_cast<const uint64_t *>(&page->call) + t,
                                                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __syncthreads();
        if (sc.seq != want) {  // (never: the host protocol forbids it) -- leave, visibly
            if (t == 0) __hip_atomic_store(g.err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            break;
        }
        const int n = g.n, me = g.me;
        const uint64_t par = want & 1;
        if (t == 0) {
            a.src = sc.src;
            a.dst = sc.dst;
            a.err = g.err;
            a.push_mask = sc.push_mask;
            a.recv_mask = sc.recv_mask;
            a.seq = want;
            a.slot_gran = g.slot_gran;
            a.nbytes = sc.nbytes;
            a.timeout_ticks = g.timeout_ticks;
            a.count = sc.count;
            a.early = sc.early;
            a.late = sc.late;
            a.split = sc.split;
            a.role_mask = sc.role_mask;
            a.mode = sc.mode;
            a.prog = sc.prog;
            a.n = n;
            a.me = me;
            a.root = sc.root;
            a.nsteps = sc.nsteps;
            a.result = sc.result;
            a.my_data = reinterpret_cast<const uint64_t *>(g.my_ll + kLLAckBytes) + par * (uint64_t)n * g.slot_gran;
            a.my_ack = reinterpret_cast<const uint64_t *>(g.my_ll);
        }
        if (t < n) {
            a.peer_data[t] = reinterpret_cast<uint64_t *>(g.peer_ll[t] + kLLAckBytes) + (par * n + me) * g.slot_gran;
            a.peer_ack[t] = reinterpret_cast<uint64_t *>(g.peer_ll[t]) + me;
            a.order[t] = sc.order[t];
        }
        if (t < kTreeSteps) a.steps[t] = sc.steps[t];
        __syncthreads();
        if (tr && t == 0) tr[2] = __builtin_amdgcn_s_memrealtime();
        // 3. my slices.  The inputs (written by kernels that completed before the call) are read
        // with system-coherent loads, the results stored write-through (ll_read16 / ll_write16<SYS>):
        // no acquire or release fence per call.
        const uint64_t nchunks = (a.nbytes + kLLChunk - 1) / kLLChunk;
        // pull forms: no granules, the inputs are read where they are
        const bool pull = a.mode == LL_PULL || a.mode == LL_PULL_AG || a.mode == LL_PULL_BC || a.mode == LL_PULL_RS;
        const bool reduce = a.mode == LL_AR || a.mode == LL_RED || a.mode == LL_PULL || a.mode == LL_PULL_RS;
        const bool evaluate = reduce ? !(a.mode == LL_RED && me != a.root) : (a.recv_mask != 0 || pull);
        // push every slice of mine (inputs read kSvcPass slices at a time, so their latencies
        // overlap; the acknowledgement wait once, behind the first reads), then receive and finish
        // them: a workgroup with several slices waits one peer round trip, not one per slice
        int failed = 0;
        // the call's participants share its work: slice / vector / word / byte k*part + wg (the
        // granule slices and 16-B vectors come 4 KiB per workgroup per step, the pull copy's words
        // and bytes less: striding by nwg while only part workgroups take part would skip some)
        const uint64_t stride = part;
        // a slice's 16-B pieces are pushed by the other half of the workgroup than the one that
        // receives and evaluates them: a wave's loads wait for its earlier stores to complete (one
        // counter for both on gfx9), so the small calls' receiving waves (the first) never queue
        // their polls behind the system-scope pushes
        const unsigned pt = ((unsigned)t + kSvcThreads / 2) % kSvcThreads;
        for (uint64_t c0 = blockIdx.x; c0 < nchunks && !failed && !pull; c0 += stride * kSvcPass) {
            uint32_t w[kSvcPass][4];
#pragma unroll
            for (int p = 0; p < kSvcPass; ++p) {
                const uint64_t c = c0 + (uint64_t)p * stride;
                if (c < nchunks) ll_read_slice<true>(a, ll_block(a, c, pt), w[p]);
            }
            if (c0 == blockIdx.x && !ll_wait_acks(a)) failed = 1;
            if (failed) break;
#pragma unroll
            for (int p = 0; p < kSvcPass; ++p) {
                const uint64_t c = c0 + (uint64_t)p * stride;
                if (c < nchunks) ll_push_slice(a, ll_block(a, c, pt), w[p]);
            }
        }
        if (tr && t == 0) tr[3] = __builtin_amdgcn_s_memrealtime();
        // the hot forms inline in the kernel: a function call costs a wait for every outstanding
        // memory operation at its entry (the pushes, written through to the peers) and its
        // register saves and scratch reloads -- ~2 us of an 8-B call's 7 on the device
        if (!failed && evaluate) {
            if (!reduce)
                failed = svc_finish_body<SvcCopy>(a, sc, nchunks, stride, tr);
            else if (sc.op == MI355X_OP_SUM && sc.type == MI355X_T_FLOAT)
                failed = svc_finish_body<SvcReduce<OpSum<float>>>(a, sc, nchunks, stride, tr);
            else if (sc.op == MI355X_OP_SUM && sc.type == MI355X_T_DOUBLE)
                failed = svc_finish_body<SvcReduce<OpSum<double>>>(a, sc, nchunks, stride, tr);
            else
                failed = svc_finish_call(sc.op, sc.type, a, sc, nchunks, stride, tr);
        }
        if (tr && t == 0) tr[7] = __builtin_amdgcn_s_memrealtime();
        // 4. every store of the workgroup has reached memory; count; the last participant
        // acknowledges the call to every peer and completes it for the host
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tr && t == 0) tr[5] = __builtin_amdgcn_s_memrealtime();
        if (t == 0) {
            bool last = part == 1;
            if (!last) {
                const uint64_t old =
                    __hip_atomic_fetch_add(&page->ctr, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                last = old + 1 == part;
                // the last participant zeroes the counter for the next call, and the reset has
                // landed before the completion word does (the next call is posted after it)
                if (last) {
                    __hip_atomic_store(&page->ctr, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
            }
            // (LL_PULL: not before every peer has read this rank's input)
            if (!failed && last && pull && !svc_pull_handshake(g, want)) failed = 1;
            if (!failed && last) {
                for (int q = 0; q < n; ++q)
                    if (q != me) ll_store(a.peer_ack[q], want);
                __hip_atomic_store(g.done, want, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            if (tr) {
                tr[6] = __builtin_amdgcn_s_memrealtime();
                uint64_t *row = g.trace + (want % kSvcTraceCalls) * kSvcTraceCols;
                for (int k = 0; k < kSvcTraceCols; ++k) row[k] = tr[k];
            }
            s_fail = failed;
        }
        __syncthreads();
        if (s_fail) break;  // the error word is set; the host ends the service
        ++want;
        idle0 = __builtin_amdgcn_s_memrealtime();
    }
    // whatever made the leader leave (quit, idle, a failed call), the followers leave with it
    if (blockIdx.x == 0 && t == 0) __hip_atomic_store(&page->go, kSvcQuit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

namespace mi355x {

int svc_probe_launch(int device)
{
    int prev = 0;
    if (hipGetDevice(&prev) != hipSuccess || hipSetDevice(device) != hipSuccess) return -1;
    SvcArgs probe;
    __builtin_memset(&probe, 0, sizeof(probe));
    probe.probe = 1;
    // on the null stream: a stream of its own would make HIP create one more hardware queue for
    // the process, and with two processes on one GPU every hardware queue beyond the second slows
    // every launch of both (profiles/r03_queue_probe.jsonl)
    hipLaunchKernelGGL(mi355x_k_svc, dim3(1), dim3(kSvcThreads), 0, nullptr, probe);
    const bool ok = hipGetLastError() == hipSuccess && hipStreamSynchronize(nullptr) == hipSuccess;
    (void)hipSetDevice(prev);
    return ok ? 0 : -1;
}

} // namespace mi355x
