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
//   1. lane 0 polls the doorbell until it carries the next call number (or kSvcQuit; or the
//      service has been idle for idle_ticks: the kernel leaves and the host relaunches it on the
//      next call);
//   2. the call's descriptor (SvcCall, in the doorbell page) is copied into LDS and expanded
//      into LLArgs;
//   3. the workgroup serves slices wg, wg + nwg, ... of the call exactly as a per-call LL block
//      serves its slice (push, receive, evaluate the reference schedule's per-element program or
//      copy), reading the inputs with system-coherent loads and storing the results write-through
//      (no kernel boundary between calls does the cache maintenance for it);
//   4. it counts itself done once its stores have reached memory; the workgroup that completes
//      the count (or the only one, for a call of one slice) acknowledges the call to every peer
//      (the LL parity protocol) and stores the call number into the host's completion word.
// Every wait is bounded (timeout_ticks; the error word is set and the workgroup leaves).
#include "coll_ll_dev.hpp"
#include "slot_list.hpp"

namespace mi355x {

static_assert(sizeof(SvcCall) % 8 == 0, "the descriptor is copied in 8-byte words");
constexpr int kSvcCallWords = (int)(sizeof(SvcCall) / 8);
static_assert(kSvcCallWords <= kSvcThreads, "one word per thread");

// one out-of-line function per slot (inlining all of them into one body makes the compiler's
// register allocation take tens of minutes)
template <class F>
static __device__ __noinline__ void svc_slot(const LLArgs &a, const LLBlock &k, const uint32_t (&w)[8][4])
{
    ll_reduce_out<F, true>(a, k, w);
}

// the evaluation for the call's (op, type): one branch per slot with a GPU kernel
static __device__ void svc_reduce_out(int op, int type, const LLArgs &a, const LLBlock &k, const uint32_t (&w)[8][4])
{
    for_each_slot([&](auto tag, int o, int t) {
        using F = typename decltype(tag)::type;
        if (o == op && t == type) svc_slot<F>(a, k, w);
    });
}

} // namespace mi355x

using namespace mi355x;

extern "C" __global__ __launch_bounds__(kSvcThreads) void mi355x_k_svc(SvcArgs g)
{
    if (g.probe) return;
    __shared__ LLArgs a;
    __shared__ SvcCall sc;
    __shared__ uint64_t s_door;
    const int t = (int)threadIdx.x;
    SvcPage *page = const_cast<SvcPage *>(g.page);
    uint64_t want = g.first;
    uint64_t ctr_base = 0;  // the doorbell page's workgroup counter before this call
    uint64_t idle0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        // 1. the doorbell
        if (t == 0) {
            uint64_t v;
            for (;;) {
                v = __hip_atomic_load(&page->door, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                if (v >= want) break;
                __builtin_amdgcn_s_sleep(2);
                if (__builtin_amdgcn_s_memrealtime() - idle0 > g.idle_ticks) {
                    v = kSvcQuit;
                    break;
                }
            }
            s_door = v;
        }
        __syncthreads();
        if (s_door != want) break;  // kSvcQuit, idle, or a number out of turn (never posted so)
        // 2. the descriptor (stored before the doorbell) into LDS
        if (t < kSvcCallWords)
            reinterpret_cast<uint64_t *>(&sc)[t] = __hip_atomic_load(reinterpret_cast<const uint64_t *>(&page->call) + t,
                                                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __syncthreads();
        if (sc.seq != want) break;
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
        // 3. my slices.  The inputs (written by kernels that completed before the call) are read
        // with system-coherent loads, the results stored write-through (ll_read16 / ll_write16<SYS>):
        // no acquire or release fence per call.  Workgroups beyond the call's slice count sit it out.
        const uint64_t nchunks = (a.nbytes + kLLChunk - 1) / kLLChunk;
        const uint64_t part = nchunks < (uint64_t)g.nwg ? nchunks : (uint64_t)g.nwg;
        if (blockIdx.x >= part) {
            if (part > 1) ctr_base += part;
            ++want;
            idle0 = __builtin_amdgcn_s_memrealtime();
            continue;
        }
        const bool reduce = a.mode == LL_AR || a.mode == LL_RED;
        const bool evaluate = reduce ? !(a.mode == LL_RED && me != a.root) : a.recv_mask != 0;
        int failed = 0;
        for (uint64_t c = blockIdx.x; c < nchunks; c += (uint64_t)g.nwg) {
            const LLBlock k = ll_block(a, c);
            if (!ll_push<true>(a, k)) {
                failed = 1;
                break;
            }
            uint32_t w[8][4];
            int bad = 0;
            if (evaluate && k.ngran) {
                if (!ll_recv(a, k, a.recv_mask, w))
                    bad = 1;
                else if (reduce)
                    svc_reduce_out(sc.op, sc.type, a, k, w);
                else
                    ll_copy_out<true>(a, k, w);
            }
            if (__syncthreads_or(bad)) {
                failed = 1;
                break;
            }
        }
        // 4. every store of the workgroup has reached memory; count; the last participant
        // acknowledges the call to every peer and completes it for the host
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (t == 0) {
            bool last = part == 1;
            if (!last) {
                const uint64_t old =
                    __hip_atomic_fetch_add(&page->ctr, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                last = old + 1 == ctr_base + part;
            }
            if (!failed && last) {
                for (int q = 0; q < n; ++q)
                    if (q != me) ll_store(a.peer_ack[q], want);
                __hip_atomic_store(g.done, want, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
        if (failed) break;  // the error word is set; the host ends the service
        if (part > 1) ctr_base += part;
        ++want;
        idle0 = __builtin_amdgcn_s_memrealtime();
    }
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
