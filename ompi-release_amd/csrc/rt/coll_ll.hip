// coll_ll.hip -- low-latency one-shot collectives for small messages (see coll_internal.hpp).
//
// The reference's recursive-doubling / small-ring region (coll_tuned_decision_fixed.c:42-85) is
// latency-bound: a host round trip (stream sync + shm barrier) costs more than the data.  Here
// one launch per rank per call, no host barrier, and -- unlike a flag-after-data protocol -- no
// memory fence on the critical path: every 4 bytes of payload travel with the call's tag in one
// naturally aligned 8-byte granule {payload, tag}, written by ONE 8-byte store (single-copy
// atomic), so a receiver that sees the tag sees the payload.  The LL region of every rank is
// uncached device memory (hipDeviceMallocUncached): remote stores land in its HBM, local polls
// read HBM, nothing stale can sit in a cache.
//
// Block b of every rank (256 threads, 4 KiB of payload, 16 B per thread):
//   1. wait until every peer it pushes to has acknowledged the call two calls back (that peer
//      then no longer reads the parity slot about to be rewritten; the wait is normally satisfied
//      at once);
//   2. pushes its 16 B into slot (parity, me) of every peer named in push_mask as 4 granules;
//   3. polls its own slots of the ranks it receives from until every granule carries this call's
//      tag (bounded: on timeout the host-visible error word is set);
//   4. finishes locally: the reference schedule's per-element program over the n inputs
//      (allreduce; reduce: the root only), or copies (allgather / bcast);
//   5. counts itself done; the last block of the call acknowledges the call to every peer.
// Slices are independent, so blocks never wait on each other.
#include "coll_ll_dev.hpp"
#include "slot_list.hpp"

namespace mi355x {

// allreduce / reduce: exchange, then this thread's 16 B of the result from the n inputs held in
// registers (<= 8 ranks: ll_usable)
template <class F> __global__ __launch_bounds__(256) void k_ll_allreduce(LLArgs a)
{
    const LLBlock k = ll_block(a, blockIdx.x);
    if (!ll_push(a, k)) return;
    const bool evaluate = !(a.mode == LL_RED && a.me != a.root);  // reduce: only the root evaluates
    uint32_t w[8][4];
    if (evaluate && ll_recv(a, k, a.recv_mask, w) && k.ngran) ll_reduce_out<F>(a, k, w);
    ll_done(a);
}

// allgather (slot q -> dst + q*nbytes) and bcast (slot root -> dst, non-roots)
__global__ __launch_bounds__(256) void k_ll_copy(LLArgs a)
{
    const LLBlock k = ll_block(a, blockIdx.x);
    if (!ll_push(a, k)) return;
    uint32_t w[8][4];
    if (a.recv_mask && ll_recv(a, k, a.recv_mask, w) && k.ngran) ll_copy_out(a, k, w);
    ll_done(a);
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
