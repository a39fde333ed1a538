// coll_pipe_host.cpp -- host side of the pipelined allreduce (coll_pipe.hip): its flag region
// and launch, plus the LL programs of the service's reduce-scatter (split out of coll_comm.cpp).

#include <fcntl.h>
#include <immintrin.h>
#include <poll.h>
#include <sched.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/un.h>
#include <unistd.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <condition_variable>
#include <cstddef>
#include <deque>
#include <functional>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "coll_internal.hpp"
#include "coll_sched.hpp"
#include "rt_internal.hpp"

#include "comm_internal.hpp"

#include "coll_comm_int.hpp"

namespace mi355x {

// ----------------------------------------------------------------- pipelined allreduce
// (Re)build the per-chunk flag region (uncached, every peer writes its row into it over xGMI)
// and the work-queue counter.  Collective: every rank reaches it in the same call.
constexpr size_t kPipeKmax = 1024;  // chunks per ring block, at most
int ensure_pipe(mi355x_comm *c)
{
    if (c->pipe_base) return MI355X_SUCCESS;
    const size_t n = (size_t)c->size;
    const size_t bytes = (n * kPipeKmax * sizeof(uint64_t) + 4095) / 4096 * 4096;
    MI_HIP(hipExtMallocWithFlags((void **)&c->pipe_base, bytes, hipDeviceMallocUncached));
    hipStream_t ss = setup_stream(c);
    MI_HIP(hipMemsetAsync(c->pipe_base, 0, bytes, ss));
    MI_HIP(hipMalloc((void **)&c->pipe_queue, sizeof(uint64_t)));
    MI_HIP(hipMemsetAsync(c->pipe_queue, 0, sizeof(uint64_t), ss));
    if (!c->ll_err) MI_HIP(hipHostMalloc((void **)&c->ll_err, sizeof(uint32_t), hipHostMallocCoherent));
    MI_HIP(hipStreamSynchronize(ss));
    c->pipe_kmax = kPipeKmax;
    c->pipe_qbase = 0;
    c->pipe_seq = 0;
    const void *mine[1] = {c->pipe_base};
    const uint64_t sig[4] = {11, bytes, 0, 0};
    std::vector<std::vector<void *>> P;
    int rc = exchange(c, 1, mine, sig, P, nullptr, true, true);
    if (rc) return rc;
    c->pipe_peer.assign(n, nullptr);
    for (size_t q = 0; q < n; ++q) c->pipe_peer[q] = (char *)P[0][q];
    TRACE(c, "pipe region %zu bytes, %d ranks on this GPU", bytes, c->pipe_share);
    return barrier(c);  // every rank has read the exchange slots
}

} // namespace mi355x

namespace mi355x {

// device-side readiness flags (coll_pipe.hip).  P[0] = every rank's input, P[1] = every rbuf.
int pipe_allreduce(mi355x_comm *c, int op, int type, const Program &pr,
                          const std::vector<std::vector<void *>> &P, size_t count, hipStream_t s)
{
    if (!c->pipe_base) return set_error(MI355X_ERR_ARG, "pipelined allreduce before its setup");
    int rc = MI355X_SUCCESS;
    const size_t esz = mi355x_type_size(type), n = (size_t)c->size;
    PipeArgs a;
    std::memset(&a, 0, sizeof(a));
    size_t maxlen = 0;
    for (int q = 0; q < c->size; ++q) {
        size_t o, l;
        ring_block(count, c->size, q, &o, &l);
        a.boff[q] = o;
        a.blen[q] = l;
        maxlen = std::max(maxlen, l);
    }
    // chunks: ~512 per block for big blocks (many more items than workgroups, so the pulls of
    // chunk k overlap the folds of the chunks after it), at least 64 KiB, whole 16-B vectors,
    // at most kPipeKmax per block
    const size_t vec = 16 / esz;
    size_t chunk = coll_tune().pipe_chunk_kib ? ((size_t)coll_tune().pipe_chunk_kib << 10) / esz
                                              : std::max<size_t>(((size_t)64 << 10) / esz, maxlen / 512);
    if (c->pipe_chunk_override) chunk = c->pipe_chunk_override;  // (the self-test's small chunks)
    chunk = std::max(chunk, (maxlen + kPipeKmax - 1) / kPipeKmax);
    chunk = (chunk + vec - 1) / vec * vec;
    const size_t nchunks = std::max<size_t>(1, (maxlen + chunk - 1) / chunk);
    const int me = c->rank;
    for (int q = 0; q < c->size; ++q) {
        a.src[q] = P[0][q];
        a.peer_rbuf[q] = (const char *)P[1][q];
        if (q != me)
            a.peer_flag[q] = reinterpret_cast<uint64_t *>(c->pipe_peer[q]) + (size_t)me * c->pipe_kmax;
    }
    a.dst = (char *)P[1][me];
    a.my_flag = reinterpret_cast<const uint64_t *>(c->pipe_base);
    a.queue = c->pipe_queue;
    a.err = c->ll_err;
    *c->ll_err = 0;
    a.qbase = c->pipe_qbase;
    a.seq = ++c->pipe_seq;
    a.timeout_ticks = (uint64_t)(c->timeout_s * 1e8);  // s_memrealtime: 100 MHz
    a.kmax = c->pipe_kmax;
    a.chunk = chunk;
    a.count = count;
    a.nchunks = (uint32_t)nchunks;
    a.n = c->size;
    a.me = me;
    for (size_t j = 0; j < pr.order.size(); ++j) a.order[j] = pr.order[j];
    a.role_mask = pr.role_mask;
    // vector paths: every fold operand shares the destination's misalignment (a whole element);
    // a pull needs only its source and destination to agree
    const uintptr_t m = (uintptr_t)a.dst & 15;
    a.wt = coll_tune().pipe_wt;
    a.co_fold = (m % esz) == 0;
    for (int q = 0; q < c->size && a.co_fold; ++q) a.co_fold = (((uintptr_t)a.src[q]) & 15) == m;
    for (int q = 0; q < c->size; ++q)
        if ((((uintptr_t)a.peer_rbuf[q]) & 15) == m) a.co_pull |= 1ull << q;
    // persistent grid: pipe_wg_per_cu workgroups of 256 per CU, split among the ranks sharing
    // this GPU.  Ranks that share a GPU must all be resident at once (rank A's pull items spin
    // until rank B's fold items have run), so their grids together stay within what the CUs hold.
    const uint64_t total = (uint64_t)nchunks * n;
    const int share = std::max(1, c->pipe_share);
    int wpc = coll_tune().pipe_wg_per_cu;
    if (share > 1) wpc = std::min(wpc, pipe_blocks_per_cu(op, type, count));
    uint64_t grid = (uint64_t)std::max(1, wpc * device_cu_count() / share);
    if (share == 1) grid = std::max<uint64_t>(grid, 8);
    if (grid > total) grid = total;
    const bool tp = c->time_phases && c->tev[0];
    if (tp) MI_HIP(hipEventRecord(c->tev[0], s));
    TRACE(c, "pipe launch seq %llu grid %llu chunks %zu x %zu elements qbase %llu co_fold %d co_pull %llx",
          (unsigned long long)a.seq, (unsigned long long)grid, nchunks, chunk, (unsigned long long)a.qbase, a.co_fold,
          (unsigned long long)a.co_pull);
    if (debug_on()) {  // progress words the host can read while the kernel runs
        if (!c->pipe_dbg) MI_HIP(hipHostMalloc((void **)&c->pipe_dbg, 4 * 4096 * sizeof(uint64_t), hipHostMallocCoherent));
        std::memset(c->pipe_dbg, 0, 4 * 4096 * sizeof(uint64_t));
        if (grid <= 4096) a.dbg = c->pipe_dbg;
    }
    rc = launch_pipe_slot(op, type, a, (unsigned)grid, s);
    if (rc) return rc;
    if (tp) MI_HIP(hipEventRecord(c->tev[1], s));
    if (a.dbg) {
        const auto t0 = std::chrono::steady_clock::now();
        double next = 2.0;
        while (hipStreamQuery(s) == hipErrorNotReady) {
            usleep(1000);
            const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            if (el > next) {
                next += 5.0;
                for (uint64_t g = 0; g < grid; ++g)
                    TRACE(c, "pipe wg %llu: item %lld stage %lld flag %lld polls %lld", (unsigned long long)g,
                          (long long)c->pipe_dbg[4 * g], (long long)c->pipe_dbg[4 * g + 1], (long long)c->pipe_dbg[4 * g + 2],
                          (long long)c->pipe_dbg[4 * g + 3]);
                uint64_t qv = 0;
                TRACE(c, "pipe err word %u", (unsigned)__atomic_load_n(c->ll_err, __ATOMIC_ACQUIRE));
                (void)qv;
            }
        }
    }
    // every peer is in this call (the exchange met them), but one may die inside it: poll, and a
    // peer that is gone sends the kernel's flag waits away through the error word
    bool gone = false;
    for (unsigned spins = 1; hipStreamQuery(s) == hipErrorNotReady; ++spins) {
        if (spins > 256) sched_yield();
        if (!gone && (spins & 0x3fffu) == 0 && peer_gone(c)) {
            gone = true;
            __atomic_store_n(c->ll_err, 1u, __ATOMIC_RELEASE);
        }
    }
    MI_HIP(hipStreamSynchronize(s));
    if (__atomic_load_n(c->ll_err, __ATOMIC_ACQUIRE)) {
        if (gone) {
            (void)hipMemsetAsync(c->pipe_queue, 0, sizeof(uint64_t), s);
            (void)hipStreamSynchronize(s);
            c->pipe_qbase = 0;
            return MI355X_ERR_PEER;
        }
        // the counter no longer has its expected value: start it over for the next call
        (void)hipMemsetAsync(c->pipe_queue, 0, sizeof(uint64_t), s);
        (void)hipStreamSynchronize(s);
        c->pipe_qbase = 0;
        c->ctrl->abort_flag.store(1);
        return set_error(MI355X_ERR_TIMEOUT, "rank %d: pipelined allreduce %llu timed out waiting for a peer", c->rank,
                         (unsigned long long)a.seq);
    }
    c->pipe_qbase += total + grid;  // every workgroup: its items + one dequeue past the end
    TRACE(c, "pipe done seq %llu", (unsigned long long)a.seq);
    if (tp) {
        MI_HIP(hipEventElapsedTime(&c->phase_ms[0], c->tev[0], c->tev[1]));
        c->phase_ms[1] = 0.f;
    }
    return barrier(c);  // peers may still read my rbuf / my input until everybody is done
}

void ll_program(LLArgs &a, const Program &pr)
{
    if (!pr.is_fold) {
        a.prog = LL_TREE;
        a.nsteps = (int)pr.steps.size();
        for (int k = 0; k < a.nsteps; ++k) a.steps[k] = pr.steps[k];
        a.result = pr.result;
        return;
    }
    a.prog = LL_FOLD;
    for (size_t j = 0; j < pr.order.size(); ++j) a.order[j] = pr.order[j];
    a.role_mask = pr.role_mask;
}

// MPI_Reduce_scatter(_block) served by the resident service (LL_PULL_RS): after the handle
// exchange every rank evaluates its own block from the n mapped inputs with the reference
// schedule's per-element program (fold order or tree, as the LL form evaluates it), stores it
// write-through into rbuf, and completes once every peer has read its input -- the launch, the
// completion wait and the finishing barrier of the host-synchronised flow are gone.  Not in place
// (MPI_IN_PLACE is all-or-none: the block would overwrite input the peers still read).  Every
// rank decides alike: the largest block, the program and the sizes are the same everywhere.
bool svc_rs_usable(const mi355x_comm *c, size_t max_block_bytes, const Program &pr)
{
    return c->svc_ok && c->svc_rs && (c->flows & MI355X_FLOW_SVC_RS) && !c->loopback && c->size >= 2 && c->size <= kLLMaxRanks && max_block_bytes <= c->svc_pull_max &&
           (pr.is_fold ? pr.order.size() == (size_t)c->size
                       : (c->size <= kTreeMax && pr.steps.size() <= (size_t)kTreeSteps));
}

// off: my block's byte offset in every rank's input; bytes: my block's length
int svc_rs_run(mi355x_comm *c, int op, int type, const Program &pr, const std::vector<std::vector<void *>> &P,
                      const void *in, size_t off, void *rbuf, size_t bytes, size_t esz)
{
    int rc = ensure_ll(c);
    if (rc) return rc;
    LLArgs a;
    std::memset(&a, 0, sizeof(a));
    ll_program(a, pr);
    SvcCall call;
    std::memset(&call, 0, sizeof(call));
    call.seq = ++c->ll_seq;
    call.src = in;
    call.dst = rbuf;
    call.nbytes = bytes;
    call.count = bytes / esz;
    call.role_mask = a.role_mask;
    call.op = op;
    call.type = type;
    call.mode = LL_PULL_RS;
    call.prog = a.prog;
    call.nsteps = a.nsteps;
    call.result = a.result;
    for (int q = 0; q < c->size; ++q) {
        call.order[q] = a.order[q];
        call.srcs[q] = (const char *)P[0][q] + off;
    }
    for (int k = 0; k < a.nsteps; ++k) call.steps[k] = a.steps[k];
    return svc_call(c, call, (bytes + kLLChunk - 1) / kLLChunk);
}

} // namespace mi355x
