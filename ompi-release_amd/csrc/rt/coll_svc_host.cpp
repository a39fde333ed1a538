// coll_svc_host.cpp -- host side of the resident LL service: launch, calls, ownership,
// handover, revocation and the process-wide service resources (split out of coll_comm.cpp).

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

// ----------------------------------------------------------------- resident LL service
// (coll_svc.hip, svc_queue.cpp).  One service per process and GPU, owned by one communicator at a
// time: the service's kernel serves one communicator's LL region, and a rank whose service were
// busy with another communicator's call could not take part in this one's (a cross-process
// circular wait for MPI_THREAD_MULTIPLE programs).  Ownership is taken where it is used: a
// communicator claims its process's service at its first service-sized call (svc_claim; every
// rank of the call claims without waiting and the communicator uses the service only if every rank
// got it), so the communicator that issues the small collectives -- typically a dup or split of
// MPI_COMM_WORLD -- gets it, not the first one created.  An owner that has been idle on every rank
// for svc_handover_s hands it over to another communicator of the process that wants it
// (svc_revoke), at a point where every one of its ranks is between the same two calls.
std::mutex g_svc_mtx;
std::map<int, mi355x_comm *> g_svc_owner;  // device -> owning communicator

uint64_t mono_ns()
{
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);  // (one clock for every process of the node)
    return (uint64_t)t.tv_sec * 1000000000ull + (uint64_t)t.tv_nsec;
}

uint64_t *svc_done_word(mi355x_comm *c) { return c->svc_host; }
uint32_t *svc_err_word(mi355x_comm *c) { return reinterpret_cast<uint32_t *>(c->svc_host + 1); }

// ring the doorbell: the page may be write-combined (BAR), so fence the stores out in order
void svc_ring(mi355x_comm *c, uint64_t v)
{
    _mm_sfence();
    __atomic_store_n(&c->svc_page->door, v, __ATOMIC_RELEASE);
    _mm_sfence();
}

int svc_launch(mi355x_comm *c, uint64_t first)
{
    SvcArgs g;
    std::memset(&g, 0, sizeof(g));
    c->svc_page->ctr = 0;  // not resident: nothing else touches them
    c->svc_page->go = 0;
    c->svc_page->shrink = 0;
    c->svc_host[2] = 0;
    _mm_sfence();
    g.page = c->svc_page;
    g.done = svc_done_word(c);
    g.err = svc_err_word(c);
    g.my_ll = c->ll_base;
    for (int q = 0; q < c->size; ++q) g.peer_ll[q] = c->ll_peer[q];
    g.first = first;
    g.slot_gran = c->ll_slot / 4;
    g.idle_ticks = (uint64_t)(c->svc_idle_s * 1e8);  // s_memrealtime: 100 MHz
    g.timeout_ticks = (uint64_t)(c->timeout_s * 1e8);
    g.shrink_ticks = (uint64_t)(c->svc_shrink_s * 1e8);
    g.shrunk = c->svc_host + 2;
    g.n = c->size;
    g.me = c->rank;
    g.nwg = c->svc_nwg;
    g.trace = c->svc_trace;
    if (svc_dispatch(c->svcq, g, c->svc_nwg)) return set_error(MI355X_ERR_HIP, "service dispatch: the previous launch is still resident");
    c->svc_launches++;
    return MI355X_SUCCESS;
}

// ask a resident service to leave and wait until it has (no call is in flight: calls complete
// before the engine returns).  False if it never left: its kernel may still poll the doorbell page
// and write the host words and the LL regions, so none of them may be freed (svc_release leaks
// them and the communicator is aborted).
bool svc_stop(mi355x_comm *c)
{
    if (c->svc_stuck) return false;
    if (!c->svcq || !svc_resident(c->svcq)) return true;
    svc_ring(c, kSvcQuit);
    if (!svc_wait_exit(c->svcq, c->timeout_s + 5.0)) {
        fprintf(stderr, "[mi355x r%d] resident service did not leave: its memory is kept, the communicator is aborted\n",
                c->rank);
        c->svc_stuck = true;
        if (c->ctrl) c->ctrl->abort_flag.store(1);
        return false;
    }
    svc_ring(c, c->ll_seq << kSvcPartBits);  // back to the last call's number: the next launch waits for the next
    return true;
}

// A call that takes a host-synchronised flow asks a resident service to leave, without waiting:
// with several processes on one GPU (the one-GPU rehearsal) a resident kernel slows every other
// launch of every process on the device (17 -> 54 us per small host-path allreduce,
// profiles/r03_queue_probe.jsonl), so the service stays only while small calls keep coming.  If
// the next service call rings the doorbell before the kernel has read the request, the kernel
// simply serves it; otherwise it has left and the call relaunches it.
void svc_park(mi355x_comm *c)
{
    if (c->svc_ok && c->svcq && svc_resident(c->svcq)) svc_ring(c, kSvcQuit);
}

// post `call` (number call.seq, `part` participating workgroups) and wait for its completion
int svc_call(mi355x_comm *c, const SvcCall &call, uint64_t part)
{
    const uint64_t seq = call.seq;
    // a service shrunk to its first workgroup while idle serves up to kSvcShrunkMaxPart slices
    // alone; a call that wants more (the pull forms) relaunches the full grid first
    if (std::min<uint64_t>(part, (uint64_t)c->svc_nwg) > kSvcShrunkMaxPart && svc_resident(c->svcq) &&
        __atomic_load_n(c->svc_host + 2, __ATOMIC_ACQUIRE)) {
        if (!svc_stop(c)) return set_error(MI355X_ERR_TIMEOUT, "rank %d: the resident service did not leave", c->rank);
        c->svc_regrows++;
    }
    std::memcpy(&c->svc_page->call, &call, sizeof(call));
    svc_ring(c, (seq << kSvcPartBits) | std::min<uint64_t>(std::max<uint64_t>(part, 1), (uint64_t)c->svc_nwg));
    int rc = MI355X_SUCCESS;
    if (!svc_resident(c->svcq)) rc = svc_launch(c, seq);
    if (rc) return rc;
    const uint64_t *done = svc_done_word(c);
    const uint32_t *err = svc_err_word(c);
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned spins = 1; __atomic_load_n(done, __ATOMIC_ACQUIRE) != seq; ++spins) {
        _mm_pause();
        if (spins & 255u) continue;
        // a peer that has not called yet may be waiting in a send for a receive of mine
        if ((spins & 1023u) == 0) barrier_progress(c, false);
        if (__atomic_load_n(err, __ATOMIC_ACQUIRE)) {
            rc = set_error(MI355X_ERR_TIMEOUT, "rank %d: service call %llu timed out waiting for a peer", c->rank,
                           (unsigned long long)seq);
            break;
        }
        if (!svc_resident(c->svcq)) {
            // it left idle just before the doorbell rang: start it again for this call
            if (__atomic_load_n(done, __ATOMIC_ACQUIRE) == seq) break;
            rc = svc_launch(c, seq);
            if (rc) break;
        }
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > c->timeout_s) {
            rc = set_error(MI355X_ERR_TIMEOUT, "rank %d: service call %llu did not complete", c->rank,
                           (unsigned long long)seq);
            break;
        }
        if ((spins & 0x3ffffu) == 0 && peer_gone(c)) {
            // the kernel may wait for that peer until its own bound: the error word sends it away
            __atomic_store_n(const_cast<uint32_t *>(err), 1u, __ATOMIC_RELEASE);
            rc = MI355X_ERR_PEER;
            break;
        }
    }
    if (rc) {
        svc_stop(c);
        *svc_err_word(c) = 0;
        return rc;
    }
    c->svc_calls++;
    c->ctrl->slot[c->rank].svc_last_ns.store(mono_ns(), std::memory_order_relaxed);
    return MI355X_SUCCESS;
}

// one LL call through the service: `a` carries the call (mode, buffers, program, masks)
int svc_run(mi355x_comm *c, LLArgs &a, int op, int type, hipStream_t s)
{
    MI_HIP(hipStreamSynchronize(s));  // the inputs: every earlier operation on the caller's stream
    SvcCall call;
    std::memset(&call, 0, sizeof(call));
    call.seq = ++c->ll_seq;
    call.src = a.src;
    call.dst = a.dst;
    call.nbytes = a.nbytes;
    call.count = a.count;
    call.early = a.early;
    call.late = a.late;
    call.split = a.split;
    call.role_mask = a.role_mask;
    call.push_mask = a.push_mask;
    call.recv_mask = a.recv_mask;
    call.op = op;
    call.type = type;
    call.mode = a.mode;
    call.prog = a.prog;
    call.root = a.root;
    call.nsteps = a.nsteps;
    call.result = a.result;
    for (int j = 0; j < c->size; ++j) call.order[j] = a.order[j];
    for (int k = 0; k < a.nsteps && k < kTreeSteps; ++k) call.steps[k] = a.steps[k];
    return svc_call(c, call, (a.nbytes + kLLChunk - 1) / kLLChunk);
}

// The one-phase ring-ordered allreduce (k_ring_all's work) served by the resident service
// (LL_PULL): the caller has exchanged every rank's input and rbuf (P[0], P[1]); the service reads
// the n inputs where they are, folds every element in its ring block's order, and completes only
// once every peer has read this rank's input -- the launch, the completion wait and the finishing
// barrier of the host-synchronised form are gone.  Same decision on every rank (sizes and every
// rank's buffer alignment, svc_pull_usable).
bool svc_pull_usable(const mi355x_comm *c, size_t bytes, size_t esz)
{
    return c->svc_ok && (c->flows & MI355X_FLOW_SVC_PULL) && !c->loopback && esz >= 4 && bytes > c->svc_max &&
           bytes <= c->svc_pull_max &&
           bytes < ((size_t)1 << 31);
}

// the same for allgather / bcast (LL_PULL_AG / LL_PULL_BC): `bytes` per rank between the LL form's
// limit and the copy limit (svc_copy_max); no alignment condition (each rank copies into its own buffer, with
// 16-B vectors where both ends allow)
bool svc_pull_copy_usable(const mi355x_comm *c, size_t bytes)
{
    return c->svc_ok && (c->flows & MI355X_FLOW_SVC_COPY) && !c->loopback && bytes > c->svc_max && bytes <= c->svc_copy_max &&
           bytes * (size_t)c->size < ((size_t)1 << 31);
}

int svc_pull_copy_run(mi355x_comm *c, int mode, const std::vector<std::vector<void *>> &P, const void *src,
                             void *dst, size_t bytes, int root)
{
    int rc = ensure_ll(c);
    if (rc) return rc;
    SvcCall call;
    std::memset(&call, 0, sizeof(call));
    call.seq = ++c->ll_seq;
    call.src = src;
    call.dst = dst;
    call.nbytes = bytes;
    call.mode = mode;
    call.root = root;
    for (int q = 0; q < c->size; ++q) call.srcs[q] = P[0][q];
    const size_t total = mode == LL_PULL_AG ? bytes * (size_t)c->size : bytes;
    return svc_call(c, call, (total + kLLChunk - 1) / kLLChunk);
}

int svc_pull_run(mi355x_comm *c, int op, int type, const std::vector<std::vector<void *>> &P, const void *in,
                        void *rbuf, size_t count, size_t esz, size_t early, size_t late, size_t split)
{
    int rc = ensure_ll(c);
    if (rc) return rc;
    SvcCall call;
    std::memset(&call, 0, sizeof(call));
    call.seq = ++c->ll_seq;
    call.src = in;
    call.dst = rbuf;
    call.nbytes = count * esz;
    call.count = count;
    call.early = early;
    call.late = late;
    call.split = split;
    call.op = op;
    call.type = type;
    call.mode = LL_PULL;
    call.prog = LL_RING;
    for (int q = 0; q < c->size; ++q) call.srcs[q] = P[0][q];
    return svc_call(c, call, (call.nbytes + kLLChunk - 1) / kLLChunk);
}

// MI355X_SVC_TRACE=1: mean microseconds between the stamped stages over the traced calls
void svc_trace_report(mi355x_comm *c)
{
    if (!c->svc_trace) return;
    std::vector<uint64_t> rows((size_t)kSvcTraceCalls * kSvcTraceCols, 0);
    if (hipMemcpy(rows.data(), c->svc_trace, rows.size() * sizeof(uint64_t), hipMemcpyDeviceToHost) != hipSuccess)
        rows.assign(rows.size(), 0);
    double acc[kSvcTraceCols] = {0};
    int nrows = 0;
    for (int r = 0; r < kSvcTraceCalls; ++r) {
        const uint64_t *row = rows.data() + (size_t)r * kSvcTraceCols;
        if (!row[0] || !row[6] || !row[7] || !row[8] || !row[9] || row[6] < row[1]) continue;
        // stages in time order: 1 door, 2 descriptor, 3 pushed, 4 received, 8 results issued (the
        // first slice), 9 workgroup joined, 7 evaluated (every slice), 5 stored, 6 completed
        const int order[] = {1, 2, 3, 4, 8, 9, 7, 5, 6};
        for (int k = 1; k < 9; ++k) acc[order[k]] += (double)(row[order[k]] - row[order[k - 1]]) * 0.01;  // 100 MHz
        ++nrows;
    }
    if (nrows)
        fprintf(stderr, "[mi355x r%d] resident service, %d traced calls, mean us: door->descriptor %.2f, "
                "->pushed %.2f, ->received %.2f, ->issued %.2f, ->joined %.2f, ->evaluated %.2f, ->stored %.2f, "
                "->completed %.2f\n", c->rank, nrows, acc[2] / nrows, acc[3] / nrows, acc[4] / nrows, acc[8] / nrows,
                acc[9] / nrows, acc[7] / nrows, acc[5] / nrows, acc[6] / nrows);
    (void)hipFree(c->svc_trace);
    c->svc_trace = nullptr;
}

std::map<int, SvcRes> g_svc_res;  // device -> resources (g_svc_mtx)

// (g_svc_mtx held) this communicator's view of the process's service resources (created if needed)
bool svc_attach(mi355x_comm *c)
{
    SvcRes &r = g_svc_res[c->device];
    if (r.stuck) return false;
    const char *inj = getenv("MI355X_SELFTEST_FAIL");  // (tests: this rank's service cannot open)
    if (inj && std::strstr(inj, "svc_open")) return false;
    if (!r.q) {
        auto *q = new SvcQueue;
        std::string why;
        if (svc_queue_create(c->device, q, &why)) {
            TRACE(c, "resident service unavailable: %s", why.c_str());
            delete q;
            return false;
        }
        void *pg = nullptr;
        if (svc_page_alloc(q, (sizeof(SvcPage) + 4095) & ~(size_t)4095, &pg, &r.page_dev)) {
            svc_queue_destroy(q);
            delete q;
            return false;
        }
        uint64_t *host = nullptr;
        if (hipHostMalloc((void **)&host, 4096, hipHostMallocCoherent) != hipSuccess) {
            svc_page_free(pg, r.page_dev);
            svc_queue_destroy(q);
            delete q;
            return false;
        }
        std::memset(host, 0, 4096);
        r.q = q;
        r.page = static_cast<SvcPage *>(pg);
        r.host = host;
    }
    if (svc_resident(r.q)) return false;  // (never: a previous owner's kernel leaves before it lets go)
    c->svcq = r.q;
    c->svc_page = r.page;
    c->svc_page_dev = r.page_dev;
    c->svc_host = r.host;
    // the previous owner's call numbers mean nothing here: the completion and error words start over
    __atomic_store_n(c->svc_host, 0ull, __ATOMIC_RELEASE);
    __atomic_store_n(reinterpret_cast<uint32_t *>(c->svc_host + 1), 0u, __ATOMIC_RELEASE);
    svc_ring(c, c->ll_seq << kSvcPartBits);
    if (!c->svc_attached) {
        r.users++;
        c->svc_attached = true;
    }
    if (!c->svc_trace && env_double("MI355X_SVC_TRACE", 0.0) != 0.0) {
        const size_t tb = sizeof(uint64_t) * kSvcTraceCalls * kSvcTraceCols;
        // (device memory: the kernel keeps a call's stamps in LDS and writes the row once the call is
        // complete, so the stamps cost no host-memory round trip inside the call)
        if (hipMalloc((void **)&c->svc_trace, tb) != hipSuccess || hipMemset(c->svc_trace, 0, tb) != hipSuccess) {
            (void)hipGetLastError();
            c->svc_trace = nullptr;
        }
    }
    return true;
}

// the kernel leaves; this communicator stops using the resources (which stay for the next owner)
void svc_detach(mi355x_comm *c)
{
    if (!svc_stop(c)) g_svc_res[c->device].stuck = true;
    c->svcq = nullptr;
    c->svc_page = nullptr;
    c->svc_host = nullptr;
    c->svc_ok = false;
}

// (g_svc_mtx held) give up ownership
void svc_unclaim_locked(mi355x_comm *c)
{
    if (!c->svc_owner) return;
    auto it = g_svc_owner.find(c->device);
    if (it != g_svc_owner.end() && it->second == c) g_svc_owner.erase(it);
    c->svc_owner = false;
}

void svc_let_go(mi355x_comm *c)
{
    std::lock_guard<std::mutex> g(g_svc_mtx);
    svc_detach(c);
    svc_unclaim_locked(c);
}

// at destruction: let go, and free the process's resources with their last user
void svc_release(mi355x_comm *c)
{
    std::lock_guard<std::mutex> g(g_svc_mtx);
    const bool had = c->svcq != nullptr;
    svc_detach(c);
    svc_unclaim_locked(c);
    if (had || c->svc_attached) svc_trace_report(c);
    if (!c->svc_attached) return;
    c->svc_attached = false;
    SvcRes &r = g_svc_res[c->device];
    if (--r.users > 0 || r.stuck) return;  // (stuck: leaked on purpose -- its kernel may still touch them)
    svc_queue_destroy(r.q);
    delete r.q;
    svc_page_free(r.page, r.page_dev);
    (void)hipHostFree(r.host);
    g_svc_res.erase(c->device);
}

// The call gate.  Every engine collective of a multi-process communicator runs inside it: the
// rank's RankSlot::gate is 1 for the call's duration and its call count advances when it leaves.
// A process that wants the service another communicator owns may take it (svc_revoke) only by
// closing the gates of every rank of the owner while all of them are between the same two calls;
// the owner's ranks then let go of the service at their next call, on every rank at the same call.
// A revoker marks a gate with its pid, (pid << 8) | 2, so a waiter can take the gate back from a
// revoker that died holding it (pids fit in 24 bits: Linux's pid_max is at most 2^22).
constexpr uint32_t kGateCall = 1u, kGateRevoker = 2u;
uint32_t gate_revoker_word() { return ((uint32_t)getpid() << 8) | kGateRevoker; }

void gate_enter(mi355x_comm *c)
{
    std::atomic<uint32_t> &g = c->ctrl->slot[c->rank].gate;
    unsigned spins = 0;
    for (uint32_t z = 0; !g.compare_exchange_weak(z, kGateCall, std::memory_order_acq_rel); z = 0) {
        _mm_pause();
        if (++spins > 256) sched_yield();  // (held only while a revoker stops this rank's service)
        if ((spins & 0xfff) == 0 && (z & 0xff) == kGateRevoker && !pid_alive((pid_t)(z >> 8))) {
            uint32_t w = z;  // the revoker died holding it
            g.compare_exchange_strong(w, 0u, std::memory_order_acq_rel);
        }
    }
    if (c->svc_ok && c->ctrl->svc_revoked.load(std::memory_order_acquire) == c->svc_epoch) {
        TRACE(c, "the resident service went to another communicator of a peer process: letting go");
        svc_let_go(c);
    }
}

void gate_exit(mi355x_comm *c)
{
    RankSlot &s = c->ctrl->slot[c->rank];
    s.calls.store(++c->gate_calls, std::memory_order_relaxed);
    s.gate.store(0u, std::memory_order_release);
}

// (g_svc_mtx held) take the process's service from its owner x: only while every rank of x is
// between the same two calls (all gates closed by us, equal call counts) and none has served a
// call for svc_handover_s.  x's ranks in other processes let go at their next call (gate_enter).
bool svc_revoke(mi355x_comm *x)
{
    if (!x->gated) return false;
    Ctrl *k = x->ctrl;
    // the gates in rank order; a gate another process's revoker holds (2) is waited for -- revokers
    // hold gates only briefly and never wait while holding a higher one, so ordered acquisition
    // cannot deadlock -- while a rank inside a call (1) ends the attempt
    int got = 0;
    const auto t0 = std::chrono::steady_clock::now();
    for (bool busy = false; got < x->size && !busy;) {
        uint32_t z = 0;
        if (k->slot[got].gate.compare_exchange_strong(z, gate_revoker_word(), std::memory_order_acq_rel)) {
            ++got;
            continue;
        }
        busy = (z & 0xff) != kGateRevoker ||
               std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > 0.1;
        _mm_pause();
    }
    bool ok = got == x->size && x->svc_ok;
    if (ok) {
        const uint64_t c0 = k->slot[0].calls.load(std::memory_order_acquire);
        uint64_t last = 0;
        for (int q = 0; q < x->size; ++q) {
            ok = ok && k->slot[q].calls.load(std::memory_order_acquire) == c0;
            last = std::max(last, k->slot[q].svc_last_ns.load(std::memory_order_acquire));
        }
        const uint64_t now = mono_ns();
        ok = ok && now > last && (double)(now - last) * 1e-9 >= x->svc_handover_s;
        if (ok) {
            k->svc_revoked.store(x->svc_epoch, std::memory_order_release);
            svc_detach(x);
            x->svc_owner = false;
            x->svc_revocations++;
        }
    }
    for (int q = 0; q < got; ++q) k->slot[q].gate.store(0u, std::memory_order_release);
    return ok;
}

// Zero the LL region and start the LL call numbering over on every rank (collective): after a
// service self-test failed somewhere, ranks may disagree on the call number or hold stale granules.
int ll_resync(mi355x_comm *c)
{
    (void)svc_stop(c);  // (every LL launch of this communicator was synchronised by its caller)
    int rc = barrier(c);
    if (rc) return rc;
    if (c->svc_stuck) return set_error(MI355X_ERR_HIP, "rank %d: the resident service did not leave", c->rank);
    hipStream_t ss = setup_stream(c);
    MI_HIP(hipMemsetAsync(c->ll_base, 0, c->ll_bytes, ss));
    MI_HIP(hipMemsetAsync(c->ll_ctr, 0, sizeof(uint64_t), ss));
    MI_HIP(hipStreamSynchronize(ss));
    c->ll_seq = 0;
    c->ll_ctr_base = 0;
    if (c->ll_err) *c->ll_err = 0;
    if (c->svc_host) {
        __atomic_store_n(c->svc_host, 0ull, __ATOMIC_RELEASE);
        __atomic_store_n(reinterpret_cast<uint32_t *>(c->svc_host + 1), 0u, __ATOMIC_RELEASE);
        svc_ring(c, 0);
    }
    return barrier(c);
}

} // namespace mi355x
