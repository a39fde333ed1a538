// coll_ll_host.cpp -- host side of the low-latency (LL) protocol: the LL region, its launch
// and the creation-time LL self-test (split out of coll_comm.cpp).

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

// ----------------------------------------------------------------- low-latency path
// Loopback communicators (threads of one process) never take it: their kernels would share the
// process's few hardware queues and a rank's spinning kernel could sit in front of the peer
// kernel it waits for.
// the resident service takes every LL-protocol call up to svc_max bytes (svc_ok: created, self-
// tested and owned on every rank -- the same decision on every rank)
bool svc_usable(const mi355x_comm *c, size_t bytes)
{
    return c->svc_ok && (c->flows & MI355X_FLOW_SVC_LL) && bytes > 0 && bytes <= c->svc_max;
}

bool ll_usable(const mi355x_comm *c, size_t bytes)
{
    if (c->loopback || c->size < 2 || c->size > kLLMaxRanks || bytes == 0) return false;
    if (svc_usable(c, bytes)) return true;
    if (bytes > c->ll_max) return false;
    // ranks sharing a GPU: every rank's blocks spin until the others' have pushed, so all of them
    // must be resident at once -- at most one block per CU for the ranks together
    const size_t blocks = (bytes + kLLChunk - 1) / kLLChunk;
    return c->pipe_share <= 1 || blocks * (size_t)c->pipe_share <= (size_t)device_cu_count();
}

bool svc_stop(mi355x_comm *c);
int svc_run(mi355x_comm *c, LLArgs &a, int op, int type, hipStream_t s);

// (Re)allocate and exchange the LL region: [ack words, one per rank][2 parities x n slots of
// ll_max payload bytes as 8-byte granules].  Collective: every rank reaches it in the same call.

int ensure_ll(mi355x_comm *c)
{
    // payload bytes per slot (at least 64 KiB: the creation-time self-test runs with ll_max 0)
    const size_t want =
        (std::max({c->ll_max, c->svc_max, (size_t)64 << 10}) + kLLChunk - 1) / kLLChunk * kLLChunk;
    if (c->ll_base && c->ll_slot >= want) return MI355X_SUCCESS;
    // a resident service holds the old region's addresses
    if (!svc_stop(c)) return set_error(MI355X_ERR_HIP, "rank %d: the resident service did not leave", c->rank);
    const size_t n = (size_t)c->size;
    const size_t total = kLLAckBytes + 2 * n * (want / 4) * sizeof(uint64_t);
    if (c->ll_base) (void)hipFree(c->ll_base);
    c->ll_base = nullptr;
    MI_HIP(hipExtMallocWithFlags((void **)&c->ll_base, total, hipDeviceMallocUncached));
    hipStream_t ss = setup_stream(c);
    MI_HIP(hipMemsetAsync(c->ll_base, 0, total, ss));
    if (!c->ll_ctr) MI_HIP(hipMalloc((void **)&c->ll_ctr, sizeof(uint64_t)));
    MI_HIP(hipMemsetAsync(c->ll_ctr, 0, sizeof(uint64_t), ss));
    MI_HIP(hipStreamSynchronize(ss));
    if (!c->ll_err) MI_HIP(hipHostMalloc((void **)&c->ll_err, sizeof(uint32_t), hipHostMallocCoherent));
    c->ll_slot = want;
    c->ll_bytes = total;
    c->ll_seq = 0;
    c->ll_ctr_base = 0;
    const void *mine[1] = {c->ll_base};
    const uint64_t sig[4] = {10, total, 0, 0};
    std::vector<std::vector<void *>> P;
    int rc = exchange(c, 1, mine, sig, P, nullptr, true, true);
    if (rc) return rc;
    c->ll_peer.assign(n, nullptr);
    for (size_t q = 0; q < n; ++q) c->ll_peer[q] = (char *)P[0][q];
    TRACE(c, "LL region %zu bytes (slot %zu payload bytes)", total, want);
    return barrier(c);  // every rank has read the exchange slots
}

// one LL call: fills the per-call fields of `a` (the caller sets mode, src, dst, nbytes,
// push_mask, the program) and runs it to completion
int ll_run(mi355x_comm *c, LLArgs &a, int op, int type, hipStream_t s)
{
    int rc = ensure_ll(c);
    if (rc) return rc;
    const size_t n = (size_t)c->size;
    const uint64_t all = (1ull << n) - 1;
    a.n = c->size;
    a.me = c->rank;
    a.push_mask &= all;
    switch (a.mode) {
    case LL_RED: a.recv_mask = (a.me == a.root) ? all : 0; break;
    case LL_BC: a.recv_mask = (a.me == a.root) ? 0 : (1ull << a.root); break;
    default: a.recv_mask = all; break;
    }
    if (svc_usable(c, a.nbytes)) return svc_run(c, a, op, type, s);
    svc_park(c);  // a per-call LL launch: the resident service steps aside as for the host flows
    const uint64_t seq = ++c->ll_seq;
    const size_t par = seq & 1, me = (size_t)c->rank;
    a.seq = seq;
    a.slot_gran = c->ll_slot / 4;
    uint64_t *my = reinterpret_cast<uint64_t *>(c->ll_base);
    for (size_t q = 0; q < n; ++q) {
        uint64_t *peer = reinterpret_cast<uint64_t *>(c->ll_peer[q]);
        a.peer_data[q] = peer + kLLAckBytes / 8 + (par * n + me) * a.slot_gran;
        a.peer_ack[q] = peer + me;
    }
    a.my_data = my + kLLAckBytes / 8 + par * n * a.slot_gran;
    a.my_ack = my;
    const uint64_t nblk = (a.nbytes + kLLChunk - 1) / kLLChunk;
    a.ctr = c->ll_ctr;
    a.ctr_target = c->ll_ctr_base + nblk;
    a.err = c->ll_err;
    *c->ll_err = 0;
    a.timeout_ticks = (uint64_t)(c->timeout_s * 1e8);  // s_memrealtime: 100 MHz
    rc = (a.mode == LL_AR || a.mode == LL_RED) ? launch_ll_slot(op, type, a, s) : launch_ll_copy(a, s);
    if (rc) return rc;
    // the kernel waits for every peer: poll instead of blocking -- a peer that has not called yet may
    // be waiting in point-to-point for this rank (MPI's progress rule), and a peer that is gone
    // sends the kernel away through the error word
    bool gone = false;
    for (unsigned spins = 1; hipStreamQuery(s) == hipErrorNotReady; ++spins) {
        if ((spins & 63u) == 0) barrier_progress(c, false);
        if (!gone && (spins & 0x3fffu) == 0 && peer_gone(c)) {
            gone = true;  // (peer_gone set the error and aborted the communicator)
            __atomic_store_n(c->ll_err, 1u, __ATOMIC_RELEASE);
        }
        if (spins > 4096) sched_yield();
    }
    MI_HIP(hipStreamSynchronize(s));
    if (__atomic_load_n(c->ll_err, __ATOMIC_ACQUIRE)) {
        (void)hipMemsetAsync(c->ll_ctr, 0, sizeof(uint64_t), s);  // its count is off now: restart it
        (void)hipStreamSynchronize(s);
        c->ll_ctr_base = 0;
        if (gone) return MI355X_ERR_PEER;
        return set_error(MI355X_ERR_TIMEOUT, "rank %d: LL call %llu timed out waiting for a peer", c->rank,
                         (unsigned long long)seq);
    }
    c->ll_ctr_base += nblk;
    return MI355X_SUCCESS;
}

double env_double(const char *name, double dflt);

// Collective, once at communicator creation: the LL region is built and one LL allgather of a
// rank-tagged 8 KiB pattern per rank runs with a short device-side bound (MI355X_LL_PROBE_S, 5 s).
// The LL path can be enabled (MI355X_KNOB_LL_MAX_BYTES) only if every rank saw every peer's bytes;
// otherwise small collectives always take the host-synchronised path (a protocol that misbehaves
// on some platform would otherwise stall every small call for timeout_s).  MI355X_LL=0 skips it.
int ll_selftest(mi355x_comm *c)
{
    const char *env = getenv("MI355X_LL");
    if ((env && atoi(env) == 0) || c->size > kLLMaxRanks) {
        c->ll_ok = false;
        c->ll_max = 0;
        return MI355X_SUCCESS;
    }
    int rc = ensure_ll(c);
    if (rc) return rc;
    const size_t per = std::min<size_t>(8192, c->ll_slot), n = (size_t)c->size;
    char *buf = nullptr;
    hipStream_t ss = setup_stream(c);
    bool ok = hipMalloc((void **)&buf, per * (n + 1)) == hipSuccess;
    if (ok) ok = hipMemsetAsync(buf, c->rank + 1, per, ss) == hipSuccess &&
                 hipMemsetAsync(buf + per, 0, per * n, ss) == hipSuccess && hipStreamSynchronize(ss) == hipSuccess;
    if (ok) {
        LLArgs a;
        std::memset(&a, 0, sizeof(a));
        a.mode = LL_AG;
        a.src = buf;
        a.dst = buf + per;
        a.nbytes = per;
        a.push_mask = ~0ull;
        const double saved = c->timeout_s;
        c->timeout_s = env_double("MI355X_LL_PROBE_S", 5.0);
        ok = ll_run(c, a, 0, 0, ss) == MI355X_SUCCESS;
        c->timeout_s = saved;
    }
    if (ok) {
        std::vector<unsigned char> h(per * n);
        ok = hipMemcpyAsync(h.data(), buf + per, per * n, hipMemcpyDeviceToHost, ss) == hipSuccess &&
             hipStreamSynchronize(ss) == hipSuccess;
        for (size_t q = 0; q < n && ok; ++q)
            for (size_t i = 0; i < per && ok; i += 509) ok = h[q * per + i] == (unsigned char)(q + 1);
    }
    (void)hipGetLastError();
    if (buf) (void)hipFree(buf);
    c->ctrl->slot[c->rank].ll_ok = ok ? 1 : 2;
    rc = barrier(c);
    if (rc) return rc;
    bool all = true;
    for (int q = 0; q < c->size; ++q) all = all && c->ctrl->slot[q].ll_ok == 1;
    c->ll_ok = all;
    if (!all) {
        c->ll_max = 0;
        if (c->rank == 0) fprintf(stderr, "[mi355x] low-latency path self-test failed: small collectives use the host-synchronised path\n");
    }
    TRACE(c, "LL self-test: %s", all ? "ok" : "failed -> LL off");
    return barrier(c);
}

} // namespace mi355x
