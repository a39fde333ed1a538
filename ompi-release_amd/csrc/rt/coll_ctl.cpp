// coll_ctl.cpp -- the engine's control segment and rendezvous: rank liveness, the host barrier,
// buffer registration (the IPC export cache), the per-call exchange of every rank's buffers and
// the call's finish, the per-communicator scratch (split out of coll_comm.cpp, no change).

#include <fcntl.h>
#include <hsa/hsa_ext_amd.h>
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

// The launch-shape knobs are per communicator (coll/tuned's forced values are per communicator too,
// coll_tuned_module.c:178-226): each engine call runs with its communicator's CollTune, installed
// for the calling thread by CallStream; outside a call (point-to-point pulls) the process defaults.
CollTune &coll_tune_default()
{
    static CollTune t;
    return t;
}
static thread_local CollTune *t_tune = nullptr;
CollTune &coll_tune() { return t_tune ? *t_tune : coll_tune_default(); }
CollTune *coll_tune_use(CollTune *t)
{
    CollTune *prev = t_tune;
    t_tune = t;
    return prev;
}

} // namespace mi355x

namespace mi355x {


// ----------------------------------------------------------------- liveness
// a process exists and has not exited (a zombie -- exited, not yet reaped by its parent -- is gone)
bool pid_alive(pid_t pid)
{
    if (pid <= 0) return false;
    if (kill(pid, 0) != 0 && errno == ESRCH) return false;
    char path[64], buf[512];
    snprintf(path, sizeof(path), "/proc/%d/stat", (int)pid);
    const int fd = open(path, O_RDONLY);
    if (fd < 0) return true;  // (no /proc: trust kill)
    const ssize_t n = read(fd, buf, sizeof(buf) - 1);
    close(fd);
    if (n <= 0) return true;
    buf[n] = 0;
    const char *p = strrchr(buf, ')');
    return !(p && p[1] == ' ' && (p[2] == 'Z' || p[2] == 'X'));
}

// A peer process that died without setting the abort flag (SIGKILL, the OOM killer) would leave
// the others spinning in an unbounded wait (the buffer-kind vote) or until timeout_s.  Waits check
// every rank's published pid now and then; a rank whose process is gone aborts the communicator.
// (Loopback ranks share this process.)
// The pid is checked only where it means the same process: in this process's PID namespace (a
// pid published from another namespace is trusted alive), and with the start time it had when
// it was published (a pid the kernel gave to a new process is a dead peer).
uint64_t pid_namespace()
{
    struct stat st;
    return stat("/proc/self/ns/pid", &st) == 0 ? (uint64_t)st.st_ino : 0;
}

bool peer_gone(mi355x_comm *c)
{
    if (c->loopback || c->size == 1) return false;
    static const uint64_t my_ns = pid_namespace();
    for (int q = 0; q < c->size; ++q) {
        const RankSlot &sl = c->ctrl->slot[q];
        const pid_t pid = (pid_t)sl.pid;
        if (q == c->rank || pid <= 0) continue;
        if (sl.pid_ns && my_ns && sl.pid_ns != my_ns) continue;  // unverifiable here: alive
        bool gone = !pid_alive(pid);
        if (!gone && sl.pid_start) {
            const uint64_t now = proc_start_time(pid);
            gone = now != 0 && now != sl.pid_start;  // (0: unreadable -- alive)
        }
        if (gone) {
            c->ctrl->abort_flag.store(1);
            set_error(MI355X_ERR_PEER, "rank %d (pid %d) is gone: the communicator is aborted", q, (int)pid);
            return true;
        }
    }
    return false;
}

// ----------------------------------------------------------------- barrier
// Point-to-point progress from inside a collective's host waits.  MPI's progress rule: a receive
// posted before the collective completes while its sender waits in a blocking send (ob1 progresses
// posted receives inside any blocking call), so the pass may read a payload and open a peer mapping
// for it -- which must not overlap a peer's closes (coll_rcache.cpp, retire_map).  The pass announces
// itself (opening) and then looks for a member that is closing; a closer announces itself (closing)
// and then waits for every opening pass to end (close_window).  Sequentially consistent stores and
// loads on both sides (Dekker): one of the two always sees the other, so a pass either opens with no
// close of this communicator in flight or defers its opens to a later pass.
void barrier_progress(mi355x_comm *c, bool drain_fds)
{
    RankSlot &me = c->ctrl->slot[c->rank];
    me.opening.store(1, std::memory_order_seq_cst);
    bool closing = false;
    for (int r = 0; r < c->size && !closing; ++r)
        closing = r != c->rank && c->ctrl->slot[r].closing.load(std::memory_order_seq_cst) != 0;
    p2p_progress_all(closing);
    // a peer may be blocked sending us dmabuf fds (full socket queue) or asking for one (serve_fd:
    // an export -- so not while a member closes either)
    if (drain_fds && !closing && c->fd_sock >= 0 && c->reg_mtx.try_lock()) {
        (void)fd_drain(c, false);
        c->reg_mtx.unlock();
    }
    // and the caller's progress engine (opal_progress: ob1's requests on other communicators, the
    // component's nonblocking requests), under the same rule for the reads it starts
    const bool prev = p2p_defer_maps(closing);
    run_progress_hook();
    (void)p2p_defer_maps(prev);
    me.opening.store(0, std::memory_order_release);
}

// close this rank's retired mappings while no member's progress pass may be opening one.  A pass
// that stays open (its read waits for a dmabuf fd from a rank that is itself waiting here) is not
// waited out: after kCloseWaitMs the closes are left for the next window (the mappings stay retired,
// so the next exchange opens one again), and nothing is exported meanwhile -- serving an fd request
// here would be an export overlapping the other closers' closes, the race the window exists for.
static int close_window(mi355x_comm *c)
{
    constexpr double kCloseWaitMs = 20.0;
    RankSlot &me = c->ctrl->slot[c->rank];
    me.closing.store(1, std::memory_order_seq_cst);
    const auto t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < c->size; ++r) {
        unsigned spins = 0;
        while (r != c->rank && c->ctrl->slot[r].opening.load(std::memory_order_seq_cst) != 0) {
            if ((++spins & 255) == 0 &&
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() > kCloseWaitMs) {
                me.closing.store(0, std::memory_order_release);
                TRACE(c, "close window: rank %d's progress pass is still open; closes left for the next window", r);
                return MI355X_SUCCESS;
            }
            sched_yield();
        }
    }
    flush_retired(c);
    me.closing.store(0, std::memory_order_release);
    return MI355X_SUCCESS;
}

int barrier(mi355x_comm *c)
{
    if (c->size == 1) return MI355X_SUCCESS;
    Ctrl *k = c->ctrl;
    const uint64_t gen = k->bar_gen.load(std::memory_order_acquire);
    if (k->bar_count.fetch_add(1, std::memory_order_acq_rel) == (uint64_t)c->size - 1) {
        k->bar_count.store(0, std::memory_order_relaxed);
        k->bar_gen.fetch_add(1, std::memory_order_release);
        return MI355X_SUCCESS;
    }
    const auto t0 = std::chrono::steady_clock::now();
    unsigned spins = 0;
    while (k->bar_gen.load(std::memory_order_acquire) == gen) {
        if (k->abort_flag.load(std::memory_order_relaxed))
            return set_error(MI355X_ERR_PEER, "a peer aborted the communicator");
        if (++spins > 2048) {
            sched_yield();
            // a peer may wait in a send for a receive of mine, or for fds (those every 256th spin:
            // each one served is an export)
            if ((spins & 63) == 0) barrier_progress(c, (spins & 255) == 0);
            if ((spins & 0xffff) == 0) {
                if (peer_gone(c)) return MI355X_ERR_PEER;
                const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
                if (el > c->timeout_s) {
                    k->abort_flag.store(1);
                    // which rank is behind: every rank's published call number
                    char who[256] = "";
                    size_t w = 0;
                    for (int r = 0; r < c->size && w + 24 < sizeof(who); ++r)
                        w += (size_t)snprintf(who + w, sizeof(who) - w, " r%d:%llu", r,
                                              (unsigned long long)k->slot[r].seq.load());
                    return set_error(MI355X_ERR_TIMEOUT, "barrier timed out after %.0f s (rank %d, %llu of %d arrived; calls%s)",
                                     el, c->rank, (unsigned long long)k->bar_count.load(), c->size, who);
                }
            }
        }
    }
    return MI355X_SUCCESS;
}

// ----------------------------------------------------------------- registration
uint64_t buffer_id(const void *p)
{
    unsigned long long id = 0;
    if (hipPointerGetAttribute(&id, HIP_POINTER_ATTRIBUTE_BUFFER_ID, (hipDeviceptr_t)p) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return (uint64_t)id;
}

// an allocation of `bytes` goes to the peers as a dmabuf fd rather than a hipIpc handle: always from
// ipc_max up (hipIpcOpenMemHandle never returns for those), and at any size while the peer-mapping
// cache is bounded -- evicting hipIpc mappings while allocations churn hands peers wrong memory on
// this platform (coll_rcache.cpp, retire_map) -- unless the dmabuf route failed its probe
static bool via_dmabuf(const mi355x_comm *c, size_t bytes)
{
    return bytes >= c->ipc_max || ((c->rcache_max_maps || c->rcache_limit) && c->dmabuf_state != -1);
}

// does the dmabuf fd `fd` name the allocation at `base` itself, from its first byte?  The runtime
// exports the whole buffer object an allocation lives in, from the object's start: the ROCr
// allocation the HIP allocation was carved from (the runtime sub-allocates small hipMallocs out of
// 2 MiB objects; an allocation of its own has an object of its size rounded up to 2 MiB --
// tools/probe/bo_sizes.py, profiles/r06_bo_sizes.jsonl).  So the check is on identity, as the
// reference's is (IPC handle bytes memcmp'd, common_cuda.c:1581; CU_POINTER_ATTRIBUTE_BUFFER_ID,
// :1937-1958), never on contents: ROCr's allocation containing `base` must start at `base`
// (hsa_amd_pointer_info's agentBaseAddress), and the fd must be that allocation (its size, read with
// dma-buf's llseek, equals ROCr's sizeInBytes).  1 yes; 0 no (such an allocation keeps the hipIpc
// route, whose handle carries the offset); -1 unknown (treated as no).
static int export_names(void *base, int fd)
{
    const off_t end = lseek(fd, 0, SEEK_END);
    if (end < 0) return -1;
    (void)lseek(fd, 0, SEEK_SET);
    hsa_amd_pointer_info_t info;
    std::memset(&info, 0, sizeof(info));
    info.size = sizeof(info);
    if (hsa_amd_pointer_info(base, &info, nullptr, nullptr, nullptr) != HSA_STATUS_SUCCESS ||
        info.type == HSA_EXT_POINTER_TYPE_UNKNOWN)
        return -1;
    return (info.agentBaseAddress == base && (size_t)end == info.sizeInBytes) ? 1 : 0;
}

int local_handle(mi355x_comm *c, const void *p, BufDesc *d, bool force)
{
    std::lock_guard<std::recursive_mutex> reg_guard(c->reg_mtx);
    std::memset(d, 0, sizeof(*d));
    if (!p) return MI355X_SUCCESS;
    d->present = 1;
    if (c->loopback) {
        d->raw = (uint64_t)(uintptr_t)p;
        if (!force) {
            void *base = nullptr;
            size_t sz = 0;
            MI_HIP(hipMemGetAddressRange(&base, &sz, (void *)p));
            d->staged = sz >= c->ipc_max;
        }
        return MI355X_SUCCESS;
    }
    const uintptr_t up = (uintptr_t)p;
    const uint64_t id = buffer_id(p);
    for (size_t i = 0; i < c->local_regs.size(); ++i) {
        const LocalReg &r = c->local_regs[i];
        if (up >= r.base && up < r.base + r.size) {
            if (r.id == id && id != 0 && (r.has_h || !force)) {
                if (!force && !r.has_h) {  // (registered for the dmabuf route)
                    d->staged = 1;
                    d->base = r.base;
                    d->off = up - r.base;
                    d->id = r.id;
                    d->size = r.size;
                    return MI355X_SUCCESS;
                }
                d->h = r.h;
                d->off = up - r.base;
                d->base = r.base;
                d->id = r.id;
                d->size = r.size;
                return MI355X_SUCCESS;
            }
            drop_reg(c->local_regs[i]);
            c->local_regs.erase(c->local_regs.begin() + (long)i);  // freed and reallocated: stale
            break;
        }
    }
    void *base = nullptr;
    size_t sz = 0;
    MI_HIP(hipMemGetAddressRange(&base, &sz, (void *)p));
    TRACE(c, "register %p: base %p size %zu id %llu", p, base, sz, (unsigned long long)id);
    LocalReg reg;
    std::memset(&reg, 0, sizeof(reg));
    reg.fd = -1;
    reg.base = (uintptr_t)base;
    reg.size = sz;
    reg.id = id;
    bool dm = !force && via_dmabuf(c, sz);
    if (dm && sz < c->ipc_max) {
        // (bounded cache) only an allocation with a buffer object of its own exports as a dmabuf --
        // the runtime sub-allocates small ones: those keep the hipIpc route
        if (hipMemGetHandleForAddressRange(&reg.fd, (hipDeviceptr_t)base, sz, hipMemRangeHandleTypeDmaBufFd, 0) !=
            hipSuccess) {
            (void)hipGetLastError();
            reg.fd = -1;
            dm = false;
        } else if (c->export_check && export_names(base, reg.fd) != 1) {
            // the fd names another range: the runtime exports the whole buffer object an allocation
            // was carved from (small allocations share one), from its start -- such an allocation
            // keeps the hipIpc route (whose handle carries the offset)
            c->export_mismatches++;
            TRACE(c, "dmabuf export of %p names another range: hipIpc route", base);
            close(reg.fd);
            reg.fd = -1;
            dm = false;
        }
    }
    if (dm) {
        // the dmabuf route (hipIpcOpenMemHandle never returns for allocations >= ipc_max): fds
        // passed by export_dmabufs, or the staged data flow when that route is off
        reg.has_h = false;
        if (id != 0) c->local_regs.push_back(reg);
        d->staged = 1;
        d->base = reg.base;
        d->off = up - reg.base;
        d->id = id;
        d->size = sz;
        return MI355X_SUCCESS;
    }
    if (hipIpcGetMemHandle(&reg.h, base) != hipSuccess) {
        // seen on ROCm 7.2 under heavy allocation churn ("invalid argument" for a live allocation):
        // this call moves the buffer through the staging buffers instead (every rank sees staged
        // = 2 and takes the staged data flow), nothing is cached
        (void)hipGetLastError();
        if (force) return set_error(MI355X_ERR_HIP, "hipIpcGetMemHandle(%p) failed", base);
        TRACE(c, "hipIpcGetMemHandle(%p) failed: staged data flow for this call", base);
        d->staged = 2;
        d->base = reg.base;
        d->off = up - reg.base;
        d->id = id;
        d->size = sz;
        return MI355X_SUCCESS;
    }
    reg.has_h = true;
    if (debug_on()) {
        uint32_t w[16];
        std::memcpy(w, &reg.h, sizeof(w));
        TRACE(c, "export %p handle %08x %08x %08x %08x %08x %08x %08x %08x %08x %08x %08x %08x", base, w[0], w[1], w[2],
              w[3], w[4], w[5], w[6], w[7], w[8], w[9], w[10], w[11]);
    }
    // without an allocation id the entry cannot be validated later: do not cache it
    if (id != 0) c->local_regs.push_back(reg);
    d->h = reg.h;
    d->off = up - reg.base;
    d->base = reg.base;
    d->id = id;
    d->size = sz;
    return MI355X_SUCCESS;
}


} // namespace mi355x

namespace mi355x {

// Publish nbuf local buffers, meet every rank, and resolve every rank's buffers:
// peers[b][r] = rank r's buffer b mapped into this process.  When any rank published a buffer
// that cannot be exported, nothing is mapped and *staged is set on every rank alike (callers
// that pass staged == NULL get an error instead).  force: export regardless of allocation size
// (the staging buffers themselves).
void svc_park(mi355x_comm *c);

int exchange(mi355x_comm *c, int nbuf, const void *const *mine, const uint64_t sig[4],
             std::vector<std::vector<void *>> &peers, bool *staged, bool force, bool persistent)
{
    if (!c->svc_keep) svc_park(c);  // a host-synchronised call: the resident service steps aside (svc_park)
    c->seq++;
    if (staged) *staged = false;
    RankSlot &s = c->ctrl->slot[c->rank];
    for (int b = 0; b < nbuf; ++b) {
        int rc = local_handle(c, mine[b], &s.buf[b], force);
        if (rc) return rc;
    }
    s.nbuf = nbuf;
    s.retiring = c->retired_maps.empty() ? 0 : 1;
    for (int i = 0; i < 4; ++i) s.sig[i] = sig[i];
    s.seq.store(c->seq, std::memory_order_release);
    TRACE(c, "published %d buffers", nbuf);
    int rc = barrier(c);
    TRACE(c, "exchange barrier passed (rc %d)", rc);
    if (rc) return rc;
    bool any_staged = false, no_export = false;
    for (int r = 0; r < c->size; ++r) {
        RankSlot &o = c->ctrl->slot[r];
        if (o.seq.load(std::memory_order_acquire) != c->seq)
            return set_error(MI355X_ERR_PEER, "rank %d is in call %llu, rank %d in call %llu", r,
                             (unsigned long long)o.seq.load(), c->rank, (unsigned long long)c->seq);
        if (o.sig[0] != sig[0] || o.sig[1] != sig[1] || o.sig[2] != sig[2] || o.sig[3] != sig[3])
            return set_error(MI355X_ERR_ARG, "collective arguments differ between rank %d and rank %d", r, c->rank);
        for (int b = 0; b < nbuf; ++b) {
            any_staged = any_staged || o.buf[b].staged;
            no_export = no_export || o.buf[b].staged == 2;
        }
    }
    // the close window (coll_rcache.cpp, retire_map): when any rank holds retired mappings, every
    // rank closes its own here -- after every rank's exports of this call, before anybody opens --
    // and meets once more, so no close overlaps a peer's IPC export or import
    bool window = false;
    for (int r = 0; r < c->size; ++r) window = window || c->ctrl->slot[r].retiring != 0;
    if (window) {
        if ((rc = close_window(c))) return rc;
        rc = barrier(c);
        if (rc) return rc;
    }
    peers.assign(nbuf, std::vector<void *>(c->size, nullptr));
    if (any_staged && !c->loopback && !no_export) {
        if (c->dmabuf_state == 0) {
            rc = barrier(c);  // every rank has read the staged flags before the probe reuses the slots
            if (rc) return rc;
            rc = probe_dmabuf(c);
            if (rc) return rc;
        }
        if (c->dmabuf_state == 1) {
            // second round: the large allocations go out as dmabuf fds, then everything is mapped
            BufDesc *ds[kMaxBufs];
            int nd = 0;
            for (int b = 0; b < nbuf; ++b)
                if (s.buf[b].staged) ds[nd++] = &s.buf[b];
            if (nd) {
                rc = export_dmabufs(c, ds, nd, ~0ull);
                if (rc) return rc;
            }
            rc = barrier(c);
            if (rc) return rc;
            any_staged = false;
        }
    }
    if (any_staged) {
        if (!staged) return set_error(MI355X_ERR_UNSUPPORTED, "buffer allocation too large to export");
        *staged = true;
        TRACE(c, "staged data flow");
        // the staged flow publishes again at once (the staging buffers): nobody may overwrite
        // its slot before every rank has read this exchange's slots
        return barrier(c);
    }
    // Every rank publishes (call, mapping state) when its opens are done.  A rank whose open failed
    // (kOpenRetry: stale mappings of that peer retired, map_peer) closes them only once every peer
    // is past its own opens -- done, or failing too -- so no close overlaps a peer's import, and
    // retries only once every failing rank has closed.  The common path costs one store.
    enum { kMapped = 1, kMapFailed = 2, kMapClosed = 3 };
    std::vector<std::pair<int, int>> failed;
    for (int r = 0; r < c->size; ++r) {
        RankSlot &o = c->ctrl->slot[r];
        for (int b = 0; b < nbuf; ++b) {
            if (r == c->rank) {
                peers[b][r] = const_cast<void *>(mine[b]);
            } else {
                PeerMap *pm = nullptr;
                rc = map_peer(c, r, o.buf[b], &peers[b][r], &pm);
                if (rc == kOpenRetry) {
                    failed.emplace_back(r, b);
                    continue;
                }
                if (rc) return rc;
                if (persistent && pm) pm->persistent = true;
            }
        }
    }
    std::atomic<uint64_t> &st = c->ctrl->slot[c->rank].map_state;
    if (failed.empty()) {
        st.store((c->seq << 2) | kMapped, std::memory_order_release);
        return MI355X_SUCCESS;
    }
    auto wait_all = [&](bool allow_failed) -> int {
        for (int r = 0; r < c->size; ++r) {
            const auto t0 = std::chrono::steady_clock::now();
            for (;;) {
                const uint64_t v = c->ctrl->slot[r].map_state.load(std::memory_order_acquire);
                if ((v >> 2) > c->seq || ((v >> 2) == c->seq && ((v & 3) != kMapFailed || allow_failed))) break;
                if (c->ctrl->abort_flag.load(std::memory_order_relaxed)) return set_error(MI355X_ERR_PEER, "a peer aborted the communicator");
                if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > c->timeout_s)
                    return set_error(MI355X_ERR_TIMEOUT, "rank %d: the mapping window timed out waiting for rank %d", c->rank, r);
                sched_yield();
            }
        }
        return MI355X_SUCCESS;
    };
    st.store((c->seq << 2) | kMapFailed, std::memory_order_release);
    if ((rc = wait_all(true))) return rc;   // every rank is past its opens
    if ((rc = close_window(c))) return rc;
    st.store((c->seq << 2) | kMapClosed, std::memory_order_release);
    if ((rc = wait_all(false))) return rc;  // every failing rank has closed
    for (const auto &f : failed) {
        PeerMap *pm = nullptr;
        rc = map_peer(c, f.first, c->ctrl->slot[f.first].buf[f.second], &peers[f.second][f.first], &pm);
        if (rc == kOpenRetry) rc = set_error(MI355X_ERR_PEER, "hipIpcOpenMemHandle(rank %d) failed twice", f.first);
        if (rc) return rc;
        if (persistent && pm) pm->persistent = true;
    }
    st.store((c->seq << 2) | kMapped, std::memory_order_release);
    return MI355X_SUCCESS;
}

// finish: every rank's work queued on its stream so far has completed (so no rank still reads a
// peer's buffer, and my results are in place).  With the control segment registered, the GPU's
// command processor writes this finish point's number into my RankSlot::done right behind my
// kernels (hipStreamWriteValue64) and I poll every rank's word: the kernel's completion reaches
// every host without a hipStreamSynchronize wake-up and without a second barrier round.
// Otherwise: stream sync + barrier.
int finish(mi355x_comm *c, hipStream_t s)
{
    if (!c->ctrl_dev || c->size == 1) {
        TRACE(c, "finish: stream sync");
        MI_HIP(hipStreamSynchronize(s));
        TRACE(c, "finish: barrier");
        return barrier(c);
    }
    const uint64_t v = ++c->done_seq;
    char *word = c->ctrl_dev + ((char *)&c->ctrl->slot[c->rank].done - (char *)c->ctrl);
    MI_HIP(hipStreamWriteValue64(s, word, v, 0));
    TRACE(c, "finish %llu: polling the ranks' completion words", (unsigned long long)v);
    Ctrl *k = c->ctrl;
    const auto t0 = std::chrono::steady_clock::now();
    for (int q = 0; q < c->size; ++q) {
        unsigned spins = 0;
        while (k->slot[q].done.load(std::memory_order_acquire) < v) {
            if (k->abort_flag.load(std::memory_order_relaxed))
                return set_error(MI355X_ERR_PEER, "a peer aborted the communicator");
            if (++spins > 4096) {
                sched_yield();
                if ((spins & 255) == 0) barrier_progress(c);  // (a peer may be asking for a dmabuf fd, serve_fd)
                if ((spins & 0xffff) == 0 && hipStreamQuery(s) != hipErrorNotReady && q == c->rank &&
                    k->slot[q].done.load(std::memory_order_acquire) < v)
                    return set_error(MI355X_ERR_HIP, "stream finished without writing its completion word");
                if ((spins & 0xffff) == 0 && peer_gone(c)) return MI355X_ERR_PEER;
                if ((spins & 0xffff) == 0 &&
                    std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > c->timeout_s) {
                    k->abort_flag.store(1);
                    return set_error(MI355X_ERR_TIMEOUT, "rank %d: finish %llu timed out waiting for rank %d (at %llu)",
                                     c->rank, (unsigned long long)v, q, (unsigned long long)k->slot[q].done.load());
                }
            }
        }
    }
    return MI355X_SUCCESS;
}

// register the control segment with HIP so the command processor can write completion words into
// it (multi-process communicators; MI355X_DONE_WORDS=0 keeps stream sync + barrier).  Every rank
// decides the same way or the finish points would not pair: the outcome is agreed on with a
// barrier round through the segment.
int setup_done_words(mi355x_comm *c)
{
    const char *env = getenv("MI355X_DONE_WORDS");
    bool ok = env && atoi(env) != 0 && c->size > 1 && !c->loopback;
    if (ok) {
        ok = hipHostRegister(c->ctrl, ctrl_bytes(c->size), hipHostRegisterMapped) == hipSuccess;
        if (ok) {
            c->ctrl_registered = true;
            void *dptr = nullptr;
            ok = hipHostGetDevicePointer(&dptr, c->ctrl, 0) == hipSuccess && dptr;
            c->ctrl_dev = ok ? (char *)dptr : nullptr;
        }
        (void)hipGetLastError();
    }
    c->ctrl->slot[c->rank].done.store(ok ? 1 : 2, std::memory_order_release);
    int rc = barrier(c);
    if (rc) return rc;
    bool all = true;
    for (int q = 0; q < c->size; ++q) all = all && c->ctrl->slot[q].done.load(std::memory_order_acquire) == 1;
    rc = barrier(c);   // every rank has read the setup words before they are reset
    if (rc) return rc;
    c->ctrl->slot[c->rank].done.store(0, std::memory_order_release);
    if (!all) c->ctrl_dev = nullptr;
    c->done_seq = 0;
    return barrier(c);
}

// The scratch may be exported to peers (MPI_Reduce's owner blocks): never a small allocation
// (small hipMallocs can fail hipIpcOpenMemHandle on the importer with "invalid device
// pointer"), and grown geometrically so it is rarely freed while peers hold a mapping.
// The stream setup-time fills and copies run on: inside a collective, the call's own stream
// (CallStream), so setup orders with the caller's work and never waits for -- or makes wait -- the
// application's other streams (no hipDeviceSynchronize anywhere on the setup paths).  Every setup
// path runs inside a collective; outside one (a communicator set up eagerly at creation) the null
// stream.  No per-communicator stream: an idle extra queue per communicator measurably slows
// co-located ranks (profiles/r05_setup_stream_bisect.txt).
hipStream_t setup_stream(mi355x_comm *c) { return c->call_depth > 0 ? c->call_s : nullptr; }

int ensure_scratch(mi355x_comm *c, size_t bytes)
{
    if (c->scratch_bytes >= bytes) return MI355X_SUCCESS;
    size_t want = std::max<size_t>((size_t)8 << 20, c->scratch_bytes * 2);
    while (want < bytes) want *= 2;
    if (c->scratch) MI_HIP(hipFree(c->scratch));
    c->scratch = nullptr;
    c->scratch_bytes = 0;
    MI_HIP(hipMalloc(&c->scratch, want));
    c->scratch_bytes = want;
    return MI355X_SUCCESS;
}


} // namespace mi355x
