// coll_comm.cpp -- host side of the coll/mi355x engine: node-local bootstrap, barrier, IPC
// registration cache, and the device-buffer collectives.
//
// Transport (replaces the PML/BTL path the reference takes for device buffers: coll/cuda host
// staging, coll_cuda_allreduce.c:30-77, and smcuda CUDA-IPC RDMA, btl/smcuda/README:13-113):
//   * ranks on one node share a small control segment (POSIX shm, or process memory for the
//     in-process "loopback" communicator used by tests);
//   * per call each rank publishes the IPC handle + offset of its buffers (hipIpcGetMemHandle on
//     the allocation base, cached per base: the reference's mpool/rgpusm registration cache,
//     common_cuda.c:971-1137); peers map them once (hipIpcOpenMemHandle, cached per handle);
//   * one kernel per rank then reads every rank's input directly over xGMI, folds it in the
//     reference schedule's order (coll_sched.cpp) and pushes the result into every destination.
// A call is: sync caller stream -> publish -> barrier -> kernel(s) -> sync -> barrier.
// Default data flow is PULL: every kernel writes only its own rank's memory and reads peers'
// memory, so coherence rests on kernel-completion release + the host barrier and never on a peer
// GPU's L2 seeing a remote write.  Allreduce: phase 1 the owner folds its ring block locally,
// phase 2 every rank pulls the other blocks (one launch, one segment per peer).  A one-phase
// PUSH variant (owners write into every peer's rbuf) is kept behind MI355X_KNOB_PUSH.
//
// Large allocations: hipIpcOpenMemHandle never returns for an allocation of 2 GiB or more on
// this platform (ROCm 7.2, dmabuf IPC; measured: 2046 MiB maps, 2048 MiB hangs).  A buffer whose
// allocation is at least `ipc_max` bytes is therefore never exported: the call switches, on every
// rank (the decision is taken after the exchange, from every rank's descriptors), to the STAGED
// data flow -- the message moves through each rank's persistent staging buffer (one allocation
// < 2 GiB, mapped once) in block-strided windows, like the segmented ring's phases.
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

namespace mi355x {

CollTune &coll_tune()
{
    static CollTune t;
    return t;
}

} // namespace mi355x

namespace mi355x {

static int fd_drain(mi355x_comm *c, bool wait);

// ----------------------------------------------------------------- liveness
// a process exists and has not exited (a zombie -- exited, not yet reaped by its parent -- is gone)
static bool pid_alive(pid_t pid)
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
static bool peer_gone(mi355x_comm *c)
{
    if (c->loopback || c->size == 1) return false;
    for (int q = 0; q < c->size; ++q) {
        const pid_t pid = (pid_t)c->ctrl->slot[q].pid;
        if (q == c->rank || pid <= 0) continue;
        if (!pid_alive(pid)) {
            c->ctrl->abort_flag.store(1);
            set_error(MI355X_ERR_PEER, "rank %d (pid %d) is gone: the communicator is aborted", q, (int)pid);
            return true;
        }
    }
    return false;
}

// ----------------------------------------------------------------- barrier
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
            // a peer may be blocked sending us dmabuf fds (full socket queue): drain it while we wait
            if (c->fd_sock >= 0 && (spins & 255) == 0 && c->reg_mtx.try_lock()) {
                (void)fd_drain(c, false);
                c->reg_mtx.unlock();
            }
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
static uint64_t buffer_id(const void *p)
{
    unsigned long long id = 0;
    if (hipPointerGetAttribute(&id, HIP_POINTER_ATTRIBUTE_BUFFER_ID, (hipDeviceptr_t)p) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return (uint64_t)id;
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
                if (!force && r.size >= c->ipc_max) {
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
    if (!force && sz >= c->ipc_max) {
        // never exported (hipIpcOpenMemHandle hangs on such allocations): staged data flow
        reg.has_h = false;
        if (id != 0) c->local_regs.push_back(reg);
        d->staged = 1;
        d->base = reg.base;
        d->off = up - reg.base;
        d->id = id;
        d->size = sz;
        return MI355X_SUCCESS;
    }
    MI_HIP(hipIpcGetMemHandle(&reg.h, base));
    reg.has_h = true;
    // without an allocation id the entry cannot be validated later: do not cache it
    if (id != 0) c->local_regs.push_back(reg);
    d->h = reg.h;
    d->off = up - reg.base;
    d->base = reg.base;
    d->id = id;
    d->size = sz;
    return MI355X_SUCCESS;
}

// ----------------------------------------------------------------- dmabuf fd passing (SCM_RIGHTS)
// hipIpcOpenMemHandle never returns for allocations of >= 2 GiB (ROCm 7.2, dmabuf IPC), but the
// allocation exported as a dmabuf fd (hipMemGetHandleForAddressRange) and imported by the peer as
// external memory maps fine.  The fd reaches the peer as SCM_RIGHTS ancillary data on an AF_UNIX
// datagram socket (the smcuda BTL's role of carrying the IPC handle, btl/smcuda/README:13-30):
// no ptrace permission is granted to anybody.  Every rank binds one socket at communicator
// creation under an abstract name derived from the control segment's (node-unique) name; the
// receiver checks the sender's pid (SO_PASSCRED) against the rank's published pid.
constexpr int kFdMax = 8;  // fds per message (a call exports at most kMaxBufs buffers)
struct FdMsg {
    int32_t from;
    int32_t nfd;
    uint64_t id[kFdMax];
};

static void fd_sock_addr(const mi355x_comm *c, int rank, sockaddr_un *a, socklen_t *len)
{
    uint64_t h = 1469598103934665603ull;
    for (char ch : c->shm_name) h = (h ^ (unsigned char)ch) * 1099511628211ull;
    for (int b = 0; b < 8; ++b) h = (h ^ ((c->ctrl->secret >> (8 * b)) & 0xff)) * 1099511628211ull;
    std::memset(a, 0, sizeof(*a));
    a->sun_family = AF_UNIX;
    // abstract namespace: sun_path[0] = 0, the name is the bytes that follow
    const int n = snprintf(a->sun_path + 1, sizeof(a->sun_path) - 1, "mi355x_fd_%016llx_%d", (unsigned long long)h, rank);
    *len = (socklen_t)(offsetof(sockaddr_un, sun_path) + 1 + (size_t)n);
}

static int fd_sock_open(mi355x_comm *c)
{
    const int s = socket(AF_UNIX, SOCK_DGRAM | SOCK_CLOEXEC, 0);
    if (s < 0) return set_error(MI355X_ERR_PEER, "socket(AF_UNIX): %s", strerror(errno));
    const int one = 1;
    sockaddr_un a;
    socklen_t len;
    fd_sock_addr(c, c->rank, &a, &len);
    if (setsockopt(s, SOL_SOCKET, SO_PASSCRED, &one, sizeof(one)) != 0 || bind(s, (sockaddr *)&a, len) != 0) {
        const int e = errno;
        close(s);
        return set_error(MI355X_ERR_PEER, "bind of the fd-passing socket: %s", strerror(e));
    }
    c->fd_sock = s;
    return MI355X_SUCCESS;
}

// receive every queued fd message into the stash; `wait`: block (bounded) for at least one.
// Caller holds reg_mtx.
static int fd_drain(mi355x_comm *c, bool wait)
{
    for (;;) {
        FdMsg m;
        iovec iov{&m, sizeof(m)};
        alignas(cmsghdr) char ctl[CMSG_SPACE(sizeof(int) * kFdMax) + CMSG_SPACE(sizeof(ucred))];
        msghdr h;
        std::memset(&h, 0, sizeof(h));
        h.msg_iov = &iov;
        h.msg_iovlen = 1;
        h.msg_control = ctl;
        h.msg_controllen = sizeof(ctl);
        if (wait) {
            pollfd p{c->fd_sock, POLLIN, 0};
            const int pr = poll(&p, 1, (int)std::min(c->timeout_s * 1000.0, 2.0e9));
            if (pr == 0) return set_error(MI355X_ERR_TIMEOUT, "rank %d: no dmabuf fd arrived", c->rank);
            if (pr < 0 && errno != EINTR) return set_error(MI355X_ERR_PEER, "poll: %s", strerror(errno));
        }
        const ssize_t got = recvmsg(c->fd_sock, &h, MSG_DONTWAIT | MSG_CMSG_CLOEXEC);
        if (got < 0) {
            if (errno == EAGAIN || errno == EWOULDBLOCK) {
                if (wait) continue;
                return MI355X_SUCCESS;
            }
            if (errno == EINTR) continue;
            return set_error(MI355X_ERR_PEER, "recvmsg: %s", strerror(errno));
        }
        int fds[kFdMax];
        int nfd = 0;
        pid_t pid = -1;
        for (cmsghdr *cm = CMSG_FIRSTHDR(&h); cm; cm = CMSG_NXTHDR(&h, cm)) {
            if (cm->cmsg_level == SOL_SOCKET && cm->cmsg_type == SCM_RIGHTS) {
                nfd = (int)((cm->cmsg_len - CMSG_LEN(0)) / sizeof(int));
                if (nfd > kFdMax) nfd = kFdMax;
                std::memcpy(fds, CMSG_DATA(cm), sizeof(int) * (size_t)nfd);
            }
            if (cm->cmsg_level == SOL_SOCKET && cm->cmsg_type == SCM_CREDENTIALS) {
                ucred cr;
                std::memcpy(&cr, CMSG_DATA(cm), sizeof(cr));
                pid = cr.pid;
            }
        }
        const bool ok = got == (ssize_t)sizeof(m) && nfd > 0 && m.nfd == nfd && m.from >= 0 && m.from < c->size &&
                        pid == (pid_t)c->ctrl->slot[m.from].pid;
        for (int i = 0; i < nfd; ++i) {
            if (!ok) {  // not from a rank of this communicator: drop it
                close(fds[i]);
                continue;
            }
            const auto key = std::make_pair((int)m.from, m.id[i]);
            auto it = c->fd_stash.find(key);
            if (it != c->fd_stash.end()) close(it->second);
            c->fd_stash[key] = fds[i];
        }
        if (wait && ok) return MI355X_SUCCESS;
    }
}

// one message carrying nfd fds and their allocation ids to `peer`.  Caller holds reg_mtx.
static int send_fds(mi355x_comm *c, int peer, const int *fds, const uint64_t *ids, int nfd)
{
    FdMsg m;
    std::memset(&m, 0, sizeof(m));
    m.from = c->rank;
    m.nfd = nfd;
    for (int i = 0; i < nfd; ++i) m.id[i] = ids[i];
    iovec iov{&m, sizeof(m)};
    alignas(cmsghdr) char ctl[CMSG_SPACE(sizeof(int) * kFdMax)];
    std::memset(ctl, 0, sizeof(ctl));
    sockaddr_un a;
    socklen_t len;
    fd_sock_addr(c, peer, &a, &len);
    msghdr h;
    std::memset(&h, 0, sizeof(h));
    h.msg_name = &a;
    h.msg_namelen = len;
    h.msg_iov = &iov;
    h.msg_iovlen = 1;
    h.msg_control = ctl;
    h.msg_controllen = CMSG_SPACE(sizeof(int) * (size_t)nfd);
    cmsghdr *cm = CMSG_FIRSTHDR(&h);
    cm->cmsg_level = SOL_SOCKET;
    cm->cmsg_type = SCM_RIGHTS;
    cm->cmsg_len = CMSG_LEN(sizeof(int) * (size_t)nfd);
    std::memcpy(CMSG_DATA(cm), fds, sizeof(int) * (size_t)nfd);
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        if (sendmsg(c->fd_sock, &h, MSG_DONTWAIT | MSG_NOSIGNAL) == (ssize_t)sizeof(m)) return MI355X_SUCCESS;
        if (errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR)
            return set_error(MI355X_ERR_PEER, "sending dmabuf fds to rank %d: %s", peer, strerror(errno));
        // the peer's queue is full (net.unix.max_dgram_qlen): it drains it whenever it waits
        // (barrier, its own sends, its imports) -- keep ours drained meanwhile too
        int rc = fd_drain(c, false);
        if (rc) return rc;
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > c->timeout_s)
            return set_error(MI355X_ERR_TIMEOUT, "rank %d: fd queue of rank %d stays full", c->rank, peer);
        usleep(50);
    }
}

static int send_fd(mi355x_comm *c, int peer, int fd, uint64_t id) { return send_fds(c, peer, &fd, &id, 1); }

// the fd rank `peer` passed for its allocation `id` (a duplicate: the stash keeps its own)
static int take_fd(mi355x_comm *c, int peer, uint64_t id, int *out)
{
    const auto key = std::make_pair(peer, id);
    int rc = fd_drain(c, false);
    if (rc) return rc;
    while (c->fd_stash.find(key) == c->fd_stash.end()) {
        rc = fd_drain(c, true);
        if (rc) return rc;
    }
    *out = fcntl(c->fd_stash[key], F_DUPFD_CLOEXEC, 0);
    if (*out < 0) return set_error(MI355X_ERR_PEER, "dup of a dmabuf fd: %s", strerror(errno));
    return MI355X_SUCCESS;
}

// forget the fd of `peer`'s allocation `id` (the allocation was freed or replaced)
static void drop_stash(mi355x_comm *c, int peer, uint64_t id)
{
    auto it = c->fd_stash.find(std::make_pair(peer, id));
    if (it == c->fd_stash.end()) return;
    close(it->second);
    c->fd_stash.erase(it);
}

// export the large allocations of ds[0..nd) as dmabuf fds and pass every one to every rank in
// `peers` that has not received it yet: one message per peer
static int export_dmabufs(mi355x_comm *c, BufDesc *const *ds, int nd, uint64_t peers)
{
    std::lock_guard<std::recursive_mutex> reg_guard(c->reg_mtx);
    LocalReg *regs[kFdMax];
    for (int i = 0; i < nd; ++i) {
        regs[i] = nullptr;
        for (LocalReg &r : c->local_regs)
            if (r.base == ds[i]->base && r.id == ds[i]->id) regs[i] = &r;
        if (!regs[i])
            return set_error(MI355X_ERR_PEER, "large allocation not registered (id %llu)", (unsigned long long)ds[i]->id);
        LocalReg &r = *regs[i];
        if (r.fd < 0) {
            MI_HIP(hipMemGetHandleForAddressRange(&r.fd, (hipDeviceptr_t)r.base, r.size,
                                                  hipMemRangeHandleTypeDmaBufFd, 0));
            r.sent = 0;
        }
        ds[i]->dmabuf = 1;
        ds[i]->fd = r.fd;
        ds[i]->size = r.size;
    }
    for (int q = 0; q < c->size; ++q) {
        if (q == c->rank || !((peers >> q) & 1u)) continue;
        int fds[kFdMax];
        uint64_t ids[kFdMax];
        int k = 0;
        for (int i = 0; i < nd; ++i) {
            if ((regs[i]->sent >> q) & 1u) continue;
            bool dup = false;  // two buffers of one allocation: one fd
            for (int j = 0; j < k; ++j) dup = dup || ids[j] == regs[i]->id;
            if (dup) continue;
            fds[k] = regs[i]->fd;
            ids[k++] = regs[i]->id;
        }
        if (!k) continue;
        int rc = send_fds(c, q, fds, ids, k);
        if (rc) return rc;
        for (int i = 0; i < nd; ++i) regs[i]->sent |= 1ull << q;
    }
    return MI355X_SUCCESS;
}

int export_dmabuf(mi355x_comm *c, BufDesc *d, uint64_t peers)
{
    BufDesc *ds[1] = {d};
    return export_dmabufs(c, ds, 1, peers);
}

static int import_dmabuf(mi355x_comm *c, int peer, uint64_t id, size_t size, void **mapped, hipExternalMemory_t *ext)
{
    int myfd = -1;
    int rc = take_fd(c, peer, id, &myfd);
    if (rc) return rc;
    hipExternalMemoryHandleDesc hd;
    std::memset(&hd, 0, sizeof(hd));
    hd.type = hipExternalMemoryHandleTypeOpaqueFd;
    hd.handle.fd = myfd;
    hd.size = size;
    hipError_t e = hipImportExternalMemory(ext, &hd);
    if (e != hipSuccess) {
        close(myfd);
        return set_error(MI355X_ERR_PEER, "hipImportExternalMemory(rank %d): %s", peer, hipGetErrorString(e));
    }
    hipExternalMemoryBufferDesc bd;
    std::memset(&bd, 0, sizeof(bd));
    bd.offset = 0;
    bd.size = size;
    e = hipExternalMemoryGetMappedBuffer(mapped, *ext, &bd);
    if (e != hipSuccess) {
        (void)hipDestroyExternalMemory(*ext);
        return set_error(MI355X_ERR_PEER, "hipExternalMemoryGetMappedBuffer(rank %d): %s", peer, hipGetErrorString(e));
    }
    TRACE(c, "dmabuf import from rank %d: %zu bytes at %p", peer, size, *mapped);
    return MI355X_SUCCESS;
}


// Collective, once per communicator: every rank exports a 4 MiB buffer as a dmabuf, every rank
// imports every peer's and checks its bytes; the path is used only if it worked everywhere.
static int probe_dmabuf(mi355x_comm *c)
{
    const char *env = getenv("MI355X_DMABUF");
    bool ok = !(env && atoi(env) == 0);
    const size_t sz = (size_t)4 << 20;
    void *buf = nullptr;
    int fd = -1;
    RankSlot &me = c->ctrl->slot[c->rank];
    if (ok && hipMalloc(&buf, sz) != hipSuccess) ok = false;
    if (ok && hipMemset(buf, c->rank + 1, sz) != hipSuccess) ok = false;
    if (ok && hipDeviceSynchronize() != hipSuccess) ok = false;
    if (ok && hipMemGetHandleForAddressRange(&fd, (hipDeviceptr_t)buf, sz, hipMemRangeHandleTypeDmaBufFd, 0) != hipSuccess)
        ok = false;
    (void)hipGetLastError();
    const uint64_t kProbeId = ~0ull;  // never an allocation id
    {
        std::lock_guard<std::recursive_mutex> reg_guard(c->reg_mtx);  // the fd stash
        for (int q = 0; q < c->size && ok; ++q)
            if (q != c->rank && send_fd(c, q, fd, kProbeId) != MI355X_SUCCESS) ok = false;
    }
    me.probe_fd = ok ? 1 : -1;  // 1: my fd went to every peer
    me.probe_size = sz;
    int rc = barrier(c);  // every sent fd is queued at its receiver
    if (rc) return rc;
    std::unique_lock<std::recursive_mutex> reg_lock(c->reg_mtx);  // the fd stash
    for (int q = 0; q < c->size && ok; ++q) {
        if (q == c->rank) continue;
        const RankSlot &o = c->ctrl->slot[q];
        if (o.probe_fd < 0) {
            ok = false;
            break;
        }
        void *mapped = nullptr;
        hipExternalMemory_t ext = nullptr;
        const int irc = import_dmabuf(c, q, kProbeId, o.probe_size, &mapped, &ext);
        drop_stash(c, q, kProbeId);
        if (irc != MI355X_SUCCESS) {
            (void)hipGetLastError();  // no sticky error for later calls
            if (c->rank == 0 || debug_on())
                fprintf(stderr, "[mi355x] rank %d: dmabuf probe import from rank %d failed: %s\n", c->rank, q,
                        mi355x_last_error());
            ok = false;
            break;
        }
        unsigned char v[2] = {0, 0};
        if (hipMemcpy(&v[0], mapped, 1, hipMemcpyDeviceToHost) != hipSuccess ||
            hipMemcpy(&v[1], (char *)mapped + sz - 1, 1, hipMemcpyDeviceToHost) != hipSuccess ||
            v[0] != (unsigned char)(q + 1) || v[1] != (unsigned char)(q + 1))
            ok = false;
        (void)hipFree(mapped);
        (void)hipDestroyExternalMemory(ext);
        (void)hipGetLastError();
    }
    for (int q = 0; q < c->size; ++q) drop_stash(c, q, kProbeId);
    reg_lock.unlock();
    me.probe_ok = ok ? 1 : 0;
    rc = barrier(c);  // every rank is done importing before the probe buffers go
    if (fd >= 0) close(fd);
    if (buf) (void)hipFree(buf);
    if (rc) return rc;
    bool all = true;
    for (int q = 0; q < c->size; ++q) all = all && c->ctrl->slot[q].probe_ok == 1;
    c->dmabuf_state = all ? 1 : -1;
    TRACE(c, "dmabuf probe: %s", all ? "usable" : "not usable -> staged flow");
    return barrier(c);  // nobody rewrites its slot before every rank has read probe_ok
}

// Bounded peer-mapping cache (mpool/rgpusm's rcache_size_limit with LRU eviction,
// mpool_rgpusm_component.c:92-100, mpool_rgpusm_module.c:104-120,396-419): when the hipIpc mappings
// of peers' allocations exceed rcache_max_maps (count) or rcache_limit (bytes), the least recently
// used ones that the current call does not use, that no point-to-point read has pinned and that
// are not the communicator's own regions are closed.  A mapping keeps the exporter's allocation
// alive on ROCm, so a long job that churns allocations would otherwise hold every freed block of
// every peer.  Both limits default to 0 = unlimited, as in the reference.  dmabuf imports (>= 2 GiB
// allocations) are not evicted: their fd reaches a peer once.
static bool evictable(const mi355x_comm *c, const PeerMap &m, const PeerMap *keep)
{
    return &m != keep && !m.persistent && m.pins == 0 && !m.ext && m.last_use != c->seq;
}

static void rcache_trim(mi355x_comm *c, const PeerMap *keep)
{
    if (!c->rcache_max_maps && !c->rcache_limit) return;
    for (;;) {
        size_t nmaps = 0, bytes = 0;
        auto lru = c->peer_maps.end();
        for (auto it = c->peer_maps.begin(); it != c->peer_maps.end(); ++it) {
            if (it->second.persistent || it->second.ext) continue;
            nmaps++;
            bytes += it->second.bytes;
            if (evictable(c, it->second, keep) && (lru == c->peer_maps.end() || it->second.last_use < lru->second.last_use))
                lru = it;
        }
        const bool over = (c->rcache_max_maps && nmaps > c->rcache_max_maps) || (c->rcache_limit && bytes > c->rcache_limit);
        if (!over || lru == c->peer_maps.end()) return;
        TRACE(c, "rcache: evict peer %d base %llx (%zu maps, %zu bytes)", lru->first.peer,
              (unsigned long long)lru->first.base, nmaps, bytes);
        close_map(lru->second);
        c->peer_maps.erase(lru);
        c->rcache_evictions++;
    }
}

size_t peer_map_count(const mi355x_comm *c)
{
    size_t n = 0;
    for (const auto &kv : c->peer_maps) n += !kv.second.persistent && !kv.second.ext;
    return n;
}

int map_peer(mi355x_comm *c, int peer, const BufDesc &d, void **out, PeerMap **entry)
{
    std::lock_guard<std::recursive_mutex> reg_guard(c->reg_mtx);
    *out = nullptr;
    if (entry) *entry = nullptr;
    if (!d.present) return MI355X_SUCCESS;
    if (c->loopback) {
        *out = (void *)(uintptr_t)d.raw;
        return MI355X_SUCCESS;
    }
    HandleKey key;
    key.peer = peer;
    key.base = d.base;
    auto it = c->peer_maps.find(key);
    if (it != c->peer_maps.end() && (it->second.id != d.id || (d.id == 0 && it->second.pins == 0))) {
        if (it->second.ext) drop_stash(c, peer, it->second.id);  // the peer replaced that allocation
        close_map(it->second);
        c->peer_maps.erase(it);
        it = c->peer_maps.end();
    }
    if (it == c->peer_maps.end() && d.dmabuf) {
        void *mapped = nullptr;
        hipExternalMemory_t ext = nullptr;
        int rc = import_dmabuf(c, peer, d.id, d.size, &mapped, &ext);
        if (rc) return rc;
        it = c->peer_maps.emplace(key, PeerMap{d.id, mapped, c->seq, ext}).first;
    }
    void *base;
    if (it != c->peer_maps.end()) {
        base = it->second.mapped;
        it->second.last_use = c->seq;
    } else {
        TRACE(c, "open peer %d base %llx id %llu", peer, (unsigned long long)d.base, (unsigned long long)d.id);
        hipError_t e = hipIpcOpenMemHandle(&base, d.h, hipIpcMemLazyEnablePeerAccess);
        TRACE(c, "opened peer %d -> %p (%s)", peer, base, hipGetErrorString(e));
        if (e != hipSuccess) {
            // A mapping of an allocation the peer has since freed can still hold the block the new
            // allocation was carved from (small allocations share blocks): the open then fails
            // with "invalid device pointer".  Drop this peer's mappings that the current call does
            // not use and try once more.
            (void)hipGetLastError();
            int dropped = 0;
            for (auto m = c->peer_maps.begin(); m != c->peer_maps.end();) {
                if (m->first.peer == peer && m->second.last_use != c->seq && m->second.pins == 0 &&
                    !m->second.persistent) {
                    close_map(m->second);
                    m = c->peer_maps.erase(m);
                    dropped++;
                } else {
                    ++m;
                }
            }
            TRACE(c, "open failed; dropped %d stale mappings of peer %d, retrying", dropped, peer);
            e = dropped ? hipIpcOpenMemHandle(&base, d.h, hipIpcMemLazyEnablePeerAccess) : e;
            if (e != hipSuccess)
                return set_error(MI355X_ERR_PEER, "hipIpcOpenMemHandle(rank %d): %s", peer, hipGetErrorString(e));
        }
        it = c->peer_maps.emplace(key, PeerMap{d.id, base, c->seq, nullptr}).first;
        it->second.bytes = d.size;
        rcache_trim(c, &it->second);
    }
    if (entry) *entry = &it->second;
    *out = (char *)base + d.off;
    return MI355X_SUCCESS;
}

// Publish nbuf local buffers, meet every rank, and resolve every rank's buffers:
// peers[b][r] = rank r's buffer b mapped into this process.  When any rank published a buffer
// that cannot be exported, nothing is mapped and *staged is set on every rank alike (callers
// that pass staged == NULL get an error instead).  force: export regardless of allocation size
// (the staging buffers themselves).
static void svc_park(mi355x_comm *c);

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
    for (int i = 0; i < 4; ++i) s.sig[i] = sig[i];
    s.seq.store(c->seq, std::memory_order_release);
    TRACE(c, "published %d buffers", nbuf);
    int rc = barrier(c);
    TRACE(c, "exchange barrier passed (rc %d)", rc);
    if (rc) return rc;
    bool any_staged = false;
    for (int r = 0; r < c->size; ++r) {
        RankSlot &o = c->ctrl->slot[r];
        if (o.seq.load(std::memory_order_acquire) != c->seq)
            return set_error(MI355X_ERR_PEER, "rank %d is in call %llu, rank %d in call %llu", r,
                             (unsigned long long)o.seq.load(), c->rank, (unsigned long long)c->seq);
        if (o.sig[0] != sig[0] || o.sig[1] != sig[1] || o.sig[2] != sig[2] || o.sig[3] != sig[3])
            return set_error(MI355X_ERR_ARG, "collective arguments differ between rank %d and rank %d", r, c->rank);
        for (int b = 0; b < nbuf; ++b) any_staged = any_staged || o.buf[b].staged;
    }
    peers.assign(nbuf, std::vector<void *>(c->size, nullptr));
    if (any_staged && !c->loopback) {
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
    for (int r = 0; r < c->size; ++r) {
        RankSlot &o = c->ctrl->slot[r];
        for (int b = 0; b < nbuf; ++b) {
            if (r == c->rank) {
                peers[b][r] = const_cast<void *>(mine[b]);
            } else {
                PeerMap *pm = nullptr;
                rc = map_peer(c, r, o.buf[b], &peers[b][r], &pm);
                if (rc) return rc;
                if (persistent && pm) pm->persistent = true;
            }
        }
    }
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
static int setup_done_words(mi355x_comm *c)
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

// ----------------------------------------------------------------- program launch
// Evaluate `pr` on elements [off, off+len) of every rank's input `in[q]`, writing dst[d] + off.
int run_program(int op, int type, const Program &pr, const std::vector<void *> &in,
                       const std::vector<void *> &dst, size_t off, size_t len, hipStream_t s)
{
    if (len == 0) return MI355X_SUCCESS;
    const size_t esz = mi355x_type_size(type);
    if (debug_on())
        fprintf(stderr, "[mi355x] run_program op %d type %d %s nr %d off %zu len %zu\n", op, type,
                pr.is_fold ? "fold" : "tree", pr.nr, off, len);
    if ((int)dst.size() > kMaxRanks || (int)in.size() > kMaxRanks)
        return set_error(MI355X_ERR_UNSUPPORTED, "communicator larger than %d ranks", kMaxRanks);
    if (pr.is_fold) {
        FoldArgs a;
        std::memset(&a, 0, sizeof(a));
        for (size_t q = 0; q < in.size(); ++q) a.src[q] = (const char *)in[q] + off * esz;
        for (size_t d = 0; d < dst.size(); ++d) a.dst[d] = (char *)dst[d] + off * esz;
        a.nr = (int)pr.order.size();
        for (int j = 0; j < a.nr; ++j) a.order[j] = pr.order[j];
        a.role_mask = pr.role_mask;
        a.nd = (int)dst.size();
        a.n = len;
        return launch_fold_slot(op, type, a, s);
    }
    if ((int)in.size() > kTreeMax) return set_error(MI355X_ERR_UNSUPPORTED, "tree program over > %d ranks", kTreeMax);
    TreeArgs t;
    std::memset(&t, 0, sizeof(t));
    for (size_t q = 0; q < in.size(); ++q) t.src[q] = (const char *)in[q] + off * esz;
    for (size_t d = 0; d < dst.size(); ++d) t.dst[d] = (char *)dst[d] + off * esz;
    t.nr = (int)in.size();
    t.nd = (int)dst.size();
    t.nsteps = (int)pr.steps.size();
    for (int k = 0; k < t.nsteps; ++k) t.steps[k] = pr.steps[k];
    t.result = pr.result;
    t.n = len;
    return launch_tree_slot(op, type, t, s);
}

// ----------------------------------------------------------------- staged data flow
// Every rank's staging buffer, exported and mapped once (cached like any other buffer).
static int stage_peers(mi355x_comm *c, std::vector<void *> &sp)
{
    if (!c->stage) MI_HIP(hipMalloc(&c->stage, c->stage_bytes));
    const void *mine[1] = {c->stage};
    const uint64_t sig[4] = {9, c->stage_bytes, 0, 0};
    std::vector<std::vector<void *>> P;
    int rc = exchange(c, 1, mine, sig, P, nullptr, true);
    if (rc) return rc;
    sp = P[0];
    return MI355X_SUCCESS;
}

// Staged reduction.  Rank b's result is elements [boff[b], boff[b] + blen[b]) of the vector; this
// rank folds its own range with program `pr` over every rank's input `in` and writes it at
// `mine_dst` (pointer of its first result element).  Window w covers elements
// [w*Wb, (w+1)*Wb) of EVERY rank's range (block-strided, as the segmented ring's phases are), so
// all ranks fold at once.  Per window: copy-in (each rank copies the other ranks' slices of its
// input into staging slot b) -> barrier -> fold (own slice read in place, peers' from their slot
// `me`) -> barrier.  With `distribute` (allreduce) the fold also writes the result into slot n,
// and every rank then pulls the other ranks' results into rbuf -> barrier.
static int staged_reduce(mi355x_comm *c, int op, int type, const Program &pr, const void *in,
                         const std::vector<size_t> &boff, const std::vector<size_t> &blen, void *mine_dst,
                         bool distribute, void *rbuf, hipStream_t s)
{
    const int n = c->size, me = c->rank;
    const size_t esz = mi355x_type_size(type);
    std::vector<void *> sp;
    int rc = stage_peers(c, sp);
    if (rc) return rc;
    const size_t slots = (size_t)n + (distribute ? 1 : 0);
    size_t wb = c->stage_bytes / (slots * esz);
    wb -= wb % 16;  // slots stay 16-byte aligned
    if (wb == 0) return set_error(MI355X_ERR_NOMEM, "staging buffer too small for %d ranks", n);
    size_t maxlen = 0;
    for (int b = 0; b < n; ++b) maxlen = std::max(maxlen, blen[b]);
    const size_t nwin = (maxlen + wb - 1) / wb;
    char *stage = (char *)c->stage;
    auto wlen = [&](int b, size_t w) -> size_t {
        const size_t lo = w * wb;
        return lo >= blen[b] ? 0 : std::min(wb, blen[b] - lo);
    };
    for (size_t w = 0; w < nwin; ++w) {
        MultiCopyArgs m;
        std::memset(&m, 0, sizeof(m));
        for (int b = 0; b < n; ++b) {
            const size_t l = wlen(b, w);
            if (b == me || l == 0) continue;
            m.src[m.nseg] = (const char *)in + (boff[b] + w * wb) * esz;
            m.dst[m.nseg] = stage + (size_t)b * wb * esz;
            m.len[m.nseg] = l * esz;
            m.nseg++;
        }
        rc = launch_multicopy(m, s);
        if (rc) return rc;
        rc = finish(c, s);
        if (rc) return rc;
        const size_t lme = wlen(me, w);
        std::vector<void *> ins(n);
        for (int q = 0; q < n; ++q)
            ins[q] = (q == me) ? (void *)((const char *)in + (boff[me] + w * wb) * esz)
                               : (void *)((char *)sp[q] + (size_t)me * wb * esz);
        std::vector<void *> dst(1, (char *)mine_dst + w * wb * esz);
        if (distribute) dst.push_back(stage + (size_t)n * wb * esz);
        rc = run_program(op, type, pr, ins, dst, 0, lme, s);
        if (rc) return rc;
        rc = finish(c, s);
        if (rc) return rc;
        if (!distribute) continue;
        std::memset(&m, 0, sizeof(m));
        for (int q = 0; q < n; ++q) {
            const size_t l = wlen(q, w);
            if (q == me || l == 0) continue;
            m.src[m.nseg] = (const char *)sp[q] + (size_t)n * wb * esz;
            m.dst[m.nseg] = (char *)rbuf + (boff[q] + w * wb) * esz;
            m.len[m.nseg] = l * esz;
            m.nseg++;
        }
        rc = launch_multicopy(m, s);
        if (rc) return rc;
        rc = finish(c, s);
        if (rc) return rc;
    }
    return MI355X_SUCCESS;
}

// Staged allgather: per window of W bytes every rank copies its slice into staging, then pulls
// the peers' slices.
static int staged_allgather(mi355x_comm *c, const void *src, void *rbuf, size_t bytes, hipStream_t s)
{
    const int n = c->size, me = c->rank;
    std::vector<void *> sp;
    int rc = stage_peers(c, sp);
    if (rc) return rc;
    char *own = (char *)rbuf + (size_t)me * bytes;
    if (src != own) MI_HIP(hipMemcpyAsync(own, src, bytes, hipMemcpyDeviceToDevice, s));
    const size_t W = c->stage_bytes & ~(size_t)15;
    for (size_t lo = 0; lo < bytes; lo += W) {
        const size_t l = std::min(W, bytes - lo);
        MI_HIP(hipMemcpyAsync(c->stage, (const char *)src + lo, l, hipMemcpyDeviceToDevice, s));
        rc = finish(c, s);
        if (rc) return rc;
        MultiCopyArgs m;
        std::memset(&m, 0, sizeof(m));
        for (int q = 0; q < n; ++q) {
            if (q == me) continue;
            m.src[m.nseg] = sp[q];
            m.dst[m.nseg] = (char *)rbuf + (size_t)q * bytes + lo;
            m.len[m.nseg] = l;
            m.nseg++;
        }
        rc = launch_multicopy(m, s);
        if (rc) return rc;
        rc = finish(c, s);
        if (rc) return rc;
    }
    return MI355X_SUCCESS;
}

// Staged bcast: per window the root copies into its staging; windows of >= 1 MiB take the
// scatter + allgather shape (each rank pulls its slice from the root into its buffer and its own
// staging, then the other slices from their owners), smaller ones a direct pull from the root.
static int staged_bcast(mi355x_comm *c, void *buf, size_t bytes, int root, hipStream_t s)
{
    const int n = c->size, me = c->rank;
    std::vector<void *> sp;
    int rc = stage_peers(c, sp);
    if (rc) return rc;
    const size_t W = c->stage_bytes & ~(size_t)15;
    for (size_t lo = 0; lo < bytes; lo += W) {
        const size_t l = std::min(W, bytes - lo);
        if (me == root) MI_HIP(hipMemcpyAsync(c->stage, (const char *)buf + lo, l, hipMemcpyDeviceToDevice, s));
        rc = finish(c, s);
        if (rc) return rc;
        MultiCopyArgs m;
        std::memset(&m, 0, sizeof(m));
        if (l < ((size_t)1 << 20)) {
            if (me != root) {
                m.src[0] = sp[root];
                m.dst[0] = (char *)buf + lo;
                m.len[0] = l;
                m.nseg = 1;
                rc = launch_multicopy(m, s);
                if (rc) return rc;
            }
            rc = finish(c, s);
            if (rc) return rc;
            continue;
        }
        size_t off, len;
        ring_block(l, n, me, &off, &len);
        if (me != root && len) {
            CopyArgs a;
            std::memset(&a, 0, sizeof(a));
            a.src = (const char *)sp[root] + off;
            a.dst[0] = (char *)buf + lo + off;
            a.dst[1] = (char *)c->stage + off;
            a.nd = 2;
            a.n = len;
            rc = launch_copy(a, s);
            if (rc) return rc;
        }
        rc = finish(c, s);
        if (rc) return rc;
        if (me != root) {
            for (int q = 0; q < n; ++q) {
                if (q == me) continue;
                size_t qo, ql;
                ring_block(l, n, q, &qo, &ql);
                if (!ql) continue;
                m.src[m.nseg] = (const char *)sp[q] + qo;  // slice q sits at rank q (and the root)
                m.dst[m.nseg] = (char *)buf + lo + qo;
                m.len[m.nseg] = ql;
                m.nseg++;
            }
            rc = launch_multicopy(m, s);
            if (rc) return rc;
        }
        rc = finish(c, s);
        if (rc) return rc;
    }
    return MI355X_SUCCESS;
}

// ----------------------------------------------------------------- low-latency path
// Loopback communicators (threads of one process) never take it: their kernels would share the
// process's few hardware queues and a rank's spinning kernel could sit in front of the peer
// kernel it waits for.
// the resident service takes every LL-protocol call up to svc_max bytes (svc_ok: created, self-
// tested and owned on every rank -- the same decision on every rank)
static bool svc_usable(const mi355x_comm *c, size_t bytes)
{
    return c->svc_ok && (c->flows & MI355X_FLOW_SVC_LL) && bytes > 0 && bytes <= c->svc_max;
}

static bool ll_usable(const mi355x_comm *c, size_t bytes)
{
    if (c->loopback || c->size < 2 || c->size > kLLMaxRanks || bytes == 0) return false;
    if (svc_usable(c, bytes)) return true;
    if (bytes > c->ll_max) return false;
    // ranks sharing a GPU: every rank's blocks spin until the others' have pushed, so all of them
    // must be resident at once -- at most one block per CU for the ranks together
    const size_t blocks = (bytes + kLLChunk - 1) / kLLChunk;
    return c->pipe_share <= 1 || blocks * (size_t)c->pipe_share <= (size_t)device_cu_count();
}

static bool svc_stop(mi355x_comm *c);
static int svc_run(mi355x_comm *c, LLArgs &a, int op, int type, hipStream_t s);

// (Re)allocate and exchange the LL region: [ack words, one per rank][2 parities x n slots of
// ll_max payload bytes as 8-byte granules].  Collective: every rank reaches it in the same call.

static int ensure_ll(mi355x_comm *c)
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
    MI_HIP(hipMemset(c->ll_base, 0, total));
    if (!c->ll_ctr) MI_HIP(hipMalloc((void **)&c->ll_ctr, sizeof(uint64_t)));
    MI_HIP(hipMemset(c->ll_ctr, 0, sizeof(uint64_t)));
    MI_HIP(hipDeviceSynchronize());
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
static int ll_run(mi355x_comm *c, LLArgs &a, int op, int type, hipStream_t s)
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
    MI_HIP(hipStreamSynchronize(s));
    if (__atomic_load_n(c->ll_err, __ATOMIC_ACQUIRE)) {
        (void)hipMemset(c->ll_ctr, 0, sizeof(uint64_t));  // its count is off now: restart it
        (void)hipDeviceSynchronize();
        c->ll_ctr_base = 0;
        return set_error(MI355X_ERR_TIMEOUT, "rank %d: LL call %llu timed out waiting for a peer", c->rank,
                         (unsigned long long)seq);
    }
    c->ll_ctr_base += nblk;
    return MI355X_SUCCESS;
}

static double env_double(const char *name, double dflt);

// Collective, once at communicator creation: the LL region is built and one LL allgather of a
// rank-tagged 8 KiB pattern per rank runs with a short device-side bound (MI355X_LL_PROBE_S, 5 s).
// The LL path can be enabled (MI355X_KNOB_LL_MAX_BYTES) only if every rank saw every peer's bytes;
// otherwise small collectives always take the host-synchronised path (a protocol that misbehaves
// on some platform would otherwise stall every small call for timeout_s).  MI355X_LL=0 skips it.
static int ll_selftest(mi355x_comm *c)
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
    bool ok = hipMalloc((void **)&buf, per * (n + 1)) == hipSuccess;
    if (ok) ok = hipMemset(buf, c->rank + 1, per) == hipSuccess && hipMemset(buf + per, 0, per * n) == hipSuccess &&
                 hipDeviceSynchronize() == hipSuccess;
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
        ok = ll_run(c, a, 0, 0, nullptr) == MI355X_SUCCESS;
        c->timeout_s = saved;
    }
    if (ok) {
        std::vector<unsigned char> h(per * n);
        ok = hipMemcpy(h.data(), buf + per, per * n, hipMemcpyDeviceToHost) == hipSuccess;
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
static std::mutex g_svc_mtx;
static std::map<int, mi355x_comm *> g_svc_owner;  // device -> owning communicator

static uint64_t mono_ns()
{
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);  // (one clock for every process of the node)
    return (uint64_t)t.tv_sec * 1000000000ull + (uint64_t)t.tv_nsec;
}

static uint64_t *svc_done_word(mi355x_comm *c) { return c->svc_host; }
static uint32_t *svc_err_word(mi355x_comm *c) { return reinterpret_cast<uint32_t *>(c->svc_host + 1); }

// ring the doorbell: the page may be write-combined (BAR), so fence the stores out in order
static void svc_ring(mi355x_comm *c, uint64_t v)
{
    _mm_sfence();
    __atomic_store_n(&c->svc_page->door, v, __ATOMIC_RELEASE);
    _mm_sfence();
}

static int svc_launch(mi355x_comm *c, uint64_t first)
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
static bool svc_stop(mi355x_comm *c)
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
static void svc_park(mi355x_comm *c)
{
    if (c->svc_ok && c->svcq && svc_resident(c->svcq)) svc_ring(c, kSvcQuit);
}

// post `call` (number call.seq, `part` participating workgroups) and wait for its completion
static int svc_call(mi355x_comm *c, const SvcCall &call, uint64_t part)
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
static int svc_run(mi355x_comm *c, LLArgs &a, int op, int type, hipStream_t s)
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
static bool svc_pull_usable(const mi355x_comm *c, size_t bytes, size_t esz)
{
    return c->svc_ok && (c->flows & MI355X_FLOW_SVC_PULL) && !c->loopback && esz >= 4 && bytes > c->svc_max &&
           bytes <= c->svc_pull_max &&
           bytes < ((size_t)1 << 31);
}

// the same for allgather / bcast (LL_PULL_AG / LL_PULL_BC): `bytes` per rank between the LL form's
// limit and the copy limit (svc_copy_max); no alignment condition (each rank copies into its own buffer, with
// 16-B vectors where both ends allow)
static bool svc_pull_copy_usable(const mi355x_comm *c, size_t bytes)
{
    return c->svc_ok && (c->flows & MI355X_FLOW_SVC_COPY) && !c->loopback && bytes > c->svc_max && bytes <= c->svc_copy_max &&
           bytes * (size_t)c->size < ((size_t)1 << 31);
}

static int svc_pull_copy_run(mi355x_comm *c, int mode, const std::vector<std::vector<void *>> &P, const void *src,
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

static int svc_pull_run(mi355x_comm *c, int op, int type, const std::vector<std::vector<void *>> &P, const void *in,
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
static void svc_trace_report(mi355x_comm *c)
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

// The service's resources -- its HSA queue, doorbell page and host words -- exist once per process
// and GPU: created with the first communicator that may use the service (svc_setup; an idle queue
// also keeps the host flows of ranks sharing a GPU fast), shared by the communicators that own the
// service in turn (a handover creates no queue), freed with the last communicator attached.
struct SvcRes {
    SvcQueue *q = nullptr;
    SvcPage *page = nullptr;
    bool page_dev = false;
    uint64_t *host = nullptr;
    int users = 0;       // communicators attached (claimed once at least, not destroyed)
    bool stuck = false;  // a service kernel never left: never freed
};
static std::map<int, SvcRes> g_svc_res;  // device -> resources (g_svc_mtx)

// (g_svc_mtx held) this communicator's view of the process's service resources (created if needed)
static bool svc_attach(mi355x_comm *c)
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
static void svc_detach(mi355x_comm *c)
{
    if (!svc_stop(c)) g_svc_res[c->device].stuck = true;
    c->svcq = nullptr;
    c->svc_page = nullptr;
    c->svc_host = nullptr;
    c->svc_ok = false;
}

// (g_svc_mtx held) give up ownership
static void svc_unclaim_locked(mi355x_comm *c)
{
    if (!c->svc_owner) return;
    auto it = g_svc_owner.find(c->device);
    if (it != g_svc_owner.end() && it->second == c) g_svc_owner.erase(it);
    c->svc_owner = false;
}

static void svc_let_go(mi355x_comm *c)
{
    std::lock_guard<std::mutex> g(g_svc_mtx);
    svc_detach(c);
    svc_unclaim_locked(c);
}

// at destruction: let go, and free the process's resources with their last user
static void svc_release(mi355x_comm *c)
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
static uint32_t gate_revoker_word() { return ((uint32_t)getpid() << 8) | kGateRevoker; }

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
static bool svc_revoke(mi355x_comm *x)
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
static int ll_resync(mi355x_comm *c)
{
    (void)svc_stop(c);
    (void)hipDeviceSynchronize();
    int rc = barrier(c);
    if (rc) return rc;
    if (c->svc_stuck) return set_error(MI355X_ERR_HIP, "rank %d: the resident service did not leave", c->rank);
    MI_HIP(hipMemset(c->ll_base, 0, c->ll_bytes));
    MI_HIP(hipMemset(c->ll_ctr, 0, sizeof(uint64_t)));
    MI_HIP(hipDeviceSynchronize());
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

// ---- the flows' self-test.  Every cross-device flow that is on by default runs one short call on
// data that changes with the communicator (its secret) and the test, into a destination poisoned
// beforehand, and every rank checks its result exactly; the outcome is agreed in the control
// segment (every rank's mask ANDed, as the LL self-test agrees ll_ok) and a flow that failed on
// any rank is turned off on every rank -- its calls take the host-synchronised flows, whose
// coherence rests on kernel completion and a host barrier.  The reference negotiates CUDA IPC per
// peer pair the same way before using it, falling back to host staging (btl/smcuda/README:41-100,
// pml_ob1_cuda.c:183-210).  MI355X_SELFTEST_FAIL=<flow,...> (svc_ll, svc_pull, svc_copy, svc_rs,
// pipe) makes this rank report those flows failed (fault injection for tests); MI355X_SELFTEST=0
// skips the tests.
static unsigned selftest_injected()
{
    const char *e = getenv("MI355X_SELFTEST_FAIL");
    if (!e) return 0;
    unsigned m = 0;
    const struct { const char *name; unsigned bit; } names[] = {{"svc_ll", MI355X_FLOW_SVC_LL}, {"svc_pull", MI355X_FLOW_SVC_PULL},
                                                                {"svc_copy", MI355X_FLOW_SVC_COPY}, {"svc_rs", MI355X_FLOW_SVC_RS},
                                                                {"pipe", MI355X_FLOW_PIPE}};
    std::string s(e);
    for (const auto &n : names)
        if (s.find(n.name) != std::string::npos) m |= n.bit;
    return m;
}

static bool selftest_on() { return env_double("MI355X_SELFTEST", 1.0) != 0.0; }

static uint32_t st_val(uint64_t seed, int q, size_t i)
{
    uint64_t x = seed ^ ((uint64_t)(q + 1) << 40) ^ ((uint64_t)i * 0x9e3779b97f4a7c15ull);
    x ^= x >> 31;
    x *= 0xbf58476d1ce4e5b9ull;
    x ^= x >> 29;
    return (uint32_t)(x & 0xffffff);  // (sums of <= 64 ranks stay below 2^31)
}

// device buffers of the self-test: my input (n x count int32 for the reduce_scatter block), output
struct SelfTest {
    mi355x_comm *c;
    uint64_t seed;
    char *in = nullptr, *out = nullptr;
    size_t cap = 0;
    bool ok = true;
    SelfTest(mi355x_comm *c_, uint64_t salt, size_t bytes) : c(c_), cap(bytes)
    {
        seed = c->ctrl->secret ^ (salt * 0x632be59bd9b4e019ull);
        ok = hipMalloc((void **)&in, cap) == hipSuccess && hipMalloc((void **)&out, cap) == hipSuccess;
    }
    ~SelfTest()
    {
        if (in) (void)hipFree(in);
        if (out) (void)hipFree(out);
        (void)hipGetLastError();
    }
    // my input: `count` int32 of test `t`; the output poisoned
    bool prepare(int t, size_t count)
    {
        std::vector<uint32_t> h(count);
        for (size_t i = 0; i < count; ++i) h[i] = st_val(seed + (uint64_t)t, c->rank, i);
        // (the null stream only: the application's other streams are not waited for)
        return ok && count * 4 <= cap && hipMemcpy(in, h.data(), count * 4, hipMemcpyHostToDevice) == hipSuccess &&
               hipMemsetAsync(out, 0xa5, cap, nullptr) == hipSuccess && hipStreamSynchronize(nullptr) == hipSuccess;
    }
    bool fetch(std::vector<uint32_t> &h, size_t count)
    {
        h.assign(count, 0);
        return hipMemcpy(h.data(), out, count * 4, hipMemcpyDeviceToHost) == hipSuccess;
    }
    // element i of the SUM over every rank's input of test t
    uint32_t sum(int t, size_t i) const
    {
        uint32_t a = 0;
        for (int q = 0; q < c->size; ++q) a += st_val(seed + (uint64_t)t, q, i);
        return a;
    }
};

// agree on the masks every rank saw pass; returns the AND (collective)
static int agree_flows(mi355x_comm *c, unsigned mine, unsigned *all)
{
    c->ctrl->slot[c->rank].flow_ok = mine;
    int rc = barrier(c);
    if (rc) return rc;
    unsigned a = ~0u;
    for (int q = 0; q < c->size; ++q) a &= c->ctrl->slot[q].flow_ok;
    *all = a;
    return barrier(c);  // nobody rewrites its word before every rank has read it
}

} // namespace mi355x
// (defined below, outside the namespace, with the public entry points)
static int allreduce_impl(mi355x_comm_t *c, const void *sbuf, void *rbuf, size_t count, int type, int op, void *stream);
static int allgather_impl(mi355x_comm_t *c, const void *sbuf, void *rbuf, size_t bytes, void *stream);
static int bcast_impl(mi355x_comm_t *c, void *buf, size_t bytes, int root, void *stream);
static int reduce_scatter_block_impl(mi355x_comm_t *c, const void *sbuf, void *rbuf, size_t rcount, int type, int op,
                                     void *stream);
namespace mi355x {

// The service's flows, at its first claim (the service is claimed on every rank; collective).
static int svc_selftest(mi355x_comm *c)
{
    c->svc_flows_tested = true;
    const unsigned tested = MI355X_FLOW_SVC_LL | MI355X_FLOW_SVC_PULL | MI355X_FLOW_SVC_COPY | MI355X_FLOW_SVC_RS;
    if (!selftest_on()) return MI355X_SUCCESS;
    const auto t0 = std::chrono::steady_clock::now();
    const int n = c->size;
    // the flows' mechanisms at fixed sizes, whatever the limits are set to now; nothing forced
    struct Saved {
        size_t svc_max, pull, copy, one;
        bool rs, ok;
        int ar, red, rs_alg;
        const mi355x_rules_t *rules;
        double timeout;
        unsigned flows;
    } sv{c->svc_max, c->svc_pull_max, c->svc_copy_max, c->one_phase_max, c->svc_rs, c->svc_ok, c->knob_allreduce,
         c->knob_reduce, c->knob_rs, c->rules, c->timeout_s, c->flows};
    c->svc_max = 8192;
    c->svc_pull_max = c->svc_copy_max = 65536;
    c->one_phase_max = std::max<size_t>(c->one_phase_max, 65536);
    c->svc_rs = true;
    c->svc_ok = true;
    c->knob_allreduce = c->knob_reduce = c->knob_rs = 0;
    c->rules = nullptr;
    c->timeout_s = env_double("MI355X_LL_PROBE_S", 5.0);
    c->flows |= tested;
    unsigned pass = 0;
    {
        SelfTest st(c, c->svc_epoch, (size_t)n * 65536);
        const int i32 = MI355X_T_INT32, sum = MI355X_OP_SUM;
        std::vector<uint32_t> h;
        // a call of `flow` served by the service: exact, and the service served `calls` of them
        auto served = [&](uint64_t before, uint64_t calls) { return c->svc_calls - before == calls; };
        // LL form: an allgather and a reducing allreduce (granules pushed into every peer)
        {
            bool ok = st.prepare(1, 2048);
            const uint64_t b = c->svc_calls;
            ok = ok && allgather_impl(c, st.in, st.out, 8192, nullptr) == MI355X_SUCCESS && st.fetch(h, 2048 * (size_t)n);
            for (int q = 0; q < n && ok; ++q)
                for (size_t i = 0; i < 2048 && ok; ++i) ok = h[(size_t)q * 2048 + i] == st_val(st.seed + 1, q, i);
            ok = ok && st.prepare(2, 2048) && allreduce_impl(c, st.in, st.out, 2048, i32, sum, nullptr) == MI355X_SUCCESS &&
                 st.fetch(h, 2048);
            for (size_t i = 0; i < 2048 && ok; ++i) ok = h[i] == st.sum(2, i);
            if (ok && served(b, 2)) pass |= MI355X_FLOW_SVC_LL;
        }
        // pull form: a one-phase ring allreduce folded from the peers' mapped inputs
        if (pass & MI355X_FLOW_SVC_LL) {
            const size_t cnt = 12288;  // 48 KiB
            bool ok = st.prepare(3, cnt);
            const uint64_t b = c->svc_calls;
            ok = ok && allreduce_impl(c, st.in, st.out, cnt, i32, sum, nullptr) == MI355X_SUCCESS && st.fetch(h, cnt);
            for (size_t i = 0; i < cnt && ok; ++i) ok = h[i] == st.sum(3, i);
            if (ok && served(b, 1)) pass |= MI355X_FLOW_SVC_PULL;
            // pull copies: allgather of every peer's block, bcast of the last rank's buffer
            ok = st.prepare(4, cnt);
            const uint64_t b2 = c->svc_calls;
            ok = ok && allgather_impl(c, st.in, st.out, cnt * 4, nullptr) == MI355X_SUCCESS && st.fetch(h, cnt * (size_t)n);
            for (int q = 0; q < n && ok; ++q)
                for (size_t i = 0; i < cnt && ok; ++i) ok = h[(size_t)q * cnt + i] == st_val(st.seed + 4, q, i);
            ok = ok && st.prepare(5, cnt) && hipMemcpy(st.out, st.in, cnt * 4, hipMemcpyDeviceToDevice) == hipSuccess &&
                 bcast_impl(c, st.out, cnt * 4, n - 1, nullptr) == MI355X_SUCCESS && st.fetch(h, cnt);
            for (size_t i = 0; i < cnt && ok; ++i) ok = h[i] == st_val(st.seed + 5, n - 1, i);
            if (ok && served(b2, 2)) pass |= MI355X_FLOW_SVC_COPY;
            // reduce-scatter form: my 16 KiB block evaluated from the peers' mapped inputs
            const size_t rc_ = 4096;
            ok = st.prepare(6, rc_ * (size_t)n);
            const uint64_t b3 = c->svc_calls;
            ok = ok && reduce_scatter_block_impl(c, st.in, st.out, rc_, i32, sum, nullptr) == MI355X_SUCCESS &&
                 st.fetch(h, rc_);
            for (size_t i = 0; i < rc_ && ok; ++i) ok = h[i] == st.sum(6, (size_t)c->rank * rc_ + i);
            if (ok && served(b3, 1)) pass |= MI355X_FLOW_SVC_RS;
        }
        (void)hipGetLastError();
    }
    pass &= ~selftest_injected();
    c->svc_max = sv.svc_max;
    c->svc_pull_max = sv.pull;
    c->svc_copy_max = sv.copy;
    c->one_phase_max = sv.one;
    c->svc_rs = sv.rs;
    c->svc_ok = sv.ok;
    c->knob_allreduce = sv.ar;
    c->knob_reduce = sv.red;
    c->knob_rs = sv.rs_alg;
    c->rules = sv.rules;
    c->timeout_s = sv.timeout;
    c->flows = sv.flows;
    unsigned all = 0;
    int rc = agree_flows(c, pass | ~tested, &all);
    if (rc) return rc;
    const unsigned failed = tested & ~all;
    c->flows &= ~failed;
    c->flows_failed |= failed;
    if (failed) {
        if (c->rank == 0)
            fprintf(stderr, "[mi355x] resident-service flow self-test failed (flows 0x%x): those calls take the "
                    "host-synchronised flows\n", failed);
        rc = ll_resync(c);
        if (rc) return rc;
    }
    c->selftest_us += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    TRACE(c, "service flow self-test: passed here 0x%x, agreed 0x%x", pass, all & tested);
    return MI355X_SUCCESS;
}

// The pipelined allreduce's per-chunk flag hand-off, at creation (multi-process, collective): one
// allreduce of 128 KiB blocks in 16 KiB chunks (8 per block), forced onto the pipelined flow.
static int pipe_selftest(mi355x_comm *c)
{
    if (!selftest_on()) return MI355X_SUCCESS;
    const auto t0 = std::chrono::steady_clock::now();
    const int n = c->size;
    const size_t count = (size_t)n * 32768;
    struct Saved {
        bool pipe, want;
        size_t one;
        int ar;
        const mi355x_rules_t *rules;
        double timeout;
    } sv{c->pipe_on, c->svc_want, c->one_phase_max, c->knob_allreduce, c->rules, c->timeout_s};
    c->pipe_on = true;
    c->svc_want = false;  // (no claim from inside this call, whatever the service limits are)
    c->one_phase_max = 0;
    c->knob_allreduce = AR_RING;
    c->rules = nullptr;
    c->pipe_chunk_override = 4096;
    c->timeout_s = env_double("MI355X_LL_PROBE_S", 5.0);
    unsigned pass = 0;
    bool admitted = false;
    {
        SelfTest st(c, 0x9e37u, count * 4);
        std::vector<uint32_t> h;
        const uint64_t refused = c->pipe_refused;
        bool ok = st.prepare(7, count) &&
                  allreduce_impl(c, st.in, st.out, count, MI355X_T_INT32, MI355X_OP_SUM, nullptr) == MI355X_SUCCESS &&
                  st.fetch(h, count);
        for (size_t i = 0; i < count && ok; ++i) ok = h[i] == st.sum(7, i);
        admitted = c->pipe_refused == refused;
        if (ok) pass |= MI355X_FLOW_PIPE;
        (void)hipGetLastError();
    }
    c->pipe_on = sv.pipe;
    c->svc_want = sv.want;
    c->one_phase_max = sv.one;
    c->knob_allreduce = sv.ar;
    c->rules = sv.rules;
    c->timeout_s = sv.timeout;
    c->pipe_chunk_override = 0;
    pass &= ~selftest_injected();
    // not admitted (another communicator's grid held a GPU): the call ran two phases -- nothing
    // learnt about the flag hand-off, so it counts as untested, not failed (every rank agrees:
    // admission is agreed per call)
    unsigned all = 0;
    int rc = agree_flows(c, (pass | ~(unsigned)MI355X_FLOW_PIPE) | (admitted ? 0u : (unsigned)MI355X_FLOW_PIPE), &all);
    if (rc) return rc;
    c->pipe_untested = !admitted;
    if (!(all & MI355X_FLOW_PIPE)) {
        c->flows &= ~(unsigned)MI355X_FLOW_PIPE;
        c->flows_failed |= MI355X_FLOW_PIPE;
        c->pipe_on = false;
        if (c->rank == 0)
            fprintf(stderr, "[mi355x] pipelined allreduce self-test failed: large allreduces take the two-phase flow\n");
    }
    c->selftest_us += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    TRACE(c, "pipelined flow self-test: %s", !admitted ? "not admitted (untested)" : (all & MI355X_FLOW_PIPE) ? "ok" : "failed -> off");
    return MI355X_SUCCESS;
}

// Collective: claim the process's service for this communicator on every rank, or on none.  Called
// from a service-sized call on every rank alike (svc_maybe_claim).  A rank whose service another
// communicator owns takes it over if that owner has been idle long enough (svc_revoke).
static int svc_claim(mi355x_comm *c)
{
    const auto t0 = std::chrono::steady_clock::now();
    int mine = 2;  // 1 claimed, 2 owned by a busy communicator, 3 the service cannot run here
    {
        std::lock_guard<std::mutex> g(g_svc_mtx);
        auto it = g_svc_owner.find(c->device);
        const bool free_ = it == g_svc_owner.end() || it->second == c;
        if (free_ || svc_revoke(it->second)) {
            if (it != g_svc_owner.end()) g_svc_owner.erase(it);  // (a revoked owner is no owner any more)
            if (!svc_attach(c)) {
                mine = 3;
            } else {
                g_svc_owner[c->device] = c;
                c->svc_owner = true;
                mine = 1;
            }
        }
    }
    c->ctrl->slot[c->rank].svc_claim = mine;
    int rc = barrier(c);
    if (rc) return rc;
    bool all = true, broken = false;
    for (int q = 0; q < c->size; ++q) {
        all = all && c->ctrl->slot[q].svc_claim == 1;
        broken = broken || c->ctrl->slot[q].svc_claim == 3;
    }
    rc = barrier(c);  // every rank has read the claims before they are rewritten
    if (rc) return rc;
    if (!all) {
        if (mine == 1) svc_let_go(c);
        if (broken) {
            c->svc_want = false;  // the service cannot run on some rank: stop trying (every rank saw it)
            if (c->rank == 0) fprintf(stderr, "[mi355x] resident LL service unavailable: small collectives use the per-call paths\n");
        }
        TRACE(c, "service claim: %s", broken ? "unavailable" : "owned by another communicator on some rank");
        return MI355X_SUCCESS;
    }
    c->svc_epoch++;
    c->ctrl->slot[c->rank].svc_last_ns.store(mono_ns(), std::memory_order_relaxed);
    if (!c->svc_flows_tested) {
        rc = svc_selftest(c);
        if (rc) return rc;
    }
    if (!(c->flows & MI355X_FLOW_SVC_LL)) {
        svc_let_go(c);
        c->svc_want = false;
        return MI355X_SUCCESS;
    }
    c->svc_ok = true;
    TRACE(c, "service claimed (epoch %llu) in %.0f us", (unsigned long long)c->svc_epoch,
          std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    return MI355X_SUCCESS;
}

// at a service-sized call: claim the service if this communicator does not have it (every
// svc_retry-th such call; the same decision on every rank: sizes and agreed state only)
static int svc_maybe_claim(mi355x_comm *c, bool sized)
{
    if (c->svc_ok || !c->svc_want || !sized) return MI355X_SUCCESS;
    if (c->svc_tries++ % c->svc_retry != 0) return MI355X_SUCCESS;
    return svc_claim(c);
}

// at creation: the service's settings (the claim itself waits for a service-sized call)
static void svc_setup(mi355x_comm *c)
{
    c->svc_max = (size_t)std::max(0.0, env_double("MI355X_SVC_MAX_BYTES", (double)c->svc_max));
    c->svc_idle_s = std::max(0.0001, env_double("MI355X_SVC_IDLE_MS", c->svc_idle_s * 1e3) * 1e-3);
    c->svc_shrink_s = std::max(0.0, env_double("MI355X_SVC_SHRINK_US", c->svc_shrink_s * 1e6) * 1e-6);
    c->svc_nwg = (int)std::min(64.0, std::max(1.0, env_double("MI355X_SVC_WGS", (double)c->svc_nwg)));
    c->svc_pull_max = (size_t)std::max(0.0, env_double("MI355X_SVC_PULL_MAX_BYTES", (double)c->svc_pull_max));
    c->svc_copy_max = (size_t)std::max(0.0, env_double("MI355X_SVC_PULL_COPY_MAX_BYTES", (double)c->svc_copy_max));
    c->svc_rs = env_double("MI355X_SVC_RS", c->svc_rs ? 1.0 : 0.0) != 0.0;
    c->svc_handover_s = std::max(0.0, env_double("MI355X_SVC_HANDOVER_MS", c->svc_handover_s * 1e3) * 1e-3);
    c->svc_retry = (uint64_t)std::max(1.0, env_double("MI355X_SVC_RETRY_CALLS", (double)c->svc_retry));
    const char *env = getenv("MI355X_SVC");
    c->svc_want = c->ll_ok && c->size <= kLLMaxRanks && !c->loopback && !(env && atoi(env) == 0);
    // The service's resources (its HSA queue above all) are created now, not at the first claim:
    // an idle HSA queue in the process changes how the GPU schedules the HIP queues of several
    // processes sharing it -- the host-synchronised small allreduce / allgather of 4 ranks on one
    // GPU takes 20 us with it and 55 us without (profiles/r04_host_flow_idle_queue.jsonl: the
    // queue alone, without any dispatch, makes the difference; hsa_init, a probe launch or a signal
    // alone do not).  MI355X_SVC_EAGER=0 defers them to the first claim; MI355X_SVC_PREP=<mask>
    // repeats the experiment (1 hsa_init, 2 probe launch, 8 a bare queue, 16 a signal).
    if (c->svc_want && env_double("MI355X_SVC_EAGER", 1.0) != 0.0) {
        std::lock_guard<std::mutex> g(g_svc_mtx);
        if (!g_svc_res[c->device].q && svc_attach(c)) svc_detach(c);
    }
    const int prep = (int)env_double("MI355X_SVC_PREP", 0.0);
    if (prep & ~4) (void)svc_prep(c->device, prep);
}

// ----------------------------------------------------------------- pipelined allreduce
// (Re)build the per-chunk flag region (uncached, every peer writes its row into it over xGMI)
// and the work-queue counter.  Collective: every rank reaches it in the same call.
constexpr size_t kPipeKmax = 1024;  // chunks per ring block, at most
static int ensure_pipe(mi355x_comm *c)
{
    if (c->pipe_base) return MI355X_SUCCESS;
    const size_t n = (size_t)c->size;
    const size_t bytes = (n * kPipeKmax * sizeof(uint64_t) + 4095) / 4096 * 4096;
    MI_HIP(hipExtMallocWithFlags((void **)&c->pipe_base, bytes, hipDeviceMallocUncached));
    MI_HIP(hipMemset(c->pipe_base, 0, bytes));
    MI_HIP(hipMalloc((void **)&c->pipe_queue, sizeof(uint64_t)));
    MI_HIP(hipMemset(c->pipe_queue, 0, sizeof(uint64_t)));
    if (!c->ll_err) MI_HIP(hipHostMalloc((void **)&c->ll_err, sizeof(uint32_t), hipHostMallocCoherent));
    MI_HIP(hipDeviceSynchronize());
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

// ---- admission of the pipelined grid.  k_pipe_allreduce is persistent and spins on flags its
// peers' grids raise, so it must never wait behind another spinning grid: two communicators whose
// grids each hold one GPU while waiting for the other's would wait forever (a cross-GPU circular
// wait, possible in any MPI_THREAD_MULTIPLE program that overlaps collectives on several
// communicators).  Every GPU therefore carries a node-wide token: one communicator at a time may
// have pipelined grids on it (its ranks sharing that GPU -- a rehearsal -- count up the same
// token).  Per call every rank tries its GPU's token WITHOUT waiting and publishes the outcome with
// the call's buffer exchange; the call is pipelined only if every rank holds its token, otherwise
// every rank releases and the call takes the two-phase flow, whose kernels never wait on a peer.
// Nothing ever spins for admission (the never-blocking progress rule of opal_progress.c:150).
// The table lives in a per-user shared-memory segment (64 GPUs) that outlives the job, so a token
// must not outlive its holder: every process that counts up a token first registers itself in the
// token's holder list (pid + process start time); a process that finds the token taken by another
// holder and no live process registered for that holder takes the count back (a holder killed
// mid-call -- SIGKILL, OOM -- would otherwise leave the GPU on the two-phase flow for every later
// job of the user on the node).  The reference keeps no node-wide state past a process's death
// (smcuda's IPC state is per endpoint, btl/smcuda/README:92-100); this is the same guarantee.
constexpr int kTokHolders = 64;       // registrations per GPU (ranks x communicators sharing it)
constexpr uint64_t kTokPending = 1ull << 63;  // registration being written (pid valid, rest not yet)
struct TokHolder {
    std::atomic<uint64_t> who;        // 0 free; pid | kTokPending while filled in; pid when complete
    std::atomic<uint64_t> start;      // the process's start time (/proc/<pid>/stat field 22)
    std::atomic<uint64_t> holder;     // the communicator id it counts up the token for
};
struct GpuTokens {
    std::atomic<uint64_t> uid[64];    // device uid (hash of the PCI bus id), 0 = free slot
    // (holder id << 32) | (generation << 8) | holders' count; count 0 = free.  The generation
    // changes on every transition, so a reclaim (compare-exchange from the value it inspected)
    // fails if anything happened in between.
    std::atomic<uint64_t> word[64];
    TokHolder h[64][kTokHolders];
};

static uint64_t proc_start_time(pid_t pid)
{
    char path[64], buf[1024];
    snprintf(path, sizeof(path), "/proc/%d/stat", (int)pid);
    const int fd = open(path, O_RDONLY);
    if (fd < 0) return 0;
    const ssize_t n = read(fd, buf, sizeof(buf) - 1);
    close(fd);
    if (n <= 0) return 0;
    buf[n] = 0;
    const char *p = strrchr(buf, ')');  // the command name may hold spaces; fields follow its ')'
    if (!p) return 0;
    int field = 2;
    for (++p; *p && field < 22; ++p)
        if (*p == ' ') ++field;
    return strtoull(p, nullptr, 10);
}

// a registered process still exists (the same process: pid reuse changes the start time)
static bool holder_alive(uint64_t who, uint64_t start)
{
    const pid_t pid = (pid_t)(who & 0x7fffffffull);
    if (!pid_alive(pid)) return false;
    if (who & kTokPending) return true;  // still registering: its start time is not written yet
    const uint64_t now = proc_start_time(pid);
    return now == 0 || now == start;
}

static GpuTokens *gpu_tokens()
{
    static GpuTokens *t = nullptr;
    static std::once_flag once;
    std::call_once(once, [] {
        char name[96];
        snprintf(name, sizeof(name), "/mi355x_gpu_tokens2_%u", (unsigned)getuid());
        const char *alt = getenv("MI355X_TOKEN_TABLE");  // (tests: a private table)
        if (alt && *alt == '/' && strlen(alt) < sizeof(name)) snprintf(name, sizeof(name), "%s", alt);
        const int fd = shm_open(name, O_CREAT | O_RDWR, 0600);
        if (fd < 0) return;
        struct stat st;
        if (fstat(fd, &st) == 0 && (size_t)st.st_size < sizeof(GpuTokens) && ftruncate(fd, sizeof(GpuTokens)) != 0) {
            close(fd);
            return;
        }
        void *m = mmap(nullptr, sizeof(GpuTokens), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        close(fd);
        if (m != MAP_FAILED) t = (GpuTokens *)m;  // a fresh segment is zero-filled: every slot free
    });
    return t;
}

// Take back a token whose count was raised only by processes that no longer exist (the value `cur`
// was read by the caller; the compare-exchange fails if anything changed since).
static bool pipe_token_reclaim(GpuTokens *t, int i, uint64_t cur)
{
    const uint64_t holder = cur >> 32;
    for (int e = 0; e < kTokHolders; ++e) {
        const uint64_t who = t->h[i][e].who.load(std::memory_order_acquire);
        if (!who) continue;
        const uint64_t start = t->h[i][e].start.load(std::memory_order_relaxed);
        const uint64_t hid = t->h[i][e].holder.load(std::memory_order_relaxed);
        if (!holder_alive(who, start)) {
            // a dead registration: free it (whatever it counted is what this reclaim takes back)
            uint64_t w = who;
            t->h[i][e].who.compare_exchange_strong(w, 0);
            continue;
        }
        // a registration still being written may belong to the dead holder's communicator too: it
        // has not counted up yet, and when it tries, its compare-exchange from the value this
        // reclaim replaces fails (the generation changed), so it does not block the reclaim
        if (who & kTokPending) continue;
        if (hid == holder) return false;  // a live process counts up this token
    }
    const uint64_t next = (((cur >> 8) + 1) & 0xffffff) << 8;  // free (holder 0, count 0), next generation
    const bool ok = t->word[i].compare_exchange_strong(cur, next, std::memory_order_acq_rel);
    if (ok) fprintf(stderr, "[mi355x] reclaimed the pipelined-grid token of a GPU from a process that died holding it\n");
    return ok;
}

static bool pipe_token_acquire(mi355x_comm *c)
{
    GpuTokens *t = gpu_tokens();
    if (!t) return false;
    if (c->pipe_token < 0) {
        const uint64_t uid = c->ctrl->slot[c->rank].dev_uid | 1;
        for (int i = 0; i < 64 && c->pipe_token < 0; ++i) {
            uint64_t cur = t->uid[i].load(std::memory_order_acquire);
            if (cur == 0 && t->uid[i].compare_exchange_strong(cur, uid)) cur = uid;
            if (cur == uid) c->pipe_token = i;
        }
        if (c->pipe_token < 0) return false;
        uint64_t h = 1469598103934665603ull;
        for (char ch : c->shm_name) h = (h ^ (unsigned char)ch) * 1099511628211ull;
        c->pipe_holder = ((h ^ (h >> 32)) & 0xffffffffull) | 1;
    }
    const int i = c->pipe_token;
    // register first (pid, start time, holder), so a reclaimer never takes a count from under me
    const uint64_t pid = (uint64_t)getpid();
    static const uint64_t my_start = proc_start_time(getpid());
    int e = -1;
    for (int k = 0; k < kTokHolders && e < 0; ++k) {
        uint64_t z = 0;
        if (t->h[i][k].who.compare_exchange_strong(z, pid | kTokPending)) e = k;
    }
    if (e < 0) return false;  // (a full list: this call simply takes the two-phase flow)
    t->h[i][e].start.store(my_start, std::memory_order_relaxed);
    t->h[i][e].holder.store(c->pipe_holder, std::memory_order_relaxed);
    t->h[i][e].who.store(pid, std::memory_order_release);
    std::atomic<uint64_t> &w = t->word[i];
    uint64_t cur = w.load(std::memory_order_acquire);
    for (int looks = 0;;) {
        const uint64_t holder = cur >> 32, cnt = cur & 0xff, gen = (cur >> 8) & 0xffffff;
        if (cnt != 0 && holder != c->pipe_holder) {
            // held by another communicator: take it back if its holders are all dead; if the word
            // changed meanwhile (a peer rank of mine reclaimed it first, or counted up), look again
            if (looks++ < 8) {
                const bool took = pipe_token_reclaim(t, i, cur);
                const uint64_t now = w.load(std::memory_order_acquire);
                if (took || now != cur) {
                    cur = now;
                    continue;
                }
            }
            break;
        }
        if (cnt == 0xff) break;
        const uint64_t next = (c->pipe_holder << 32) | (((gen + 1) & 0xffffff) << 8) | (cnt + 1);
        if (w.compare_exchange_weak(cur, next, std::memory_order_acq_rel)) {
            c->pipe_entry = e;
            return true;
        }
    }
    t->h[i][e].who.store(0, std::memory_order_release);
    return false;
}

static void pipe_token_release(mi355x_comm *c)
{
    GpuTokens *t = gpu_tokens();
    std::atomic<uint64_t> &w = t->word[c->pipe_token];
    uint64_t cur = w.load(std::memory_order_acquire);
    for (;;) {
        const uint64_t cnt = cur & 0xff, gen = (cur >> 8) & 0xffffff;
        const uint64_t next = cnt <= 1 ? (((gen + 1) & 0xffffff) << 8)
                                       : (cur & ~0xffffffffull) | (((gen + 1) & 0xffffff) << 8) | (cnt - 1);
        if (w.compare_exchange_weak(cur, next, std::memory_order_acq_rel)) break;
    }
    if (c->pipe_entry >= 0) t->h[c->pipe_token][c->pipe_entry].who.store(0, std::memory_order_release);
    c->pipe_entry = -1;
}

// One launch per rank: fold my ring block and pull the other blocks, chunk by chunk, with
// device-side readiness flags (coll_pipe.hip).  P[0] = every rank's input, P[1] = every rbuf.
static int pipe_allreduce(mi355x_comm *c, int op, int type, const Program &pr,
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
    MI_HIP(hipStreamSynchronize(s));
    if (__atomic_load_n(c->ll_err, __ATOMIC_ACQUIRE)) {
        // the counter no longer has its expected value: start it over for the next call
        (void)hipMemset(c->pipe_queue, 0, sizeof(uint64_t));
        (void)hipDeviceSynchronize();
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

static void ll_program(LLArgs &a, const Program &pr)
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
static bool svc_rs_usable(const mi355x_comm *c, size_t max_block_bytes, const Program &pr)
{
    return c->svc_ok && c->svc_rs && (c->flows & MI355X_FLOW_SVC_RS) && !c->loopback && c->size >= 2 && c->size <= kLLMaxRanks && max_block_bytes <= c->svc_pull_max &&
           (pr.is_fold ? pr.order.size() == (size_t)c->size
                       : (c->size <= kTreeMax && pr.steps.size() <= (size_t)kTreeSteps));
}

// off: my block's byte offset in every rank's input; bytes: my block's length
static int svc_rs_run(mi355x_comm *c, int op, int type, const Program &pr, const std::vector<std::vector<void *>> &P,
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

// ----------------------------------------------------------------- algorithm choice
// The order of coll/tuned's dec_dynamic functions (coll_tuned_decision_dynamic.c:59-99): a file
// rule for this communicator size and message size, else the forced (MCA) algorithm, else the
// fixed decision.
static int rule_alg(const mi355x_comm *c, int coll, size_t bytes, int *faninout)
{
    int alg = 0;
    if (c->rules) mi355x_rules_decide(c->rules, coll, c->size, bytes, &alg, faninout, nullptr);
    return alg;
}

static int pick_allreduce(const mi355x_comm *c, size_t count, size_t esz)
{
    const int r = rule_alg(c, MI355X_COLL_ALLREDUCE, count * esz, nullptr);
    if (r) return r;
    return c->knob_allreduce ? c->knob_allreduce : allreduce_decision(c->size, count, esz);
}

// what comm->c_coll.coll_reduce would run for `count` elements (ompi_coll_tuned_reduce_intra_
// dec_dynamic): used by MPI_Reduce and by the algorithms that call it (nonoverlapping allreduce,
// coll/basic reduce_scatter_block, nonoverlapping reduce_scatter)
static int pick_reduce(const mi355x_comm *c, size_t count, size_t esz, int *chain_fanout)
{
    int fio = 0;
    const int r = rule_alg(c, MI355X_COLL_REDUCE, count * esz, &fio);
    if (r) {
        *chain_fanout = fio;
        return r;
    }
    *chain_fanout = c->chain_fanout;
    return c->knob_reduce ? c->knob_reduce : reduce_decision(c->size, count, esz);
}

static int pick_reduce_scatter(const mi355x_comm *c, size_t total, size_t esz)
{
    const int r = rule_alg(c, MI355X_COLL_REDUCESCATTER, total * esz, nullptr);
    if (r) return r;
    return c->knob_rs ? c->knob_rs : reduce_scatter_decision(c->size, total, esz);
}

// per-element program of a reduce to `root` of `count` elements
static bool reduce_program(const mi355x_comm *c, size_t count, size_t esz, int root, Program *pr, int *alg)
{
    int fanout = kDefaultChainFanout;
    *alg = pick_reduce(c, count, esz, &fanout);
    ExprPool ep;
    return compile_expr(ep, expr_reduce(ep, *alg, c->size, root, fanout), c->size, pr);
}

// program of the non-ring allreduce algorithms: recursive doubling, or reduce to 0 + bcast
// (nonoverlapping: comm->c_coll.coll_reduce, coll_tuned_allreduce.c:67-100; linear: the linear
// reduce, :897-929)
static bool allreduce_tree_program(mi355x_comm *c, int alg, size_t count, size_t esz, Program *pr)
{
    if (alg == AR_RECDBL || alg == AR_LINEAR) {
        // these depend on the communicator size only: compiled once (the symbolic re-execution of
        // the schedule costs about a microsecond, a visible share of a small allreduce)
        std::lock_guard<std::mutex> g(c->prog_mtx);
        auto it = c->prog_cache.find(alg);
        if (it != c->prog_cache.end()) {
            *pr = it->second;
            return true;
        }
        ExprPool ep;
        const bool ok = compile_expr(ep, alg == AR_RECDBL ? expr_allreduce_recursive_doubling(ep, c->size)
                                                          : expr_reduce(ep, RED_LINEAR, c->size, 0),
                                     c->size, pr);
        if (ok) c->prog_cache.emplace(alg, *pr);
        return ok;
    }
    int ra;
    return reduce_program(c, count, esz, 0, pr, &ra);
}

int check_common(mi355x_comm *c, int op, int type)
{
    if (!c) return set_error(MI355X_ERR_ARG, "comm is NULL");
    if (!mi355x_comm_op_supported(op, type))
        return set_error(MI355X_ERR_UNSUPPORTED, "no engine fold for op %d type %d", op, type);
    return MI355X_SUCCESS;
}

static double env_double(const char *name, double dflt)
{
    const char *v = getenv(name);
    return v ? atof(v) : dflt;
}

// ----------------------------------------------------------------- nonblocking
// Wait until every posted nonblocking call of this communicator has finished (MPI orders a
// blocking collective after the nonblocking ones posted before it on every rank).
void drain(mi355x_comm *c)
{
    std::unique_lock<std::mutex> g(c->q_mtx);
    c->q_cv.wait(g, [c] { return c->pending == 0; });
}

static void worker_main(mi355x_comm *c)
{
    (void)hipSetDevice(c->device);
    for (;;) {
        mi355x_request *r;
        {
            std::unique_lock<std::mutex> g(c->q_mtx);
            c->q_cv.wait(g, [c] { return c->stop || !c->queue.empty(); });
            if (c->queue.empty()) return;  // stop requested and nothing left
            r = c->queue.front();
            c->queue.pop_front();
        }
        int rc = MI355X_SUCCESS;
        if (hipStreamWaitEvent(c->nb_stream, r->ev, 0) != hipSuccess)
            rc = set_error(MI355X_ERR_HIP, "hipStreamWaitEvent failed");
        if (rc == MI355X_SUCCESS) {
            CallGate gate(c);
            rc = r->run(c->nb_stream);
        }
        r->rc = rc;
        if (rc != MI355X_SUCCESS) r->err = mi355x_last_error();
        r->run = nullptr;
        r->done.store(1, std::memory_order_release);
        {
            std::lock_guard<std::mutex> g(c->q_mtx);
            c->pending--;
        }
        c->q_cv.notify_all();
    }
}

// queue `run` after the caller's work on `stream`; the request completes when it has run
int post(mi355x_comm *c, void *stream, std::function<int(hipStream_t)> run, mi355x_request **out)
{
    if (!out) return set_error(MI355X_ERR_ARG, "request pointer is NULL");
    *out = nullptr;
    if (!c->nb_stream) {
        DeviceGuard dg(c->device);
        MI_HIP(hipStreamCreateWithFlags(&c->nb_stream, hipStreamNonBlocking));
    }
    auto *r = new mi355x_request();
    hipError_t e = hipEventCreateWithFlags(&r->ev, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventRecord(r->ev, resolve_stream(stream));
    if (e != hipSuccess) {
        if (r->ev) (void)hipEventDestroy(r->ev);
        delete r;
        return set_error(MI355X_ERR_HIP, "event on the caller stream: %s", hipGetErrorString(e));
    }
    r->run = std::move(run);
    {
        std::lock_guard<std::mutex> g(c->q_mtx);
        if (!c->worker.joinable()) c->worker = std::thread(worker_main, c);
        c->queue.push_back(r);
        c->pending++;
    }
    c->q_cv.notify_all();
    *out = r;
    return MI355X_SUCCESS;
}

} // namespace mi355x

using namespace mi355x;

extern "C" {

int mi355x_comm_create(const char *key, int rank, int size, int device, mi355x_comm_t **out)
{
    if (!key || !out || size < 1 || size > kMaxRanks || rank < 0 || rank >= size)
        return set_error(MI355X_ERR_ARG, "bad comm_create arguments");
    *out = nullptr;
    const auto t_create = std::chrono::steady_clock::now();
    DeviceGuard dg(device);
    char bus[64] = "";
    MI_HIP(hipDeviceGetPCIBusId(bus, (int)sizeof(bus), device));
    auto *c = new mi355x_comm();
    c->rank = rank;
    c->size = size;
    c->device = device;
    c->timeout_s = env_double("MI355X_TIMEOUT_S", 600.0);
    c->shm_name = std::string("/mi355x_") + key;
    for (char &ch : c->shm_name)
        if (ch != '/' && !isalnum((unsigned char)ch) && ch != '_' && ch != '-') ch = '_';
    const size_t bytes = ctrl_bytes(size);
    int fd = -1;
    if (rank == 0) {
        // the key must be node-unique (coll/mi355x: rank 0's pid + a counter + random bits,
        // broadcast at enable time); an existing segment of that name belongs to somebody else
        // and is never unlinked here
        fd = shm_open(c->shm_name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
        if (fd < 0) {
            const int e = errno;
            delete c;
            return set_error(MI355X_ERR_PEER, "control segment %s: %s%s", key, strerror(e),
                             e == EEXIST ? " (the rendezvous key is in use by another communicator)" : "");
        }
        if (ftruncate(fd, (off_t)bytes) != 0) {
            close(fd);
            shm_unlink(c->shm_name.c_str());
            delete c;
            return set_error(MI355X_ERR_PEER, "ftruncate of control segment %s failed", key);
        }
    } else {
        const auto t0 = std::chrono::steady_clock::now();
        for (;;) {
            fd = shm_open(c->shm_name.c_str(), O_RDWR, 0600);
            if (fd >= 0) {
                struct stat st;
                if (fstat(fd, &st) == 0 && (size_t)st.st_size >= bytes) break;
                close(fd);
                fd = -1;
            }
            if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > c->timeout_s) {
                delete c;
                return set_error(MI355X_ERR_TIMEOUT, "rank %d: control segment %s never appeared", rank, key);
            }
            usleep(1000);
        }
    }
    void *m = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (m == MAP_FAILED) {
        delete c;
        return set_error(MI355X_ERR_PEER, "mmap of the control segment failed");
    }
    c->ctrl = (Ctrl *)m;
    if (rank == 0) {
        std::memset(m, 0, bytes);
        c->ctrl->size = (uint32_t)size;
        uint64_t secret = 0;
        FILE *ur = fopen("/dev/urandom", "rb");
        if (!ur || fread(&secret, sizeof(secret), 1, ur) != 1)
            secret = (uint64_t)std::chrono::steady_clock::now().time_since_epoch().count() ^ ((uint64_t)getpid() << 32);
        if (ur) fclose(ur);
        c->ctrl->secret = secret;
        std::atomic_thread_fence(std::memory_order_release);
        __atomic_store_n(&c->ctrl->magic, kMagic, __ATOMIC_RELEASE);
    } else {
        const auto t0 = std::chrono::steady_clock::now();
        while (__atomic_load_n(&c->ctrl->magic, __ATOMIC_ACQUIRE) != kMagic) {
            if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > c->timeout_s) {
                munmap(m, bytes);
                delete c;
                return set_error(MI355X_ERR_TIMEOUT, "rank %d: control segment never initialised", rank);
            }
            usleep(200);
        }
    }
    c->ctrl->slot[rank].pid = (int32_t)getpid();
    c->ctrl->slot[rank].dev = device;
    uint64_t uid = 1469598103934665603ull;
    for (const char *p = bus; *p; ++p) uid = (uid ^ (unsigned char)tolower((unsigned char)*p)) * 1099511628211ull;
    c->ctrl->slot[rank].dev_uid = uid;
    c->ctrl->attached.fetch_add(1);
    int rc = size > 1 ? fd_sock_open(c) : MI355X_SUCCESS;
    if (rc) {
        c->ctrl->abort_flag.store(1);  // the others leave their creation barrier with an error
        if (rank == 0) shm_unlink(c->shm_name.c_str());
        const std::string msg = mi355x_last_error();
        mi355x_comm_destroy(c);
        return set_error(rc, "%s", msg.c_str());
    }
    rc = barrier(c);  // everybody mapped the segment and bound its socket: the name can go
    if (rank == 0) shm_unlink(c->shm_name.c_str());
    // ranks of this communicator on my GPU (a one-GPU rehearsal, or an oversubscribed node): they
    // split the CUs, and a persistent or spinning launch of one must stay co-resident with the others'
    int share = 0;
    for (int q = 0; q < size; ++q) share += c->ctrl->slot[q].dev_uid == uid;
    c->pipe_share = std::max(1, share);
    c->ll_max = (size_t)std::max(0.0, env_double("MI355X_LL_MAX_BYTES", 0.0));
    // pipelined allreduce by default from 4 ranks up: ahead of the two-phase flow at n = 4 and 8,
    // behind at n = 2 in the one-GPU rehearsal (profiles/r02_bench_n{2,4,8}_*); MI355X_PIPE=0/1 decides
    c->pipe_on = env_double("MI355X_PIPE", size >= 4 ? 1.0 : 0.0) != 0.0;
    c->one_phase_max = (size_t)std::max(0.0, env_double("MI355X_ONE_PHASE_MAX_BYTES", (double)c->one_phase_max));
    c->lat_on = env_double("MI355X_LAT_PROFILE", 0.0) != 0.0;
    c->rcache_max_maps = (size_t)std::max(0.0, env_double("MI355X_RCACHE_MAX_MAPS", 0.0));
    c->rcache_limit = (size_t)std::max(0.0, env_double("MI355X_RCACHE_SIZE_LIMIT", 0.0));
    c->gated = size > 1;
    if (rc == MI355X_SUCCESS && size > 1) rc = setup_done_words(c);
    if (rc == MI355X_SUCCESS && size > 1) rc = ll_selftest(c);
    if (rc == MI355X_SUCCESS && size > 1) {
        svc_setup(c);
        rc = pipe_selftest(c);
    }
    if (rc) {
        mi355x_comm_destroy(c);
        return rc;
    }
    c->create_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t_create).count();
    *out = c;
    return MI355X_SUCCESS;
}

int mi355x_comm_create_loopback(int size, int device, mi355x_comm_t **comms)
{
    if (!comms || size < 1 || size > kMaxRanks) return set_error(MI355X_ERR_ARG, "bad loopback arguments");
    auto shared = std::make_shared<LoopShared>();
    shared->ctrl = (Ctrl *)calloc(1, ctrl_bytes(size));
    if (!shared->ctrl) return set_error(MI355X_ERR_NOMEM, "calloc");
    shared->ctrl->magic = kMagic;
    shared->ctrl->size = (uint32_t)size;
    for (int r = 0; r < size; ++r) {
        auto *c = new mi355x_comm();
        c->rank = r;
        c->size = size;
        c->device = device;
        c->ctrl = shared->ctrl;
        c->loopback = true;
        c->loop = shared;
        c->timeout_s = env_double("MI355X_TIMEOUT_S", 600.0);
        shared->refs++;
        comms[r] = c;
    }
    return MI355X_SUCCESS;
}

int mi355x_comm_destroy(mi355x_comm_t *c)
{
    if (!c) return MI355X_SUCCESS;
    if (c->worker.joinable()) {
        {
            std::lock_guard<std::mutex> g(c->q_mtx);
            c->stop = true;
        }
        c->q_cv.notify_all();
        c->worker.join();
    }
    DeviceGuard dg(c->device);
    if (c->gated) gate_enter(c);  // (never while another process's revoker is taking the service from it)
    svc_release(c);
    p2p_destroy(c);
    for (hipEvent_t e : c->tev)
        if (e) (void)hipEventDestroy(e);
    if (c->nb_stream) (void)hipStreamDestroy(c->nb_stream);
    for (auto &kv : c->peer_maps) close_map(kv.second);
    for (LocalReg &r : c->local_regs) drop_reg(r);
    for (auto &kv : c->fd_stash) close(kv.second);
    if (c->fd_sock >= 0) close(c->fd_sock);
    if (c->pipe_base) (void)hipFree(c->pipe_base);
    if (c->pipe_queue) (void)hipFree(c->pipe_queue);
    if (c->pipe_dbg) (void)hipHostFree(c->pipe_dbg);
    if (c->scratch) (void)hipFree(c->scratch);
    if (c->stage) (void)hipFree(c->stage);
    if (!c->svc_stuck) {  // (a service kernel that never left may still read and write these)
        if (c->ll_base) (void)hipFree(c->ll_base);
        if (c->ll_ctr) (void)hipFree(c->ll_ctr);
        if (c->ll_err) (void)hipHostFree(c->ll_err);
    }
    if (c->lat_on && c->lat_n)
        fprintf(stderr, "[mi355x r%d] small allreduce steps over %llu calls (us): input sync %.2f, exchange %.2f, "
                "launch %.2f, finish %.2f\n", c->rank, (unsigned long long)c->lat_n, c->lat_acc[0] / c->lat_n,
                c->lat_acc[1] / c->lat_n, c->lat_acc[2] / c->lat_n, c->lat_acc[3] / c->lat_n);
    if (c->ctrl_registered) (void)hipHostUnregister(c->ctrl);
    if (c->loopback) {
        std::lock_guard<std::mutex> g(c->loop->mtx);
        if (--c->loop->refs == 0) free(c->loop->ctrl);
    } else if (c->ctrl) {
        munmap(c->ctrl, ctrl_bytes(c->size));
    }
    delete c;
    return MI355X_SUCCESS;
}

int mi355x_comm_set_rules(mi355x_comm_t *c, const mi355x_rules_t *rules)
{
    if (!c) return set_error(MI355X_ERR_ARG, "comm is NULL");
    DeviceGuard dg(c->device);
    drain(c);
    c->rules = rules;
    return MI355X_SUCCESS;
}

int mi355x_comm_rank(const mi355x_comm_t *c) { return c ? c->rank : -1; }
int mi355x_comm_size(const mi355x_comm_t *c) { return c ? c->size : -1; }
int mi355x_comm_barrier(mi355x_comm_t *c)
{
    if (!c) return set_error(MI355X_ERR_ARG, "comm is NULL");
    DeviceGuard dg(c->device);
    drain(c);
    return barrier(c);
}
static void (*g_progress_hook)(void) = nullptr;
int mi355x_set_progress_hook(void (*progress)(void))
{
    g_progress_hook = progress;
    return MI355X_SUCCESS;
}

// A host-buffer rank waits here for its peers' votes.  It must not stall other work meanwhile: the
// wait drives the caller's progress engine (opal_progress through the hook) and this
// communicator's point-to-point, so a peer that first needs an outstanding send of ours to
// complete still gets there (ob1's blocking waits progress the same way, req_wait.c).  The wait is
// unbounded, like a host collective's receive: a rank that is late by minutes (checkpoint I/O) is
// not an error, and nothing poisons the communicator.
int mi355x_comm_vote(mi355x_comm_t *c, int device, int *any_device)
{
    if (!c || !any_device) return set_error(MI355X_ERR_ARG, "NULL argument");
    *any_device = device ? 1 : 0;
    if (c->size == 1) return MI355X_SUCCESS;
    const uint64_t s = ++c->vote_seq;
    Ctrl *k = c->ctrl;
    k->slot[c->rank].vote[s % kVoteRing].store((s << 1) | (device ? 1u : 0u), std::memory_order_release);
    if (device) return MI355X_SUCCESS;
    for (int r = 0; r < c->size; ++r) {
        if (r == c->rank) continue;
        unsigned spins = 0;
        for (;;) {
            const uint64_t v = k->slot[r].vote[s % kVoteRing].load(std::memory_order_acquire);
            if ((v >> 1) == s) {
                if (v & 1u) *any_device = 1;
                break;
            }
            if ((v >> 1) > s)
                return set_error(MI355X_ERR_PEER, "rank %d is %d or more collectives ahead of rank %d", r,
                                 kVoteRing, c->rank);
            if (k->abort_flag.load(std::memory_order_relaxed))
                return set_error(MI355X_ERR_PEER, "a peer aborted the communicator");
            if (++spins > 2048) {
                if ((spins & 63) == 0) {
                    if (c->p2p) (void)p2p_progress(c);
                    if (g_progress_hook) g_progress_hook();
                }
                if ((spins & 0xffff) == 0 && peer_gone(c)) return MI355X_ERR_PEER;
                sched_yield();
            }
        }
    }
    return MI355X_SUCCESS;
}

int mi355x_comm_last_algorithm(const mi355x_comm_t *c) { return c ? c->last_alg : -1; }

// test hook without a GPU: the token table's holder protocol for a device uid, as a communicator
// named `name` would use it (op 1: try to take it; 0: give it back).  Returns 1 while held.  The
// CPU tests kill a holder process and check that the next process takes the token back.
int mi355x_debug_token(uint64_t dev_uid, const char *name, int op)
{
    static std::mutex mtx;
    static std::map<std::string, mi355x_comm *> comms;
    if (!name) return set_error(MI355X_ERR_ARG, "name is NULL");
    std::lock_guard<std::mutex> g(mtx);
    mi355x_comm *&c = comms[name];
    if (!c) {
        c = new mi355x_comm();
        c->ctrl = (Ctrl *)calloc(1, ctrl_bytes(1));
        c->ctrl->slot[0].dev_uid = dev_uid;
        c->shm_name = std::string("/mi355x_") + name;
    }
    if (op) return (c->pipe_entry >= 0 || pipe_token_acquire(c)) ? 1 : 0;
    if (c->pipe_entry >= 0) pipe_token_release(c);
    return 0;
}

// test hook: take (1) or give back (0) this communicator's pipelined-grid token of its GPU outside
// any call, as a rank inside a pipelined allreduce holds it (tests kill a holder, then check that
// the next communicator on the GPU is admitted again)
int mi355x_debug_pipe_token(mi355x_comm_t *c, int acquire)
{
    if (!c) return set_error(MI355X_ERR_ARG, "comm is NULL");
    if (acquire) return pipe_token_acquire(c) ? 1 : 0;
    if (c->pipe_entry >= 0) pipe_token_release(c);
    return 0;
}
int mi355x_comm_get(const mi355x_comm_t *c, int knob, long *value)
{
    if (!c || !value) return set_error(MI355X_ERR_ARG, "NULL argument");
    switch (knob) {
    case MI355X_KNOB_ALLREDUCE_ALG: *value = c->knob_allreduce; break;
    case MI355X_KNOB_REDUCE_ALG: *value = c->knob_reduce; break;
    case MI355X_KNOB_REDUCE_SCATTER_ALG: *value = c->knob_rs; break;
    case MI355X_KNOB_BLOCKS_PER_CU: *value = coll_tune().blocks_per_cu; break;
    case MI355X_KNOB_TIMEOUT_S: *value = (long)c->timeout_s; break;
    case MI355X_KNOB_PUSH: *value = coll_tune().push; break;
    case MI355X_KNOB_IPC_MAX_BYTES: *value = (long)c->ipc_max; break;
    case MI355X_KNOB_STAGE_BYTES: *value = (long)c->stage_bytes; break;
    case MI355X_KNOB_PIPE_REFUSED: *value = (long)c->pipe_refused; break;
    case MI355X_KNOB_LL_MAX_BYTES: *value = (long)c->ll_max; break;
    case MI355X_KNOB_REDUCE_CHAIN_FANOUT: *value = c->chain_fanout; break;
    case MI355X_KNOB_TIME_PHASES: *value = c->time_phases ? 1 : 0; break;
    case MI355X_KNOB_COPY_BLOCK_KIB: *value = coll_tune().copy_block_kib; break;
    case MI355X_KNOB_PIPE: *value = c->pipe_on ? 1 : 0; break;
    case MI355X_KNOB_PIPE_WG_PER_CU: *value = coll_tune().pipe_wg_per_cu; break;
    case MI355X_KNOB_PIPE_CHUNK_KIB: *value = coll_tune().pipe_chunk_kib; break;
    case MI355X_KNOB_PIPE_WT: *value = coll_tune().pipe_wt; break;
    case MI355X_KNOB_ONE_PHASE_MAX_BYTES: *value = (long)c->one_phase_max; break;
    case MI355X_KNOB_SVC_MAX_BYTES: *value = (c->svc_ok || c->svc_want) ? (long)c->svc_max : 0; break;
    case MI355X_KNOB_SVC_CALLS: *value = (long)c->svc_calls; break;
    case MI355X_KNOB_SVC_LAUNCHES: *value = (long)c->svc_launches; break;
    case MI355X_KNOB_SVC_RESIDENT: *value = c->svcq && svc_resident(c->svcq) ? 1 : 0; break;
    case MI355X_KNOB_SVC_PULL_MAX_BYTES: *value = (c->svc_ok || c->svc_want) ? (long)c->svc_pull_max : 0; break;
    case MI355X_KNOB_SVC_PULL_COPY_MAX_BYTES: *value = (c->svc_ok || c->svc_want) ? (long)c->svc_copy_max : 0; break;
    case MI355X_KNOB_FLOWS: *value = (long)c->flows; break;
    case MI355X_KNOB_FLOWS_FAILED: *value = (long)c->flows_failed; break;
    case MI355X_KNOB_CREATE_US: *value = (long)c->create_us; break;
    case MI355X_KNOB_SELFTEST_US: *value = (long)c->selftest_us; break;
    case MI355X_KNOB_SVC_OWNER: *value = c->svc_ok ? 1 : 0; break;
    case MI355X_KNOB_SVC_CLAIMS: *value = (long)c->svc_epoch; break;
    case MI355X_KNOB_SVC_IDLE_US: *value = (long)(c->svc_idle_s * 1e6 + 0.5); break;
    case MI355X_KNOB_SVC_SHRINK_US: *value = (long)(c->svc_shrink_s * 1e6 + 0.5); break;
    case MI355X_KNOB_SVC_REGROWS: *value = (long)c->svc_regrows; break;
    case MI355X_KNOB_RCACHE_MAX_MAPS: *value = (long)c->rcache_max_maps; break;
    case MI355X_KNOB_RCACHE_SIZE_LIMIT: *value = (long)c->rcache_limit; break;
    case MI355X_KNOB_PEER_MAPS: {
        std::lock_guard<std::recursive_mutex> g(const_cast<mi355x_comm *>(c)->reg_mtx);
        *value = (long)peer_map_count(c);
        break;
    }
    case MI355X_KNOB_RCACHE_EVICTIONS: *value = (long)c->rcache_evictions; break;
    default: return set_error(MI355X_ERR_ARG, "unknown knob %d", knob);
    }
    return MI355X_SUCCESS;
}

int mi355x_comm_phase_ms(const mi355x_comm_t *c, float *phase1_ms, float *phase2_ms)
{
    if (!c || !phase1_ms || !phase2_ms) return set_error(MI355X_ERR_ARG, "NULL argument");
    *phase1_ms = c->phase_ms[0];
    *phase2_ms = c->phase_ms[1];
    return MI355X_SUCCESS;
}

int mi355x_comm_set(mi355x_comm_t *c, int knob, long value)
{
    if (!c) return set_error(MI355X_ERR_ARG, "comm is NULL");
    switch (knob) {
    case MI355X_KNOB_ALLREDUCE_ALG: c->knob_allreduce = (int)value; break;
    case MI355X_KNOB_REDUCE_ALG: c->knob_reduce = (int)value; break;
    case MI355X_KNOB_REDUCE_SCATTER_ALG: c->knob_rs = (int)value; break;
    case MI355X_KNOB_BLOCKS_PER_CU:
        // up to 1024: with that many the streaming kernels' grids are one-shot (every thread one pass)
        if (value < 1 || value > 1024) return set_error(MI355X_ERR_ARG, "blocks_per_cu out of range");
        coll_tune().blocks_per_cu = (int)value;
        break;
    case MI355X_KNOB_TIMEOUT_S: c->timeout_s = (double)value; break;
    case MI355X_KNOB_PUSH: coll_tune().push = value ? 1 : 0; break;
    case MI355X_KNOB_IPC_MAX_BYTES:
        if (value < 0) return set_error(MI355X_ERR_ARG, "ipc_max_bytes < 0");
        c->ipc_max = (size_t)value;
        break;
    case MI355X_KNOB_REDUCE_CHAIN_FANOUT:
        if (value < 1 || value > 32) return set_error(MI355X_ERR_ARG, "chain fan-out out of range");
        c->chain_fanout = (int)value;
        break;
    case MI355X_KNOB_COPY_BLOCK_KIB:
        if (value < 4 || value > 256) return set_error(MI355X_ERR_ARG, "copy_block_kib out of range");
        coll_tune().copy_block_kib = (int)value;
        break;
    case MI355X_KNOB_PIPE: c->pipe_on = value != 0 && (c->flows & MI355X_FLOW_PIPE); break;  // (a failed self-test keeps it off)
    case MI355X_KNOB_PIPE_WG_PER_CU:
        if (value < 1 || value > 8) return set_error(MI355X_ERR_ARG, "pipe_wg_per_cu out of range");
        coll_tune().pipe_wg_per_cu = (int)value;
        break;
    case MI355X_KNOB_PIPE_CHUNK_KIB:
        if (value < 0 || value > (1l << 20)) return set_error(MI355X_ERR_ARG, "pipe_chunk_kib out of range");
        coll_tune().pipe_chunk_kib = (int)value;
        break;
    case MI355X_KNOB_PIPE_WT: coll_tune().pipe_wt = value != 0; break;
    case MI355X_KNOB_ONE_PHASE_MAX_BYTES:
        if (value < 0 || value > (1l << 30)) return set_error(MI355X_ERR_ARG, "one_phase_max_bytes out of range");
        c->one_phase_max = (size_t)value;
        break;
    case MI355X_KNOB_TIME_PHASES:
        c->time_phases = value != 0;
        if (c->time_phases && !c->tev[0]) {
            DeviceGuard dg(c->device);
            for (hipEvent_t &e : c->tev) MI_HIP(hipEventCreate(&e));
        }
        break;
    case MI355X_KNOB_LL_MAX_BYTES:
        if (value < 0 || value > (64l << 20)) return set_error(MI355X_ERR_ARG, "ll_max_bytes out of range");
        c->ll_max = c->ll_ok ? (size_t)value : 0;  // a failed (or skipped) self-test keeps it off
        break;
    case MI355X_KNOB_SVC_PULL_MAX_BYTES:
        if (value < 0 || value > (1l << 30)) return set_error(MI355X_ERR_ARG, "svc_pull_max_bytes out of range");
        if (c->svc_ok || c->svc_want) {
            drain(c);
            c->svc_pull_max = (size_t)value;
        }
        break;
    case MI355X_KNOB_SVC_PULL_COPY_MAX_BYTES:
        if (value < 0 || value > (1l << 30)) return set_error(MI355X_ERR_ARG, "svc_pull_copy_max_bytes out of range");
        if (c->svc_ok || c->svc_want) {
            drain(c);
            c->svc_copy_max = (size_t)value;
        }
        break;
    case MI355X_KNOB_SVC_MAX_BYTES:
        if (value < 0 || value > (64l << 20)) return set_error(MI355X_ERR_ARG, "svc_max_bytes out of range");
        if (c->svc_ok || c->svc_want) {  // a communicator that cannot have the service keeps 0
            drain(c);
            c->svc_max = (size_t)value;
        }
        break;
    case MI355X_KNOB_RCACHE_MAX_MAPS:
    case MI355X_KNOB_RCACHE_SIZE_LIMIT: {
        if (value < 0) return set_error(MI355X_ERR_ARG, "rcache bound < 0");
        drain(c);
        std::lock_guard<std::recursive_mutex> g(c->reg_mtx);
        (knob == MI355X_KNOB_RCACHE_MAX_MAPS ? c->rcache_max_maps : c->rcache_limit) = (size_t)value;
        rcache_trim(c, nullptr);
        break;
    }
    case MI355X_KNOB_SVC_SHRINK_US:
    case MI355X_KNOB_SVC_IDLE_US:
        if (knob == MI355X_KNOB_SVC_SHRINK_US ? (value < 0 || value > 60000000) : (value < 100 || value > 60000000))
            return set_error(MI355X_ERR_ARG, "%s out of range", knob == MI355X_KNOB_SVC_SHRINK_US ? "svc_shrink_us" : "svc_idle_us");
        drain(c);
        (knob == MI355X_KNOB_SVC_SHRINK_US ? c->svc_shrink_s : c->svc_idle_s) = (double)value * 1e-6;
        {  // a resident service picks the new limit up at its next launch (g_svc_mtx: not while a
           // revoker detaches this communicator)
            std::lock_guard<std::mutex> g(g_svc_mtx);
            if (c->svc_ok && c->svcq) svc_park(c);
        }
        break;
    case MI355X_KNOB_STAGE_BYTES:
        if (value < 4096 || value >= (1l << 31)) return set_error(MI355X_ERR_ARG, "stage_bytes out of range");
        if (c->stage) (void)hipFree(c->stage);
        c->stage = nullptr;
        c->stage_bytes = (size_t)value & ~(size_t)4095;
        break;
    default: return set_error(MI355X_ERR_ARG, "unknown knob %d", knob);
    }
    return MI355X_SUCCESS;
}

// Describe the per-element program the engine runs (host only, no GPU needed).  Layout:
//   fold: [1, nr, len, order[0..len-1], role[0..len-1]]
//   tree: [0, nr, nsteps, result, (dst, out, in) x nsteps]
// kind 1: allreduce (alg 3 = recursive doubling, 4/5 = ring block `block`,
//                    1/2 = reduce-to-0 with reduce algorithm `block` (1..5) + bcast)
// kind 2: reduce to rank `block` with reduce algorithm `alg`;  kind 3: reduce_scatter ring block;
// kind 4: reduce_scatter recursive halving block; kind 5: reduce chain to 0 with fan-out `block`.
// Returns the number of ints written or < 0.
int mi355x_sched_program(int kind, int n, int alg, int block, int *out, int cap)
{
    if (!out || n < 1 || n > kMaxRanks) return set_error(MI355X_ERR_ARG, "bad arguments");
    Program pr;
    ExprPool ep;
    bool ok = true;
    switch (kind) {
    case 1:
        if (alg == AR_RING || alg == AR_RING_SEGMENTED) pr = ring_block_program(n, block);
        else if (alg == AR_RECDBL) ok = compile_expr(ep, expr_allreduce_recursive_doubling(ep, n), n, &pr);
        else ok = compile_expr(ep, expr_reduce(ep, block, n, 0), n, &pr);
        break;
    case 2: ok = compile_expr(ep, expr_reduce(ep, alg, n, block), n, &pr); break;  // block = root
    case 5: ok = compile_expr(ep, expr_reduce(ep, RED_CHAIN, n, 0, block), n, &pr); break;  // block = fan-out
    case 3: pr = reduce_scatter_ring_block_program(n, block); break;
    case 4: {
        std::vector<int> roots = expr_reduce_scatter_rechalving(ep, n);
        ok = compile_expr(ep, roots[block], n, &pr);
        break;
    }
    default: return set_error(MI355X_ERR_ARG, "unknown kind %d", kind);
    }
    if (!ok) return set_error(MI355X_ERR_UNSUPPORTED, "schedule does not compile");
    std::vector<int> v;
    if (pr.is_fold) {
        v = {1, pr.nr, (int)pr.order.size()};
        for (int r : pr.order) v.push_back(r);
        for (size_t j = 0; j < pr.order.size(); ++j) v.push_back((int)((pr.role_mask >> j) & 1u));
    } else {
        v = {0, pr.nr, (int)pr.steps.size(), pr.result};
        for (const TreeStep &t : pr.steps) {
            v.push_back(t.dst);
            v.push_back(t.out);
            v.push_back(t.in);
        }
    }
    if ((int)v.size() > cap) return set_error(MI355X_ERR_ARG, "cap too small");
    for (size_t i = 0; i < v.size(); ++i) out[i] = v[i];
    return (int)v.size();
}

// MPI_Allreduce (coll_tuned_allreduce_intra_dec_fixed order; sbuf NULL = MPI_IN_PLACE)
static int allreduce_impl(mi355x_comm_t *c, const void *sbuf, void *rbuf, size_t count, int type, int op,
                     void *stream)
{
    int rc = check_common(c, op, type);
    if (rc) return rc;
    if (count == 0) return MI355X_SUCCESS;
    hipStream_t s = resolve_stream(stream);
    const size_t esz = mi355x_type_size(type);
    const void *in = sbuf ? sbuf : rbuf;
    if (c->size == 1) {
        c->last_alg = AR_RING;
        if (sbuf && sbuf != rbuf) MI_HIP(hipMemcpyAsync(rbuf, sbuf, count * esz, hipMemcpyDeviceToDevice, s));
        MI_HIP(hipStreamSynchronize(s));
        return MI355X_SUCCESS;
    }
    rc = svc_maybe_claim(c, count * esz <= std::max(c->svc_max, c->svc_pull_max));
    if (rc) return rc;
    int alg = pick_allreduce(c, count, esz);
    // the reference's own fallbacks: segmented ring -> ring when count < n * segcount
    // (coll_tuned_allreduce.c:672-679), ring -> recursive doubling when count < n (:398-405)
    if (alg == AR_RING_SEGMENTED && count < (size_t)c->size * computed_segcount(1u << 20, esz, count))
        alg = AR_RING;
    if (alg == AR_RING && count < (size_t)c->size) alg = AR_RECDBL;
    c->last_alg = alg;
    const bool ring = (alg == AR_RING || alg == AR_RING_SEGMENTED);
    if (ll_usable(c, count * esz) && (ring || c->size <= kTreeMax)) {
        // one-shot: every rank evaluates the whole vector with the reference's per-element order
        LLArgs a;
        std::memset(&a, 0, sizeof(a));
        a.mode = LL_AR;
        a.src = in;
        a.dst = rbuf;
        a.nbytes = count * esz;
        a.count = count;
        a.push_mask = ~0ull;
        if (ring) {
            size_t o1, l0, l1;
            ring_block(count, c->size, 0, &o1, &l0);
            ring_block(count, c->size, c->size - 1, &o1, &l1);
            a.prog = LL_RING;
            a.early = l0;
            a.late = l1;
            a.split = count % (size_t)c->size;
            if (a.late == 0) a.late = 1;  // count < n never reaches the ring (recursive doubling)
        } else {
            Program pr;
            if (!allreduce_tree_program(c, alg, count, esz, &pr))
                return set_error(MI355X_ERR_UNSUPPORTED, "schedule too large");
            ll_program(a, pr);
        }
        return ll_run(c, a, op, type, s);
    }
    bool pipe = ring && !c->loopback && c->pipe_on && (c->flows & MI355X_FLOW_PIPE) && !coll_tune().push;
    if (pipe) {  // collective setup first: it reuses the exchange slots
        rc = ensure_pipe(c);
        if (rc) return rc;
    }
    // admission (above): try my GPU's token, publish the outcome with the exchange
    const bool held = pipe && pipe_token_acquire(c);
    if (pipe) c->ctrl->slot[c->rank].pipe_adm.store(((c->seq + 1) << 1) | (held ? 1u : 0u), std::memory_order_release);
    using lclk = std::chrono::steady_clock;
    lclk::time_point lt[4];
    if (c->lat_on) lt[0] = lclk::now();
    MI_HIP(hipStreamSynchronize(s));  // every rank's input is complete before it is published
    if (c->lat_on) lt[1] = lclk::now();
    const void *mine[2] = {in, rbuf};
    const uint64_t sig[4] = {1, count, (uint64_t)type, (uint64_t)op};
    std::vector<std::vector<void *>> P;
    bool staged = false;
    // the one-phase ring sizes may go to the resident service (svc_pull_run): its exchange then
    // leaves the service resident (the same decision on every rank: sizes only)
    const bool one_phase = ring && sbuf && sbuf != rbuf && !coll_tune().push && count * esz <= c->one_phase_max &&
                           count <= 0xffffffffull;
    const bool pull_cand = one_phase && svc_pull_usable(c, count * esz, esz);
    c->svc_keep = pull_cand;
    rc = exchange(c, 2, mine, sig, P, &staged);
    c->svc_keep = false;
    if (c->lat_on) lt[2] = lclk::now();
    auto lat_done = [&](int rc2) {  // the one-launch paths: launch done at lt[3], then finish
        if (!c->lat_on || rc2) return rc2;
        lt[3] = lclk::now();
        rc2 = finish(c, s);
        const lclk::time_point e = lclk::now();
        for (int i = 0; i < 3; ++i) c->lat_acc[i] += std::chrono::duration<double, std::micro>(lt[i + 1] - lt[i]).count();
        c->lat_acc[3] += std::chrono::duration<double, std::micro>(e - lt[3]).count();
        c->lat_n++;
        return rc2;
    };
    if (rc) {
        if (held) pipe_token_release(c);
        return rc;
    }
    if (pipe) {
        bool all = true;
        for (int q = 0; q < c->size; ++q)
            all = all && c->ctrl->slot[q].pipe_adm.load(std::memory_order_acquire) == ((c->seq << 1) | 1u);
        if (!all) {
            pipe = false;
            c->pipe_refused++;
            TRACE(c, "pipelined grid not admitted on every GPU: two-phase flow");
        }
        if (held && !all) pipe_token_release(c);
    }
    struct TokenGuard {  // an admitted grid gives its token back once the call is over
        mi355x_comm *c;
        bool on;
        ~TokenGuard()
        {
            if (on) pipe_token_release(c);
        }
    } token_guard{c, pipe && held};
    Program pr;
    if (!ring) {
        if (!allreduce_tree_program(c, alg, count, esz, &pr))
            return set_error(MI355X_ERR_UNSUPPORTED, "schedule too large");
        if (sbuf && sbuf != rbuf && !staged) {
            // tree orders (small messages): every rank evaluates the whole vector from the n
            // inputs and writes only its own rbuf -- one phase, reads only
            std::vector<void *> dst(1, rbuf);
            rc = run_program(op, type, pr, P[0], dst, 0, count, s);
            if (rc) return rc;
            if (c->lat_on) return lat_done(rc);
            return finish(c, s);
        }
    }
    bool pull = pull_cand && !staged;
    for (int q = 0; q < c->size && pull; ++q)
        pull = !((((uintptr_t)P[0][q]) | ((uintptr_t)P[1][q])) & 15);  // every rank's buffers 16-B aligned
    if (pull) {
        size_t o1, l0, l1;
        ring_block(count, c->size, 0, &o1, &l0);
        ring_block(count, c->size, c->size - 1, &o1, &l1);
        return svc_pull_run(c, op, type, P, in, rbuf, count, esz, l0, l1 ? l1 : 1, count % (size_t)c->size);
    }
    if (pull_cand) svc_park(c);  // (kept for this call, which now takes a host-synchronised flow)
    if (one_phase && !staged) {
        // small ring-ordered messages: every rank evaluates every block from the n inputs (reads
        // n x S, writes only its own rbuf) -- one launch and one barrier, like the tree orders
        RingAllArgs ra;
        std::memset(&ra, 0, sizeof(ra));
        for (int q = 0; q < c->size; ++q) ra.src[q] = P[0][q];
        ra.dst = rbuf;
        ra.n = c->size;
        size_t o1, l0, l1;
        ring_block(count, c->size, 0, &o1, &l0);
        ring_block(count, c->size, c->size - 1, &o1, &l1);
        ra.count = (uint32_t)count;
        ra.early = (uint32_t)l0;
        ra.late = (uint32_t)(l1 ? l1 : 1);
        ra.split = (uint32_t)(count % (size_t)c->size);
        rc = launch_ring_all_slot(op, type, ra, s);
        if (rc) return rc;
        if (c->lat_on) return lat_done(rc);
        return finish(c, s);
    }
    // owner-computes: rank r evaluates ring block r (the reference's block partition, so the
    // ring's per-block order is one program per launch)
    size_t off, len;
    ring_block(count, c->size, c->rank, &off, &len);
    if (ring) pr = ring_block_program(c->size, c->rank);
    if (staged) {
        std::vector<size_t> boff(c->size), blen(c->size);
        for (int q = 0; q < c->size; ++q) ring_block(count, c->size, q, &boff[q], &blen[q]);
        return staged_reduce(c, op, type, pr, in, boff, blen, (char *)rbuf + off * esz, true, rbuf, s);
    }
    if (coll_tune().push) {
        // one phase: the owner writes its block into every rank's rbuf
        rc = run_program(op, type, pr, P[0], P[1], off, len, s);
        if (rc) return rc;
        return finish(c, s);
    }
    // multi-process: the fold of my block and the pulls of the others in one pipelined launch
    // (coll_pipe.hip); loopback ranks share one process's queues, so they keep two phases
    if (pipe) return pipe_allreduce(c, op, type, pr, P, count, s);
    // phase 1: reduce own block locally; phase 2: pull every other block from its owner
    const bool tp = c->time_phases && c->tev[0];
    if (tp) MI_HIP(hipEventRecord(c->tev[0], s));
    std::vector<void *> dst(1, rbuf);
    rc = run_program(op, type, pr, P[0], dst, off, len, s);
    if (rc) return rc;
    if (tp) MI_HIP(hipEventRecord(c->tev[1], s));
    rc = finish(c, s);
    if (rc) return rc;
    if (tp) MI_HIP(hipEventRecord(c->tev[2], s));
    MultiCopyArgs m;
    std::memset(&m, 0, sizeof(m));
    for (int q = 0; q < c->size; ++q) {
        if (q == c->rank) continue;
        size_t qo, ql;
        ring_block(count, c->size, q, &qo, &ql);
        m.src[m.nseg] = (const char *)P[1][q] + qo * esz;
        m.dst[m.nseg] = (char *)rbuf + qo * esz;
        m.len[m.nseg] = ql * esz;
        m.nseg++;
    }
    rc = launch_multicopy(m, s);
    if (rc) return rc;
    if (tp) MI_HIP(hipEventRecord(c->tev[3], s));
    rc = finish(c, s);
    if (rc == MI355X_SUCCESS && tp) {
        MI_HIP(hipEventElapsedTime(&c->phase_ms[0], c->tev[0], c->tev[1]));
        MI_HIP(hipEventElapsedTime(&c->phase_ms[1], c->tev[2], c->tev[3]));
    }
    return rc;
}

// MPI_Reduce to `root` (ompi_coll_tuned_reduce_intra_dec_fixed, coll_tuned_decision_fixed.c:343-446,
// and the forced algorithms of coll_tuned_reduce.c).  sbuf NULL = MPI_IN_PLACE (root only, input in
// rbuf); rbuf is read on the root only.  The result of every element is the reference tree's
// expression (linear / chain / pipeline / binary / binomial), evaluated:
//   small  : LL one-shot, every rank pushes to the root, the root evaluates (when enabled);
//   <= one_phase_max: the root evaluates everything from the mapped inputs, one launch;
//   large  : owner-computes -- rank r evaluates ring block r from the n inputs into its own
//            memory, then the root pulls the blocks (each link carries 2 S/n, writes stay local);
//   staged : (allocations >= ipc_max) the root evaluates everything through the staging buffers.
static int reduce_impl(mi355x_comm_t *c, const void *sbuf, void *rbuf, size_t count, int type, int op, int root,
                  void *stream)
{
    int rc = check_common(c, op, type);
    if (rc) return rc;
    if (root < 0 || root >= c->size) return set_error(MI355X_ERR_ARG, "bad root");
    if (!sbuf && c->rank != root) return set_error(MI355X_ERR_ARG, "MPI_IN_PLACE is only valid at the root");
    if (count == 0) return MI355X_SUCCESS;
    hipStream_t s = resolve_stream(stream);
    const size_t esz = mi355x_type_size(type);
    const void *in = sbuf ? sbuf : rbuf;
    const bool am_root = (c->rank == root);
    if (c->size == 1) {
        c->last_alg = RED_LINEAR;
        if (sbuf && sbuf != rbuf) MI_HIP(hipMemcpyAsync(rbuf, sbuf, count * esz, hipMemcpyDeviceToDevice, s));
        MI_HIP(hipStreamSynchronize(s));
        return MI355X_SUCCESS;
    }
    Program pr;
    int ra;
    if (!reduce_program(c, count, esz, root, &pr, &ra)) return set_error(MI355X_ERR_UNSUPPORTED, "schedule too large");
    c->last_alg = ra;
    rc = svc_maybe_claim(c, count * esz <= c->svc_max);
    if (rc) return rc;
    if (ll_usable(c, count * esz) && (pr.is_fold || c->size <= kTreeMax)) {
        LLArgs a;
        std::memset(&a, 0, sizeof(a));
        a.mode = LL_RED;
        a.root = root;
        a.src = in;
        a.dst = am_root ? rbuf : nullptr;
        a.nbytes = count * esz;
        a.count = count;
        a.push_mask = 1ull << root;
        ll_program(a, pr);
        return ll_run(c, a, op, type, s);
    }
    size_t off, len;
    ring_block(count, c->size, c->rank, &off, &len);
    if (!am_root) {
        rc = ensure_scratch(c, len * esz);
        if (rc) return rc;
    }
    MI_HIP(hipStreamSynchronize(s));
    const void *mine[2] = {in, am_root ? nullptr : c->scratch};
    const uint64_t sig[4] = {6, count, ((uint64_t)type << 32) | (uint64_t)op, (uint64_t)root};
    std::vector<std::vector<void *>> P;
    bool staged = false;
    rc = exchange(c, 2, mine, sig, P, &staged);
    if (rc) return rc;
    if (staged) {
        std::vector<size_t> boff(c->size, 0), blen(c->size, 0);
        blen[root] = count;
        return staged_reduce(c, op, type, pr, in, boff, blen, am_root ? rbuf : nullptr, false, nullptr, s);
    }
    if (count * esz <= c->one_phase_max) {
        // small messages: the root evaluates every element from the n inputs (one launch, reads
        // only; in place at the root each lane reads its element of rbuf before writing it); the
        // others wait in the closing barrier until the root is done with their inputs
        if (am_root) {
            std::vector<void *> d0(1, rbuf);
            rc = run_program(op, type, pr, P[0], d0, 0, count, s);
            if (rc) return rc;
        }
        return finish(c, s);
    }
    // phase 1: every rank evaluates its ring block from the n inputs into its own memory (the root
    // straight into rbuf); phase 2: the root pulls the other blocks (one segment per peer).  Only
    // local writes: a remote write would land in HBM behind the root's L2, which may hold the
    // old lines of rbuf (coarse-grained memory is not probed).
    void *mydst = am_root ? (void *)((char *)rbuf + off * esz) : c->scratch;
    std::vector<void *> d0(1, (char *)mydst - off * esz);  // run_program offsets by off
    rc = run_program(op, type, pr, P[0], d0, off, len, s);
    if (rc) return rc;
    rc = finish(c, s);
    if (rc) return rc;
    if (am_root) {
        MultiCopyArgs m;
        std::memset(&m, 0, sizeof(m));
        for (int q = 0; q < c->size; ++q) {
            size_t qo, ql;
            ring_block(count, c->size, q, &qo, &ql);
            if (q == root || ql == 0) continue;
            m.src[m.nseg] = P[1][q];
            m.dst[m.nseg] = (char *)rbuf + qo * esz;
            m.len[m.nseg] = ql * esz;
            m.nseg++;
        }
        rc = launch_multicopy(m, s);
        if (rc) return rc;
    }
    return finish(c, s);  // the peers keep their scratch until the root has pulled it
}

// MPI_Reduce_scatter_block as coll/basic runs it: tuned reduce to 0 + scatter
// (coll_basic_reduce_scatter_block.c:54-111); sbuf NULL = MPI_IN_PLACE (input in rbuf).
static int reduce_scatter_block_impl(mi355x_comm_t *c, const void *sbuf, void *rbuf, size_t rcount, int type,
                                int op, void *stream)
{
    int rc = check_common(c, op, type);
    if (rc) return rc;
    const size_t count = rcount * (size_t)c->size;
    if (count == 0) return MI355X_SUCCESS;
    hipStream_t s = resolve_stream(stream);
    const size_t esz = mi355x_type_size(type);
    const void *in = sbuf ? sbuf : rbuf;
    Program pr;
    int ra;
    if (!reduce_program(c, count, esz, 0, &pr, &ra)) return set_error(MI355X_ERR_UNSUPPORTED, "schedule too large");
    c->last_alg = ra;
    const bool inplace = (in == (const void *)rbuf);
    rc = svc_maybe_claim(c, !inplace && c->svc_rs && rcount * esz <= c->svc_pull_max);
    if (rc) return rc;
    if (inplace) {
        rc = ensure_scratch(c, rcount * esz);
        if (rc) return rc;
    }
    MI_HIP(hipStreamSynchronize(s));
    const void *mine[1] = {in};
    const uint64_t sig[4] = {2, rcount, (uint64_t)type, (uint64_t)op};
    std::vector<std::vector<void *>> P;
    bool staged = false;
    const bool pull_cand = !inplace && svc_rs_usable(c, rcount * esz, pr);  // the resident service evaluates
    c->svc_keep = pull_cand;
    rc = exchange(c, 1, mine, sig, P, &staged);
    c->svc_keep = false;
    if (rc) return rc;
    if (pull_cand && !staged) return svc_rs_run(c, op, type, pr, P, in, (size_t)c->rank * rcount * esz, rbuf, rcount * esz, esz);
    if (pull_cand) svc_park(c);
    if (staged) {
        std::vector<size_t> boff(c->size), blen(c->size, rcount);
        for (int q = 0; q < c->size; ++q) boff[q] = (size_t)q * rcount;
        rc = staged_reduce(c, op, type, pr, in, boff, blen, inplace ? c->scratch : rbuf, false, nullptr, s);
        if (rc) return rc;
        if (inplace) {
            MI_HIP(hipMemcpyAsync(rbuf, c->scratch, rcount * esz, hipMemcpyDeviceToDevice, s));
            MI_HIP(hipStreamSynchronize(s));
        }
        return MI355X_SUCCESS;
    }
    std::vector<void *> dst(1, inplace ? c->scratch : rbuf);
    // the result block r is written at offset 0 of the destination: shift the destination back
    std::vector<void *> d0(1, (char *)dst[0] - (size_t)c->rank * rcount * esz);
    rc = run_program(op, type, pr, P[0], d0, (size_t)c->rank * rcount, rcount, s);
    if (rc) return rc;
    rc = finish(c, s);
    if (rc) return rc;
    if (inplace) {
        MI_HIP(hipMemcpyAsync(rbuf, c->scratch, rcount * esz, hipMemcpyDeviceToDevice, s));
        MI_HIP(hipStreamSynchronize(s));
    }
    return MI355X_SUCCESS;
}

// MPI_Reduce_scatter with vector counts (coll_tuned_reduce_scatter_intra_dec_fixed order)
static int reduce_scatter_impl(mi355x_comm_t *c, const void *sbuf, void *rbuf, const int *rcounts, int type,
                          int op, void *stream)
{
    int rc = check_common(c, op, type);
    if (rc) return rc;
    if (!rcounts) return set_error(MI355X_ERR_ARG, "rcounts is NULL");
    std::vector<size_t> disp(c->size + 1, 0);
    for (int r = 0; r < c->size; ++r) {
        if (rcounts[r] < 0) return set_error(MI355X_ERR_ARG, "negative rcount");
        disp[r + 1] = disp[r] + (size_t)rcounts[r];
    }
    const size_t count = disp[c->size];
    if (count == 0) return MI355X_SUCCESS;
    hipStream_t s = resolve_stream(stream);
    const size_t esz = mi355x_type_size(type);
    const void *in = sbuf ? sbuf : rbuf;
    const int alg = pick_reduce_scatter(c, count, esz);
    c->last_alg = alg;
    const size_t mine_n = (size_t)rcounts[c->rank];
    const bool inplace = (in == (const void *)rbuf);
    {
        size_t mb = 0;
        for (int r = 0; r < c->size; ++r) mb = std::max(mb, (size_t)rcounts[r]);
        rc = svc_maybe_claim(c, !inplace && c->svc_rs && mb * esz <= c->svc_pull_max);
        if (rc) return rc;
    }
    if (inplace) {
        rc = ensure_scratch(c, mine_n * esz);
        if (rc) return rc;
    }
    MI_HIP(hipStreamSynchronize(s));
    const void *mine[1] = {in};
    uint64_t h = 1469598103934665603ull;
    for (int r = 0; r < c->size; ++r) h = (h ^ (uint64_t)rcounts[r]) * 1099511628211ull;
    const uint64_t sig[4] = {3, h, (uint64_t)type, (uint64_t)op};
    std::vector<std::vector<void *>> P;
    bool staged = false;
    Program pr;
    if (c->size == 1) {
        pr.is_fold = true;
        pr.order = {0};
        pr.nr = 1;
    } else if (alg == RS_RING) {
        pr = reduce_scatter_ring_block_program(c->size, c->rank);
    } else if (alg == RS_NONOVERLAPPING) {
        // reduce of the whole vector to rank 0 (comm->c_coll.coll_reduce) + scatterv
        // (coll_tuned_reduce_scatter.c:60-121): every block carries the reduce tree's order
        int ra;
        if (!reduce_program(c, count, esz, 0, &pr, &ra)) return set_error(MI355X_ERR_UNSUPPORTED, "schedule too large");
    } else {
        ExprPool ep;
        std::vector<int> roots = expr_reduce_scatter_rechalving(ep, c->size);
        if (!compile_expr(ep, roots[c->rank], c->size, &pr))
            return set_error(MI355X_ERR_UNSUPPORTED, "schedule too large");
    }
    size_t max_block = 0;
    for (int r = 0; r < c->size; ++r) max_block = std::max(max_block, (size_t)rcounts[r]);
    const bool pull_cand = !inplace && svc_rs_usable(c, max_block * esz, pr);  // the resident service evaluates
    c->svc_keep = pull_cand;
    rc = exchange(c, 1, mine, sig, P, &staged);
    c->svc_keep = false;
    if (rc) return rc;
    if (pull_cand && !staged) return svc_rs_run(c, op, type, pr, P, in, disp[c->rank] * esz, rbuf, mine_n * esz, esz);
    if (pull_cand) svc_park(c);
    void *dst0 = inplace ? c->scratch : rbuf;
    if (staged) {
        std::vector<size_t> boff(disp.begin(), disp.end() - 1), blen(c->size);
        for (int q = 0; q < c->size; ++q) blen[q] = (size_t)rcounts[q];
        rc = staged_reduce(c, op, type, pr, in, boff, blen, dst0, false, nullptr, s);
        if (rc) return rc;
        if (inplace && mine_n) {
            MI_HIP(hipMemcpyAsync(rbuf, c->scratch, mine_n * esz, hipMemcpyDeviceToDevice, s));
            MI_HIP(hipStreamSynchronize(s));
        }
        return MI355X_SUCCESS;
    }
    std::vector<void *> d0(1, (char *)dst0 - disp[c->rank] * esz);
    rc = run_program(op, type, pr, P[0], d0, disp[c->rank], mine_n, s);
    if (rc) return rc;
    rc = finish(c, s);
    if (rc) return rc;
    if (inplace && mine_n) {
        MI_HIP(hipMemcpyAsync(rbuf, c->scratch, mine_n * esz, hipMemcpyDeviceToDevice, s));
        MI_HIP(hipStreamSynchronize(s));
    }
    return MI355X_SUCCESS;
}

// MPI_Allgather of `bytes` per rank (contiguous); sbuf NULL = MPI_IN_PLACE.  Pull: one launch
// copies every peer's block concurrently (one segment per peer -> every link busy).
static int allgather_impl(mi355x_comm_t *c, const void *sbuf, void *rbuf, size_t bytes, void *stream)
{
    if (!c) return set_error(MI355X_ERR_ARG, "comm is NULL");
    if (bytes == 0) return MI355X_SUCCESS;
    hipStream_t s = resolve_stream(stream);
    const void *src = sbuf ? sbuf : (const char *)rbuf + (size_t)c->rank * bytes;
    int rc0 = svc_maybe_claim(c, bytes <= std::max(c->svc_max, c->svc_copy_max));
    if (rc0) return rc0;
    if (ll_usable(c, bytes)) {
        c->last_alg = 3;
        LLArgs a;
        std::memset(&a, 0, sizeof(a));
        a.mode = LL_AG;
        a.src = src;
        a.dst = rbuf;
        a.nbytes = bytes;
        a.push_mask = ~0ull;
        return ll_run(c, a, 0, 0, s);
    }
    MI_HIP(hipStreamSynchronize(s));
    // pull reads only the peers' send blocks; push also writes into their rbufs
    const bool push = coll_tune().push != 0;
    const void *mine[2] = {src, rbuf};
    const uint64_t sig[4] = {4, bytes, (uint64_t)push, 0};
    std::vector<std::vector<void *>> P;
    bool staged = false;
    const bool pull_cand = !push && svc_pull_copy_usable(c, bytes);  // the resident service copies
    c->svc_keep = pull_cand;
    int rc = exchange(c, push ? 2 : 1, mine, sig, P, &staged);
    c->svc_keep = false;
    if (rc) return rc;
    c->last_alg = 1;
    if (pull_cand && !staged) return svc_pull_copy_run(c, LL_PULL_AG, P, src, rbuf, bytes, 0);
    if (pull_cand) svc_park(c);
    if (staged) return staged_allgather(c, src, rbuf, bytes, s);
    if (push) {
        CopyArgs a;
        std::memset(&a, 0, sizeof(a));
        a.src = src;
        a.nd = c->size;
        for (int q = 0; q < c->size; ++q) a.dst[q] = (char *)P[1][q] + (size_t)c->rank * bytes;
        a.n = bytes;
        rc = launch_copy(a, s);
        if (rc) return rc;
        return finish(c, s);
    }
    MultiCopyArgs m;
    std::memset(&m, 0, sizeof(m));
    for (int q = 0; q < c->size; ++q) {
        char *d = (char *)rbuf + (size_t)q * bytes;
        if (P[0][q] == d) continue;  // in place: own block already there
        m.src[m.nseg] = P[0][q];
        m.dst[m.nseg] = d;
        m.len[m.nseg] = bytes;
        m.nseg++;
    }
    rc = launch_multicopy(m, s);
    if (rc) return rc;
    return finish(c, s);
}

// MPI_Bcast of `bytes` from root.  Small messages: every rank pulls the whole buffer from the
// root.  Large: scatter + allgather shape (each rank first pulls its slice from the root, then the
// other slices from their owners), so each xGMI link carries ~2/n of the message instead of the
// root's links carrying all of it.
static int bcast_impl(mi355x_comm_t *c, void *buf, size_t bytes, int root, void *stream)
{
    if (!c) return set_error(MI355X_ERR_ARG, "comm is NULL");
    if (root < 0 || root >= c->size) return set_error(MI355X_ERR_ARG, "bad root");
    if (bytes == 0 || c->size == 1) return MI355X_SUCCESS;
    hipStream_t s = resolve_stream(stream);
    int rc0 = svc_maybe_claim(c, bytes <= std::max(c->svc_max, c->svc_copy_max));
    if (rc0) return rc0;
    if (ll_usable(c, bytes)) {
        c->last_alg = 3;
        LLArgs a;
        std::memset(&a, 0, sizeof(a));
        a.mode = LL_BC;
        a.root = root;
        a.src = (c->rank == root) ? buf : nullptr;
        a.dst = buf;
        a.nbytes = bytes;
        a.push_mask = ~0ull & ~(1ull << root);
        return ll_run(c, a, 0, 0, s);
    }
    MI_HIP(hipStreamSynchronize(s));
    const void *mine[1] = {buf};
    const uint64_t sig[4] = {5, bytes, (uint64_t)root, 0};
    std::vector<std::vector<void *>> P;
    bool staged = false;
    const bool split = bytes >= ((size_t)1 << 20);
    const bool pull_cand = !split && svc_pull_copy_usable(c, bytes);  // the resident service copies
    c->svc_keep = pull_cand;
    int rc = exchange(c, 1, mine, sig, P, &staged);
    c->svc_keep = false;
    if (rc) return rc;
    c->last_alg = split ? 2 : 1;
    if (pull_cand && !staged) return svc_pull_copy_run(c, LL_PULL_BC, P, buf, buf, bytes, root);
    if (pull_cand) svc_park(c);
    if (staged) return staged_bcast(c, buf, bytes, root, s);
    MultiCopyArgs m;
    std::memset(&m, 0, sizeof(m));
    if (!split) {
        if (c->rank != root) {
            m.src[0] = P[0][root];
            m.dst[0] = buf;
            m.len[0] = bytes;
            m.nseg = 1;
            rc = launch_multicopy(m, s);
            if (rc) return rc;
        }
        return finish(c, s);
    }
    size_t off, len;
    ring_block(bytes, c->size, c->rank, &off, &len);
    if (c->rank != root) {
        m.src[0] = (const char *)P[0][root] + off;
        m.dst[0] = (char *)buf + off;
        m.len[0] = len;
        m.nseg = 1;
        rc = launch_multicopy(m, s);
        if (rc) return rc;
    }
    rc = finish(c, s);
    if (rc) return rc;
    std::memset(&m, 0, sizeof(m));
    if (c->rank != root) {
        for (int q = 0; q < c->size; ++q) {
            if (q == c->rank) continue;
            size_t qo, ql;
            ring_block(bytes, c->size, q, &qo, &ql);
            m.src[m.nseg] = (const char *)P[0][q] + qo;  // slice q is complete at rank q (or root)
            m.dst[m.nseg] = (char *)buf + qo;
            m.len[m.nseg] = ql;
            m.nseg++;
        }
        rc = launch_multicopy(m, s);
        if (rc) return rc;
    }
    return finish(c, s);
}

// ----------------------------------------------------------------- public entry points
int mi355x_allreduce(mi355x_comm_t *c, const void *sbuf, void *rbuf, size_t count, int type, int op, void *stream)
{
    if (!c) return set_error(MI355X_ERR_ARG, "comm is NULL");
    DeviceGuard dg(c->device);
    drain(c);
    CallGate gate(c);
    return allreduce_impl(c, sbuf, rbuf, count, type, op, stream);
}
int mi355x_reduce(mi355x_comm_t *c, const void *sbuf, void *rbuf, size_t count, int type, int op, int root,
                  void *stream)
{
    if (!c) return set_error(MI355X_ERR_ARG, "comm is NULL");
    DeviceGuard dg(c->device);
    drain(c);
    CallGate gate(c);
    return reduce_impl(c, sbuf, rbuf, count, type, op, root, stream);
}
int mi355x_reduce_scatter_block(mi355x_comm_t *c, const void *sbuf, void *rbuf, size_t rcount, int type, int op,
                                void *stream)
{
    if (!c) return set_error(MI355X_ERR_ARG, "comm is NULL");
    DeviceGuard dg(c->device);
    drain(c);
    CallGate gate(c);
    return reduce_scatter_block_impl(c, sbuf, rbuf, rcount, type, op, stream);
}
int mi355x_reduce_scatter(mi355x_comm_t *c, const void *sbuf, void *rbuf, const int *rcounts, int type, int op,
                          void *stream)
{
    if (!c) return set_error(MI355X_ERR_ARG, "comm is NULL");
    DeviceGuard dg(c->device);
    drain(c);
    CallGate gate(c);
    return reduce_scatter_impl(c, sbuf, rbuf, rcounts, type, op, stream);
}
int mi355x_allgather(mi355x_comm_t *c, const void *sbuf, void *rbuf, size_t bytes, void *stream)
{
    if (!c) return set_error(MI355X_ERR_ARG, "comm is NULL");
    DeviceGuard dg(c->device);
    drain(c);
    CallGate gate(c);
    return allgather_impl(c, sbuf, rbuf, bytes, stream);
}
int mi355x_bcast(mi355x_comm_t *c, void *buf, size_t bytes, int root, void *stream)
{
    if (!c) return set_error(MI355X_ERR_ARG, "comm is NULL");
    DeviceGuard dg(c->device);
    drain(c);
    CallGate gate(c);
    return bcast_impl(c, buf, bytes, root, stream);
}

// nonblocking: argument checks at post time, the collective itself on the progress thread
int mi355x_iallreduce(mi355x_comm_t *c, const void *sbuf, void *rbuf, size_t count, int type, int op, void *stream,
                      mi355x_request_t **req)
{
    int rc = check_common(c, op, type);
    if (rc) return rc;
    return post(c, stream, [=](hipStream_t s) { return allreduce_impl(c, sbuf, rbuf, count, type, op, s); }, req);
}
int mi355x_ireduce(mi355x_comm_t *c, const void *sbuf, void *rbuf, size_t count, int type, int op, int root,
                   void *stream, mi355x_request_t **req)
{
    int rc = check_common(c, op, type);
    if (rc) return rc;
    if (root < 0 || root >= c->size) return set_error(MI355X_ERR_ARG, "bad root");
    return post(c, stream, [=](hipStream_t s) { return reduce_impl(c, sbuf, rbuf, count, type, op, root, s); }, req);
}
int mi355x_ireduce_scatter_block(mi355x_comm_t *c, const void *sbuf, void *rbuf, size_t rcount, int type, int op,
                                 void *stream, mi355x_request_t **req)
{
    int rc = check_common(c, op, type);
    if (rc) return rc;
    return post(c, stream,
                [=](hipStream_t s) { return reduce_scatter_block_impl(c, sbuf, rbuf, rcount, type, op, s); }, req);
}
int mi355x_iallgather(mi355x_comm_t *c, const void *sbuf, void *rbuf, size_t bytes, void *stream,
                      mi355x_request_t **req)
{
    if (!c) return set_error(MI355X_ERR_ARG, "comm is NULL");
    return post(c, stream, [=](hipStream_t s) { return allgather_impl(c, sbuf, rbuf, bytes, s); }, req);
}
int mi355x_ibcast(mi355x_comm_t *c, void *buf, size_t bytes, int root, void *stream, mi355x_request_t **req)
{
    if (!c) return set_error(MI355X_ERR_ARG, "comm is NULL");
    if (root < 0 || root >= c->size) return set_error(MI355X_ERR_ARG, "bad root");
    return post(c, stream, [=](hipStream_t s) { return bcast_impl(c, buf, bytes, root, s); }, req);
}

int mi355x_request_test(mi355x_request_t *r, int *done)
{
    if (!r || !done) return set_error(MI355X_ERR_ARG, "NULL request");
    if (r->kind != 0 && !r->done.load(std::memory_order_acquire)) p2p_progress(r->comm);
    *done = r->done.load(std::memory_order_acquire);
    if (*done && r->rc != MI355X_SUCCESS) return set_error(r->rc, "%s", r->err.c_str());
    return MI355X_SUCCESS;
}
int mi355x_request_wait(mi355x_request_t *r)
{
    if (!r) return set_error(MI355X_ERR_ARG, "NULL request");
    if (r->kind != 0) return p2p_wait(r);
    unsigned spins = 0;
    while (!r->done.load(std::memory_order_acquire)) {
        if (++spins > 64) sched_yield();
    }
    if (r->rc != MI355X_SUCCESS) return set_error(r->rc, "%s", r->err.c_str());
    return MI355X_SUCCESS;
}
int mi355x_request_free(mi355x_request_t *r)
{
    if (!r) return MI355X_SUCCESS;
    if (!r->done.load(std::memory_order_acquire)) return set_error(MI355X_ERR_ARG, "request still active");
    if (r->ev) (void)hipEventDestroy(r->ev);
    delete r;
    return MI355X_SUCCESS;
}

} // extern "C"
