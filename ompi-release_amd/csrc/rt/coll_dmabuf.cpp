// coll_dmabuf.cpp -- dmabuf IPC of allocations hipIpc cannot export: fd passing between the
// ranks (SCM_RIGHTS), import, and the creation-time probe (split out of coll_comm.cpp).

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

// ----------------------------------------------------------------- dmabuf fd passing (SCM_RIGHTS)
// hipIpcOpenMemHandle never returns for allocations of >= 2 GiB (ROCm 7.2, dmabuf IPC), but the
// allocation exported as a dmabuf fd (hipMemGetHandleForAddressRange) and imported by the peer as
// external memory maps fine.  The fd reaches the peer as SCM_RIGHTS ancillary data on an AF_UNIX
// datagram socket (the smcuda BTL's role of carrying the IPC handle, btl/smcuda/README:13-30):
// no ptrace permission is granted to anybody.  Every rank binds one socket at communicator
// creation under an abstract name derived from the control segment's (node-unique) name; the
// receiver checks the sender's pid (SO_PASSCRED) against the rank's published pid.
constexpr int kFdMax = 8;  // fds per message (a call exports at most kMaxBufs buffers)
// kind 0: nfd fds for allocations id[0..nfd); kind 1: a request for allocation id[0]'s fd (an
// importer that closed its import, or never got the fd, asks its exporter again); kind 2: that
// allocation is not registered with the exporter any more
enum : int32_t { kFdGive = 0, kFdAsk = 1, kFdGone = 2 };
constexpr int kStashGone = -2;  // fd_stash value for a kFdGone answer
struct FdMsg {
    int32_t from;
    int32_t nfd;
    int32_t kind;
    int32_t pad;
    uint64_t id[kFdMax];
};

static int send_msg(mi355x_comm *c, int peer, const FdMsg &m, const int *fds, int nfd);

void fd_sock_addr(const mi355x_comm *c, int rank, sockaddr_un *a, socklen_t *len)
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

int fd_sock_open(mi355x_comm *c)
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
int fd_drain(mi355x_comm *c, bool wait)
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
        const bool from_rank = got == (ssize_t)sizeof(m) && m.from >= 0 && m.from < c->size &&
                               pid == (pid_t)c->ctrl->slot[m.from].pid;
        if (from_rank && nfd == 0 && m.nfd == 0 && m.kind == kFdAsk) {
            int rc = serve_fd(c, m.from, m.id[0]);
            if (rc) return rc;
            continue;
        }
        if (from_rank && nfd == 0 && m.nfd == 0 && m.kind == kFdGone) {
            c->fd_stash[std::make_pair((int)m.from, m.id[0])] = kStashGone;
            if (wait) return MI355X_SUCCESS;
            continue;
        }
        const bool ok = from_rank && nfd > 0 && m.nfd == nfd && m.kind == kFdGive;
        for (int i = 0; i < nfd; ++i) {
            if (!ok) {  // not from a rank of this communicator: drop it
                close(fds[i]);
                continue;
            }
            const auto key = std::make_pair((int)m.from, m.id[i]);
            auto it = c->fd_stash.find(key);
            if (it != c->fd_stash.end() && it->second >= 0) close(it->second);
            c->fd_stash[key] = fds[i];
        }
        if (wait && ok) return MI355X_SUCCESS;
    }
}

// one message to `peer`: nfd fds (SCM_RIGHTS) and their allocation ids, or a request / answer
// without fds.  Caller holds reg_mtx.
static int send_msg(mi355x_comm *c, int peer, const FdMsg &m, const int *fds, int nfd)
{
    iovec iov{const_cast<FdMsg *>(&m), sizeof(m)};
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
    if (nfd > 0) {
        h.msg_control = ctl;
        h.msg_controllen = CMSG_SPACE(sizeof(int) * (size_t)nfd);
        cmsghdr *cm = CMSG_FIRSTHDR(&h);
        cm->cmsg_level = SOL_SOCKET;
        cm->cmsg_type = SCM_RIGHTS;
        cm->cmsg_len = CMSG_LEN(sizeof(int) * (size_t)nfd);
        std::memcpy(CMSG_DATA(cm), fds, sizeof(int) * (size_t)nfd);
    }
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        if (sendmsg(c->fd_sock, &h, MSG_DONTWAIT | MSG_NOSIGNAL) == (ssize_t)sizeof(m)) return MI355X_SUCCESS;
        if (errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR)
            return set_error(MI355X_ERR_PEER, "sending dmabuf fds to rank %d: %s", peer, strerror(errno));
        // the peer's queue is full (net.unix.max_dgram_qlen): it drains it whenever it waits
        // (barrier, finish, its own sends, its imports) -- keep ours drained meanwhile too
        int rc = fd_drain(c, false);
        if (rc) return rc;
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > c->timeout_s)
            return set_error(MI355X_ERR_TIMEOUT, "rank %d: fd queue of rank %d stays full", c->rank, peer);
        usleep(50);
    }
}

int send_fds(mi355x_comm *c, int peer, const int *fds, const uint64_t *ids, int nfd)
{
    FdMsg m;
    std::memset(&m, 0, sizeof(m));
    m.from = c->rank;
    m.nfd = nfd;
    m.kind = kFdGive;
    for (int i = 0; i < nfd; ++i) m.id[i] = ids[i];
    return send_msg(c, peer, m, fds, nfd);
}

// a peer asks for the fd of my allocation `id` again: export it afresh, send it, close my copy (an
// exporter keeps no fd of its own, so a freed allocation is held only by the imports of it)
int serve_fd(mi355x_comm *c, int peer, uint64_t id)
{
    FdMsg m;
    std::memset(&m, 0, sizeof(m));
    m.from = c->rank;
    m.id[0] = id;
    for (const LocalReg &r : c->local_regs) {
        if (r.id != id || r.has_h) continue;  // (an allocation on the hipIpc route never went out as a dmabuf)
        int fd = -1;
        if (hipMemGetHandleForAddressRange(&fd, (hipDeviceptr_t)r.base, r.size, hipMemRangeHandleTypeDmaBufFd, 0) !=
            hipSuccess) {
            (void)hipGetLastError();
            break;
        }
        TRACE(c, "dmabuf: rank %d asked again for allocation %llu", peer, (unsigned long long)id);
        m.kind = kFdGive;
        m.nfd = 1;
        const int rc = send_msg(c, peer, m, &fd, 1);
        close(fd);
        return rc;
    }
    m.kind = kFdGone;
    return send_msg(c, peer, m, nullptr, 0);
}

int send_fd(mi355x_comm *c, int peer, int fd, uint64_t id) { return send_fds(c, peer, &fd, &id, 1); }

// the fd rank `peer` passed for its allocation `id` (a duplicate: the stash keeps its own)
int take_fd(mi355x_comm *c, int peer, uint64_t id, int *out)
{
    const auto key = std::make_pair(peer, id);
    int rc = fd_drain(c, false);
    if (rc) return rc;
    if (c->fd_stash.find(key) == c->fd_stash.end()) {  // (closed an import of it, or never got it: ask)
        FdMsg m;
        std::memset(&m, 0, sizeof(m));
        m.from = c->rank;
        m.kind = kFdAsk;
        m.id[0] = id;
        rc = send_msg(c, peer, m, nullptr, 0);
        if (rc) return rc;
    }
    while (c->fd_stash.find(key) == c->fd_stash.end()) {
        rc = fd_drain(c, true);
        if (rc) return rc;
    }
    if (c->fd_stash[key] == kStashGone) {
        c->fd_stash.erase(key);
        return set_error(MI355X_ERR_PEER, "rank %d no longer has allocation %llu registered", peer, (unsigned long long)id);
    }
    *out = fcntl(c->fd_stash[key], F_DUPFD_CLOEXEC, 0);
    if (*out < 0) return set_error(MI355X_ERR_PEER, "dup of a dmabuf fd: %s", strerror(errno));
    return MI355X_SUCCESS;
}

// forget the fd of `peer`'s allocation `id` (the allocation was freed or replaced)
void drop_stash(mi355x_comm *c, int peer, uint64_t id)
{
    auto it = c->fd_stash.find(std::make_pair(peer, id));
    if (it == c->fd_stash.end()) return;
    if (it->second >= 0) close(it->second);
    c->fd_stash.erase(it);
}

// pass the dmabuf fds of the allocations of ds[0..nd) to every rank in `peers` that has not had
// them yet: one message per peer.  The export is made for the sends and closed after them (the
// fds in flight and the peers' imports hold the allocation; a peer that later needs one again asks,
// serve_fd), so an exporter never keeps a freed allocation alive itself.
int export_dmabufs(mi355x_comm *c, BufDesc *const *ds, int nd, uint64_t peers)
{
    std::lock_guard<std::recursive_mutex> reg_guard(c->reg_mtx);
    LocalReg *regs[kFdMax];
    for (int i = 0; i < nd; ++i) {
        regs[i] = nullptr;
        for (LocalReg &r : c->local_regs)
            if (r.base == ds[i]->base && r.id == ds[i]->id) regs[i] = &r;
        if (!regs[i])
            return set_error(MI355X_ERR_PEER, "large allocation not registered (id %llu)", (unsigned long long)ds[i]->id);
        ds[i]->dmabuf = 1;
        ds[i]->fd = -1;
        ds[i]->size = regs[i]->size;
    }
    int rc = MI355X_SUCCESS;
    for (int q = 0; q < c->size && !rc; ++q) {
        if (q == c->rank || !((peers >> q) & 1u)) continue;
        int fds[kFdMax];
        uint64_t ids[kFdMax];
        int k = 0;
        for (int i = 0; i < nd; ++i) {
            LocalReg &r = *regs[i];
            if ((r.sent >> q) & 1u) continue;
            bool dup = false;  // two buffers of one allocation: one fd
            for (int j = 0; j < k; ++j) dup = dup || ids[j] == r.id;
            if (dup) continue;
            if (r.fd < 0) {
                MI_HIP(hipMemGetHandleForAddressRange(&r.fd, (hipDeviceptr_t)r.base, r.size,
                                                      hipMemRangeHandleTypeDmaBufFd, 0));
            }
            fds[k] = r.fd;
            ids[k++] = r.id;
        }
        if (!k) continue;
        rc = send_fds(c, q, fds, ids, k);
        if (!rc)
            for (int i = 0; i < nd; ++i) regs[i]->sent |= 1ull << q;
    }
    for (int i = 0; i < nd; ++i) drop_reg(*regs[i]);  // (closes this call's exports; the registration stays)
    return rc;
}

int export_dmabuf(mi355x_comm *c, BufDesc *d, uint64_t peers)
{
    BufDesc *ds[1] = {d};
    return export_dmabufs(c, ds, 1, peers);
}

int import_dmabuf(mi355x_comm *c, int peer, uint64_t id, size_t size, void **mapped, hipExternalMemory_t *ext)
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
    drop_stash(c, peer, id);  // (the import holds the allocation now)
    return MI355X_SUCCESS;
}


// Collective, once per communicator: every rank exports a 4 MiB buffer as a dmabuf, every rank
// imports every peer's and checks its bytes; the path is used only if it worked everywhere.
int probe_dmabuf(mi355x_comm *c)
{
    const char *env = getenv("MI355X_DMABUF");
    bool ok = !(env && atoi(env) == 0);
    const size_t sz = (size_t)4 << 20;
    void *buf = nullptr;
    int fd = -1;
    RankSlot &me = c->ctrl->slot[c->rank];
    if (ok && hipMalloc(&buf, sz) != hipSuccess) ok = false;
    hipStream_t ss = setup_stream(c);
    if (ok && hipMemsetAsync(buf, c->rank + 1, sz, ss) != hipSuccess) ok = false;
    if (ok && hipStreamSynchronize(ss) != hipSuccess) ok = false;
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

} // namespace mi355x
