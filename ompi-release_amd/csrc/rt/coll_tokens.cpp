// coll_tokens.cpp -- node-wide admission tokens of the pipelined grid (split out of
// coll_comm.cpp).

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

uint64_t proc_start_time(pid_t pid)
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
bool holder_alive(uint64_t who, uint64_t start)
{
    const pid_t pid = (pid_t)(who & 0x7fffffffull);
    if (!pid_alive(pid)) return false;
    if (who & kTokPending) return true;  // still registering: its start time is not written yet
    const uint64_t now = proc_start_time(pid);
    return now == 0 || now == start;
}

GpuTokens *gpu_tokens()
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
bool pipe_token_reclaim(GpuTokens *t, int i, uint64_t cur)
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

bool pipe_token_acquire(mi355x_comm *c)
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

void pipe_token_release(mi355x_comm *c)
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


} // namespace mi355x
