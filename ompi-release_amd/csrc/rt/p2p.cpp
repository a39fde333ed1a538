// p2p.cpp -- point-to-point (MPI_Send / MPI_Recv / MPI_Isend / MPI_Irecv / MPI_Sendrecv /
// MPI_Iprobe / MPI_Improbe + MPI_Imrecv) between the ranks of a coll/mi355x communicator, on device
// and host buffers, in one matching queue.
//
// What it replaces: ob1 matches every message of a communicator in one queue whatever the buffer
// kind, and decides per request, on each side, how the bytes move (pml_ob1_cuda.c:52-100 on the
// send side, pml_ob1_recvreq.c:647-663 on the receive side).  A device message goes by RGET over
// btl/smcuda: the sender registers its buffer (CUDA IPC handle, mpool/rgpusm cache) and sends a
// rendezvous header carrying the handle; the receiver matches it (pml_ob1_recvfrag.c match loop:
// per-source order, posted receives in posting order, MPI_ANY_SOURCE / MPI_ANY_TAG), opens the
// handle and copies out of the sender's GPU buffer (mca_btl_smcuda_get_cuda,
// btl_smcuda.c:1083-1168), then returns a FIN so the send completes.  A host message (and a small
// device one) goes through the sm BTL's shared-memory fragments: eager up to 4 KiB
// (btl_sm_component.c:244), rendezvous beyond.
//
// Here, MI355X-first:
//   * the match / RGET header is an Envelope in the communicator's shared control segment: one
//     ring of kP2PSlots per ordered pair (src, dst), filled by src, drained by dst in order
//     (comm_internal.hpp); `full` announces message m, `done` is the FIN;
//   * where the bytes wait for the receiver:
//       - a device payload above 4 KiB: the sender's own buffer, exported once (the registration
//         cache of coll_comm.cpp; dmabuf for allocations of 2 GiB or more), or -- a non-contiguous
//         layout, or a buffered send -- a copy in the communicator's exportable device arena
//         (the GPU convertor packs into it);
//       - a host payload, or a device payload of at most 4 KiB: a copy in the sender's host
//         arena, a POSIX shared-memory segment the receiver maps (the sm BTL's role);
//   * the receiver PULLS: a device payload is read over xGMI by one kernel on its own GPU
//     (k_multicopy, or the convertor's unpack kernel for a derived datatype) into the receive
//     buffer -- or into a device staging slot, then to host memory, for a host receive; a host
//     payload is copied out of the mapped segment (memcpy / host convertor, or host-to-device
//     copy).  Nothing is ever written into the peer's memory;
//   * completion of a send: eager (the caller's request completes once the payload is copied --
//     the engine keeps an internal request for the envelope) for messages of at most 4 KiB and
//     buffered sends, rendezvous (the FIN) otherwise and for synchronous sends;
//   * progress is polled (mi355x_p2p_progress, the opal_progress hook; test / wait call it):
//     queued sends are announced, mailboxes drained, posted receives matched, finished reads
//     acknowledged, acknowledged sends completed.
// Truncation follows ob1 (pml_ob1_recvreq.h:172-180): the receive gets as many bytes as its
// buffer holds, status.bytes is the message size and status.error MI355X_ERR_TRUNCATE.
#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <new>

#include "comm_internal.hpp"
#include "ddt_internal.hpp"

namespace mi355x {

constexpr size_t kEagerLimit = 4096;          // btl_sm_component.c:244, btl_smcuda_component.c:183
constexpr int32_t kEnvPacked = 1;             // the payload is a packed copy (layout unused)
constexpr int32_t kEnvHost = 2;               // the payload is in the sender's host arena
constexpr int32_t kEnvStream = 4;             // ... and is being copied in: a StreamHdr precedes it
constexpr int32_t kEnvInline = 8;             // the payload is inside the envelope (<= kP2PInline bytes)
constexpr int32_t kEnvDual = 16;              // a small device payload offered two ways (Envelope::claim)
static_assert(sizeof(BufDesc) >= kP2PInline, "an inline payload fits the envelope's descriptor space");
// host payloads of at least kStreamMin bytes are announced before they are copied into the arena
// and copied in kStreamFrag fragments, the receiver copying fragment k out while the sender copies
// k + 1 in (the sm BTL's fragment pipeline, btl_sm_sendi / mca_btl_sm_component_progress)
constexpr size_t kStreamMin = (size_t)1 << 20;   // MI355X_P2P_STREAM_MIN overrides (A/B timing)
constexpr size_t kStreamFrag = (size_t)256 << 10;  // smallest fragment (stream_frag)
struct alignas(64) StreamHdr {
    std::atomic<uint64_t> ready;   // payload bytes copied in so far
    char pad[56];
};
static_assert(sizeof(StreamHdr) == 64, "StreamHdr is one cache line");

// fragment of a streamed n-byte payload: n / 16 within [256 KiB, 1 MiB] (two-process one-way
// host -> host, profiles/r03_host_p2p.jsonl: 1 MiB fragments lead at 64 MiB, 256 KiB at 1-8 MiB);
// sender and receiver may fragment differently -- the receiver waits for `ready` to cover its own
static size_t stream_frag(size_t n)
{
    static const size_t env = [] {
        const char *e = getenv("MI355X_P2P_STREAM_FRAG");
        return e ? std::max<size_t>((size_t)strtoull(e, nullptr, 0), 4096) : (size_t)0;
    }();
    if (env) return env;
    return std::min<size_t>(std::max<size_t>((n / 16) & ~(size_t)4095, kStreamFrag), kStreamFrag * 4);
}

static size_t stream_min()
{
    static const size_t v = [] {
        const char *e = getenv("MI355X_P2P_STREAM_MIN");
        return e ? (size_t)strtoull(e, nullptr, 0) : kStreamMin;
    }();
    return v;
}

struct P2PMsg {   // an announced message not matched yet (ob1's unexpected queue)
    int src;
    uint64_t m;
    Envelope *env;
};

// bump-allocated staging; reset when no slot is in use; a full arena is replaced by a larger one
// and kept (retired) until its last slot is released
struct DevArena {
    char *base = nullptr;
    size_t bytes = 0, used = 0;
    int users = 0;
    std::vector<void *> retired;
};

// the sender's host arena: one shared-memory segment per generation, named after the control
// segment, the rank and the generation; receivers map it on first use
struct HostSeg {
    char *base;
    size_t bytes;
    uint32_t gen;
    std::string name;
    bool reg = false;  // registered with HIP (seg_register)
    char *dbase = nullptr;  // its device-side address (registered and mapped), else null
    int pins = 0;           // (a peer's segment) copy kernels still reading it: never unmapped meanwhile
};
struct HostArena {
    HostSeg cur{nullptr, 0, 0, std::string(), false};
    size_t used = 0;
    int users = 0;
    std::vector<HostSeg> retired;
};

struct P2P {
    std::recursive_mutex mtx;
    hipStream_t stream = nullptr;
    unsigned fd_polls = 0;                  // p2p_progress calls (a dmabuf fd request check every 32)
    std::vector<uint64_t> send_seq;        // next message number, per destination
    std::vector<uint64_t> recv_seq;        // next message number to drain, per source
    std::deque<P2PMsg> unexpected;         // arrival order (per source: send order)
    std::deque<mi355x_request *> posted;   // receives not matched yet, posting order
    std::deque<mi355x_request *> queued;   // sends waiting for a free envelope, posting order
    std::vector<mi355x_request *> sending; // announced, waiting for the receiver's FIN
    std::vector<mi355x_request *> reading; // matched receives whose pull is in flight
    // matched receives of a dual message whose device buffer could not be mapped here: they wait
    // for the sender's host copy (claim 1) instead of claiming the pull
    std::vector<std::pair<mi355x_request *, P2PMsg>> dual_wait;
    // matched receives whose read needs a peer mapping, matched in a progress pass that must not
    // open one (a member of the collective it runs from is closing, barrier_progress): started at
    // the next pass that may
    std::vector<std::pair<mi355x_request *, P2PMsg>> deferred;
    DevArena arena;                        // exportable: packed / buffered device payloads
    DevArena rstage;                       // receive side: device staging of host receives
    HostArena harena;                      // host payloads (shared memory)
    char *bounce = nullptr;                // registered host bounce for an inline payload bound for the device
    std::vector<hipEvent_t> evpool;        // completion events of dual sends' host copies, for reuse
    std::map<std::pair<int, uint32_t>, HostSeg> peer_segs;  // peers' host arenas, mapped
};

static void seg_drop(HostSeg &g, bool owner);

// Every communicator with point-to-point state, so that any of the engine's host-side waits can
// progress all of them -- as ob1's waits run opal_progress over every pending request: an eager
// send that found its peer's ring full completed for its caller but is announced only by a later
// progress pass, and its receiver may be what the waiting rank is waiting for.
static std::mutex g_p2p_mtx;
static std::vector<mi355x_comm *> g_p2p_comms;

static P2P *p2p_of(mi355x_comm *c)
{
    if (!c->p2p) {
        auto *p = new P2P();
        p->send_seq.assign((size_t)c->size, 0);
        p->recv_seq.assign((size_t)c->size, 0);
        c->p2p = p;
        std::lock_guard<std::mutex> g(g_p2p_mtx);
        g_p2p_comms.push_back(c);
    }
    return c->p2p;
}

// fault injection for tests (MI355X_P2P_INJECT, read once): 1 the dual offer's host copy fails
// (sender), 2 the first mapping of a dual sender's device buffer fails (receiver), 4 every such
// mapping fails (receiver)
static unsigned p2p_inject()
{
    static const unsigned v = (unsigned)atoi(getenv("MI355X_P2P_INJECT") ? getenv("MI355X_P2P_INJECT") : "0");
    return v;
}

// set while a progress pass must not open peer mappings -- from inside a collective's barrier while
// a member closes its retired ones (coll_ctl.cpp, barrier_progress / close_window: hipIpc opens must
// not overlap a peer's closes, coll_rcache.cpp): reads that would open one wait for a later pass
static thread_local bool t_defer_maps = false;

bool p2p_defer_maps(bool on)
{
    const bool prev = t_defer_maps;
    t_defer_maps = on;
    return prev;
}

void p2p_progress_all(bool defer_maps)
{
    std::unique_lock<std::mutex> g(g_p2p_mtx, std::try_to_lock);  // (another thread progresses them now)
    if (!g.owns_lock()) return;
    const bool saved = t_defer_maps;
    t_defer_maps = defer_maps;
    for (mi355x_comm *c : g_p2p_comms) (void)p2p_progress(c);
    t_defer_maps = saved;
}

static int p2p_stream(mi355x_comm *c, P2P *p, hipStream_t *s)
{
    if (!p->stream) {
        DeviceGuard dg(c->device);
        MI_HIP(hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking));
    }
    *s = p->stream;
    return MI355X_SUCCESS;
}

void p2p_destroy(mi355x_comm *c)
{
    P2P *p = c->p2p;
    if (!p) return;
    {
        std::lock_guard<std::mutex> g(g_p2p_mtx);  // (waits out a progress pass over it)
        g_p2p_comms.erase(std::remove(g_p2p_comms.begin(), g_p2p_comms.end(), c), g_p2p_comms.end());
    }
    if (p->stream) {
        (void)hipStreamSynchronize(p->stream);
        (void)hipStreamDestroy(p->stream);
    }
    for (mi355x_request *r : p->reading)
        if (r->pin) r->pin->pins--;  // (the stream was synchronised above: nothing reads any more)
    // sends the engine owns (eager / buffered) that never saw their FIN
    for (mi355x_request *r : p->queued)
        if (r->internal) delete r;
    for (mi355x_request *r : p->sending)
        if (r->internal) delete r;
    for (DevArena *a : {&p->arena, &p->rstage}) {
        if (a->base) (void)hipFree(a->base);
        for (void *x : a->retired) (void)hipFree(x);
    }
    seg_drop(p->harena.cur, true);
    for (HostSeg &g : p->harena.retired) seg_drop(g, true);
    if (p->bounce) (void)hipHostFree(p->bounce);
    for (hipEvent_t e : p->evpool) (void)hipEventDestroy(e);
    for (auto &kv : p->peer_segs) seg_drop(kv.second, false);
    delete p;
    c->p2p = nullptr;
}

static int arena_alloc(DevArena &a, size_t bytes, void **out)
{
    const size_t need = (bytes + 255) & ~(size_t)255;
    if (a.used + need > a.bytes) {
        if (a.base) {
            if (a.users > 0) a.retired.push_back(a.base);  // peers may still read it
            else MI_HIP(hipFree(a.base));
        }
        a.base = nullptr;
        size_t want = std::max<size_t>((size_t)8 << 20, a.bytes * 2);
        while (want < need) want *= 2;
        a.bytes = 0;
        a.used = 0;
        MI_HIP(hipMalloc((void **)&a.base, want));
        a.bytes = want;
    }
    *out = a.base + a.used;
    a.used += need;
    a.users++;
    return MI355X_SUCCESS;
}

static void arena_release(DevArena &a)
{
    if (--a.users > 0) return;
    a.used = 0;
    for (void *x : a.retired) (void)hipFree(x);
    a.retired.clear();
}

// Host arenas are registered with HIP (pinned and GPU-mapped; the receiver's mapping read-only), so
// a small device payload's device-to-host copy into the sender's slot and the receiver's
// host-to-device copy out of it are one DMA each, not a staged copy through HIP's own pinned
// buffer (MI355X_P2P_REGISTER=0 leaves them unregistered)
static void seg_register(HostSeg &g, bool readonly)
{
    static const bool on = !(getenv("MI355X_P2P_REGISTER") && atoi(getenv("MI355X_P2P_REGISTER")) == 0);
    if (!on || !g.base) return;
    const unsigned flags = hipHostRegisterMapped | (readonly ? hipHostRegisterReadOnly : 0u);
    g.reg = hipHostRegister(g.base, g.bytes, flags) == hipSuccess;
    void *d = nullptr;
    if (g.reg && hipHostGetDevicePointer(&d, g.base, 0) == hipSuccess) g.dbase = static_cast<char *>(d);
    (void)hipGetLastError();
}

static void seg_drop(HostSeg &g, bool owner)
{
    if (!g.base) return;
    if (g.reg) (void)hipHostUnregister(g.base);
    g.reg = false;
    g.dbase = nullptr;
    munmap(g.base, g.bytes);
    if (owner && !g.name.empty()) shm_unlink(g.name.c_str());
    g.base = nullptr;
}

static std::string seg_name(const mi355x_comm *c, int rank, uint32_t gen)
{
    return c->shm_name + "_h" + std::to_string(rank) + "_" + std::to_string(gen);
}

// a slot of `bytes` in my host arena; desc describes it to the receiver
static int harena_alloc(mi355x_comm *c, P2P *p, size_t bytes, void **out, BufDesc *desc)
{
    HostArena &h = p->harena;
    const size_t need = (bytes + 63) & ~(size_t)63;
    if (h.used + need > h.cur.bytes) {
        if (h.cur.base) {
            if (h.users > 0) h.retired.push_back(h.cur);
            else seg_drop(h.cur, true);
        }
        size_t want = std::max<size_t>((size_t)1 << 20, h.cur.bytes * 2);
        while (want < need) want *= 2;
        HostSeg g{nullptr, want, h.cur.gen + 1, std::string(), false};
        if (c->loopback) {  // threads of one process: plain memory, read through the pointer
            void *m = mmap(nullptr, want, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
            if (m == MAP_FAILED) return set_error(MI355X_ERR_NOMEM, "host arena of %zu bytes", want);
            g.base = (char *)m;
        } else {
            g.name = seg_name(c, c->rank, g.gen);
            const int fd = shm_open(g.name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
            if (fd < 0) return set_error(MI355X_ERR_NOMEM, "host arena %s: %s", g.name.c_str(), strerror(errno));
            void *m = MAP_FAILED;
            if (ftruncate(fd, (off_t)want) == 0) m = mmap(nullptr, want, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
            close(fd);
            if (m == MAP_FAILED) {
                shm_unlink(g.name.c_str());
                return set_error(MI355X_ERR_NOMEM, "host arena %s of %zu bytes", g.name.c_str(), want);
            }
            g.base = (char *)m;
            seg_register(g, false);
        }
        h.cur = g;
        h.used = 0;
    }
    *out = h.cur.base + h.used;
    std::memset(desc, 0, sizeof(*desc));
    desc->present = 1;
    desc->raw = (uint64_t)(uintptr_t)*out;
    desc->off = h.used;
    desc->id = h.cur.gen;
    desc->size = h.cur.bytes;
    h.used += need;
    h.users++;
    return MI355X_SUCCESS;
}

static void harena_release(P2P *p)
{
    HostArena &h = p->harena;
    if (--h.users > 0) return;
    h.used = 0;
    for (HostSeg &g : h.retired) seg_drop(g, true);
    h.retired.clear();
}

// where a peer's host payload is readable: the pointer itself (same process), else the peer's
// segment of that generation, mapped once (older generations of that peer are unmapped: their
// slots were read synchronously, and a message still pending keeps its segment alive on the
// sender's side, so it can be mapped again by name)
static int host_src(mi355x_comm *c, P2P *p, int src, const BufDesc &d, const char **out, const char **dev_out = nullptr,
                    HostSeg **seg = nullptr)
{
    if (dev_out) *dev_out = nullptr;
    if (seg) *seg = nullptr;
    if (c->loopback || src == c->rank) {
        *out = (const char *)(uintptr_t)d.raw;
        return MI355X_SUCCESS;
    }
    const uint32_t gen = (uint32_t)d.id;
    auto it = p->peer_segs.find({src, gen});
    if (it == p->peer_segs.end()) {
        for (auto j = p->peer_segs.begin(); j != p->peer_segs.end();) {
            if (j->first.first == src && j->first.second < gen && j->second.pins == 0) {
                seg_drop(j->second, false);
                j = p->peer_segs.erase(j);
            } else {
                ++j;
            }
        }
        HostSeg g{nullptr, 0, gen, seg_name(c, src, gen), false};
        const int fd = shm_open(g.name.c_str(), O_RDONLY, 0600);
        if (fd < 0) return set_error(MI355X_ERR_PEER, "host arena %s of rank %d: %s", g.name.c_str(), src, strerror(errno));
        struct stat st;
        void *m = MAP_FAILED;
        if (fstat(fd, &st) == 0) {
            g.bytes = (size_t)st.st_size;
            m = mmap(nullptr, g.bytes, PROT_READ, MAP_SHARED, fd, 0);
        }
        close(fd);
        if (m == MAP_FAILED) return set_error(MI355X_ERR_PEER, "mapping host arena %s failed", g.name.c_str());
        g.base = (char *)m;
        g.name.clear();  // not ours to unlink
        seg_register(g, true);
        it = p->peer_segs.emplace(std::make_pair(src, gen), g).first;
    }
    if (d.off > it->second.bytes) return set_error(MI355X_ERR_PEER, "host payload outside rank %d's arena", src);
    *out = it->second.base + d.off;
    if (dev_out && it->second.dbase) *dev_out = it->second.dbase + d.off;  // the same bytes, device-mapped
    if (seg) *seg = &it->second;
    return MI355X_SUCCESS;
}

static void complete(mi355x_request *r, int rc)
{
    r->rc = rc;
    if (rc != MI355X_SUCCESS) r->err = mi355x_last_error();
    r->done.store(1, std::memory_order_release);
}

// a receive whose data is in place: MPI_Wait reports the status's error (truncation)
static void complete_recv(mi355x_request *r)
{
    if (r->st_error == MI355X_ERR_TRUNCATE)
        complete(r, set_error(MI355X_ERR_TRUNCATE, "message of %zu bytes from rank %d truncated to %zu",
                              r->st_bytes, r->st_source, r->bytes));
    else
        complete(r, MI355X_SUCCESS);
}

// Envelope::claim of message `msg` in state 0 (undecided), 1 (host copy) or 2 (device pull)
static inline uint64_t claim_word(uint64_t msg, uint64_t state) { return ((msg + 1) << 2) | state; }

// announce send r in its envelope if the slot is free (the message K before it is done)
static bool try_announce(mi355x_comm *c, mi355x_request *r)
{
    Envelope *env = &p2p_ring(c->ctrl, c->size, c->rank, r->peer)[r->msg % kP2PSlots];
    // `done` of a slot only grows (by kP2PSlots per reuse): compare with >=
    if (r->msg >= (uint64_t)kP2PSlots &&
        env->done.load(std::memory_order_acquire) < r->msg - (uint64_t)kP2PSlots + 1)
        return false;
    env->tag = r->tag;
    env->flags = r->env_flags;
    env->bytes = r->bytes;
    if (r->env_flags & kEnvInline) std::memcpy(env->inl, r->inl, r->bytes);
    else std::memcpy(&env->buf, &r->desc, sizeof(BufDesc));
    env->hoff = r->hoff;
    env->hgen = r->hgen;
    env->claim.store(claim_word(r->msg, 0), std::memory_order_relaxed);
    env->full.store(r->msg + 1, std::memory_order_release);
    r->env = env;
    return true;
}

// bytes [0, need) of a streamed host payload are in the sender's arena
static int stream_wait(mi355x_comm *c, const StreamHdr *h, uint64_t need, int src)
{
    if (h->ready.load(std::memory_order_acquire) >= need) return MI355X_SUCCESS;
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned spins = 1;; ++spins) {
        if (h->ready.load(std::memory_order_acquire) >= need) return MI355X_SUCCESS;
        if ((spins & 0xff) == 0) {
            sched_yield();
            if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > c->timeout_s)
                return set_error(MI355X_ERR_TIMEOUT, "rank %d: streamed message from rank %d stalled at %llu of %llu bytes",
                                 c->rank, src, (unsigned long long)h->ready.load(), (unsigned long long)need);
        }
    }
}

// copy out a streamed host payload (hdr at `src`, payload after it) fragment by fragment as the
// sender copies it in: into host memory (memcpy / host convertor window), or into device memory
// (host-to-device copies; a layout through device staging, unpacked once at the end)
static int read_stream(mi355x_comm *c, P2P *p, mi355x_request *r, const char *src, size_t n, bool contig, char *dst,
                       hipStream_t s)
{
    const auto *h = reinterpret_cast<const StreamHdr *>(src);
    const char *pay = src + sizeof(StreamHdr);
    const int from = r->st_source;
    void *stage = nullptr;
    int rc = MI355X_SUCCESS;
    if (!r->host && !contig && (rc = arena_alloc(p->rstage, n, &stage))) return rc;
    const size_t frag = stream_frag(n);
    for (size_t off = 0; off < n && !rc; off += frag) {
        const size_t k = std::min(frag, n - off);
        if ((rc = stream_wait(c, h, off + k, from))) break;
        if (r->host) {
            if (contig) std::memcpy(dst + off, pay + off, k);
            else rc = mi355x_unpack_host(r->ddt, r->count, r->buf, off, pay + off, k);
        } else if (hipMemcpy((contig ? dst : (char *)stage) + off, pay + off, k, hipMemcpyHostToDevice) != hipSuccess) {
            rc = set_error(MI355X_ERR_HIP, "host-to-device copy of a %zu-byte message failed", n);
        }
    }
    if (stage) {
        if (!rc) rc = mi355x_unpack(r->ddt, r->count, r->buf, 0, stage, n, nullptr, s);
        if (!rc && hipStreamSynchronize(s) != hipSuccess) rc = set_error(MI355X_ERR_HIP, "unpack of a message failed");
        arena_release(p->rstage);
    }
    return rc;
}

// matched receive r <- message msg: copy the bytes into place (complete now), or start the pull
static void start_read(mi355x_comm *c, P2P *p, mi355x_request *r, const P2PMsg &msg)
{
    Envelope *env = msg.env;
    r->env = env;
    r->msg = msg.m;
    r->st_source = msg.src;
    r->st_tag = env->tag;
    r->st_bytes = env->bytes;
    r->st_error = env->bytes > r->bytes ? MI355X_ERR_TRUNCATE : MI355X_SUCCESS;
    const size_t n = std::min<size_t>(env->bytes, r->bytes);
    if (t_defer_maps && n && msg.src != c->rank && !c->loopback && !(env->flags & (kEnvHost | kEnvInline)) &&
        !((env->flags & kEnvDual) && env->claim.load(std::memory_order_acquire) == claim_word(msg.m, 1))) {
        p->deferred.emplace_back(r, msg);  // (its read opens a peer mapping: not from inside a barrier)
        return;
    }
    auto fin = [&]() { env->done.store(msg.m + 1, std::memory_order_release); };
    auto fail = [&](int rc) {
        fin();  // the sender must not hang
        complete(r, rc);
    };
    if (n == 0) {
        fin();
        complete_recv(r);
        return;
    }
    int64_t first = 0;
    const bool contig = !r->ddt || ddt_contiguous(r->ddt, r->count, &first);
    char *dst = (char *)r->buf + first;
    hipStream_t s = nullptr;
    int rc = MI355X_SUCCESS;
    // a small device payload offered two ways: pull it from the device buffer unless the sender's
    // host copy was taken first (claim 1).  The device pull is claimed only once the sender's buffer
    // is mapped here: if the mapping fails (an allocation a peer freed and reused can make hipIpc
    // refuse it) the receive waits for the host copy, which the sender takes when nobody claims.
    bool dual_host = false;
    if (env->flags & kEnvDual) {
        dual_host = env->claim.load(std::memory_order_acquire) == claim_word(msg.m, 1);
        if (!dual_host && msg.src != c->rank && !c->loopback) {
            void *mapped = nullptr;
            static std::atomic<int> injected_once{0};
            const bool inject = (p2p_inject() & 4) || ((p2p_inject() & 2) && injected_once.exchange(1) == 0);
            if (inject || map_peer(c, msg.src, env->buf, &mapped, nullptr, false) != MI355X_SUCCESS) {
                (void)hipGetLastError();
                p->dual_wait.emplace_back(r, msg);
                return;
            }
        }
        uint64_t z = claim_word(msg.m, 0);
        // (a failed CAS leaves the word in z: 1 the host copy was taken; 3 it failed -- pull the
        // device buffer, which is mapped, and the sender waits for this FIN)
        if (!dual_host && !env->claim.compare_exchange_strong(z, claim_word(msg.m, 2), std::memory_order_acq_rel))
            dual_host = z == claim_word(msg.m, 1);
    }
    BufDesc hdesc = env->buf;
    if (dual_host) {
        std::memset(&hdesc, 0, sizeof(hdesc));
        hdesc.present = 1;
        hdesc.id = env->hgen;
        hdesc.off = env->hoff;
    }
    const bool hostpay = dual_host || (env->flags & (kEnvHost | kEnvInline)) != 0;
    // (the stream only where a kernel or an async copy runs: not for a host payload into host memory)
    if ((!hostpay || !r->host || !contig) && (rc = p2p_stream(c, p, &s))) return fail(rc);
    if (hostpay) {
        // host payload (sm-BTL style): copied out synchronously, FIN at once -- from the envelope
        // itself (inline), or from the sender's host arena
        const char *src = nullptr;
        if (env->flags & kEnvInline) {
            src = reinterpret_cast<const char *>(env->inl);
            if (!r->host) {  // bound for the device: through a registered bounce (one DMA)
                if (!p->bounce && hipHostMalloc((void **)&p->bounce, kP2PInline, hipHostMallocDefault) != hipSuccess) {
                    p->bounce = nullptr;
                    (void)hipGetLastError();
                }
                if (p->bounce) {
                    std::memcpy(p->bounce, src, std::min<size_t>(n, kP2PInline));
                    src = p->bounce;
                }
            }
        } else {
            const char *dsrc = nullptr;
            HostSeg *seg = nullptr;
            if ((rc = host_src(c, p, msg.src, hdesc, &src, &dsrc, &seg))) return fail(rc);
            if (dsrc && !r->host && contig && !(env->flags & kEnvStream)) {
                // into device memory from the registered, device-mapped arena: one copy kernel on
                // the point-to-point stream, completed (and FINed) by progress like a device pull
                MultiCopyArgs m;
                std::memset(&m, 0, sizeof(m));
                m.src[0] = dsrc;
                m.dst[0] = dst;
                m.len[0] = n;
                m.nseg = 1;
                rc = launch_multicopy(m, s);
                if (!rc && !r->ev && hipEventCreateWithFlags(&r->ev, hipEventDisableTiming) != hipSuccess)
                    rc = set_error(MI355X_ERR_HIP, "hipEventCreate failed");
                if (!rc && hipEventRecord(r->ev, s) != hipSuccess)
                    rc = set_error(MI355X_ERR_HIP, "hipEventRecord on the point-to-point stream failed");
                if (rc) {
                    (void)hipStreamSynchronize(s);
                    return fail(rc);
                }
                if (seg) {
                    seg->pins++;
                    r->hpin = seg;
                }
                p->reading.push_back(r);
                return;
            }
        }
        if (env->flags & kEnvStream) {
            rc = read_stream(c, p, r, src, n, contig, dst, s);
            if (rc) return fail(rc);
            fin();
            complete_recv(r);
            return;
        }
        if (r->host) {
            if (contig) std::memcpy(dst, src, n);
            else rc = mi355x_unpack_host(r->ddt, r->count, r->buf, 0, src, n);
        } else if (contig) {
            if (hipMemcpy(dst, src, n, hipMemcpyHostToDevice) != hipSuccess)
                rc = set_error(MI355X_ERR_HIP, "host-to-device copy of a %zu-byte message failed", n);
        } else {
            void *stage = nullptr;
            if ((rc = arena_alloc(p->rstage, n, &stage))) return fail(rc);
            if (hipMemcpy(stage, src, n, hipMemcpyHostToDevice) != hipSuccess)
                rc = set_error(MI355X_ERR_HIP, "host-to-device copy of a %zu-byte message failed", n);
            if (!rc) rc = mi355x_unpack(r->ddt, r->count, r->buf, 0, stage, n, nullptr, s);
            if (!rc && hipStreamSynchronize(s) != hipSuccess) rc = set_error(MI355X_ERR_HIP, "unpack of a message failed");
            arena_release(p->rstage);
        }
        if (rc) return fail(rc);
        fin();
        complete_recv(r);
        return;
    }
    const void *src = nullptr;
    if (msg.src == c->rank || c->loopback) {
        src = (const void *)(uintptr_t)(env->buf.raw);
    } else {
        void *mapped = nullptr;
        PeerMap *pm = nullptr;
        rc = map_peer(c, msg.src, env->buf, &mapped, &pm, false);
        if (rc) return fail(rc);
        if (pm) {
            pm->pins++;
            r->pin = pm;
        }
        src = mapped;
    }
    auto pull = [&](void *to) {  // one launch reads the sender's bytes over xGMI
        MultiCopyArgs m;
        std::memset(&m, 0, sizeof(m));
        m.src[0] = src;
        m.dst[0] = to;
        m.len[0] = n;
        m.nseg = 1;
        return launch_multicopy(m, s);
    };
    if (!r->host) {
        rc = contig ? pull(dst) : mi355x_unpack(r->ddt, r->count, r->buf, 0, src, n, nullptr, s);
    } else {
        // host receive of a device payload: pull into device staging, then one device-to-host copy
        // (ob1's receive-side CUDA convertor does the same copy, pml_ob1_recvreq.c:647-663)
        if (!(rc = arena_alloc(p->rstage, n, &r->stage))) {
            rc = pull(r->stage);
            void *to = dst;
            if (!contig) {
                r->htmp.resize(n);
                to = r->htmp.data();
            }
            if (!rc && hipMemcpyAsync(to, r->stage, n, hipMemcpyDeviceToHost, s) != hipSuccess)
                rc = set_error(MI355X_ERR_HIP, "device-to-host copy of a %zu-byte message failed", n);
        }
    }
    if (rc == MI355X_SUCCESS && !r->ev && hipEventCreateWithFlags(&r->ev, hipEventDisableTiming) != hipSuccess)
        rc = set_error(MI355X_ERR_HIP, "hipEventCreate failed");
    if (rc == MI355X_SUCCESS && hipEventRecord(r->ev, s) != hipSuccess)
        rc = set_error(MI355X_ERR_HIP, "hipEventRecord on the point-to-point stream failed");
    if (rc) {
        (void)hipStreamSynchronize(s);
        if (r->pin) {
            r->pin->pins--;
            r->pin = nullptr;
        }
        if (r->stage) {
            arena_release(p->rstage);
            r->stage = nullptr;
        }
        r->htmp.clear();
        return fail(rc);
    }
    p->reading.push_back(r);
}

// ob1's match test: MPI_ANY_TAG matches user tags only (tag >= 0), pml_ob1_recvfrag.c:487
static bool matches(const mi355x_request *r, const P2PMsg &m)
{
    const int t = m.env->tag;
    return (r->peer == MI355X_ANY_SOURCE || r->peer == m.src) && (r->tag == MI355X_ANY_TAG ? t >= 0 : r->tag == t);
}

static void drain_mailboxes(mi355x_comm *c, P2P *p)
{
    for (int q = 0; q < c->size; ++q) {
        Envelope *ring = p2p_ring(c->ctrl, c->size, q, c->rank);
        for (;;) {
            const uint64_t m = p->recv_seq[(size_t)q];
            Envelope *env = &ring[m % kP2PSlots];
            if (env->full.load(std::memory_order_acquire) != m + 1) break;
            p->unexpected.push_back(P2PMsg{q, m, env});
            p->recv_seq[(size_t)q] = m + 1;
        }
    }
}

// a send whose FIN arrived: its payload slot is free; an engine-owned send is finished
static void send_done(P2P *p, mi355x_request *r)
{
    if (r->twin) {  // (kEnvDual) delivered before the host copy was taken
        complete(r->twin, MI355X_SUCCESS);
        r->twin = nullptr;
    }
    if (r->ev && (r->env_flags & kEnvDual)) {
        p->evpool.push_back(r->ev);
        r->ev = nullptr;
    }
    if (r->packed) arena_release(p->arena);
    if (r->hslot) harena_release(p);
    r->packed = r->hslot = nullptr;
    if (r->internal) delete r;
    else complete(r, MI355X_SUCCESS);
}

// (kEnvDual) time to take the host copy: nobody claimed the device buffer within the delay
static bool dual_copy_due(const mi355x_request *r)
{
    static const double delay = std::max(0.0, (getenv("MI355X_P2P_DUAL_DELAY_US") ? atof(getenv("MI355X_P2P_DUAL_DELAY_US"))
                                                                                   : 10.0)) * 1e-6;
    const double now = std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
    return now - r->dual_t0 >= delay;
}

// (kEnvDual) the copy kernel of the caller's bytes into the registered arena slot, and its event
static int dual_copy_launch(mi355x_comm *c, P2P *p, mi355x_request *r)
{
    r->copy_launched = true;
    hipStream_t s = nullptr;
    int rc = p2p_stream(c, p, &s);
    if (rc) return rc;
    HostSeg *g = nullptr;  // the segment the slot is in (the current one, or a retired generation)
    if (p->harena.cur.gen == r->hgen) g = &p->harena.cur;
    for (HostSeg &x : p->harena.retired)
        if (x.gen == r->hgen) g = &x;
    if (!g || !g->dbase) return set_error(MI355X_ERR_HIP, "host arena slot without a device mapping");
    MultiCopyArgs m;
    std::memset(&m, 0, sizeof(m));
    m.src[0] = r->dual_src;
    m.dst[0] = g->dbase + r->hoff;
    m.len[0] = r->bytes;
    m.nseg = 1;
    if ((rc = launch_multicopy(m, s))) return rc;
    if (!r->ev) {
        if (!p->evpool.empty()) {
            r->ev = p->evpool.back();
            p->evpool.pop_back();
        } else if (hipEventCreateWithFlags(&r->ev, hipEventDisableTiming) != hipSuccess) {
            r->ev = nullptr;
            (void)hipStreamSynchronize(s);
            return set_error(MI355X_ERR_HIP, "hipEventCreate failed");
        }
    }
    if (hipEventRecord(r->ev, s) != hipSuccess) {
        (void)hipStreamSynchronize(s);
        return set_error(MI355X_ERR_HIP, "hipEventRecord on the point-to-point stream failed");
    }
    return MI355X_SUCCESS;
}

int p2p_progress(mi355x_comm *c)
{
    DeviceGuard dg(c->device);
    P2P *p = p2p_of(c);
    std::lock_guard<std::recursive_mutex> g(p->mtx);
    // a receiver that closed its import of one of my send buffers asks me for its dmabuf fd again
    // (serve_fd): serve it while I wait in point-to-point too (now and then: one syscall)
    // (not in a pass that must not open mappings: serving one is an export, which must not overlap a
    // member's closes either)
    if (!t_defer_maps && c->dmabuf_state != -1 && c->fd_sock >= 0 && (++p->fd_polls & 31) == 0 &&
        c->reg_mtx.try_lock()) {
        (void)fd_drain(c, false);
        c->reg_mtx.unlock();
    }
    // 1. announce queued sends, in order; a destination whose ring is full holds its later sends
    uint64_t blocked = 0;  // destinations whose ring is full (bit per rank; kMaxRanks = 64)
    for (auto it = p->queued.begin(); it != p->queued.end();) {
        mi355x_request *r = *it;
        if (!((blocked >> r->peer) & 1u) && try_announce(c, r)) {
            p->sending.push_back(r);
            it = p->queued.erase(it);
        } else {
            blocked |= 1ull << r->peer;
            ++it;
        }
    }
    // 2. new envelopes, 3. match posted receives in posting order against the arrivals (first the
    //    matched dual receives whose host copy has come)
    if (!t_defer_maps && !p->deferred.empty()) {
        std::vector<std::pair<mi355x_request *, P2PMsg>> d;
        d.swap(p->deferred);
        for (const auto &w : d) start_read(c, p, w.first, w.second);
    }
    for (size_t i = 0; i < p->dual_wait.size();) {
        const auto w = p->dual_wait[i];
        const uint64_t cl = w.second.env->claim.load(std::memory_order_acquire);
        if (cl == claim_word(w.second.m, 3)) {
            // the sender's host copy failed: the device buffer is the only source left -- one more
            // try to map it (outside a barrier), else the receive fails (the FIN lets the send end)
            if (t_defer_maps) {
                ++i;
                continue;
            }
            p->dual_wait.erase(p->dual_wait.begin() + (ptrdiff_t)i);
            void *mapped = nullptr;
            if ((p2p_inject() & 4) || map_peer(c, w.second.src, w.second.env->buf, &mapped, nullptr, false) != MI355X_SUCCESS) {
                (void)hipGetLastError();
                w.second.env->done.store(w.second.m + 1, std::memory_order_release);
                complete(w.first, set_error(MI355X_ERR_PEER, "rank %d: neither the device buffer of rank %d's small "
                                                             "send nor its host copy is readable", c->rank, w.second.src));
                continue;
            }
            start_read(c, p, w.first, w.second);
            continue;
        }
        if (cl != claim_word(w.second.m, 1)) {
            ++i;
            continue;
        }
        p->dual_wait.erase(p->dual_wait.begin() + (ptrdiff_t)i);
        start_read(c, p, w.first, w.second);
    }
    drain_mailboxes(c, p);
    for (auto it = p->posted.begin(); it != p->posted.end();) {
        mi355x_request *r = *it;
        auto m = std::find_if(p->unexpected.begin(), p->unexpected.end(),
                              [r](const P2PMsg &x) { return matches(r, x); });
        if (m == p->unexpected.end()) {
            ++it;
            continue;
        }
        const P2PMsg msg = *m;
        p->unexpected.erase(m);
        it = p->posted.erase(it);
        start_read(c, p, r, msg);
    }
    // 4. finished pulls: host receives get their host-convertor pass, FIN to the sender, complete
    for (auto it = p->reading.begin(); it != p->reading.end();) {
        mi355x_request *r = *it;
        const hipError_t e = hipEventQuery(r->ev);
        if (e == hipErrorNotReady) {
            ++it;
            continue;
        }
        if (r->pin) {
            r->pin->pins--;
            r->pin = nullptr;
        }
        if (r->hpin) {
            static_cast<HostSeg *>(r->hpin)->pins--;
            r->hpin = nullptr;
        }
        if (r->stage) {
            arena_release(p->rstage);
            r->stage = nullptr;
        }
        r->env->done.store(r->msg + 1, std::memory_order_release);
        int rc = e == hipSuccess ? MI355X_SUCCESS
                                 : set_error(MI355X_ERR_HIP, "point-to-point read: %s", hipGetErrorString(e));
        if (!rc && !r->htmp.empty()) rc = mi355x_unpack_host(r->ddt, r->count, r->buf, 0, r->htmp.data(), r->htmp.size());
        r->htmp.clear();
        r->htmp.shrink_to_fit();
        if (rc == MI355X_SUCCESS) complete_recv(r);
        else complete(r, rc);
        it = p->reading.erase(it);
    }
    // 5. acknowledged sends (a dual send's caller completes as soon as its host copy is taken --
    // unless the receiver already chose to pull from the device buffer -- and the slot is released
    // only once the copy kernel has finished writing it)
    // (once the FIN is in, the slot may already carry a later message: nothing of r's touches it)
    for (auto it = p->sending.begin(); it != p->sending.end();) {
        mi355x_request *r = *it;
        // >=: the receiver may already have finished the slot's next message too
        const bool fin = r->env->done.load(std::memory_order_acquire) >= r->msg + 1;
        if ((r->env_flags & kEnvDual) && !fin && !r->copy_launched &&
            r->env->claim.load(std::memory_order_acquire) == claim_word(r->msg, 0) && dual_copy_due(r)) {
            if ((p2p_inject() & 1) || dual_copy_launch(c, p, r) != MI355X_SUCCESS) {
                // no host copy: tell a receiver that could not map the device buffer (claim 3) --
                // it tries the mapping once more or fails its receive, and its FIN ends this send
                // (without this both sides waited for each other)
                (void)hipGetLastError();
                r->copy_done = true;
                uint64_t z = claim_word(r->msg, 0);
                (void)r->env->claim.compare_exchange_strong(z, claim_word(r->msg, 3), std::memory_order_acq_rel);
            }
        }
        if ((r->env_flags & kEnvDual) && r->copy_launched && !r->copy_done) {
            const hipError_t e = hipEventQuery(r->ev);
            if (e != hipErrorNotReady) {
                r->copy_done = true;
                uint64_t z = claim_word(r->msg, 0);  // (fails after the FIN: the receiver claimed first)
                if (e == hipSuccess && r->env->claim.compare_exchange_strong(z, claim_word(r->msg, 1), std::memory_order_acq_rel) &&
                    r->twin) {
                    complete(r->twin, MI355X_SUCCESS);
                    r->twin = nullptr;
                } else if (e != hipSuccess) {  // the copy failed: as a failed launch (claim 3)
                    (void)hipGetLastError();
                    (void)r->env->claim.compare_exchange_strong(z, claim_word(r->msg, 3), std::memory_order_acq_rel);
                }
            }
        }
        if (!fin) {
            ++it;
            continue;
        }
        if ((r->env_flags & kEnvDual) && r->copy_launched && !r->copy_done) {
            // delivered (the receiver pulled from the device buffer): the caller completes now; the
            // engine keeps the arena slot until its copy kernel -- whose bytes nobody reads -- is done
            if (r->twin) {
                complete(r->twin, MI355X_SUCCESS);
                r->twin = nullptr;
            }
            ++it;
            continue;
        }
        it = p->sending.erase(it);
        send_done(p, r);
    }
    return MI355X_SUCCESS;
}

// 1 when `buf` is device memory; 0 for host memory (or an empty message)
static int buffer_kind(const void *buf, size_t bytes, int *dev)
{
    *dev = 0;
    if (bytes == 0) return MI355X_SUCCESS;
    if (!buf) return set_error(MI355X_ERR_ARG, "NULL buffer");
    return mi355x_ptr_is_device(buf, dev);
}

static mi355x_request *new_request(mi355x_comm *c, int kind)
{
    auto *r = new mi355x_request();
    r->kind = kind;
    r->comm = c;
    return r;
}

// (kEnvDual, not announced yet) turn r into a plain host-arena send: the copy into its slot now
static int dual_to_host(mi355x_comm *c, P2P *p, mi355x_request *r)
{
    int rc = dual_copy_launch(c, p, r);
    if (rc == MI355X_SUCCESS && hipEventSynchronize(r->ev) != hipSuccess)
        rc = set_error(MI355X_ERR_HIP, "device-to-host copy of a small send failed");
    if (r->ev) {
        p->evpool.push_back(r->ev);
        r->ev = nullptr;
    }
    if (rc) return rc;
    r->env_flags = kEnvHost;
    std::memcpy(&r->desc, &r->hdesc, sizeof(r->desc));
    return MI355X_SUCCESS;
}

// announce r (queue it behind an earlier send to the same destination); the caller's request is
// r, or -- eager -- a completed twin while the engine keeps r until the FIN
static mi355x_request *post_send(mi355x_comm *c, P2P *p, mi355x_request *r, bool eager, bool dual = false)
{
    r->msg = p->send_seq[(size_t)r->peer]++;
    mi355x_request *user = r;
    if (eager || dual) {
        r->internal = true;
        user = new_request(c, 1);
        user->peer = r->peer;
        user->tag = r->tag;
        user->bytes = r->bytes;
        user->mode = r->mode;
        if (dual) r->twin = user;  // completed by progress: host copy taken, or FIN
        else complete(user, MI355X_SUCCESS);
    }
    bool earlier = false;   // an earlier send to the same destination still queued: keep order
    for (mi355x_request *q : p->queued) earlier = earlier || q->peer == r->peer;
    if (!earlier && try_announce(c, r)) {
        p->sending.push_back(r);
        return user;
    }
    if (dual && dual_to_host(c, p, r) == MI355X_SUCCESS) {
        // no envelope free for it now: it cannot be offered two ways, so it takes the host form at
        // once and its caller completes (eager), as every small send must even when the peer's
        // ring is full
        complete(user, MI355X_SUCCESS);
        r->twin = nullptr;
    }
    p->queued.push_back(r);
    return user;
}

// a host payload of >= kStreamMin bytes: announced first, then copied into the arena fragment by
// fragment behind a StreamHdr the receiver polls (the caller holds p->mtx)
static int isend_stream(mi355x_comm *c, P2P *p, mi355x_request *r, bool eager, mi355x_request **out)
{
    void *slot = nullptr;
    BufDesc desc;
    int rc = harena_alloc(c, p, sizeof(StreamHdr) + r->bytes, &slot, &desc);
    if (rc) {
        delete r;
        return rc;
    }
    auto *h = new (slot) StreamHdr();
    h->ready.store(0, std::memory_order_relaxed);
    char *pay = static_cast<char *>(slot) + sizeof(StreamHdr);
    r->hslot = slot;
    r->env_flags = kEnvHost | kEnvStream;
    std::memcpy(&r->desc, &desc, sizeof(desc));
    int64_t first = 0;
    const bool contig = !r->ddt || ddt_contiguous(r->ddt, r->count, &first);
    const char *ubuf = static_cast<const char *>(r->buf) + first;
    // the payload must be complete before the receiver is told: a pack that fails is reported
    // after the fact, so pack into the slot up front when the layout is not contiguous
    if (!contig && (rc = mi355x_pack_host(r->ddt, r->count, r->buf, 0, pay, r->bytes))) {
        harena_release(p);
        delete r;
        return rc;
    }
    if (!contig) h->ready.store(r->bytes, std::memory_order_release);
    *out = post_send(c, p, r, eager);
    if (contig) {
        const size_t frag = stream_frag(r->bytes);
        for (size_t off = 0; off < r->bytes; off += frag) {
            const size_t k = std::min(frag, r->bytes - off);
            std::memcpy(pay + off, ubuf + off, k);
            h->ready.store(off + k, std::memory_order_release);
        }
    }
    return MI355X_SUCCESS;
}

static int isend(mi355x_comm *c, const void *buf, size_t count, const mi355x_ddt_t *d, int dest, int tag, int mode,
                 void *stream, mi355x_request **out)
{
    if (!c || !out) return set_error(MI355X_ERR_ARG, "NULL argument");
    *out = nullptr;
    if (dest != MI355X_PROC_NULL && (dest < 0 || dest >= c->size)) return set_error(MI355X_ERR_ARG, "bad destination %d", dest);
    if (tag == MI355X_ANY_TAG) return set_error(MI355X_ERR_ARG, "a send cannot carry MPI_ANY_TAG");
    if (mode < MI355X_SEND_SYNCHRONOUS || mode > MI355X_SEND_STANDARD) return set_error(MI355X_ERR_ARG, "bad send mode %d", mode);
    const size_t bytes = d ? count * mi355x_ddt_size(d) : count;
    mi355x_request *r = new_request(c, 1);
    r->peer = dest;
    r->tag = tag;
    r->ddt = d;
    r->count = count;
    r->buf = const_cast<void *>(buf);
    r->bytes = bytes;
    r->mode = mode;
    if (dest == MI355X_PROC_NULL) {
        complete(r, MI355X_SUCCESS);
        *out = r;
        return MI355X_SUCCESS;
    }
    int dev = 0;
    int rc = buffer_kind(buf, bytes, &dev);
    if (rc) {
        delete r;
        return rc;
    }
    r->host = !dev;
    DeviceGuard dg(c->device);
    P2P *p = p2p_of(c);
    std::lock_guard<std::recursive_mutex> g(p->mtx);
    auto bail = [&](int code) {
        if (r->packed) arena_release(p->arena);
        if (r->hslot) harena_release(p);
        if (r->ev) (void)hipEventDestroy(r->ev);
        delete r;
        return code;
    };
    // the send buffer is complete once the caller's prior work on `stream` is
    if (bytes && (dev || stream) && hipStreamSynchronize(resolve_stream(stream)) != hipSuccess)
        return bail(set_error(MI355X_ERR_HIP, "caller stream failed"));
    const bool small = bytes <= kEagerLimit && mode != MI355X_SEND_SYNCHRONOUS;
    const bool eager = small || mode == MI355X_SEND_BUFFERED;
    if (!dev && bytes >= stream_min()) return isend_stream(c, p, r, eager, out);
    int64_t first = 0;
    const bool contig = !d || ddt_contiguous(d, count, &first);
    const char *ubuf = (const char *)buf + first;
    if (!dev && bytes && bytes <= kP2PInline && contig && mode != MI355X_SEND_SYNCHRONOUS) {
        // a few host bytes (an MPI scalar, a small header): inside the envelope -- no arena slot,
        // no export; the request holds them until the envelope is posted.  (A device payload goes
        // to the registered arena: one DMA into pinned memory beats a staged copy into the heap.)
        std::memcpy(r->inl, ubuf, bytes);
        r->env_flags = kEnvInline;
        *out = post_send(c, p, r, eager);
        return MI355X_SUCCESS;
    }
    BufDesc desc;
    std::memset(&desc, 0, sizeof(desc));
    hipStream_t s = nullptr;
    // A small device payload is offered two ways at once (kEnvDual): the envelope carries the export
    // of the caller's buffer AND a copy kernel writes the bytes into the sender's registered host
    // arena.  A receiver that matches before the copy is taken pulls straight from the device buffer
    // (one launch on its side, as a rendezvous); otherwise the send completes as soon as the copy is
    // done (eager: both ranks may send first) and the receiver reads the host copy.  One GPU round
    // trip per message where a receiver waits, instead of a device-to-host and a host-to-device copy
    // one after the other.  The copy is launched only if no receiver has claimed the device buffer
    // within MI355X_P2P_DUAL_DELAY_US (10 us) of the announcement (p2p_progress), so a waiting
    // receiver's pull never competes with it.  MI355X_P2P_DUAL=0 keeps the host-arena-only form.
    static const bool dual_on = !(getenv("MI355X_P2P_DUAL") && atoi(getenv("MI355X_P2P_DUAL")) == 0);
    // (MPI_Bsend is local: it keeps the eager host form, never waiting on a receiver's claim)
    if (dual_on && dev && small && contig && bytes && mode != MI355X_SEND_BUFFERED && dest != c->rank && !c->loopback &&
        p->harena.cur.dbase != nullptr) {
        BufDesc hd;
        void *slot = nullptr;
        if ((rc = local_handle(c, ubuf, &desc, false))) return bail(rc);
        if (!desc.staged) {
            desc.raw = (uint64_t)(uintptr_t)ubuf;
            if ((rc = harena_alloc(c, p, bytes, &slot, &hd))) return bail(rc);
            r->hslot = slot;
            if (!p->harena.cur.dbase) return bail(set_error(MI355X_ERR_HIP, "host arena without a device mapping"));
            r->dual_src = ubuf;
            r->dual_t0 = std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
            r->env_flags = kEnvDual;
            r->hoff = hd.off;
            r->hgen = (uint32_t)hd.id;
            std::memcpy(&r->hdesc, &hd, sizeof(hd));
            std::memcpy(&r->desc, &desc, sizeof(desc));
            *out = post_send(c, p, r, false, true);
            return MI355X_SUCCESS;
        }
        std::memset(&desc, 0, sizeof(desc));  // (an allocation of >= ipc_max: the host-arena form)
    }
    if (bytes && (!dev || small)) {
        // the host arena: host payloads of any size, device payloads up to the eager limit
        void *slot = nullptr;
        if ((rc = harena_alloc(c, p, bytes, &slot, &desc))) return bail(rc);
        r->hslot = slot;
        r->env_flags = kEnvHost;
        if (!dev) {
            if (contig) std::memcpy(slot, ubuf, bytes);
            else if ((rc = mi355x_pack_host(d, count, buf, 0, slot, bytes))) return bail(rc);
        } else if (contig) {
            // the copy kernel writes the registered slot through its device mapping: one launch on
            // the point-to-point stream (a DMA-engine copy costs more than a launch for a few KiB)
            char *dslot = p->harena.cur.dbase ? p->harena.cur.dbase + desc.off : nullptr;
            if (dslot && !(rc = p2p_stream(c, p, &s))) {
                MultiCopyArgs m;
                std::memset(&m, 0, sizeof(m));
                m.src[0] = ubuf;
                m.dst[0] = dslot;
                m.len[0] = bytes;
                m.nseg = 1;
                rc = launch_multicopy(m, s);
                if (!rc && hipStreamSynchronize(s) != hipSuccess) rc = set_error(MI355X_ERR_HIP, "device-to-host copy failed");
                if (rc) return bail(rc);
            } else if (hipMemcpy(slot, ubuf, bytes, hipMemcpyDeviceToHost) != hipSuccess) {
                return bail(set_error(MI355X_ERR_HIP, "device-to-host copy of a %zu-byte send failed", bytes));
            }
        } else {
            void *tmp = nullptr;
            if ((rc = p2p_stream(c, p, &s)) || (rc = arena_alloc(p->arena, bytes, &tmp))) return bail(rc);
            rc = mi355x_pack(d, count, buf, 0, tmp, bytes, nullptr, s);
            if (!rc && hipStreamSynchronize(s) != hipSuccess) rc = set_error(MI355X_ERR_HIP, "pack for send failed");
            if (!rc && hipMemcpy(slot, tmp, bytes, hipMemcpyDeviceToHost) != hipSuccess)
                rc = set_error(MI355X_ERR_HIP, "device-to-host copy of a %zu-byte send failed", bytes);
            arena_release(p->arena);
            if (rc) return bail(rc);
        }
    } else if (bytes) {
        // device payload: the caller's buffer itself, or a copy in the exportable device arena
        // (a layout to pack, or a buffered send whose buffer the caller may reuse at once)
        const void *src = ubuf;
        if (!contig || mode == MI355X_SEND_BUFFERED) {
            if ((rc = p2p_stream(c, p, &s))) return bail(rc);
            void *copy = nullptr;
            if ((rc = arena_alloc(p->arena, bytes, &copy))) return bail(rc);
            r->packed = copy;
            if (!contig) {
                r->env_flags = kEnvPacked;
                rc = mi355x_pack(d, count, buf, 0, copy, bytes, nullptr, s);
            } else if (hipMemcpyAsync(copy, ubuf, bytes, hipMemcpyDeviceToDevice, s) != hipSuccess) {
                rc = set_error(MI355X_ERR_HIP, "copy of a buffered send failed");
            }
            if (!rc && hipStreamSynchronize(s) != hipSuccess) rc = set_error(MI355X_ERR_HIP, "pack for send failed");
            if (rc) return bail(rc);
            src = copy;
        }
        if ((rc = local_handle(c, src, &desc, false))) return bail(rc);
        desc.raw = (uint64_t)(uintptr_t)src;
        if (desc.staged == 2 && !c->loopback && dest != c->rank)
            return bail(set_error(MI355X_ERR_HIP, "send buffer could not be exported (hipIpcGetMemHandle failed)"));
        if (desc.staged && !c->loopback && dest != c->rank) {
            const char *env = getenv("MI355X_DMABUF");
            if ((env && atoi(env) == 0) || c->dmabuf_state == -1)
                return bail(set_error(MI355X_ERR_UNSUPPORTED,
                                      "send buffer in an allocation of >= %zu bytes needs the dmabuf export", c->ipc_max));
            if ((rc = export_dmabuf(c, &desc, 1ull << dest))) return bail(rc);
        }
    }
    std::memcpy(&r->desc, &desc, sizeof(desc));
    *out = post_send(c, p, r, eager);
    return MI355X_SUCCESS;
}

// a receive request for (buf, count, d), not posted yet
static int make_recv(mi355x_comm *c, void *buf, size_t count, const mi355x_ddt_t *d, int source, int tag, void *stream,
                     mi355x_request **out)
{
    const size_t bytes = d ? count * mi355x_ddt_size(d) : count;
    mi355x_request *r = new_request(c, 2);
    r->peer = source;
    r->tag = tag;
    r->ddt = d;
    r->count = count;
    r->buf = buf;
    r->bytes = bytes;
    int dev = 0;
    int rc = buffer_kind(buf, bytes, &dev);
    if (rc) {
        delete r;
        return rc;
    }
    r->host = !dev;
    DeviceGuard dg(c->device);
    // (the completion event of a device-side read is created when one starts, start_read: a host
    // payload copied out on the host needs none -- hipEventCreate would be most of its latency)
    // the receive buffer may be written once the caller's prior work on `stream` is done
    if (bytes && (dev || stream) && hipStreamSynchronize(resolve_stream(stream)) != hipSuccess) {
        delete r;
        return set_error(MI355X_ERR_HIP, "caller stream failed");
    }
    *out = r;
    return MI355X_SUCCESS;
}

static int irecv(mi355x_comm *c, void *buf, size_t count, const mi355x_ddt_t *d, int source, int tag, void *stream,
                 mi355x_request **out)
{
    if (!c || !out) return set_error(MI355X_ERR_ARG, "NULL argument");
    *out = nullptr;
    if (source != MI355X_PROC_NULL && source != MI355X_ANY_SOURCE && (source < 0 || source >= c->size))
        return set_error(MI355X_ERR_ARG, "bad source %d", source);
    if (source == MI355X_PROC_NULL) {   // MPI: source PROC_NULL, tag ANY_TAG, count 0
        mi355x_request *r = new_request(c, 2);
        r->peer = source;
        r->tag = tag;
        r->st_source = MI355X_PROC_NULL;
        r->st_tag = MI355X_ANY_TAG;
        complete(r, MI355X_SUCCESS);
        *out = r;
        return MI355X_SUCCESS;
    }
    mi355x_request *r = nullptr;
    int rc = make_recv(c, buf, count, d, source, tag, stream, &r);
    if (rc) return rc;
    P2P *p = p2p_of(c);
    {
        std::lock_guard<std::recursive_mutex> g(p->mtx);
        p->posted.push_back(r);
    }
    p2p_progress(c);
    *out = r;
    return MI355X_SUCCESS;
}

// wait for r, driving this communicator's point-to-point progress
int p2p_wait(mi355x_request *r)
{
    mi355x_comm *c = r->comm;
    const auto t0 = std::chrono::steady_clock::now();
    unsigned spins = 0;
    while (!r->done.load(std::memory_order_acquire)) {
        p2p_progress(c);
        if (r->done.load(std::memory_order_acquire)) break;
        if (++spins > 64) {
            if ((spins & 63) == 0) {
                p2p_progress_all();  // (the other communicators' queued sends)
                run_progress_hook();  // (and the caller's: ob1's requests a peer may need first)
            }
            sched_yield();
            if ((spins & 0x3ff) == 0 &&
                std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > c->timeout_s)
                return set_error(MI355X_ERR_TIMEOUT, "rank %d: %s rank %d (tag %d) not complete after %.0f s",
                                 c->rank, r->kind == 1 ? "send to" : "receive from", r->peer, r->tag, c->timeout_s);
        }
    }
    if (r->rc != MI355X_SUCCESS) return set_error(r->rc, "%s", r->err.c_str());
    return MI355X_SUCCESS;
}

static void fill_status(const mi355x_request *r, mi355x_status_t *st)
{
    if (!st) return;
    st->source = r->st_source;
    st->tag = r->st_tag;
    st->error = r->st_error;
    st->bytes = r->st_bytes;
}

} // namespace mi355x

struct mi355x_message {   // a message taken out of the queue by a matched probe
    mi355x_comm *comm;
    mi355x::P2PMsg m;
};

using namespace mi355x;

extern "C" {

int mi355x_isend(mi355x_comm_t *c, const void *buf, size_t count, const mi355x_ddt_t *d, int dest, int tag,
                 void *stream, mi355x_request_t **req)
{
    return isend(c, buf, count, d, dest, tag, MI355X_SEND_STANDARD, stream, req);
}

int mi355x_isend_mode(mi355x_comm_t *c, const void *buf, size_t count, const mi355x_ddt_t *d, int dest, int tag,
                      int mode, void *stream, mi355x_request_t **req)
{
    return isend(c, buf, count, d, dest, tag, mode, stream, req);
}

int mi355x_irecv(mi355x_comm_t *c, void *buf, size_t count, const mi355x_ddt_t *d, int source, int tag,
                 void *stream, mi355x_request_t **req)
{
    return irecv(c, buf, count, d, source, tag, stream, req);
}

int mi355x_send_mode(mi355x_comm_t *c, const void *buf, size_t count, const mi355x_ddt_t *d, int dest, int tag,
                     int mode, void *stream)
{
    mi355x_request *r = nullptr;
    int rc = isend(c, buf, count, d, dest, tag, mode, stream, &r);
    if (rc) return rc;
    rc = p2p_wait(r);
    if (rc == MI355X_ERR_TIMEOUT) return rc;  // still announced: the request cannot be freed
    (void)mi355x_request_free(r);
    return rc;
}

int mi355x_send(mi355x_comm_t *c, const void *buf, size_t count, const mi355x_ddt_t *d, int dest, int tag,
                void *stream)
{
    return mi355x_send_mode(c, buf, count, d, dest, tag, MI355X_SEND_STANDARD, stream);
}

int mi355x_recv(mi355x_comm_t *c, void *buf, size_t count, const mi355x_ddt_t *d, int source, int tag,
                void *stream, mi355x_status_t *status)
{
    mi355x_request *r = nullptr;
    int rc = irecv(c, buf, count, d, source, tag, stream, &r);
    if (rc) return rc;
    rc = p2p_wait(r);
    if (rc == MI355X_ERR_TIMEOUT) return rc;
    fill_status(r, status);
    (void)mi355x_request_free(r);
    return rc;
}

int mi355x_sendrecv(mi355x_comm_t *c, const void *sbuf, size_t scount, const mi355x_ddt_t *sd, int dest, int stag,
                    void *rbuf, size_t rcount, const mi355x_ddt_t *rd, int source, int rtag, void *stream,
                    mi355x_status_t *status)
{
    mi355x_request *rr = nullptr, *sr = nullptr;
    int rc = irecv(c, rbuf, rcount, rd, source, rtag, stream, &rr);
    if (rc) return rc;
    rc = isend(c, sbuf, scount, sd, dest, stag, MI355X_SEND_STANDARD, stream, &sr);
    if (rc) {
        // the receive stays posted; wait for it so nothing is left behind
        (void)p2p_wait(rr);
        (void)mi355x_request_free(rr);
        return rc;
    }
    int rc_s = p2p_wait(sr);
    int rc_r = p2p_wait(rr);
    fill_status(rr, status);
    if (rc_s != MI355X_ERR_TIMEOUT) (void)mi355x_request_free(sr);
    if (rc_r != MI355X_ERR_TIMEOUT) (void)mi355x_request_free(rr);
    return rc_s ? rc_s : rc_r;
}

static void proc_null_status(mi355x_status_t *status)
{
    if (!status) return;
    status->source = MI355X_PROC_NULL;
    status->tag = MI355X_ANY_TAG;
    status->error = 0;
    status->bytes = 0;
}

int mi355x_iprobe(mi355x_comm_t *c, int source, int tag, int *flag, mi355x_status_t *status)
{
    if (!c || !flag) return set_error(MI355X_ERR_ARG, "NULL argument");
    *flag = 0;
    if (source == MI355X_PROC_NULL) {
        *flag = 1;
        proc_null_status(status);
        return MI355X_SUCCESS;
    }
    p2p_progress(c);
    P2P *p = p2p_of(c);
    std::lock_guard<std::recursive_mutex> g(p->mtx);
    mi355x_request probe;
    probe.peer = source;
    probe.tag = tag;
    for (const P2PMsg &m : p->unexpected)
        if (matches(&probe, m)) {
            *flag = 1;
            if (status) {
                status->source = m.src;
                status->tag = m.env->tag;
                status->error = 0;
                status->bytes = m.env->bytes;
            }
            break;
        }
    return MI355X_SUCCESS;
}

int mi355x_improbe(mi355x_comm_t *c, int source, int tag, int *flag, mi355x_message_t **msg, mi355x_status_t *status)
{
    if (!c || !flag || !msg) return set_error(MI355X_ERR_ARG, "NULL argument");
    *flag = 0;
    *msg = nullptr;
    if (source == MI355X_PROC_NULL) {  // the MPI layer answers this itself (ompi_message_no_proc)
        *flag = 1;
        proc_null_status(status);
        return MI355X_SUCCESS;
    }
    p2p_progress(c);
    P2P *p = p2p_of(c);
    std::lock_guard<std::recursive_mutex> g(p->mtx);
    mi355x_request probe;
    probe.peer = source;
    probe.tag = tag;
    auto it = std::find_if(p->unexpected.begin(), p->unexpected.end(),
                           [&](const P2PMsg &x) { return matches(&probe, x); });
    if (it == p->unexpected.end()) return MI355X_SUCCESS;
    *msg = new mi355x_message{c, *it};
    p->unexpected.erase(it);
    *flag = 1;
    if (status) {
        status->source = (*msg)->m.src;
        status->tag = (*msg)->m.env->tag;
        status->error = 0;
        status->bytes = (*msg)->m.env->bytes;
    }
    return MI355X_SUCCESS;
}

int mi355x_imrecv(mi355x_comm_t *c, void *buf, size_t count, const mi355x_ddt_t *d, mi355x_message_t *msg,
                  void *stream, mi355x_request_t **req)
{
    if (!c || !msg || !req || msg->comm != c) return set_error(MI355X_ERR_ARG, "bad matched receive arguments");
    *req = nullptr;
    mi355x_request *r = nullptr;
    int rc = make_recv(c, buf, count, d, msg->m.src, msg->m.env->tag, stream, &r);
    if (rc) return rc;  // msg stays valid: the caller may retry
    DeviceGuard dg(c->device);
    P2P *p = p2p_of(c);
    {
        std::lock_guard<std::recursive_mutex> g(p->mtx);
        start_read(c, p, r, msg->m);
    }
    delete msg;
    *req = r;
    return MI355X_SUCCESS;
}

int mi355x_request_cancel(mi355x_request_t *r)
{
    if (!r) return set_error(MI355X_ERR_ARG, "NULL request");
    if (r->kind != 2 || r->done.load(std::memory_order_acquire)) return MI355X_SUCCESS;
    P2P *p = p2p_of(r->comm);
    std::lock_guard<std::recursive_mutex> g(p->mtx);
    auto it = std::find(p->posted.begin(), p->posted.end(), r);
    if (it == p->posted.end()) return MI355X_SUCCESS;  // matched already: too late (ob1 likewise)
    p->posted.erase(it);
    r->cancelled = true;
    complete(r, MI355X_SUCCESS);
    return MI355X_SUCCESS;
}

int mi355x_request_cancelled(const mi355x_request_t *r, int *cancelled)
{
    if (!r || !cancelled) return set_error(MI355X_ERR_ARG, "NULL argument");
    *cancelled = r->cancelled ? 1 : 0;
    return MI355X_SUCCESS;
}

int mi355x_p2p_progress(mi355x_comm_t *c)
{
    if (!c) return set_error(MI355X_ERR_ARG, "comm is NULL");
    return p2p_progress(c);
}

int mi355x_request_get_status(const mi355x_request_t *r, mi355x_status_t *status)
{
    if (!r || !status) return set_error(MI355X_ERR_ARG, "NULL argument");
    fill_status(r, status);
    return MI355X_SUCCESS;
}

} // extern "C"
