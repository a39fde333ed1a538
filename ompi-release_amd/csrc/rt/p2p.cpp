// p2p.cpp -- device point-to-point (MPI_Send / MPI_Recv / MPI_Isend / MPI_Irecv / MPI_Sendrecv /
// MPI_Iprobe) between the ranks of a coll/mi355x communicator.
//
// What it replaces: the reference moves a device message with ob1's RGET protocol over
// btl/smcuda.  The sender registers its buffer (CUDA IPC handle, mpool/rgpusm cache) and sends a
// rendezvous header carrying the handle (pml_ob1_cuda.c:52-100, pml_ob1_sendreq.c RGET start);
// the receiver matches it (pml_ob1_recvfrag.c match loop: per-source order, posted receives in
// posting order, MPI_ANY_SOURCE / MPI_ANY_TAG), opens the handle and copies out of the sender's
// GPU buffer (mca_btl_smcuda_get_cuda, btl_smcuda.c:1083-1168), then returns a FIN so the send
// completes.  Non-contiguous layouts go through the GPU convertor (opal_datatype_cuda.c).
//
// Here, MI355X-first:
//   * the rendezvous header is an Envelope in the communicator's shared control segment: one
//     ring of kP2PSlots per ordered pair (src, dst), filled by src, drained by dst in order
//     (comm_internal.hpp); `full` announces message m, `done` is the FIN;
//   * the sender exports its buffer once (the registration cache of coll_comm.cpp; dmabuf for
//     allocations of 2 GiB or more); a non-contiguous send is first packed by the GPU convertor
//     into the communicator's exportable arena;
//   * the receiver PULLS: one kernel on its own GPU reads the sender's bytes over xGMI and writes
//     them into the receive buffer (k_multicopy for a contiguous receive, the unpack kernel for a
//     derived datatype) -- nothing is ever written into the peer's memory;
//   * progress is polled (mi355x_p2p_progress, the opal_progress hook; test / wait call it):
//     queued sends are announced, mailboxes drained, posted receives matched, finished reads
//     acknowledged, acknowledged sends completed.
// Truncation follows ob1 (pml_ob1_recvreq.h:172-180): the receive gets as many bytes as its
// buffer holds, status.bytes is the message size and status.error MI355X_ERR_TRUNCATE.
#include <sched.h>

#include <algorithm>
#include <chrono>
#include <cstring>

#include "comm_internal.hpp"
#include "ddt_internal.hpp"

namespace mi355x {

struct P2PMsg {   // an announced message not matched yet (ob1's unexpected queue)
    int src;
    uint64_t m;
    Envelope *env;
};

struct P2P {
    std::recursive_mutex mtx;
    hipStream_t stream = nullptr;
    std::vector<uint64_t> send_seq;        // next message number, per destination
    std::vector<uint64_t> recv_seq;        // next message number to drain, per source
    std::deque<P2PMsg> unexpected;         // arrival order (per source: send order)
    std::deque<mi355x_request *> posted;   // receives not matched yet, posting order
    std::deque<mi355x_request *> queued;   // sends waiting for a free envelope, posting order
    std::vector<mi355x_request *> sending; // announced, waiting for the receiver's FIN
    std::vector<mi355x_request *> reading; // matched receives whose pull is in flight
    // exportable arena for packed copies of non-contiguous sends (bump allocated; reset when no
    // packed send is outstanding; never a small allocation, see ensure_scratch)
    char *arena = nullptr;
    size_t arena_bytes = 0, arena_used = 0;
    int arena_users = 0;
    std::vector<void *> retired;
};

static P2P *p2p_of(mi355x_comm *c)
{
    if (!c->p2p) {
        auto *p = new P2P();
        p->send_seq.assign((size_t)c->size, 0);
        p->recv_seq.assign((size_t)c->size, 0);
        c->p2p = p;
    }
    return c->p2p;
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
    if (p->stream) {
        (void)hipStreamSynchronize(p->stream);
        (void)hipStreamDestroy(p->stream);
    }
    for (mi355x_request *r : p->reading)
        if (r->pin) r->pin->pins--;
    if (p->arena) (void)hipFree(p->arena);
    for (void *a : p->retired) (void)hipFree(a);
    delete p;
    c->p2p = nullptr;
}

static int arena_alloc(P2P *p, size_t bytes, void **out)
{
    const size_t need = (bytes + 255) & ~(size_t)255;
    if (p->arena_used + need > p->arena_bytes) {
        if (p->arena) {
            if (p->arena_users > 0) p->retired.push_back(p->arena);  // peers may still read it
            else MI_HIP(hipFree(p->arena));
        }
        p->arena = nullptr;
        size_t want = std::max<size_t>((size_t)8 << 20, p->arena_bytes * 2);
        while (want < need) want *= 2;
        p->arena_bytes = 0;
        p->arena_used = 0;
        MI_HIP(hipMalloc((void **)&p->arena, want));
        p->arena_bytes = want;
    }
    *out = p->arena + p->arena_used;
    p->arena_used += need;
    p->arena_users++;
    return MI355X_SUCCESS;
}

static void arena_release(P2P *p)
{
    if (--p->arena_users > 0) return;
    p->arena_used = 0;
    for (void *a : p->retired) (void)hipFree(a);
    p->retired.clear();
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

// announce send r in its envelope if the slot is free (the message K before it is done)
static bool try_announce(mi355x_comm *c, mi355x_request *r)
{
    Envelope *env = &p2p_ring(c->ctrl, c->size, c->rank, r->peer)[r->msg % kP2PSlots];
    // `done` of a slot only grows (by kP2PSlots per reuse): compare with >=
    if (r->msg >= (uint64_t)kP2PSlots &&
        env->done.load(std::memory_order_acquire) < r->msg - (uint64_t)kP2PSlots + 1)
        return false;
    env->tag = r->tag;
    env->flags = r->packed ? 1 : 0;
    env->bytes = r->bytes;
    std::memcpy(&env->buf, &r->desc, sizeof(BufDesc));
    env->full.store(r->msg + 1, std::memory_order_release);
    r->env = env;
    return true;
}

// matched receive r <- message msg: pull the bytes (or complete at once for an empty message)
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
    auto fail = [&](int rc) {
        env->done.store(msg.m + 1, std::memory_order_release);  // the sender must not hang
        complete(r, rc);
    };
    if (n == 0) {
        env->done.store(msg.m + 1, std::memory_order_release);
        complete_recv(r);
        return;
    }
    const void *src = nullptr;
    if (msg.src == c->rank || c->loopback) {
        src = (const void *)(uintptr_t)(env->buf.raw);
    } else {
        void *mapped = nullptr;
        PeerMap *pm = nullptr;
        int rc = map_peer(c, msg.src, env->buf, &mapped, &pm);
        if (rc) return fail(rc);
        if (pm) {
            pm->pins++;
            r->pin = pm;
        }
        src = mapped;
    }
    hipStream_t s;
    int rc = p2p_stream(c, p, &s);
    if (rc) return fail(rc);
    int64_t first = 0;
    if (!r->ddt || ddt_contiguous(r->ddt, r->count, &first)) {
        MultiCopyArgs m;
        std::memset(&m, 0, sizeof(m));
        m.src[0] = src;
        m.dst[0] = (char *)r->buf + first;
        m.len[0] = n;
        m.nseg = 1;
        rc = launch_multicopy(m, s);
    } else {
        rc = mi355x_unpack(r->ddt, r->count, r->buf, 0, src, n, nullptr, s);
    }
    if (rc == MI355X_SUCCESS && hipEventRecord(r->ev, s) != hipSuccess)
        rc = set_error(MI355X_ERR_HIP, "hipEventRecord on the point-to-point stream failed");
    if (rc) {
        if (r->pin) {
            (void)hipStreamSynchronize(s);
            r->pin->pins--;
            r->pin = nullptr;
        }
        return fail(rc);
    }
    p->reading.push_back(r);
}

static bool matches(const mi355x_request *r, const P2PMsg &m)
{
    return (r->peer == MI355X_ANY_SOURCE || r->peer == m.src) && (r->tag == MI355X_ANY_TAG || r->tag == m.env->tag);
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

int p2p_progress(mi355x_comm *c)
{
    DeviceGuard dg(c->device);
    P2P *p = p2p_of(c);
    std::lock_guard<std::recursive_mutex> g(p->mtx);
    // 1. announce queued sends, in order; a destination whose ring is full holds its later sends
    std::vector<char> blocked((size_t)c->size, 0);
    for (auto it = p->queued.begin(); it != p->queued.end();) {
        mi355x_request *r = *it;
        if (!blocked[(size_t)r->peer] && try_announce(c, r)) {
            p->sending.push_back(r);
            it = p->queued.erase(it);
        } else {
            blocked[(size_t)r->peer] = 1;
            ++it;
        }
    }
    // 2. new envelopes, 3. match posted receives in posting order against the arrivals
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
    // 4. finished pulls: FIN to the sender, receive complete
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
        r->env->done.store(r->msg + 1, std::memory_order_release);
        if (e == hipSuccess) complete_recv(r);
        else complete(r, set_error(MI355X_ERR_HIP, "point-to-point read: %s", hipGetErrorString(e)));
        it = p->reading.erase(it);
    }
    // 5. acknowledged sends
    for (auto it = p->sending.begin(); it != p->sending.end();) {
        mi355x_request *r = *it;
        // >=: the receiver may already have finished the slot's next message too
        if (r->env->done.load(std::memory_order_acquire) < r->msg + 1) {
            ++it;
            continue;
        }
        if (r->packed) arena_release(p);
        r->packed = nullptr;
        complete(r, MI355X_SUCCESS);
        it = p->sending.erase(it);
    }
    return MI355X_SUCCESS;
}

static int check_buffer(const void *buf, size_t bytes)
{
    if (bytes == 0) return MI355X_SUCCESS;
    if (!buf) return set_error(MI355X_ERR_ARG, "NULL buffer");
    int dev = 0;
    int rc = mi355x_ptr_is_device(buf, &dev);
    if (rc) return rc;
    if (!dev) return set_error(MI355X_ERR_ARG, "point-to-point buffers must be device memory");
    return MI355X_SUCCESS;
}

static mi355x_request *new_request(mi355x_comm *c, int kind)
{
    auto *r = new mi355x_request();
    r->kind = kind;
    r->comm = c;
    return r;
}

static int isend(mi355x_comm *c, const void *buf, size_t count, const mi355x_ddt_t *d, int dest, int tag,
                 void *stream, mi355x_request **out)
{
    if (!c || !out) return set_error(MI355X_ERR_ARG, "NULL argument");
    *out = nullptr;
    if (dest != MI355X_PROC_NULL && (dest < 0 || dest >= c->size)) return set_error(MI355X_ERR_ARG, "bad destination %d", dest);
    if (tag < 0) return set_error(MI355X_ERR_ARG, "bad tag %d", tag);
    const size_t bytes = d ? count * mi355x_ddt_size(d) : count;
    mi355x_request *r = new_request(c, 1);
    r->peer = dest;
    r->tag = tag;
    r->ddt = d;
    r->count = count;
    r->buf = const_cast<void *>(buf);
    r->bytes = bytes;
    if (dest == MI355X_PROC_NULL) {
        complete(r, MI355X_SUCCESS);
        *out = r;
        return MI355X_SUCCESS;
    }
    int rc = check_buffer(buf, bytes);
    if (rc) {
        delete r;
        return rc;
    }
    DeviceGuard dg(c->device);
    P2P *p = p2p_of(c);
    std::lock_guard<std::recursive_mutex> g(p->mtx);
    auto bail = [&](int code) {
        if (r->packed) arena_release(p);
        delete r;
        return code;
    };
    // the send buffer is complete once the caller's prior work on `stream` is
    if (bytes && hipStreamSynchronize(resolve_stream(stream)) != hipSuccess)
        return bail(set_error(MI355X_ERR_HIP, "caller stream failed"));
    const void *src = buf;
    int64_t first = 0;
    if (bytes && d && !ddt_contiguous(d, count, &first)) {
        hipStream_t s;
        if ((rc = p2p_stream(c, p, &s))) return bail(rc);
        void *packed = nullptr;
        if ((rc = arena_alloc(p, bytes, &packed))) return bail(rc);
        r->packed = packed;
        if ((rc = mi355x_pack(d, count, buf, 0, packed, bytes, nullptr, s))) return bail(rc);
        if (hipStreamSynchronize(s) != hipSuccess) return bail(set_error(MI355X_ERR_HIP, "pack for send failed"));
        src = packed;
    } else if (bytes) {
        src = (const char *)buf + first;
    }
    BufDesc desc;
    std::memset(&desc, 0, sizeof(desc));
    if (bytes) {
        if ((rc = local_handle(c, src, &desc, false))) return bail(rc);
        desc.raw = (uint64_t)(uintptr_t)src;
        if (desc.staged && !c->loopback && dest != c->rank) {
            const char *env = getenv("MI355X_DMABUF");
            if ((env && atoi(env) == 0) || c->dmabuf_state == -1)
                return bail(set_error(MI355X_ERR_UNSUPPORTED,
                                      "send buffer in an allocation of >= %zu bytes needs the dmabuf export", c->ipc_max));
            if ((rc = export_dmabuf(c, &desc, 1ull << dest))) return bail(rc);
        }
    }
    std::memcpy(&r->desc, &desc, sizeof(desc));
    r->msg = p->send_seq[(size_t)dest]++;
    bool earlier = false;   // an earlier send to the same destination still queued: keep order
    for (mi355x_request *q : p->queued) earlier = earlier || q->peer == dest;
    if (!earlier && try_announce(c, r)) p->sending.push_back(r);
    else p->queued.push_back(r);
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
    if (tag < 0 && tag != MI355X_ANY_TAG) return set_error(MI355X_ERR_ARG, "bad tag %d", tag);
    const size_t bytes = d ? count * mi355x_ddt_size(d) : count;
    mi355x_request *r = new_request(c, 2);
    r->peer = source;
    r->tag = tag;
    r->ddt = d;
    r->count = count;
    r->buf = buf;
    r->bytes = bytes;
    if (source == MI355X_PROC_NULL) {   // MPI: source PROC_NULL, tag ANY_TAG, count 0
        r->st_source = MI355X_PROC_NULL;
        r->st_tag = MI355X_ANY_TAG;
        complete(r, MI355X_SUCCESS);
        *out = r;
        return MI355X_SUCCESS;
    }
    int rc = check_buffer(buf, bytes);
    if (rc) {
        delete r;
        return rc;
    }
    if (hipEventCreateWithFlags(&r->ev, hipEventDisableTiming) != hipSuccess) {
        delete r;
        return set_error(MI355X_ERR_HIP, "hipEventCreate failed");
    }
    // the receive buffer may be written once the caller's prior work on `stream` is done
    if (bytes && hipStreamSynchronize(resolve_stream(stream)) != hipSuccess) {
        (void)hipEventDestroy(r->ev);
        delete r;
        return set_error(MI355X_ERR_HIP, "caller stream failed");
    }
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

using namespace mi355x;

extern "C" {

int mi355x_isend(mi355x_comm_t *c, const void *buf, size_t count, const mi355x_ddt_t *d, int dest, int tag,
                 void *stream, mi355x_request_t **req)
{
    return isend(c, buf, count, d, dest, tag, stream, req);
}

int mi355x_irecv(mi355x_comm_t *c, void *buf, size_t count, const mi355x_ddt_t *d, int source, int tag,
                 void *stream, mi355x_request_t **req)
{
    return irecv(c, buf, count, d, source, tag, stream, req);
}

int mi355x_send(mi355x_comm_t *c, const void *buf, size_t count, const mi355x_ddt_t *d, int dest, int tag,
                void *stream)
{
    mi355x_request *r = nullptr;
    int rc = isend(c, buf, count, d, dest, tag, stream, &r);
    if (rc) return rc;
    rc = p2p_wait(r);
    if (rc == MI355X_ERR_TIMEOUT) return rc;  // still announced: the request cannot be freed
    (void)mi355x_request_free(r);
    return rc;
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
    rc = isend(c, sbuf, scount, sd, dest, stag, stream, &sr);
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

int mi355x_iprobe(mi355x_comm_t *c, int source, int tag, int *flag, mi355x_status_t *status)
{
    if (!c || !flag) return set_error(MI355X_ERR_ARG, "NULL argument");
    *flag = 0;
    if (source == MI355X_PROC_NULL) {
        *flag = 1;
        if (status) {
            status->source = MI355X_PROC_NULL;
            status->tag = MI355X_ANY_TAG;
            status->error = 0;
            status->bytes = 0;
        }
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
