// coll_staged.cpp -- program launch and the staged data flow (buffers that cannot be
// exported move through each rank's staging buffer) (split out of coll_comm.cpp).

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
int stage_peers(mi355x_comm *c, std::vector<void *> &sp)
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
int staged_reduce(mi355x_comm *c, int op, int type, const Program &pr, const void *in,
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
int staged_allgather(mi355x_comm *c, const void *src, void *rbuf, size_t bytes, hipStream_t s)
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
int staged_bcast(mi355x_comm *c, void *buf, size_t bytes, int root, hipStream_t s)
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

} // namespace mi355x
