// coll_flows.cpp -- the device-buffer collectives' data flows and their public entry points
// (split out of coll_comm.cpp).

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

// MPI_Allreduce (coll_tuned_allreduce_intra_dec_fixed order; sbuf NULL = MPI_IN_PLACE)
int allreduce_impl(mi355x_comm_t *c, const void *sbuf, void *rbuf, size_t count, int type, int op,
                     void *stream)
{
    int rc = check_common(c, op, type);
    if (rc) return rc;
    if (count == 0) return MI355X_SUCCESS;
    hipStream_t s = resolve_stream(stream);
    CallStream call_stream(c, s);  // (the setup work of this call, if any, runs on its stream)
    if (const int rs_ = dev_setup(c)) return rs_;  // (first device-buffer collective: collective setup)
    if (!coll_slot_supported(op, type)) {  // (no fold kernel carries the slot: gather-then-fold, coll_gfold.cpp)
        return gfold_allreduce(c, sbuf ? sbuf : rbuf, rbuf, count, type, op, s);
    }
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
    if (pipe) {
        c->pipe_calls++;
        return pipe_allreduce(c, op, type, pr, P, count, s);
    }
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
int reduce_impl(mi355x_comm_t *c, const void *sbuf, void *rbuf, size_t count, int type, int op, int root,
                  void *stream)
{
    int rc = check_common(c, op, type);
    if (rc) return rc;
    if (root < 0 || root >= c->size) return set_error(MI355X_ERR_ARG, "bad root");
    if (!sbuf && c->rank != root) return set_error(MI355X_ERR_ARG, "MPI_IN_PLACE is only valid at the root");
    if (count == 0) return MI355X_SUCCESS;
    hipStream_t s = resolve_stream(stream);
    CallStream call_stream(c, s);  // (the setup work of this call, if any, runs on its stream)
    if (const int rs_ = dev_setup(c)) return rs_;  // (first device-buffer collective: collective setup)
    if (!coll_slot_supported(op, type)) {  // (no fold kernel carries the slot: gather-then-fold, coll_gfold.cpp)
        return gfold_reduce(c, sbuf ? sbuf : rbuf, rbuf, count, type, op, root, s);
    }
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
int reduce_scatter_block_impl(mi355x_comm_t *c, const void *sbuf, void *rbuf, size_t rcount, int type,
                                int op, void *stream)
{
    int rc = check_common(c, op, type);
    if (rc) return rc;
    const size_t count = rcount * (size_t)c->size;
    if (count == 0) return MI355X_SUCCESS;
    hipStream_t s = resolve_stream(stream);
    CallStream call_stream(c, s);  // (the setup work of this call, if any, runs on its stream)
    if (const int rs_ = dev_setup(c)) return rs_;  // (first device-buffer collective: collective setup)
    if (!coll_slot_supported(op, type)) {  // (no fold kernel carries the slot: gather-then-fold, coll_gfold.cpp)
        return gfold_reduce_scatter_block(c, sbuf ? sbuf : rbuf, rbuf, rcount, type, op, s);
    }
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
int reduce_scatter_impl(mi355x_comm_t *c, const void *sbuf, void *rbuf, const int *rcounts, int type,
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
    CallStream call_stream(c, s);  // (the setup work of this call, if any, runs on its stream)
    if (const int rs_ = dev_setup(c)) return rs_;  // (first device-buffer collective: collective setup)
    if (!coll_slot_supported(op, type)) {  // (no fold kernel carries the slot: gather-then-fold, coll_gfold.cpp)
        return gfold_reduce_scatter(c, sbuf ? sbuf : rbuf, rbuf, disp.data(), type, op, s);
    }
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
int allgather_impl(mi355x_comm_t *c, const void *sbuf, void *rbuf, size_t bytes, void *stream)
{
    if (!c) return set_error(MI355X_ERR_ARG, "comm is NULL");
    if (bytes == 0) return MI355X_SUCCESS;
    hipStream_t s = resolve_stream(stream);
    CallStream call_stream(c, s);  // (the setup work of this call, if any, runs on its stream)
    if (const int rs_ = dev_setup(c)) return rs_;  // (first device-buffer collective: collective setup)
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
int bcast_impl(mi355x_comm_t *c, void *buf, size_t bytes, int root, void *stream)
{
    if (!c) return set_error(MI355X_ERR_ARG, "comm is NULL");
    if (root < 0 || root >= c->size) return set_error(MI355X_ERR_ARG, "bad root");
    if (bytes == 0 || c->size == 1) return MI355X_SUCCESS;
    hipStream_t s = resolve_stream(stream);
    CallStream call_stream(c, s);  // (the setup work of this call, if any, runs on its stream)
    if (const int rs_ = dev_setup(c)) return rs_;  // (first device-buffer collective: collective setup)
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


} // namespace mi355x

using namespace mi355x;

extern "C" {

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
