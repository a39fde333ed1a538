// coll_move.cpp -- the remaining collectives of the reduction path's callers on device buffers:
// MPI_Gather(v), MPI_Scatter(v), MPI_Allgatherv, MPI_Alltoall(v) (data movement) and MPI_Scan /
// MPI_Exscan (reductions).  Without them the reference stages every such call through host memory
// (coll/cuda covers only the reductions, coll_cuda_module.c:118-140; everything else goes to
// tuned/basic over the PML, whose device path is ob1 RGET over smcuda).
//
// One data flow for all of them, MI355X-first: every rank publishes its send buffer (the IPC /
// dmabuf registration cache of coll_comm.cpp), meets the others, and PULLS what it must receive
// straight from the owners' memory with one k_multicopy launch (one segment per peer, so every
// xGMI link runs at once), then meets them again so no buffer is reused while a peer still reads
// it.  Counts and displacements a receiver cannot know (scatterv's at the root, alltoallv's
// senders') are published in the control segment next to the buffers.
//
// Scan / Exscan replicate coll/basic's linear chain (coll_basic_scan.c:40-120,
// coll_basic_exscan.c:40-110): rank r's result is ((x0 op x1) op ...) op x_r, each step
// ompi_op_reduce(op, partial, x_k) -- the partial is the `in` operand -- so rank r evaluates that
// left fold over the n inputs directly (k_fold, order 0..r, every step role `in`), bit-identical
// to the chain without its n-1 sequential hops.
#include <cstring>

#include "comm_internal.hpp"
#include "coll_comm_int.hpp"

namespace mi355x {

static int copy_segments(MultiCopyArgs &m, hipStream_t s)
{
    if (m.nseg == 0) return MI355X_SUCCESS;
    return launch_multicopy(m, s);
}

static void add_seg(MultiCopyArgs &m, const void *src, void *dst, size_t len)
{
    if (len == 0 || src == dst) return;
    m.src[m.nseg] = src;
    m.dst[m.nseg] = dst;
    m.len[m.nseg] = len;
    m.nseg++;
}

static int check_comm(mi355x_comm *c, int root)
{
    if (!c) return set_error(MI355X_ERR_ARG, "comm is NULL");
    if (c->size > kMaxSegs) return set_error(MI355X_ERR_UNSUPPORTED, "communicator larger than %d ranks", kMaxSegs);
    if (root < 0 || root >= c->size) return set_error(MI355X_ERR_ARG, "bad root %d", root);
    return MI355X_SUCCESS;
}

// MPI_Gatherv: the root pulls rank q's sbytes into rbuf + displs[q] (at most rcounts[q] bytes).
// sbuf NULL at the root = MPI_IN_PLACE (its block is already in rbuf).
static int gatherv_impl(mi355x_comm *c, const void *sbuf, size_t sbytes, void *rbuf, const size_t *rcounts,
                        const size_t *displs, int root, void *stream)
{
    int rc = check_comm(c, root);
    if (rc) return rc;
    const bool am_root = c->rank == root;
    if (am_root && (!rcounts || !displs)) return set_error(MI355X_ERR_ARG, "gatherv: counts at the root are NULL");
    if (!am_root && !sbuf && sbytes) return set_error(MI355X_ERR_ARG, "MPI_IN_PLACE is only valid at the root");
    hipStream_t s = resolve_stream(stream);
    CallStream call_stream(c, s);
    MI_HIP(hipStreamSynchronize(s));
    c->ctrl->slot[c->rank].varg[0] = (int64_t)(sbuf ? sbytes : 0);
    const void *mine[1] = {sbytes ? sbuf : nullptr};
    const uint64_t sig[4] = {20, (uint64_t)root, 0, 0};
    std::vector<std::vector<void *>> P;
    rc = exchange(c, 1, mine, sig, P);
    if (rc) return rc;
    c->last_alg = 1;
    if (am_root) {
        MultiCopyArgs m;
        std::memset(&m, 0, sizeof(m));
        for (int q = 0; q < c->size; ++q) {
            const size_t qb = (size_t)c->ctrl->slot[q].varg[0];
            if (qb > rcounts[q])
                return set_error(MI355X_ERR_TRUNCATE, "gatherv: rank %d sends %zu bytes, root expects %zu", q, qb,
                                 rcounts[q]);
            if (qb) add_seg(m, P[0][q], (char *)rbuf + displs[q], qb);
        }
        rc = copy_segments(m, s);
        if (rc) return rc;
    }
    return finish(c, s);
}

// MPI_Scatterv: rank r pulls scounts[r] bytes at root's sbuf + displs[r] (both published by the
// root) into rbuf (at most rbytes).  rbuf NULL at the root = MPI_IN_PLACE.
static int scatterv_impl(mi355x_comm *c, const void *sbuf, const size_t *scounts, const size_t *displs, void *rbuf,
                         size_t rbytes, int root, void *stream)
{
    int rc = check_comm(c, root);
    if (rc) return rc;
    const bool am_root = c->rank == root;
    if (am_root && (!scounts || !displs)) return set_error(MI355X_ERR_ARG, "scatterv: counts at the root are NULL");
    if (!am_root && !rbuf && rbytes) return set_error(MI355X_ERR_ARG, "MPI_IN_PLACE is only valid at the root");
    hipStream_t s = resolve_stream(stream);
    CallStream call_stream(c, s);
    MI_HIP(hipStreamSynchronize(s));
    bool any = false;
    if (am_root)
        for (int q = 0; q < c->size; ++q) {
            c->ctrl->slot[c->rank].varg[q] = (int64_t)scounts[q];
            c->ctrl->slot[c->rank].varg[kMaxRanks + q] = (int64_t)displs[q];
            any = any || scounts[q];
        }
    const void *mine[1] = {am_root && any ? sbuf : nullptr};
    const uint64_t sig[4] = {21, (uint64_t)root, 0, 0};
    std::vector<std::vector<void *>> P;
    rc = exchange(c, 1, mine, sig, P);
    if (rc) return rc;
    c->last_alg = 1;
    const RankSlot &rs = c->ctrl->slot[root];
    const size_t len = (size_t)rs.varg[c->rank];
    if (rbuf && len) {
        if (len > rbytes)
            return set_error(MI355X_ERR_TRUNCATE, "scatterv: root sends %zu bytes to rank %d, which expects %zu", len,
                             c->rank, rbytes);
        MultiCopyArgs m;
        std::memset(&m, 0, sizeof(m));
        add_seg(m, (const char *)P[0][root] + rs.varg[kMaxRanks + c->rank], rbuf, len);
        rc = copy_segments(m, s);
        if (rc) return rc;
    }
    return finish(c, s);
}

// MPI_Allgatherv: every rank pulls rank q's block (rcounts[q] bytes) into rbuf + displs[q].
// sbuf NULL = MPI_IN_PLACE (the rank's block is at rbuf + displs[rank]).
static int allgatherv_impl(mi355x_comm *c, const void *sbuf, size_t sbytes, void *rbuf, const size_t *rcounts,
                           const size_t *displs, void *stream)
{
    int rc = check_comm(c, 0);
    if (rc) return rc;
    if (!rcounts || !displs) return set_error(MI355X_ERR_ARG, "allgatherv: counts are NULL");
    hipStream_t s = resolve_stream(stream);
    CallStream call_stream(c, s);
    MI_HIP(hipStreamSynchronize(s));
    const int me = c->rank;
    const void *src = sbuf ? sbuf : (const char *)rbuf + displs[me];
    const size_t mybytes = sbuf ? sbytes : rcounts[me];
    if (mybytes > rcounts[me])
        return set_error(MI355X_ERR_TRUNCATE, "allgatherv: rank %d sends %zu bytes, %zu expected", me, mybytes,
                         rcounts[me]);
    const void *mine[1] = {mybytes ? src : nullptr};
    const uint64_t sig[4] = {22, 0, 0, 0};
    std::vector<std::vector<void *>> P;
    rc = exchange(c, 1, mine, sig, P);
    if (rc) return rc;
    c->last_alg = 1;
    MultiCopyArgs m;
    std::memset(&m, 0, sizeof(m));
    for (int q = 0; q < c->size; ++q)
        if (rcounts[q] && P[0][q]) add_seg(m, P[0][q], (char *)rbuf + displs[q], q == me ? mybytes : rcounts[q]);
    rc = copy_segments(m, s);
    if (rc) return rc;
    return finish(c, s);
}

// MPI_Alltoallv: rank r pulls from rank q the scounts_q[r] bytes at q's sbuf + sdispls_q[r]
// (published by q) into rbuf + rdispls[q] (at most rcounts[q]).  sbuf NULL = MPI_IN_PLACE: the
// data to send is rbuf laid out by rcounts / rdispls, snapshotted into scratch first.
static int alltoallv_impl(mi355x_comm *c, const void *sbuf, const size_t *scounts, const size_t *sdispls, void *rbuf,
                          const size_t *rcounts, const size_t *rdispls, void *stream)
{
    int rc = check_comm(c, 0);
    if (rc) return rc;
    if (!rcounts || !rdispls || (sbuf && (!scounts || !sdispls)))
        return set_error(MI355X_ERR_ARG, "alltoallv: counts are NULL");
    hipStream_t s = resolve_stream(stream);
    CallStream call_stream(c, s);
    const int n = c->size, me = c->rank;
    const void *src = sbuf;
    if (!sbuf) {
        scounts = rcounts;
        sdispls = rdispls;
        size_t extent = 0;
        for (int q = 0; q < n; ++q) extent = std::max(extent, rdispls[q] + rcounts[q]);
        if (extent) {
            rc = ensure_scratch(c, extent);
            if (rc) return rc;
            MI_HIP(hipMemcpyAsync(c->scratch, rbuf, extent, hipMemcpyDeviceToDevice, s));
        }
        src = c->scratch;
    }
    MI_HIP(hipStreamSynchronize(s));
    bool any = false;
    for (int q = 0; q < n; ++q) {
        c->ctrl->slot[me].varg[q] = (int64_t)scounts[q];
        c->ctrl->slot[me].varg[kMaxRanks + q] = (int64_t)sdispls[q];
        any = any || scounts[q];
    }
    const void *mine[1] = {any ? src : nullptr};
    const uint64_t sig[4] = {23, 0, 0, 0};
    std::vector<std::vector<void *>> P;
    rc = exchange(c, 1, mine, sig, P);
    if (rc) return rc;
    c->last_alg = 1;
    MultiCopyArgs m;
    std::memset(&m, 0, sizeof(m));
    for (int k = 0; k < n; ++k) {
        const int q = (me + k) % n;   // own block first, then the peers in ring order
        const RankSlot &qs = c->ctrl->slot[q];
        const size_t len = (size_t)qs.varg[me];
        if (len > rcounts[q])
            return set_error(MI355X_ERR_TRUNCATE, "alltoallv: rank %d sends %zu bytes to rank %d, which expects %zu",
                             q, len, me, rcounts[q]);
        if (len) add_seg(m, (const char *)P[0][q] + qs.varg[kMaxRanks + me], (char *)rbuf + rdispls[q], len);
    }
    rc = copy_segments(m, s);
    if (rc) return rc;
    return finish(c, s);
}

// MPI_Scan (exclusive = false) / MPI_Exscan (true) in coll/basic's order (see the file header).
// sbuf NULL = MPI_IN_PLACE.  Exscan leaves rank 0's rbuf untouched.
static int scan_impl(mi355x_comm *c, const void *sbuf, void *rbuf, size_t count, int type, int op, bool exclusive,
                     void *stream)
{
    int rc = check_common(c, op, type);
    if (rc) return rc;
    if (c->size > kMaxRanks) return set_error(MI355X_ERR_UNSUPPORTED, "communicator larger than %d ranks", kMaxRanks);
    if (count == 0) return MI355X_SUCCESS;
    hipStream_t s = resolve_stream(stream);
    CallStream call_stream(c, s);
    const size_t esz = mi355x_type_size(type);
    const int me = c->rank;
    const void *in = sbuf ? sbuf : rbuf;
    const int last = exclusive ? me - 1 : me;   // fold over ranks 0..last
    if (!coll_slot_supported(op, type)) {  // (no fold kernel carries the slot: gather-then-fold, coll_gfold.cpp)
        return gfold_scan(c, in, rbuf, count, type, op, last, s);
    }
    // in place, rbuf is also an input the later ranks read: the result goes to scratch first
    const bool via_scratch = !sbuf && last >= 0 && !(last == 0 && me == 0);
    if (via_scratch) {
        rc = ensure_scratch(c, count * esz);
        if (rc) return rc;
    }
    MI_HIP(hipStreamSynchronize(s));
    const void *mine[1] = {in};
    const uint64_t sig[4] = {exclusive ? 25u : 24u, count, ((uint64_t)type << 32) | (uint64_t)op, 0};
    std::vector<std::vector<void *>> P;
    rc = exchange(c, 1, mine, sig, P);
    if (rc) return rc;
    c->last_alg = 1;
    void *target = via_scratch ? c->scratch : rbuf;
    if (last == 0) {   // rank 0 of scan, rank 1 of exscan: a copy of x0
        MultiCopyArgs m;
        std::memset(&m, 0, sizeof(m));
        add_seg(m, P[0][0], target, count * esz);
        rc = copy_segments(m, s);
        if (rc) return rc;
    } else if (last > 0) {
        Program pr;
        pr.is_fold = true;
        for (int q = 0; q <= last; ++q) pr.order.push_back(q);
        pr.role_mask = 0;   // ompi_op_reduce(op, partial, x_k): the partial is `in`
        pr.nr = last + 1;
        std::vector<void *> dst(1, target);
        rc = run_program(op, type, pr, P[0], dst, 0, count, s);
        if (rc) return rc;
    }
    rc = finish(c, s);   // every rank has read every input
    if (rc) return rc;
    if (via_scratch) {
        MI_HIP(hipMemcpyAsync(rbuf, c->scratch, count * esz, hipMemcpyDeviceToDevice, s));
        MI_HIP(hipStreamSynchronize(s));
    }
    return MI355X_SUCCESS;
}

} // namespace mi355x

using namespace mi355x;

extern "C" {

int mi355x_gatherv(mi355x_comm_t *c, const void *sbuf, size_t sbytes, void *rbuf, const size_t *rcounts,
                   const size_t *displs, int root, void *stream)
{
    if (!c) return set_error(MI355X_ERR_ARG, "comm is NULL");
    DeviceGuard dg(c->device);
    drain(c);
    CallGate gate(c);
    return gatherv_impl(c, sbuf, sbytes, rbuf, rcounts, displs, root, stream);
}

int mi355x_gather(mi355x_comm_t *c, const void *sbuf, void *rbuf, size_t bytes, int root, void *stream)
{
    if (!c) return set_error(MI355X_ERR_ARG, "comm is NULL");
    std::vector<size_t> cnt((size_t)c->size, bytes), dsp((size_t)c->size);
    for (int q = 0; q < c->size; ++q) dsp[(size_t)q] = (size_t)q * bytes;
    DeviceGuard dg(c->device);
    drain(c);
    CallGate gate(c);
    return gatherv_impl(c, sbuf, bytes, rbuf, cnt.data(), dsp.data(), root, stream);
}

int mi355x_scatterv(mi355x_comm_t *c, const void *sbuf, const size_t *scounts, const size_t *displs, void *rbuf,
                    size_t rbytes, int root, void *stream)
{
    if (!c) return set_error(MI355X_ERR_ARG, "comm is NULL");
    DeviceGuard dg(c->device);
    drain(c);
    CallGate gate(c);
    return scatterv_impl(c, sbuf, scounts, displs, rbuf, rbytes, root, stream);
}

int mi355x_scatter(mi355x_comm_t *c, const void *sbuf, void *rbuf, size_t bytes, int root, void *stream)
{
    if (!c) return set_error(MI355X_ERR_ARG, "comm is NULL");
    std::vector<size_t> cnt((size_t)c->size, bytes), dsp((size_t)c->size);
    for (int q = 0; q < c->size; ++q) dsp[(size_t)q] = (size_t)q * bytes;
    DeviceGuard dg(c->device);
    drain(c);
    CallGate gate(c);
    return scatterv_impl(c, sbuf, cnt.data(), dsp.data(), rbuf, bytes, root, stream);
}

int mi355x_allgatherv(mi355x_comm_t *c, const void *sbuf, size_t sbytes, void *rbuf, const size_t *rcounts,
                      const size_t *displs, void *stream)
{
    if (!c) return set_error(MI355X_ERR_ARG, "comm is NULL");
    DeviceGuard dg(c->device);
    drain(c);
    CallGate gate(c);
    return allgatherv_impl(c, sbuf, sbytes, rbuf, rcounts, displs, stream);
}

int mi355x_alltoallv(mi355x_comm_t *c, const void *sbuf, const size_t *scounts, const size_t *sdispls, void *rbuf,
                     const size_t *rcounts, const size_t *rdispls, void *stream)
{
    if (!c) return set_error(MI355X_ERR_ARG, "comm is NULL");
    DeviceGuard dg(c->device);
    drain(c);
    CallGate gate(c);
    return alltoallv_impl(c, sbuf, scounts, sdispls, rbuf, rcounts, rdispls, stream);
}

int mi355x_alltoall(mi355x_comm_t *c, const void *sbuf, void *rbuf, size_t bytes, void *stream)
{
    if (!c) return set_error(MI355X_ERR_ARG, "comm is NULL");
    std::vector<size_t> cnt((size_t)c->size, bytes), dsp((size_t)c->size);
    for (int q = 0; q < c->size; ++q) dsp[(size_t)q] = (size_t)q * bytes;
    DeviceGuard dg(c->device);
    drain(c);
    CallGate gate(c);
    return alltoallv_impl(c, sbuf, cnt.data(), dsp.data(), rbuf, cnt.data(), dsp.data(), stream);
}

int mi355x_scan(mi355x_comm_t *c, const void *sbuf, void *rbuf, size_t count, int type, int op, void *stream)
{
    if (!c) return set_error(MI355X_ERR_ARG, "comm is NULL");
    DeviceGuard dg(c->device);
    drain(c);
    CallGate gate(c);
    return scan_impl(c, sbuf, rbuf, count, type, op, false, stream);
}

int mi355x_exscan(mi355x_comm_t *c, const void *sbuf, void *rbuf, size_t count, int type, int op, void *stream)
{
    if (!c) return set_error(MI355X_ERR_ARG, "comm is NULL");
    DeviceGuard dg(c->device);
    drain(c);
    CallGate gate(c);
    return scan_impl(c, sbuf, rbuf, count, type, op, true, stream);
}

int mi355x_iscan(mi355x_comm_t *c, const void *sbuf, void *rbuf, size_t count, int type, int op, void *stream,
                 mi355x_request_t **req)
{
    int rc = check_common(c, op, type);
    if (rc) return rc;
    return post(c, stream, [=](hipStream_t s) { return scan_impl(c, sbuf, rbuf, count, type, op, false, s); }, req);
}

int mi355x_ialltoall(mi355x_comm_t *c, const void *sbuf, void *rbuf, size_t bytes, void *stream,
                     mi355x_request_t **req)
{
    if (!c) return set_error(MI355X_ERR_ARG, "comm is NULL");
    return post(c, stream,
                [=](hipStream_t s) {
                    std::vector<size_t> cnt((size_t)c->size, bytes), dsp((size_t)c->size);
                    for (int q = 0; q < c->size; ++q) dsp[(size_t)q] = (size_t)q * bytes;
                    return alltoallv_impl(c, sbuf, cnt.data(), dsp.data(), rbuf, cnt.data(), dsp.data(), s);
                },
                req);
}

} // extern "C"
