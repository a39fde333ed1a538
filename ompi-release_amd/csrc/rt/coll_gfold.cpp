// coll_gfold.cpp -- the engine's form for the op/hip slots its fold families do not carry.
//
// MPI_LONG_DOUBLE_INT's pairs and MPI_C_LONG_DOUBLE_COMPLEX's values are 32 bytes, twice the
// 16-byte vector the engine's fold, pipelined and LL kernel families are built around; op/hip
// reduces them on the GPU (k_wide_halves: exact x87 compare on the 80-bit encoding, x87 add /
// multiply in integer arithmetic).  The engine serves such a slot as gather-then-fold: every rank's
// input is gathered window by window into a per-communicator device buffer (mi355x_allgather's
// flows, over xGMI), then each rank evaluates the elements it owns with op/hip's 2-buff kernel, in
// the per-element order of the algorithm coll/tuned would run for the call -- the same programs
// the fold kernels evaluate for every other slot (coll_sched.cpp):
//   * MPI_Allreduce: the fixed decision / forced algorithm / dynamic rule (coll_tuned_decision_
//     fixed.c:42-85) with the reference's fallbacks; ring and segmented ring evaluate ring block b
//     with block b's left fold, the local value as `out` and the received partial as `in`
//     (coll_tuned_allreduce.c:470-497); recursive doubling, nonoverlapping and linear their trees;
//   * MPI_Reduce and MPI_Reduce_scatter_block (coll/basic: tuned reduce to 0 + scatter): the reduce
//     tree decision_fixed.c:343-446 picks (coll_tuned_reduce.c:66-361);
//   * MPI_Reduce_scatter: recursive halving / ring / non-overlapping (coll_tuned_reduce_scatter.c);
//   * MPI_Scan / MPI_Exscan: coll/basic's rank chain (coll_basic_scan.c:84-110,
//     coll_basic_exscan.c:63-104).
// The operand roles matter: the pair rule keeps `out` when a compare is unordered (a NaN value,
// op_base_functions.c:96-101), so op2(out = x, in = y) and op2(out = y, in = x) differ there.  A
// program node op2(out = A, in = B) is one 2-buff launch with inout = A's block and in = B's block;
// every leaf appears once in a program, so the gathered blocks are evaluated in place.
// Traffic: n x the input per rank (a gather, not a reduce-scatter) -- this form is for the slots no
// fold kernel carries, never for the bandwidth path.  Memory: n x one window (32 MiB per rank),
// whatever the message size; the buffer grows on the call's stream and is dropped after
// kGfoldIdle without a gather-then-fold call (gfold_idle, from every engine call's CallStream).
#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "coll_internal.hpp"
#include "coll_sched.hpp"
#include "rt_internal.hpp"

#include "comm_internal.hpp"

#include "coll_comm_int.hpp"

namespace mi355x {

namespace {

constexpr double kGfoldIdle = 1.0;  // seconds without a call before the buffer goes

// bytes per rank gathered per window: 32 MiB, or MI355X_GFOLD_WINDOW_KIB (tests; same on every rank)
size_t window_bytes()
{
    const char *e = getenv("MI355X_GFOLD_WINDOW_KIB");
    const long kib = e ? atol(e) : 0;
    return kib > 0 ? (size_t)kib << 10 : (size_t)32 << 20;
}

double now_s()
{
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// one program evaluated over `len` elements of the gathered window: blk(q) = rank q's elements
int eval_program(const Program &pr, int op, int type, char *g, size_t wbytes, size_t lo_bytes, size_t len,
                 char *dst, hipStream_t s)
{
    const size_t esz = mi355x_type_size(type);
    auto blk = [&](int q) { return g + (size_t)q * wbytes + lo_bytes; };
    const char *res;
    int rc;
    if (pr.is_fold) {
        char *acc = blk(pr.order[0]);
        for (size_t j = 1; j < pr.order.size(); ++j) {
            char *x = blk(pr.order[j]);
            if ((pr.role_mask >> j) & 1) {  // op2(out = acc, in = x)
                if ((rc = mi355x_op_reduce(op, type, x, acc, len, s))) return rc;
            } else {                        // op2(out = x, in = acc)
                if ((rc = mi355x_op_reduce(op, type, acc, x, len, s))) return rc;
                acc = x;
            }
        }
        res = acc;
    } else {
        for (const TreeStep &st : pr.steps)  // R[dst = out] = op2(out = R[out], in = R[in])
            if ((rc = mi355x_op_reduce(op, type, blk(st.in), blk(st.out), len, s))) return rc;
        res = blk(pr.result);
    }
    if (dst) MI_HIP(hipMemcpyAsync(dst, res, len * esz, hipMemcpyDeviceToDevice, s));
    return MI355X_SUCCESS;
}

int grow(mi355x_comm *c, size_t need, size_t cap, hipStream_t s)
{
    if (c->gf_bytes >= need) return MI355X_SUCCESS;
    size_t want = std::max(need, std::min(cap, 2 * c->gf_bytes));
    if (c->gf_buf) MI_HIP(hipFreeAsync(c->gf_buf, s));
    c->gf_buf = nullptr;
    c->gf_bytes = 0;
    MI_HIP(hipMallocAsync(&c->gf_buf, want, s));
    c->gf_bytes = want;
    return MI355X_SUCCESS;
}

} // namespace

void gfold_idle(mi355x_comm *c, hipStream_t s)
{
    if (!c->gf_buf || now_s() - c->gf_used < kGfoldIdle) return;
    (void)hipFreeAsync(c->gf_buf, s);
    c->gf_buf = nullptr;
    c->gf_bytes = 0;
}

int gather_fold(mi355x_comm *c, const void *in, size_t count, int type, int op, const std::vector<GfSeg> &segs,
                hipStream_t s)
{
    const size_t esz = mi355x_type_size(type), n = (size_t)c->size;
    if (count == 0) return MI355X_SUCCESS;
    c->gf_used = now_s();
    // A result is written to dst as soon as its window is evaluated.  With MPI_IN_PLACE dst is also
    // an input the peers gather, so every result must land at or before its element's position
    // (true of every caller: the same element, or the rank's block moved to the buffer's start):
    // those positions belong to windows every rank has already gathered.
    const size_t wmax = std::max<size_t>(1, window_bytes() / esz);
    size_t win = wmax;
    const char *ib = static_cast<const char *>(in);
    for (const GfSeg &sg : segs)
        if (sg.dst && sg.ne && sg.dst > ib + sg.e0 * esz && sg.dst < ib + count * esz) win = count;  // (never: one window)
    win = std::min(win, count);
    int rc = grow(c, n * win * esz, n * wmax * esz, s);
    if (rc) return rc;
    char *g = static_cast<char *>(c->gf_buf);
    for (size_t w0 = 0; w0 < count; w0 += win) {
        const size_t w1 = std::min(count, w0 + win), wbytes = (w1 - w0) * esz;
        rc = allgather_impl(c, ib + w0 * esz, g, wbytes, s);  // collective: returns with the blocks in place
        if (rc) return rc;
        for (const GfSeg &sg : segs) {
            const size_t a = std::max(w0, sg.e0), b = std::min(w1, sg.e0 + sg.ne);
            if (a >= b) continue;
            rc = eval_program(sg.pr, op, type, g, wbytes, (a - w0) * esz, b - a,
                              sg.dst ? sg.dst + (a - sg.e0) * esz : nullptr, s);
            if (rc) return rc;
        }
    }
    MI_HIP(hipStreamSynchronize(s));
    c->gf_used = now_s();
    return MI355X_SUCCESS;
}

// ---- the collectives' segments -------------------------------------------------------------------

int gfold_allreduce(mi355x_comm *c, const void *in, void *rbuf, size_t count, int type, int op, hipStream_t s)
{
    const size_t esz = mi355x_type_size(type);
    int alg = pick_allreduce(c, count, esz);
    // the reference's fallbacks (coll_tuned_allreduce.c:672-679, :398-405), as allreduce_impl
    if (alg == AR_RING_SEGMENTED && count < (size_t)c->size * computed_segcount(1u << 20, esz, count)) alg = AR_RING;
    if (alg == AR_RING && count < (size_t)c->size) alg = AR_RECDBL;
    c->last_alg = alg;
    std::vector<GfSeg> segs;
    if (alg == AR_RING || alg == AR_RING_SEGMENTED) {
        for (int b = 0; b < c->size; ++b) {
            GfSeg sg;
            ring_block(count, c->size, b, &sg.e0, &sg.ne);
            sg.pr = ring_block_program(c->size, b);
            sg.dst = static_cast<char *>(rbuf) + sg.e0 * esz;
            segs.push_back(sg);
        }
    } else {
        GfSeg sg;
        sg.e0 = 0;
        sg.ne = count;
        if (!allreduce_tree_program(c, alg, count, esz, &sg.pr)) return set_error(MI355X_ERR_UNSUPPORTED, "schedule too large");
        sg.dst = static_cast<char *>(rbuf);
        segs.push_back(sg);
    }
    return gather_fold(c, in, count, type, op, segs, s);
}

int gfold_reduce(mi355x_comm *c, const void *in, void *rbuf, size_t count, int type, int op, int root, hipStream_t s)
{
    const size_t esz = mi355x_type_size(type);
    GfSeg sg;
    int ra;
    if (!reduce_program(c, count, esz, root, &sg.pr, &ra)) return set_error(MI355X_ERR_UNSUPPORTED, "schedule too large");
    c->last_alg = ra;
    std::vector<GfSeg> segs;
    if (c->rank == root) {
        sg.e0 = 0;
        sg.ne = count;
        sg.dst = static_cast<char *>(rbuf);
        segs.push_back(sg);
    }
    return gather_fold(c, in, count, type, op, segs, s);
}

int gfold_reduce_scatter_block(mi355x_comm *c, const void *in, void *rbuf, size_t rcount, int type, int op,
                               hipStream_t s)
{
    // coll/basic: the tuned reduce of the whole vector to rank 0, then a scatter
    // (coll_basic_reduce_scatter_block.c:54-111)
    const size_t count = rcount * (size_t)c->size, esz = mi355x_type_size(type);
    GfSeg sg;
    int ra;
    if (!reduce_program(c, count, esz, 0, &sg.pr, &ra)) return set_error(MI355X_ERR_UNSUPPORTED, "schedule too large");
    c->last_alg = ra;
    sg.e0 = (size_t)c->rank * rcount;
    sg.ne = rcount;
    sg.dst = static_cast<char *>(rbuf);
    return gather_fold(c, in, count, type, op, std::vector<GfSeg>(1, sg), s);
}

int gfold_reduce_scatter(mi355x_comm *c, const void *in, void *rbuf, const size_t *disp, int type, int op,
                         hipStream_t s)
{
    const size_t count = disp[c->size], esz = mi355x_type_size(type);
    const int alg = pick_reduce_scatter(c, count, esz);
    c->last_alg = alg;
    GfSeg sg;
    if (c->size == 1) {
        sg.pr.is_fold = true;
        sg.pr.order = {0};
        sg.pr.nr = 1;
    } else if (alg == RS_RING) {
        sg.pr = reduce_scatter_ring_block_program(c->size, c->rank);
    } else if (alg == RS_NONOVERLAPPING) {
        int ra;
        if (!reduce_program(c, count, esz, 0, &sg.pr, &ra)) return set_error(MI355X_ERR_UNSUPPORTED, "schedule too large");
    } else {
        ExprPool ep;
        std::vector<int> roots = expr_reduce_scatter_rechalving(ep, c->size);
        if (!compile_expr(ep, roots[c->rank], c->size, &sg.pr)) return set_error(MI355X_ERR_UNSUPPORTED, "schedule too large");
    }
    sg.e0 = disp[c->rank];
    sg.ne = disp[c->rank + 1] - disp[c->rank];
    sg.dst = static_cast<char *>(rbuf);
    return gather_fold(c, in, count, type, op, std::vector<GfSeg>(1, sg), s);
}

int gfold_scan(mi355x_comm *c, const void *in, void *rbuf, size_t count, int type, int op, int last, hipStream_t s)
{
    // coll/basic's chain: p = r[0]; p = op2(out = r[k], in = p) for k = 1..last
    std::vector<GfSeg> segs;
    if (last >= 0) {
        GfSeg sg;
        sg.pr.is_fold = true;
        sg.pr.nr = last + 1;
        for (int k = 0; k <= last; ++k) sg.pr.order.push_back(k);
        sg.pr.role_mask = 0;
        sg.e0 = 0;
        sg.ne = count;
        sg.dst = static_cast<char *>(rbuf);
        segs.push_back(sg);
    }
    c->last_alg = 1;
    return gather_fold(c, in, count, type, op, segs, s);
}

} // namespace mi355x
