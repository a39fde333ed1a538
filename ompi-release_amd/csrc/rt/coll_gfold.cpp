// coll_gfold.cpp -- the engine's form for the op/hip slots its fold families do not carry.
//
// MPI_LONG_DOUBLE_INT's pairs are 32 bytes, twice the 16-byte vector the engine's fold, pipelined
// and LL kernel families are built around; op/hip reduces them on the GPU (k_wide, exact x87
// compare on the 80-bit encoding).  The engine serves such a slot as gather-then-fold: every
// rank's input is gathered into a per-communicator device buffer (mi355x_allgather's flows, over
// xGMI), then each rank folds the elements it owns with op/hip's 2-buff kernel in coll/basic's
// orders -- reduce / allreduce / reduce_scatter linear (coll_basic_reduce.c:215-250: rbuf =
// r[n-1], then ompi_op_reduce(op, r[i], rbuf) for i = n-2..0; coll/tuned's allreduce and reduce
// algorithm 1), scan / exscan the rank chain (coll_basic_scan.c:84-110, coll_basic_exscan.c:63-104).
// MAXLOC / MINLOC over ordered values give the same bits under every coll/tuned algorithm (the pair
// rule is commutative and associative, ties go to the smaller index); with NaN values the result is
// the basic-linear algorithm's.  Traffic: n x the input per rank (a gather, not a reduce-scatter) --
// this form is for the slots no fold kernel carries, never for the bandwidth path.
#include <cstring>
#include <vector>

#include "coll_internal.hpp"
#include "rt_internal.hpp"

#include "comm_internal.hpp"

#include "coll_comm_int.hpp"

namespace mi355x {

int gather_fold(mi355x_comm *c, const void *in, size_t count, int type, int op, size_t e0, size_t ne, int chain,
                void *dst, hipStream_t s)
{
    const size_t esz = mi355x_type_size(type), bytes = count * esz, n = (size_t)c->size;
    if (bytes == 0) return MI355X_SUCCESS;
    if (c->gf_bytes < n * bytes) {
        if (c->gf_buf) MI_HIP(hipFree(c->gf_buf));
        c->gf_buf = nullptr;
        c->gf_bytes = 0;
        MI_HIP(hipMalloc(&c->gf_buf, n * bytes));
        c->gf_bytes = n * bytes;
    }
    char *g = static_cast<char *>(c->gf_buf);
    int rc = allgather_impl(c, in, g, bytes, s);  // collective; returns with the blocks in place
    if (rc || !dst || ne == 0) return rc;
    auto blk = [&](size_t q) { return g + q * bytes + e0 * esz; };
    if (chain < 0) {  // linear: acc = r[n-1]; acc = r[q] op acc for q = n-2..0
        MI_HIP(hipMemcpyAsync(dst, blk(n - 1), ne * esz, hipMemcpyDeviceToDevice, s));
        for (size_t q = n - 1; q-- > 0;)
            if ((rc = mi355x_op_reduce(op, type, blk(q), dst, ne, s))) return rc;
    } else {  // chain: p = r[0]; p = p op r[k] (the partial is `in`) for k = 1..chain, in the gathered blocks
        for (int k = 1; k <= chain; ++k)
            if ((rc = mi355x_op_reduce(op, type, blk((size_t)k - 1), blk((size_t)k), ne, s))) return rc;
        MI_HIP(hipMemcpyAsync(dst, blk((size_t)chain), ne * esz, hipMemcpyDeviceToDevice, s));
    }
    MI_HIP(hipStreamSynchronize(s));
    return MI355X_SUCCESS;
}

} // namespace mi355x
