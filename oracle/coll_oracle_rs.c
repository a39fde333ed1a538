/*
 * coll_oracle_rs.c -- MPI_Reduce_scatter (vector counts) of Open MPI 1.8.5 coll/tuned, simulated
 * over n ranks in one process with real data.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).
 *   non-overlapping    coll_tuned_reduce_scatter.c:60-121 (reduce to 0 + scatterv)
 *   recursive halving  coll_tuned_reduce_scatter.c:141-400
 *   ring               coll_tuned_reduce_scatter.c:466-636
 *   decision           coll_tuned_decision_fixed.c:456-502
 * Each step snapshots what the senders hold before anyone reduces (the blocking send/recv pairs
 * of the reference never let a rank reduce into a range it is sending in the same step).
 */
#include "oracle.h"

#include <stdlib.h>
#include <string.h>

static int pow2_le(int n)
{
    int p = 1;
    while ((p << 1) <= n) p <<= 1;
    return p;
}

static int rs_rechalving(int n, const int *rcounts, int type, int op, const void *const *sbufs,
                         void *const *rbufs)
{
    size_t esz = oracle_type_size(type);
    int *disps = malloc(sizeof(int) * (size_t)n);
    disps[0] = 0;
    for (int i = 0; i < n - 1; ++i) disps[i + 1] = disps[i] + rcounts[i];
    size_t count = (size_t)disps[n - 1] + (size_t)rcounts[n - 1];
    size_t bytes = count * esz;
    char **res = malloc(sizeof(char *) * (size_t)n);
    char **snap = malloc(sizeof(char *) * (size_t)n);
    for (int r = 0; r < n; ++r) {
        res[r] = malloc(bytes + 1);
        snap[r] = malloc(bytes + 1);
        memcpy(res[r], sbufs[r] ? sbufs[r] : rbufs[r], bytes);
    }
    int tmp_size = pow2_le(n), remain = n - tmp_size;
    int *tmp_rank = malloc(sizeof(int) * (size_t)n);
    /* pre-step: even r < 2*remain sends everything to r+1 which reduces result = result (op) recv */
    for (int r = 0; r < n; ++r) {
        if (r < 2 * remain) {
            if ((r & 1) == 0) {
                tmp_rank[r] = -1;
            } else {
                oracle_op_2buff(op, type, res[r - 1], res[r], count);
                tmp_rank[r] = r / 2;
            }
        } else {
            tmp_rank[r] = r - remain;
        }
    }
    int *tmp_rc = malloc(sizeof(int) * (size_t)tmp_size), *tmp_d = malloc(sizeof(int) * (size_t)tmp_size);
    for (int i = 0; i < tmp_size; ++i)
        tmp_rc[i] = (i < remain) ? rcounts[2 * i + 1] + rcounts[2 * i] : rcounts[i + remain];
    tmp_d[0] = 0;
    for (int i = 0; i < tmp_size - 1; ++i) tmp_d[i + 1] = tmp_d[i] + tmp_rc[i];
    int *sidx = calloc((size_t)n, sizeof(int)), *ridx = calloc((size_t)n, sizeof(int));
    int *lidx = malloc(sizeof(int) * (size_t)n);
    for (int r = 0; r < n; ++r) lidx[r] = tmp_size;
    for (int mask = tmp_size >> 1; mask > 0; mask >>= 1) {
        for (int r = 0; r < n; ++r) memcpy(snap[r], res[r], bytes);
        for (int r = 0; r < n; ++r) {
            int tr = tmp_rank[r];
            if (tr < 0) continue;
            int tp = tr ^ mask;
            int peer = (tp < remain) ? tp * 2 + 1 : tp + remain;
            int rlo, rhi;
            if (tr < tp) {
                sidx[r] = ridx[r] + mask;
                rlo = ridx[r];
                rhi = sidx[r];
            } else {
                ridx[r] = sidx[r] + mask;
                rlo = ridx[r];
                rhi = lidx[r];
            }
            int rcount = 0;
            for (int i = rlo; i < rhi; ++i) rcount += tmp_rc[i];
            if (rcount > 0) {
                size_t o = (size_t)tmp_d[rlo] * esz;
                oracle_op_2buff(op, type, snap[peer] + o, res[r] + o, (size_t)rcount);
            }
            sidx[r] = ridx[r];
            lidx[r] = ridx[r] + mask;
        }
    }
    for (int r = 0; r < n; ++r) {
        if (tmp_rank[r] >= 0 && rcounts[r])
            memcpy(rbufs[r], res[r] + (size_t)disps[r] * esz, (size_t)rcounts[r] * esz);
    }
    for (int r = 0; r < 2 * remain; r += 2)
        if (rcounts[r]) memcpy(rbufs[r], res[r + 1] + (size_t)disps[r] * esz, (size_t)rcounts[r] * esz);
    for (int r = 0; r < n; ++r) { free(res[r]); free(snap[r]); }
    free(res); free(snap); free(tmp_rank); free(tmp_rc); free(tmp_d); free(sidx); free(ridx); free(lidx);
    free(disps);
    return 2;
}

static int rs_ring(int n, const int *rcounts, int type, int op, const void *const *sbufs,
                   void *const *rbufs)
{
    size_t esz = oracle_type_size(type);
    int *displs = malloc(sizeof(int) * (size_t)n);
    int total = rcounts[0], maxb = rcounts[0];
    displs[0] = 0;
    for (int i = 1; i < n; ++i) {
        displs[i] = total;
        total += rcounts[i];
        if (rcounts[i] > maxb) maxb = rcounts[i];
    }
    char **acc = malloc(sizeof(char *) * (size_t)n);
    char *msg = malloc((size_t)maxb * esz * (size_t)n + 1), *nxt = malloc((size_t)maxb * esz * (size_t)n + 1);
    int *mb = malloc(sizeof(int) * (size_t)n), *nb = malloc(sizeof(int) * (size_t)n);
    for (int r = 0; r < n; ++r) {
        acc[r] = malloc((size_t)total * esz + 1);
        memcpy(acc[r], sbufs[r] ? sbufs[r] : rbufs[r], (size_t)total * esz);
    }
    /* rank r first sends block r-1 of its accumbuf (:568-577) */
    for (int r = 0; r < n; ++r) {
        int b = (r + n - 1) % n;
        mb[r] = b;
        memcpy(msg + (size_t)r * maxb * esz, acc[r] + (size_t)displs[b] * esz, (size_t)rcounts[b] * esz);
    }
    /* steps k = 2..n: receive block (r - k) from r-1, accum[b] = inbuf (op) accum[b], forward */
    for (int k = 2; k <= n; ++k) {
        for (int r = 0; r < n; ++r) {
            int left = (r + n - 1) % n, b = mb[left];
            char *in = msg + (size_t)left * maxb * esz;
            oracle_op_2buff(op, type, in, acc[r] + (size_t)displs[b] * esz, (size_t)rcounts[b]);
            nb[r] = b;
        }
        for (int r = 0; r < n; ++r) {
            memcpy(nxt + (size_t)r * maxb * esz, acc[r] + (size_t)displs[nb[r]] * esz, (size_t)rcounts[nb[r]] * esz);
            mb[r] = nb[r];
        }
        char *t = msg; msg = nxt; nxt = t;
    }
    for (int r = 0; r < n; ++r) {
        memcpy(rbufs[r], acc[r] + (size_t)displs[r] * esz, (size_t)rcounts[r] * esz);
        free(acc[r]);
    }
    free(acc); free(msg); free(nxt); free(mb); free(nb); free(displs);
    return 3;
}

/* ompi_coll_tuned_reduce_scatter_intra_nonoverlapping (coll_tuned_reduce_scatter.c:60-121):
 * reduce the whole vector to rank 0 through comm->c_coll.coll_reduce (the tuned reduce
 * decision on the total count), then scatterv */
static int rs_nonoverlapping(int n, const int *rcounts, int type, int op, const void *const *sbufs,
                             void *const *rbufs)
{
    size_t total = 0;
    for (int r = 0; r < n; ++r) total += (size_t)rcounts[r];
    const size_t esz = oracle_type_size(type);
    char *full = malloc(total * esz + 1);
    int rc = oracle_reduce(0, n, 0, total, type, op, 0, sbufs, full);
    if (rc < 0) {
        free(full);
        return rc;
    }
    size_t off = 0;
    for (int r = 0; r < n; ++r) {
        memcpy(rbufs[r], full + off * esz, (size_t)rcounts[r] * esz);
        off += (size_t)rcounts[r];
    }
    free(full);
    return 1;
}

int oracle_reduce_scatter(int n, const int *rcounts, int type, int op,
                          const void *const *sbufs, void *const *rbufs)
{
    if (n < 1 || !oracle_has_op(op, type)) return MI355X_ERR_ARG;
    size_t total = 0;
    for (int r = 0; r < n; ++r) total += (size_t)rcounts[r];
    if (total == 0) return 0;
    if (n == 1) {
        memcpy(rbufs[0], sbufs[0] ? sbufs[0] : rbufs[0], total * oracle_type_size(type));
        return 3;
    }
    /* decision_fixed.c:456-502 (commutative) */
    size_t tot_bytes = total * oracle_type_size(type);
    int pow2 = 1;
    while (pow2 < n) pow2 <<= 1;
    if (tot_bytes <= 12 * 1024 || (tot_bytes <= 256 * 1024 && pow2 == n) ||
        (n >= 0.0012 * (double)tot_bytes + 8.0))
        return rs_rechalving(n, rcounts, type, op, sbufs, rbufs);
    return rs_ring(n, rcounts, type, op, sbufs, rbufs);
}

int oracle_reduce_scatter_alg(int alg, int n, const int *rcounts, int type, int op,
                              const void *const *sbufs, void *const *rbufs)
{
    if (alg == 1) return rs_nonoverlapping(n, rcounts, type, op, sbufs, rbufs);
    if (alg == 2) return rs_rechalving(n, rcounts, type, op, sbufs, rbufs);
    if (alg == 3) return rs_ring(n, rcounts, type, op, sbufs, rbufs);
    return oracle_reduce_scatter(n, rcounts, type, op, sbufs, rbufs);
}
