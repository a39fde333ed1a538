/*
 * coll_oracle.c -- single-process simulation of the Open MPI 1.8.5 coll/tuned schedules on the
 * reduction path, driven by the restated op loops of op_oracle.c.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Every simulated rank owns the buffers the reference
 * algorithm would own; a point-to-point message is a memcpy from the sender's buffer as it is at
 * that step (each step takes a snapshot before anybody reduces, which is exactly the ordering the
 * reference's irecv/send/wait sequence enforces).  The op applications use the reference's
 * operand roles: ompi_op_reduce(op, source, target) == oracle_op_2buff(source -> in,
 * target -> inout) (ompi/op/op.h:540-574).
 */
#include "oracle.h"

#include <stdlib.h>
#include <string.h>

#define CHK(x) do { int rc_ = (x); if (rc_ < 0) return rc_; } while (0)

/* COLL_TUNED_COMPUTE_BLOCKCOUNT (coll_tuned.h:546-552) */
static void blockcount(size_t count, int nblocks, size_t *split, size_t *early, size_t *late)
{
    *early = *late = count / (size_t)nblocks;
    *split = count % (size_t)nblocks;
    if (*split != 0) *early += 1;
}

/* block offset of block b (coll_tuned_allreduce.c:459-462 and every later use) */
static size_t block_off(size_t b, size_t split, size_t early, size_t late)
{
    return (b < split) ? b * early : b * late + split;
}
static size_t block_len(size_t b, size_t split, size_t early, size_t late)
{
    return (b < split) ? early : late;
}

/* COLL_TUNED_COMPUTED_SEGCOUNT (coll_tuned.h:525-533) */
static size_t computed_segcount(size_t segsize, size_t typelng, size_t segcount)
{
    if (segsize >= typelng && segsize < typelng * segcount) {
        size_t sc = segsize / typelng;
        size_t residual = segsize - sc * typelng;
        if (residual > (typelng >> 1)) sc++;
        return sc;
    }
    return segcount;
}

static int next_pow2_incl(int v) /* opal_next_poweroftwo_inclusive */
{
    int p = 1;
    while (p < v) p <<= 1;
    return p;
}

/* ------------------------------------------------------------- recursive doubling */
/* coll_tuned_allreduce.c:143-294 */
static int ar_recursive_doubling(int n, size_t count, int type, int op,
                                 const void *const *sbufs, void *const *rbufs)
{
    size_t esz = oracle_type_size(type), bytes = esz * count;
    if (n == 1) {
        if (sbufs[0]) memcpy(rbufs[0], sbufs[0], bytes);
        return ORACLE_AR_RECURSIVE_DOUBLING;
    }
    char **inplace = calloc((size_t)n, sizeof(char *));
    char **tsend = calloc((size_t)n, sizeof(char *));
    char **trecv = calloc((size_t)n, sizeof(char *));
    int *newrank = calloc((size_t)n, sizeof(int));
    char *stage = malloc(bytes ? bytes * (size_t)n : 1);
    for (int r = 0; r < n; ++r) {
        inplace[r] = malloc(bytes ? bytes : 1);
        memcpy(inplace[r], sbufs[r] ? sbufs[r] : rbufs[r], bytes);
        tsend[r] = inplace[r];
        trecv[r] = (char *)rbufs[r];
    }
    /* opal_next_poweroftwo(size) >> 1 (bit_ops.h:115-129): largest power of two <= size */
    int adjsize = next_pow2_incl(n + 1) >> 1;
    int extra = n - adjsize;
    /* pre-step: even r < 2*extra sends to r+1; odd receives and reduces tsend = trecv (op) tsend */
    for (int r = 0; r < n; ++r) {
        if (r < 2 * extra) {
            if (r % 2 == 0) {
                newrank[r] = -1;
            } else {
                memcpy(trecv[r], tsend[r - 1], bytes);
                CHK(oracle_op_2buff(op, type, trecv[r], tsend[r], count));
                newrank[r] = r >> 1;
            }
        } else {
            newrank[r] = r - extra;
        }
    }
    for (int dist = 1; dist < adjsize; dist <<= 1) {
        int *remote = calloc((size_t)n, sizeof(int));
        /* snapshot exchange: everybody receives the partner's tsend first */
        for (int r = 0; r < n; ++r) {
            if (newrank[r] < 0) continue;
            int nr = newrank[r] ^ dist;
            remote[r] = (nr < extra) ? (nr * 2 + 1) : (nr + extra);
            memcpy(stage + (size_t)r * bytes, tsend[remote[r]], bytes);
        }
        for (int r = 0; r < n; ++r) {
            if (newrank[r] < 0) continue;
            memcpy(trecv[r], stage + (size_t)r * bytes, bytes);
            if (r < remote[r]) {
                /* tmprecv = tmpsend (op) tmprecv, then swap (:249-254) */
                CHK(oracle_op_2buff(op, type, tsend[r], trecv[r], count));
                char *t = trecv[r]; trecv[r] = tsend[r]; tsend[r] = t;
            } else {
                /* tmpsend = tmprecv (op) tmpsend (:255-257) */
                CHK(oracle_op_2buff(op, type, trecv[r], tsend[r], count));
            }
        }
        free(remote);
    }
    /* post-step (:265-278) */
    for (int r = 0; r < n; ++r) {
        if (r < 2 * extra && r % 2 == 0) {
            memcpy(rbufs[r], tsend[r + 1], bytes);
            tsend[r] = (char *)rbufs[r];
        }
    }
    for (int r = 0; r < n; ++r) {
        if (tsend[r] != (char *)rbufs[r]) memcpy(rbufs[r], tsend[r], bytes);
        free(inplace[r]);
    }
    free(inplace); free(tsend); free(trecv); free(newrank); free(stage);
    return ORACLE_AR_RECURSIVE_DOUBLING;
}

/* ------------------------------------------------------------- ring / segmented ring */
/* One ring reduce-scatter pass over sub-blocks.  sub(b) gives [offset,len) of the piece of
 * block b handled in this pass.  Rank r first sends piece r; in round j it receives piece
 * (r - j) from rank r-1, reduces rbuf[piece] = rbuf[piece] (op) received, and forwards it.
 * coll_tuned_allreduce.c:459-512 (ring) and :721-831 (segmented, per phase). */
struct piece { size_t off, len; };

static int ring_rs_pass(int n, int type, int op, void *const *rbufs, const struct piece *pc)
{
    size_t esz = oracle_type_size(type), maxlen = 0;
    for (int b = 0; b < n; ++b) if (pc[b].len > maxlen) maxlen = pc[b].len;
    char *msg = malloc(maxlen * esz * (size_t)n + 1), *nxt = malloc(maxlen * esz * (size_t)n + 1);
    int *msgblk = malloc(sizeof(int) * (size_t)n);
    for (int r = 0; r < n; ++r) {
        memcpy(msg + (size_t)r * maxlen * esz, (char *)rbufs[r] + pc[r].off * esz, pc[r].len * esz);
        msgblk[r] = r;
    }
    for (int j = 1; j < n; ++j) {
        for (int r = 0; r < n; ++r) {
            int left = (r + n - 1) % n, b = msgblk[left];
            char *tgt = (char *)rbufs[r] + pc[b].off * esz;
            char *in = msg + (size_t)left * maxlen * esz;
            /* stage a private copy: the receive buffer (inbuf) of rank r */
            memcpy(nxt + (size_t)r * maxlen * esz, in, pc[b].len * esz);
            CHK(oracle_op_2buff(op, type, nxt + (size_t)r * maxlen * esz, tgt, pc[b].len));
        }
        /* what each rank sends next round is the block it just reduced */
        int *nb = malloc(sizeof(int) * (size_t)n);
        for (int r = 0; r < n; ++r) {
            int left = (r + n - 1) % n, b = msgblk[left];
            nb[r] = b;
            memcpy(nxt + (size_t)r * maxlen * esz, (char *)rbufs[r] + pc[b].off * esz,
                   pc[b].len * esz);
        }
        memcpy(msgblk, nb, sizeof(int) * (size_t)n);
        free(nb);
        char *t = msg; msg = nxt; nxt = t;
    }
    free(msg); free(nxt); free(msgblk);
    return 0;
}

/* ring allgather with ranks shifted by one (coll_tuned_allreduce.c:515-541 / :834-860):
 * round k: rank r receives block (r - k) from rank r-1. */
static void ring_allgather_shifted(int n, int type, void *const *rbufs, size_t split, size_t early,
                                   size_t late)
{
    size_t esz = oracle_type_size(type);
    for (int k = 0; k < n - 1; ++k) {
        for (int r = 0; r < n; ++r) {
            int left = (r + n - 1) % n;
            size_t b = (size_t)((r + n - k) % n);
            memcpy((char *)rbufs[r] + block_off(b, split, early, late) * esz,
                   (char *)rbufs[left] + block_off(b, split, early, late) * esz,
                   block_len(b, split, early, late) * esz);
        }
    }
}

static int ar_ring(int n, size_t count, int type, int op, const void *const *sbufs,
                   void *const *rbufs)
{
    size_t esz = oracle_type_size(type);
    if (n == 1) {
        if (sbufs[0]) memcpy(rbufs[0], sbufs[0], count * esz);
        return ORACLE_AR_RING;
    }
    if (count < (size_t)n) return ar_recursive_doubling(n, count, type, op, sbufs, rbufs);
    for (int r = 0; r < n; ++r)
        if (sbufs[r]) memcpy(rbufs[r], sbufs[r], count * esz);
    size_t split, early, late;
    blockcount(count, n, &split, &early, &late);
    struct piece *pc = malloc(sizeof(struct piece) * (size_t)n);
    for (int b = 0; b < n; ++b) {
        pc[b].off = block_off((size_t)b, split, early, late);
        pc[b].len = block_len((size_t)b, split, early, late);
    }
    CHK(ring_rs_pass(n, type, op, rbufs, pc));
    ring_allgather_shifted(n, type, rbufs, split, early, late);
    free(pc);
    return ORACLE_AR_RING;
}

static int ar_ring_segmented(int n, size_t count, int type, int op, uint32_t segsize,
                             const void *const *sbufs, void *const *rbufs)
{
    size_t esz = oracle_type_size(type);
    if (n == 1) {
        if (sbufs[0]) memcpy(rbufs[0], sbufs[0], count * esz);
        return ORACLE_AR_RING_SEGMENTED;
    }
    size_t segcount = computed_segcount(segsize, esz, count);
    if (count < (size_t)n * segcount) return ar_ring(n, count, type, op, sbufs, rbufs);
    /* num_phases (coll_tuned_allreduce.c:685-689) */
    size_t ns = (size_t)n * segcount;
    size_t num_phases = count / ns;
    if ((count % ns >= (size_t)n) && (count % ns > ns / 2)) num_phases++;
    for (int r = 0; r < n; ++r)
        if (sbufs[r]) memcpy(rbufs[r], sbufs[r], count * esz);
    size_t split, early, late;
    blockcount(count, n, &split, &early, &late);
    struct piece *pc = malloc(sizeof(struct piece) * (size_t)n);
    for (size_t ph = 0; ph < num_phases; ++ph) {
        for (int b = 0; b < n; ++b) {
            size_t boff = block_off((size_t)b, split, early, late);
            size_t blen = block_len((size_t)b, split, early, late);
            size_t psplit, pearly, plate;
            blockcount(blen, (int)num_phases, &psplit, &pearly, &plate);
            pc[b].off = boff + block_off(ph, psplit, pearly, plate);
            pc[b].len = block_len(ph, psplit, pearly, plate);
        }
        CHK(ring_rs_pass(n, type, op, rbufs, pc));
    }
    ring_allgather_shifted(n, type, rbufs, split, early, late);
    free(pc);
    return ORACLE_AR_RING_SEGMENTED;
}

int oracle_allreduce_decision(int n, size_t count, int type, uint32_t *segsize_out)
{
    /* coll_tuned_decision_fixed.c:42-85; every predefined op is commutative */
    size_t bytes = oracle_type_size(type) * count;
    if (segsize_out) *segsize_out = 0;
    if (bytes < 10000) return ORACLE_AR_RECURSIVE_DOUBLING;
    if (count > (size_t)n) {
        const size_t seg = 1u << 20;
        if ((size_t)n * seg >= bytes) return ORACLE_AR_RING;
        if (segsize_out) *segsize_out = (uint32_t)seg;
        return ORACLE_AR_RING_SEGMENTED;
    }
    return ORACLE_AR_NONOVERLAPPING;
}

int oracle_ring_fold_order(int n, size_t count, size_t index, int *order)
{
    size_t split, early, late;
    blockcount(count, n, &split, &early, &late);
    size_t b = (index < split * early) ? index / early : split + (index - split * early) / late;
    for (int j = 0; j < n; ++j) order[j] = (int)((b + (size_t)j) % (size_t)n);
    return 0;
}

/* forward declaration; reduce trees live in coll_oracle_reduce.c */
int oracle_bcast_copy(int n, int root, size_t bytes, void *const *bufs);

int oracle_allreduce(int alg, int n, size_t count, int type, int op, uint32_t segsize,
                     const void *const *sbufs, void *const *rbufs)
{
    if (n < 1 || !oracle_has_op(op, type)) return MI355X_ERR_ARG;
    if (alg == ORACLE_AR_DECISION) alg = oracle_allreduce_decision(n, count, type, &segsize);
    switch (alg) {
    case ORACLE_AR_RECURSIVE_DOUBLING:
        return ar_recursive_doubling(n, count, type, op, sbufs, rbufs);
    case ORACLE_AR_RING:
        return ar_ring(n, count, type, op, sbufs, rbufs);
    case ORACLE_AR_RING_SEGMENTED:
        return ar_ring_segmented(n, count, type, op, segsize ? segsize : (1u << 20), sbufs, rbufs);
    case ORACLE_AR_LINEAR:
    case ORACLE_AR_NONOVERLAPPING: {
        /* reduce to rank 0 then bcast (coll_tuned_allreduce.c:84-99, :897-929) */
        size_t bytes = oracle_type_size(type) * count;
        const void **in = malloc(sizeof(void *) * (size_t)n);
        for (int r = 0; r < n; ++r) in[r] = sbufs[r] ? sbufs[r] : rbufs[r];
        /* snapshot in-place inputs before rank 0's rbuf is overwritten */
        void *tmp0 = NULL;
        if (!sbufs[0]) { tmp0 = malloc(bytes ? bytes : 1); memcpy(tmp0, rbufs[0], bytes); in[0] = tmp0; }
        int rc = oracle_reduce(alg == ORACLE_AR_LINEAR ? ORACLE_RED_LINEAR : ORACLE_RED_DECISION,
                               n, 0, count, type, op, 0, in, rbufs[0]);
        free(tmp0); free(in);
        if (rc < 0) return rc;
        oracle_bcast_copy(n, 0, bytes, rbufs);
        return alg;
    }
    default:
        return MI355X_ERR_ARG;
    }
}
