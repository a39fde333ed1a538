/*
 * coll_oracle_reduce.c -- MPI_Reduce / MPI_Reduce_scatter_block / MPI_Bcast results of the
 * Open MPI 1.8.5 tuned + basic components, for commutative (= every predefined) ops.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * ompi_coll_tuned_reduce_generic (coll_tuned_reduce.c:66-361) applies, at a tree node with
 * children c0..c(k-1) (tree_next order) and its own data x, for every segment:
 *     k == 1 : acc = c0 (op) x                      (the child's partial is received straight
 *                                                     into accumbuf, :150-160; own data is the
 *                                                     `in` operand, :214-221)
 *     k >= 2 : acc = ((c0 (op) x) (op) c1) ... (op) c(k-1)     (:189-222)
 * with acc always the `out` (target) operand.  Leaves send x unchanged.  Segmentation does not
 * change the per-element order, so a whole-vector evaluation over the tree is exact.
 * Trees: chain (coll_tuned_topo.c:457-603; fanout 1 = pipeline; reduce_intra_chain uses the
 * chain_fanout MCA value, default 4), binary (build_tree(2),
 * :76-189), binomial (build_bmtree, :324-398).  basic_linear (coll_tuned_reduce.c:618-721)
 * is rbuf = x(n-1); rbuf = rbuf (op) x(i) for i = n-2..0 -- the chain's order.
 */
#include "oracle.h"

#include <stdlib.h>
#include <string.h>

#define MAXF 32

struct tnode { int nchild; int child[MAXF]; };

static int pown(int fanout, int num)
{
    int p = 1;
    if (num < 0) return 0;
    for (int j = 0; j < num; ++j) p *= fanout;
    return p;
}
static int calc_level(int fanout, int rank)
{
    int level, num;
    if (rank < 0) return -1;
    for (level = 0, num = 0; num <= rank; level++) num += pown(fanout, level);
    return level - 1;
}

/* children of `rank` in ompi_coll_tuned_topo_build_tree(fanout, comm, root) */
static void tree_children(int fanout, int n, int root, int rank, struct tnode *t)
{
    t->nchild = 0;
    if (n < 2) return;
    int sr = rank - root;
    if (sr < 0) sr += n;
    int level = calc_level(fanout, sr);
    int delta = pown(fanout, level);
    for (int i = 0; i < fanout; ++i) {
        int sc = sr + delta * (i + 1);
        if (sc < n) t->child[t->nchild++] = (sc + root) % n;
        else break;
    }
}

/* children in ompi_coll_tuned_topo_build_bmtree(comm, root) */
static void bmtree_children(int n, int root, int rank, struct tnode *t)
{
    t->nchild = 0;
    int index = rank - root;
    if (index < 0) index += n;
    /* opal_next_poweroftwo(index): smallest power of two strictly greater (1 for 0) */
    int mask = 1;
    while (mask <= index) mask <<= 1;
    while (mask < n) {
        int remote = index ^ mask;
        if (remote >= n) break;
        remote += root;
        if (remote >= n) remote -= n;
        t->child[t->nchild++] = remote;
        mask <<= 1;
    }
}

/* children in ompi_coll_tuned_topo_build_chain(fanout, comm, root) (coll_tuned_topo.c:457-603):
 * the non-root ranks form `fanout` chains hanging off the root; fanout 1 is the pipeline */
static void chain_children(int fanout, int n, int root, int rank, struct tnode *t)
{
    int sr = rank - root;
    if (sr < 0) sr += n;
    t->nchild = 0;
    if (fanout < 1) fanout = 1;
    if (fanout > MAXF) fanout = MAXF;
    if (n - 1 < fanout) fanout = n - 1;
    if (fanout == 1) {
        if (sr + 1 < n) t->child[t->nchild++] = (sr + 1 + root) % n;
        return;
    }
    if (n == 1) return;
    int maxchainlen = (n - 1) / fanout, mark;
    if ((n - 1) % fanout != 0) {
        maxchainlen++;
        mark = (n - 1) % fanout;
    } else {
        mark = fanout + 1;
    }
    if (sr == 0) {
        int next = (root + 1) % n;
        t->child[t->nchild++] = next;
        for (int i = 1; i < fanout; ++i) {
            next = next + maxchainlen;
            if (i > mark) next--;
            next %= n;
            t->child[t->nchild++] = next;
        }
        return;
    }
    int head, len;
    if (sr - 1 < mark * maxchainlen) {
        int column = (sr - 1) / maxchainlen;
        head = 1 + column * maxchainlen;
        len = maxchainlen;
    } else {
        int column = mark + (sr - 1 - mark * maxchainlen) / (maxchainlen - 1);
        head = mark * maxchainlen + 1 + (column - mark) * (maxchainlen - 1);
        len = maxchainlen - 1;
    }
    if (sr != head + len - 1 && sr + 1 < n) t->child[t->nchild++] = (sr + 1 + root) % n;
}

struct rctx {
    int n, type, op;
    size_t count, bytes;
    const void *const *x;
    struct tnode *nodes;
};

/* evaluate the partial result the subtree rooted at r sends upwards, into out */
static int eval_node(struct rctx *c, int r, void *out)
{
    struct tnode *t = &c->nodes[r];
    if (t->nchild == 0) {
        memcpy(out, c->x[r], c->bytes);
        return 0;
    }
    void *tmp = malloc(c->bytes ? c->bytes : 1);
    int rc = eval_node(c, t->child[0], out);            /* acc = c0 */
    if (rc == 0) rc = oracle_op_2buff(c->op, c->type, c->x[r], out, c->count); /* acc (op)= x */
    for (int i = 1; rc == 0 && i < t->nchild; ++i) {
        rc = eval_node(c, t->child[i], tmp);
        if (rc == 0) rc = oracle_op_2buff(c->op, c->type, tmp, out, c->count);   /* acc (op)= ci */
    }
    free(tmp);
    return rc;
}

/* coll_tuned_decision_fixed.c:343-446, commutative branch */
int oracle_reduce_decision(int n, size_t count, int type, uint32_t *segsize_out)
{
    const double a1 = 0.6016 / 1024.0, b1 = 1.3496;
    const double a2 = 0.0410 / 1024.0, b2 = 9.7128;
    const double a3 = 0.0422 / 1024.0, b3 = 1.1614;
    const double a4 = 0.0033 / 1024.0, b4 = 1.6761;
    size_t msg = oracle_type_size(type) * count;
    uint32_t seg = 0;
    int alg;
    if (n < 8 && msg < 512) {
        alg = ORACLE_RED_LINEAR;
    } else if ((n < 8 && msg < 20480) || msg < 2048 || count <= 1) {
        alg = ORACLE_RED_BINOMIAL; seg = 0;
    } else if (n > a1 * (double)msg + b1) {
        alg = ORACLE_RED_BINOMIAL; seg = 1024;
    } else if (n > a2 * (double)msg + b2) {
        alg = ORACLE_RED_PIPELINE; seg = 1024;
    } else if (n > a3 * (double)msg + b3) {
        alg = ORACLE_RED_BINARY; seg = 32 * 1024;
    } else if (n > a4 * (double)msg + b4) {
        alg = ORACLE_RED_PIPELINE; seg = 32 * 1024;
    } else {
        alg = ORACLE_RED_PIPELINE; seg = 64 * 1024;
    }
    if (segsize_out) *segsize_out = seg;
    return alg;
}

int oracle_reduce(int alg, int n, int root, size_t count, int type, int op, uint32_t segsize,
                  const void *const *sbufs, void *root_rbuf)
{
    (void)segsize; /* segmentation does not change the per-element order */
    /* chain fanout: the MCA default ompi_coll_tuned_init_chain_fanout = 4 (coll_tuned_component.c:51) */
    return oracle_reduce_fo(alg, n, root, 4, count, type, op, sbufs, root_rbuf);
}

int oracle_reduce_fo(int alg, int n, int root, int chain_fanout, size_t count, int type, int op,
                     const void *const *sbufs, void *root_rbuf)
{
    if (n < 1 || root < 0 || root >= n || !oracle_has_op(op, type)) return MI355X_ERR_ARG;
    if (alg == ORACLE_RED_DECISION) alg = oracle_reduce_decision(n, count, type, NULL);
    struct rctx c;
    c.n = n; c.type = type; c.op = op; c.count = count;
    c.bytes = oracle_type_size(type) * count;
    c.x = sbufs;
    c.nodes = calloc((size_t)n, sizeof(struct tnode));
    for (int r = 0; r < n; ++r) {
        switch (alg) {
        case ORACLE_RED_LINEAR:
            /* linear folds x(n-1), x(n-2), .., x(0) whatever the root: the order of a
             * fanout-1 chain rooted at rank 0 */
        case ORACLE_RED_PIPELINE:
            chain_children(1, n, alg == ORACLE_RED_LINEAR ? 0 : root, r, &c.nodes[r]);
            break;
        case ORACLE_RED_CHAIN: chain_children(chain_fanout, n, root, r, &c.nodes[r]); break;
        case ORACLE_RED_BINARY: tree_children(2, n, root, r, &c.nodes[r]); break;
        case ORACLE_RED_BINOMIAL: bmtree_children(n, root, r, &c.nodes[r]); break;
        default: free(c.nodes); return MI355X_ERR_ARG;
        }
    }
    int rc = eval_node(&c, alg == ORACLE_RED_LINEAR ? 0 : root, root_rbuf);
    free(c.nodes);
    return rc < 0 ? rc : alg;
}

int oracle_bcast_copy(int n, int root, size_t bytes, void *const *bufs)
{
    for (int r = 0; r < n; ++r)
        if (r != root) memcpy(bufs[r], bufs[root], bytes);
    return 0;
}

/* coll_basic_reduce_scatter_block.c:54-111: reduce(sbuf -> tmp at rank 0) + scatter(tmp) */
int oracle_reduce_scatter_block(int n, size_t rcount, int type, int op,
                                const void *const *sbufs, void *const *rbufs)
{
    size_t esz = oracle_type_size(type), count = rcount * (size_t)n;
    if (count == 0) return 0;
    const void **in = malloc(sizeof(void *) * (size_t)n);
    for (int r = 0; r < n; ++r) in[r] = sbufs[r] ? sbufs[r] : rbufs[r]; /* IN_PLACE: sbuf=rbuf */
    char *tmp = malloc(count * esz);
    int alg = oracle_reduce(ORACLE_RED_DECISION, n, 0, count, type, op, 0, in, tmp);
    if (alg >= 0)
        for (int r = 0; r < n; ++r) memcpy(rbufs[r], tmp + (size_t)r * rcount * esz, rcount * esz);
    free(tmp);
    free(in);
    return alg;
}
