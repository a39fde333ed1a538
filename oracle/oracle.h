/*
 * oracle.h -- CPU restatement of the reference (Open MPI 1.8.5) collective-reduction path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may load liboracle.so, and only as the checker / the timed CPU baseline.  Nothing in
 * ompi-release_amd/ links or calls it.
 *
 * Parity status: the reference's own op loops (ompi/mca/op/base/op_base_functions.c) cannot be
 * compiled here without writing a stand-in for the configure-generated opal_config.h, which
 * the task rules forbid, and the reference holds no op/coll tests or golden vectors
 * (SURVEY.md §4).  The op and coll parts of this oracle are therefore "parity unpinned": they
 * restate the reference expression-for-expression (file:line cited per function) and are
 * checked against the hand-derived known answers in tests/golden/.  The datatype part is pinned
 * by the reference's own known-answer tests test/datatype/{position_noncontig,checksum}.c,
 * restated in tests/test_oracle_ddt.py.
 */
#ifndef MI355X_ORACLE_H
#define MI355X_ORACLE_H

#include <stddef.h>
#include <stdint.h>
#include "../include/mi355x_types.h"

#ifdef __cplusplus
extern "C" {
#endif

/* size in bytes of one element of `type` on this host (x86-64 C ABI); 0 if unknown */
size_t oracle_type_size(int type);
/* 1 if the reference base table (Fortran disabled) has a non-NULL 2-buff fn for (op,type) */
int oracle_has_op(int op, int type);

/* 2-buff: inout[i] = inout[i] (op) in[i]          op_base_functions.c:39-103 */
int oracle_op_2buff(int op, int type, const void *in, void *inout, size_t count);
/* 3-buff: out[i]   = in1[i] (op) in2[i]            op_base_functions.c:606-683 */
int oracle_op_3buff(int op, int type, const void *in1, const void *in2, void *out, size_t count);
/* same loops with multiple host threads (cpu_baseline "all cores" leg) */
int oracle_op_3buff_mt(int op, int type, const void *in1, const void *in2, void *out,
                       size_t count, int nthreads);

/* reference op-table signatures (ompi/mca/op/op.h:253-266), for use as the "base" component
 * in the mini-OMPI harness tests */
typedef void (*oracle_ompi_fn2_t)(void *, void *, int *, void **, void *);
typedef void (*oracle_ompi_fn3_t)(void *, void *, void *, int *, void **, void *);
oracle_ompi_fn2_t oracle_ompi_fn2(int op, int type);
oracle_ompi_fn3_t oracle_ompi_fn3(int op, int type);

/* ---------------- collective schedules (single-process simulation of n ranks) -------------- */

/* algorithm ids, numbered like coll_tuned_allreduce_algorithm (coll_tuned_allreduce.c:46-54) */
enum oracle_allreduce_alg {
    ORACLE_AR_DECISION = 0,          /* ompi_coll_tuned_allreduce_intra_dec_fixed */
    ORACLE_AR_LINEAR = 1,            /* basic linear: reduce to 0 + bcast      (:897-929) */
    ORACLE_AR_NONOVERLAPPING = 2,    /* reduce + bcast                          (:67-100)  */
    ORACLE_AR_RECURSIVE_DOUBLING = 3,/*                                         (:143-294) */
    ORACLE_AR_RING = 4,              /*                                         (:360-554) */
    ORACLE_AR_RING_SEGMENTED = 5     /*                                         (:635-873) */
};

/* MPI_Allreduce over n simulated ranks.  sbufs[r], rbufs[r]: count elements of `type`.
 * sbufs[r] == NULL means MPI_IN_PLACE (input taken from rbufs[r]).  segsize is used only by
 * RING_SEGMENTED (bytes).  Returns the algorithm actually run (after fallbacks) or < 0. */
int oracle_allreduce(int alg, int n, size_t count, int type, int op, uint32_t segsize,
                     const void *const *sbufs, void *const *rbufs);

/* The reference's CPU allreduce (segmented ring over sm-BTL-style 32 KiB shared-memory fragments)
 * run by n concurrent ranks (threads pinned to cores core0..core0+n-1; core0 < 0: unpinned);
 * 1 warm-up + reps timed calls, *sec_per_call = slowest rank's time per call.  segsize 0 = ring.
 * cpu_ring.c; its results equal oracle_allreduce(RING_SEGMENTED / RING). */
int oracle_cpu_allreduce(int n, size_t count, int type, int op, uint32_t segsize, const void *const *sbufs,
                         void *const *rbufs, int reps, int core0, double *sec_per_call);

/* The algorithm ompi_coll_tuned_allreduce_intra_dec_fixed picks (decision_fixed.c:42-85). */
int oracle_allreduce_decision(int n, size_t count, int type, uint32_t *segsize_out);

/* MPI_Reduce (root) over n simulated ranks with the tuned decision (decision_fixed.c:343-446);
 * rbuf used on root only.  Returns the algorithm id run (see oracle_reduce_alg). */
enum oracle_reduce_alg {
    ORACLE_RED_DECISION = 0,
    ORACLE_RED_LINEAR = 1,
    ORACLE_RED_CHAIN = 2,
    ORACLE_RED_PIPELINE = 3,
    ORACLE_RED_BINARY = 4,
    ORACLE_RED_BINOMIAL = 5
};
int oracle_reduce(int alg, int n, int root, size_t count, int type, int op, uint32_t segsize,
                  const void *const *sbufs, void *root_rbuf);
int oracle_reduce_decision(int n, size_t count, int type, uint32_t *segsize_out);
/* same with an explicit chain fanout for ORACLE_RED_CHAIN (oracle_reduce uses the default 4) */
int oracle_reduce_fo(int alg, int n, int root, int chain_fanout, size_t count, int type, int op,
                     const void *const *sbufs, void *root_rbuf);

/* MPI_Reduce_scatter_block as run by coll/basic (coll_basic_reduce_scatter_block.c:54-111):
 * tuned reduce to rank 0 + scatter.  sbufs[r]: n*rcount elems; rbufs[r]: rcount elems. */
int oracle_reduce_scatter_block(int n, size_t rcount, int type, int op,
                                const void *const *sbufs, void *const *rbufs);

/* MPI_Reduce_scatter (vector counts) with the tuned decision (decision_fixed.c:456-502):
 * recursive halving or ring.  Algorithm ids are coll/tuned's (coll_tuned_reduce_scatter.c:46-52):
 * 1 = non-overlapping (reduce to 0 + scatterv), 2 = recursive halving, 3 = ring. */
int oracle_reduce_scatter(int n, const int *rcounts, int type, int op,
                          const void *const *sbufs, void *const *rbufs);
/* same with a forced algorithm (ids above, 0 = decision) */
int oracle_reduce_scatter_alg(int alg, int n, const int *rcounts, int type, int op,
                              const void *const *sbufs, void *const *rbufs);

/* MPI_Scan (exclusive 0) / MPI_Exscan (1) in coll/basic's linear-chain order (coll_oracle_scan.c) */
int oracle_scan(int exclusive, int n, size_t count, int type, int op, const void *const *sbufs,
                void *const *rbufs);

/* ---------------- datatypes / convertor (ddt_oracle.c) ------------------------------------- */
typedef struct oracle_ddt oracle_ddt_t;
oracle_ddt_t *oracle_ddt_contiguous(int64_t count, int64_t elem);
oracle_ddt_t *oracle_ddt_vector(int64_t count, int64_t blocklen, int64_t stride, int64_t elem);
oracle_ddt_t *oracle_ddt_indexed(int count, const int *blocklens, const int *disps, int64_t elem);
oracle_ddt_t *oracle_ddt_struct(int n, const int64_t *disp, const int64_t *len, const int64_t *elem,
                                int64_t extent);
void oracle_ddt_free(oracle_ddt_t *d);
int64_t oracle_ddt_size(const oracle_ddt_t *d);
int64_t oracle_ddt_extent(const oracle_ddt_t *d);
int64_t oracle_ddt_round_position(const oracle_ddt_t *d, int64_t count, int64_t pos);
int oracle_ddt_pack(const oracle_ddt_t *d, int64_t count, const void *base, int64_t pos, void *dst, int64_t bytes);
int oracle_ddt_unpack(const oracle_ddt_t *d, int64_t count, void *base, int64_t pos, const void *src,
                      int64_t bytes);
unsigned long oracle_uicsum_partial(const void *source, size_t csumlen, unsigned int *lastPartialInt,
                                    size_t *lastPartialLength);
uint32_t oracle_ddt_pack_checksum(const oracle_ddt_t *d, int64_t count, const void *base, void *dst);
void oracle_ddt_pack_runs(const oracle_ddt_t *d, int64_t count, const void *base, void *dst);

/* Expression-order description of the allreduce fold actually applied to element `index`:
 * writes the rank fold order into order[0..n-1] for ring / segmented ring (acc starts at
 * order[0]; each later rank's local value is the `out` operand).  Returns 0 if the element's
 * order is a left fold, 1 if the algorithm is a tree (rec. doubling). */
int oracle_ring_fold_order(int n, size_t count, size_t index, int *order);

#ifdef __cplusplus
}
#endif
#endif
