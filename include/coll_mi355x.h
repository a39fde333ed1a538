/*
 * coll_mi355x.h -- the coll/mi355x MCA component (lib/mca_coll_mi355x.so).
 *
 * Plugs into the coll framework (ompi/mca/coll/coll.h:357-451) at priority 90 -- above
 * coll/tuned (30) and coll/cuda (78) -- for intra-communicators whose ranks all live on this
 * node.  It provides allreduce, reduce, reduce_scatter, reduce_scatter_block, allgather, bcast,
 * gather(v), scatter(v), allgatherv, alltoall(v), scan and exscan, and the nonblocking iallreduce,
 * ireduce, ireduce_scatter_block, iallgather and ibcast; every other slot (alltoallw, barrier,
 * the other nonblocking and neighborhood ones) stays with the lower-priority modules.  Entry points have exactly the reference
 * signatures (coll.h:181-239) and replace, for device buffers:
 *   mca_coll_cuda_allreduce            (ompi/mca/coll/cuda/coll_cuda_allreduce.c:30-77)
 *   mca_coll_cuda_reduce_scatter_block (coll_cuda_reduce_scatter_block.c:34-83)
 *   ompi_coll_tuned_*_intra_dec_fixed  (coll_tuned_decision_fixed.c) reached on device buffers,
 *                                      incl. ompi_coll_tuned_reduce_intra_dec_fixed (:343-446)
 * with results identical to the tuned/basic schedules (same per-element operand order).
 *
 * Host buffers, user-defined ops and types the engine has no fold for go to the function that
 * was installed in the slot before this module (snapshotted at enable time, retained, as coll/cuda
 * does at coll_cuda_module.c:120-157) -- with every device buffer of such a call staged through
 * host memory around it, as coll/cuda stages every call it intercepts
 * (coll_cuda_allreduce.c:43-75, coll_cuda_reduce_scatter_block.c:45-83).
 *
 * Host facts the component reads from the Open MPI 1.8 launcher environment:
 *   OMPI_COMM_WORLD_SIZE / OMPI_COMM_WORLD_LOCAL_SIZE  (orte/mca/ess/base/ess_base_put.c:76,87)
 *     -> the job is single-node (else the component declines);
 *   OMPI_COMM_WORLD_LOCAL_RANK (orte/mca/odls/base/odls_base_default_fns.c:863) -> GPU index;
 *   OMPI_MCA_ess_base_jobid (:817) + the communicator's c_contextid -> node-unique rendezvous key.
 * The mini-OMPI harness (libompi_mini) sets the same variables.
 */
#ifndef MI355X_COLL_MI355X_H
#define MI355X_COLL_MI355X_H

#include "ompi_abi.h"

#ifdef __cplusplus
extern "C" {
#endif

extern mca_coll_base_component_t mca_coll_mi355x_component;

int mca_coll_mi355x_allreduce(void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                              struct ompi_op_t *op, struct ompi_communicator_t *comm,
                              mca_coll_base_module_t *module);
int mca_coll_mi355x_reduce(void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                           int root, struct ompi_communicator_t *comm, mca_coll_base_module_t *module);
/* nonblocking (coll.h:241-356; reference: coll/libnbc) */
int mca_coll_mi355x_iallreduce(void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                               struct ompi_communicator_t *comm, ompi_request_t **request,
                               mca_coll_base_module_t *module);
int mca_coll_mi355x_ireduce(void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                            int root, struct ompi_communicator_t *comm, ompi_request_t **request,
                            mca_coll_base_module_t *module);
int mca_coll_mi355x_ireduce_scatter_block(void *sbuf, void *rbuf, int rcount, struct ompi_datatype_t *dtype,
                                          struct ompi_op_t *op, struct ompi_communicator_t *comm,
                                          ompi_request_t **request, mca_coll_base_module_t *module);
int mca_coll_mi355x_iallgather(void *sbuf, int scount, struct ompi_datatype_t *sdtype, void *rbuf, int rcount,
                               struct ompi_datatype_t *rdtype, struct ompi_communicator_t *comm,
                               ompi_request_t **request, mca_coll_base_module_t *module);
int mca_coll_mi355x_ibcast(void *buff, int count, struct ompi_datatype_t *datatype, int root,
                           struct ompi_communicator_t *comm, ompi_request_t **request, mca_coll_base_module_t *module);
int mca_coll_mi355x_reduce_scatter_block(void *sbuf, void *rbuf, int rcount, struct ompi_datatype_t *dtype,
                                         struct ompi_op_t *op, struct ompi_communicator_t *comm,
                                         mca_coll_base_module_t *module);
int mca_coll_mi355x_reduce_scatter(void *sbuf, void *rbuf, int *rcounts, struct ompi_datatype_t *dtype,
                                   struct ompi_op_t *op, struct ompi_communicator_t *comm,
                                   mca_coll_base_module_t *module);
int mca_coll_mi355x_allgather(void *sbuf, int scount, struct ompi_datatype_t *sdtype, void *rbuf, int rcount,
                              struct ompi_datatype_t *rdtype, struct ompi_communicator_t *comm,
                              mca_coll_base_module_t *module);
int mca_coll_mi355x_bcast(void *buff, int count, struct ompi_datatype_t *datatype, int root,
                          struct ompi_communicator_t *comm, mca_coll_base_module_t *module);

/* the callers either side of the reduction path (coll.h:185-238; reference: coll/tuned, coll/basic
 * over the PML); dense datatypes on device buffers, everything else to the previous owner */
int mca_coll_mi355x_gather(void *sbuf, int scount, struct ompi_datatype_t *sdtype, void *rbuf, int rcount,
                           struct ompi_datatype_t *rdtype, int root, struct ompi_communicator_t *comm,
                           mca_coll_base_module_t *module);
int mca_coll_mi355x_gatherv(void *sbuf, int scount, struct ompi_datatype_t *sdtype, void *rbuf, int *rcounts,
                            int *disps, struct ompi_datatype_t *rdtype, int root, struct ompi_communicator_t *comm,
                            mca_coll_base_module_t *module);
int mca_coll_mi355x_scatter(void *sbuf, int scount, struct ompi_datatype_t *sdtype, void *rbuf, int rcount,
                            struct ompi_datatype_t *rdtype, int root, struct ompi_communicator_t *comm,
                            mca_coll_base_module_t *module);
int mca_coll_mi355x_scatterv(void *sbuf, int *scounts, int *disps, struct ompi_datatype_t *sdtype, void *rbuf,
                             int rcount, struct ompi_datatype_t *rdtype, int root, struct ompi_communicator_t *comm,
                             mca_coll_base_module_t *module);
int mca_coll_mi355x_allgatherv(void *sbuf, int scount, struct ompi_datatype_t *sdtype, void *rbuf, int *rcounts,
                               int *disps, struct ompi_datatype_t *rdtype, struct ompi_communicator_t *comm,
                               mca_coll_base_module_t *module);
int mca_coll_mi355x_alltoall(void *sbuf, int scount, struct ompi_datatype_t *sdtype, void *rbuf, int rcount,
                             struct ompi_datatype_t *rdtype, struct ompi_communicator_t *comm,
                             mca_coll_base_module_t *module);
int mca_coll_mi355x_alltoallv(void *sbuf, int *scounts, int *sdisps, struct ompi_datatype_t *sdtype, void *rbuf,
                              int *rcounts, int *rdisps, struct ompi_datatype_t *rdtype,
                              struct ompi_communicator_t *comm, mca_coll_base_module_t *module);
/* MPI_Scan / MPI_Exscan in coll/basic's chain order (coll_basic_scan.c, coll_basic_exscan.c) */
int mca_coll_mi355x_scan(void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                         struct ompi_communicator_t *comm, mca_coll_base_module_t *module);
int mca_coll_mi355x_exscan(void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                           struct ompi_communicator_t *comm, mca_coll_base_module_t *module);

/* Point-to-point through the PML slot: installed over the selected PML's table (`mca_pml`,
 * pml.h:558) when the component is initialised, the way pml/v parasites the host PML
 * (pml_v_component.c:110-131).  On a communicator with the engine EVERY point-to-point call goes to
 * the engine -- device and host buffers, every send mode, persistent and matched-probe requests --
 * so all of its messages share one matching queue, as ob1's do (pml_ob1_cuda.c:52-100,
 * pml_ob1_recvreq.c:647-663, pml_ob1_recvfrag.c:487); other communicators keep the saved entries.
 * Each function has the signature of the pml.h:146-470 slot it fills.
 * OMPI_MCA_coll_mi355x_pml_hook=0 leaves the PML untouched. */
int mca_coll_mi355x_pml_isend(void *buf, size_t count, struct ompi_datatype_t *dt, int dst, int tag,
                              mca_pml_base_send_mode_t mode, struct ompi_communicator_t *comm,
                              ompi_request_t **request);
int mca_coll_mi355x_pml_send(void *buf, size_t count, struct ompi_datatype_t *dt, int dst, int tag,
                             mca_pml_base_send_mode_t mode, struct ompi_communicator_t *comm);
int mca_coll_mi355x_pml_irecv(void *buf, size_t count, struct ompi_datatype_t *dt, int src, int tag,
                              struct ompi_communicator_t *comm, ompi_request_t **request);
int mca_coll_mi355x_pml_recv(void *buf, size_t count, struct ompi_datatype_t *dt, int src, int tag,
                             struct ompi_communicator_t *comm, ompi_status_public_t *status);
int mca_coll_mi355x_pml_iprobe(int src, int tag, struct ompi_communicator_t *comm, int *matched,
                               ompi_status_public_t *status);
int mca_coll_mi355x_pml_probe(int src, int tag, struct ompi_communicator_t *comm, ompi_status_public_t *status);
int mca_coll_mi355x_pml_improbe(int src, int tag, struct ompi_communicator_t *comm, int *matched,
                                struct ompi_message_t **message, ompi_status_public_t *status);
int mca_coll_mi355x_pml_mprobe(int src, int tag, struct ompi_communicator_t *comm, struct ompi_message_t **message,
                               ompi_status_public_t *status);
int mca_coll_mi355x_pml_imrecv(void *buf, size_t count, struct ompi_datatype_t *dt, struct ompi_message_t **message,
                               ompi_request_t **request);
int mca_coll_mi355x_pml_mrecv(void *buf, size_t count, struct ompi_datatype_t *dt, struct ompi_message_t **message,
                              ompi_status_public_t *status);
int mca_coll_mi355x_pml_isend_init(void *buf, size_t count, struct ompi_datatype_t *dt, int dst, int tag,
                                   mca_pml_base_send_mode_t mode, struct ompi_communicator_t *comm,
                                   ompi_request_t **request);
int mca_coll_mi355x_pml_irecv_init(void *buf, size_t count, struct ompi_datatype_t *dt, int src, int tag,
                                   struct ompi_communicator_t *comm, ompi_request_t **request);
int mca_coll_mi355x_pml_start(size_t count, ompi_request_t **requests);

/* MCA parameters coll_mi355x_<name>: registered with mca_base_component_var_register when the
 * component is loaded by an Open MPI that provides it, else read from OMPI_MCA_coll_mi355x_<name> */
extern int mca_coll_mi355x_priority;            /* 90 */
extern int mca_coll_mi355x_allreduce_algorithm; /* 0 = tuned decision, else coll_tuned numbering */
extern int mca_coll_mi355x_pml_hook;            /* 1 = point-to-point on engine communicators through the engine */
extern int mca_coll_mi355x_mixed_buffers;       /* 1 = ranks may mix host and device buffers in a call */
extern int mca_coll_mi355x_rcache_max_maps;     /* peer mappings kept open per communicator (0 = unlimited) */
extern unsigned long long mca_coll_mi355x_rcache_size_limit; /* the same in bytes (mpool_rgpusm_rcache_size_limit) */
/* the engine's crossovers and flow parameters (MI355X_KNOB_* on every communicator's engine) */
extern int mca_coll_mi355x_pipe_min_ranks;               /* 4: pipelined allreduce from this many ranks (0 never) */
extern int mca_coll_mi355x_pipe_chunk_kib;               /* 0: auto */
extern int mca_coll_mi355x_pipe_wg_per_cu;               /* 2 */
extern int mca_coll_mi355x_pipe_wt;                      /* 1: write-through fold results */
extern unsigned long long mca_coll_mi355x_one_phase_max; /* 1 MiB */
extern unsigned long long mca_coll_mi355x_svc_max;       /* 32 KiB */
extern unsigned long long mca_coll_mi355x_svc_pull_max;  /* 128 KiB */
extern unsigned long long mca_coll_mi355x_svc_copy_max;  /* 1 MiB */
extern int mca_coll_mi355x_svc_idle_us;                  /* 1000 */
extern int mca_coll_mi355x_svc_shrink_us;                /* 100 */
extern int mca_coll_mi355x_selftest;                     /* 1 */
/* the engine of a communicator coll/mi355x serves (NULL otherwise): for tools and tests */
struct mi355x_comm *mca_coll_mi355x_engine_of(struct ompi_communicator_t *comm);

/* Reductions the engine declines (user-defined ops; types with no engine slot) go to the
 * lower-priority component with every device buffer staged through host memory, as coll/cuda does
 * (coll_cuda_allreduce.c:43-75): this counts those staged calls. */
extern unsigned long mca_coll_mi355x_staged_calls;
/* the op slot the engine reduces a datatype as (OMPI-predefined, ompi_op_ddt_map, extent = the
 * slot's element), or -1 */
int mca_coll_mi355x_reducible_type(const struct ompi_datatype_t *dt);

#ifdef __cplusplus
}
#endif
#endif
