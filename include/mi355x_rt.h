/*
 * mi355x_rt.h -- C ABI of libmi355x_rt.so, the thin HIP layer under op/hip and coll/mi355x.
 *
 * It replaces, for device buffers, the roles the reference gives to:
 *   - the CPU op loops            ompi/mca/op/base/op_base_functions.c:39-683 (mi355x_op_*)
 *   - the CUDA driver shim         ompi/mca/common/cuda/common_cuda.c (pointer query :1687-1783,
 *                                  memcpy :1796-1889, IPC handles :971-1221)  (mi355x_ptr_*,
 *                                  mi355x_memcpy*, mi355x_ipc_*)
 *   - the datatype CUDA hooks      opal/datatype/opal_datatype_cuda.c:43-192 (mi355x_pack_*)
 *   - the tuned schedules on device buffers, coll/cuda staging   coll_cuda_allreduce.c:30-77
 *                                  (mi355x_coll_*)
 * Plain C types only: pointers, sizes, ints.  `stream` is a hipStream_t passed as void*; NULL
 * is the HIP default (null) stream.  Every function returns MI355X_SUCCESS (0) or a
 * negative mi355x_status; mi355x_last_error() gives the text of the last failure.
 * Nothing here falls back to the CPU: when no GPU / no HIP runtime is present the calls fail
 * with MI355X_ERR_HIP.
 */
#ifndef MI355X_RT_H
#define MI355X_RT_H

#include <stddef.h>
#include <stdint.h>

#include "mi355x_types.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------- runtime / diagnostics */
const char *mi355x_last_error(void);
int mi355x_version(void);                 /* 100*major + minor of this library */
int mi355x_device_count(int *count);
int mi355x_set_device(int dev);
int mi355x_get_device(int *dev);
int mi355x_stream_create(void **stream);
int mi355x_stream_destroy(void *stream);
int mi355x_stream_sync(void *stream);
int mi355x_device_sync(void);
int mi355x_malloc(void **p, size_t bytes);
int mi355x_free(void *p);
int mi355x_host_alloc(void **p, size_t bytes);   /* pinned */
int mi355x_host_free(void *p);
int mi355x_memcpy(void *dst, const void *src, size_t bytes);                /* synchronous */
int mi355x_memcpy_async(void *dst, const void *src, size_t bytes, void *stream);
int mi355x_memset_async(void *dst, int value, size_t bytes, void *stream);

/* Pointer classification (replaces mca_common_cuda_is_gpu_buffer, common_cuda.c:1687-1783):
 * *is_device = 1 for hipMalloc'd / IPC-mapped device memory, 0 for host memory. */
int mi355x_ptr_is_device(const void *p, int *is_device);

/* Timing helpers around launches on `stream` (hipEvent based). */
int mi355x_event_create(void **ev);
int mi355x_event_destroy(void *ev);
int mi355x_event_record(void *ev, void *stream);
int mi355x_event_elapsed_ms(void *start, void *stop, float *ms);

/* ---------------------------------------------------------------- op/hip kernels */
/* 1 if (op,type) has a GPU kernel.  Slots absent from the reference table are 0, and so are
 * the x87 `long double` SUM/PROD slots (no 80-bit arithmetic on CDNA4; op/hip stages those to the
 * host base loops).  The x87 compare-only slots -- MAX/MIN on MPI_LONG_DOUBLE, MAXLOC/MINLOC on
 * MPI_LONG_DOUBLE_INT -- are GPU kernels (exact x87 ordering on the 80-bit encoding). */
int mi355x_op_supported(int op, int type);
/* 1 if the collective engine (mi355x_allreduce & co.) reduces (op,type) on the device: the
 * op/hip slots less MPI_LONG_DOUBLE_INT (32-byte pairs).  coll/mi355x stages the others to the
 * lower-priority component through host memory (coll/cuda's rule, coll_cuda_allreduce.c:43-75). */
int mi355x_comm_op_supported(int op, int type);
size_t mi355x_type_size(int type);

/* 2-buff: inout[i] = inout[i] (op) in[i], count elements, asynchronous on `stream`.
 * Device pointers only.  Replaces ompi_op_base_2buff_<op>_<type> (op_base_functions.c:39-103). */
int mi355x_op_reduce(int op, int type, const void *in, void *inout, size_t count, void *stream);
/* 3-buff: out[i] = in1[i] (op) in2[i]; in1/in2/out must not overlap (restrict, op.h:625-630).
 * Replaces ompi_op_base_3buff_<op>_<type> (op_base_functions.c:606-683). */
int mi355x_op_reduce_3buff(int op, int type, const void *in1, const void *in2, void *out,
                           size_t count, void *stream);

/* Launch-shape knobs for the streaming op kernels.  unroll in {1,2,4,8} (16-byte vectors per
 * operand per lane; 0 = keep), blocks_per_cu in 1..64 (grid-stride mode; 0 = keep),
 * nontemporal: -2 keep, -1 auto (non-temporal when the three streams exceed 256 MiB), or a mask
 * 0..3 (1 = loads, 2 = stores).  Only the fp32/fp64 SUM kernels have every variant compiled;
 * the other slots run unroll 1 with masks 0 or 3. */
int mi355x_op_tune(int unroll, int blocks_per_cu, int nontemporal);
int mi355x_op_get_tune(int *unroll, int *blocks_per_cu, int *nontemporal);
/* grid shape: 0 = persistent grid-stride (blocks_per_cu x CUs), 1 = one-shot chunked grid */
int mi355x_op_set_mode(int mode);
int mi355x_op_get_mode(void);
int mi355x_op_set_threads(int threads);   /* block size of the one-shot grid (64..1024) */


/* ---------------------------------------------------------------- coll/mi355x engine */
/* A communicator of `size` ranks on one node, one process (or, for tests, one thread) per rank
 * and GPU.  Buffers are exchanged per call through hipIpcGetMemHandle / hipIpcOpenMemHandle
 * (cached), and every collective is blocking: it returns once the result is in place and no peer
 * still reads this rank's buffers.  `stream` orders the call after the caller's prior work on
 * that stream.  Results replicate the reference coll/tuned (+ coll/basic) schedule's operand
 * order per element, so they are bit-identical to the reference's for the same algorithm. */
typedef struct mi355x_comm mi355x_comm_t;

/* Multi-process: every rank calls with the same `key` (node-unique, e.g. job id + comm id). */
int mi355x_comm_create(const char *key, int rank, int size, int device, mi355x_comm_t **comm);
/* In-process: `size` communicator handles over one device; rank r must be driven from its own
 * thread (the collectives block until every rank has joined). */
int mi355x_comm_create_loopback(int size, int device, mi355x_comm_t **comms);
int mi355x_comm_destroy(mi355x_comm_t *comm);
int mi355x_comm_rank(const mi355x_comm_t *comm);
int mi355x_comm_size(const mi355x_comm_t *comm);
int mi355x_comm_barrier(mi355x_comm_t *comm);
/* Buffer-kind agreement for one collective call.  coll/cuda tolerates ranks that mix host and
 * device buffers in one collective (each rank stages its own, coll_cuda_allreduce.c:30-77); the
 * engine needs every rank in the same protocol.  Every rank calls this once per collective, in the
 * collective's call order, and learns whether the call runs in the engine (*engine = 1: a host rank
 * joins on device copies) or in the lower-priority host component (*engine = 0: a device rank
 * stages its buffers to the host, as coll/cuda does).  Only one side of a call waits for the
 * others' votes, and which one is agreed window by window: every 32nd call every rank waits (a
 * checkpoint: all ranks see every vote, and learn whether any rank used device buffers in the
 * window just ended); in a window after device use the host ranks wait and the device ranks only
 * publish (a mixed call runs in the engine), in a window without it the device ranks wait and the
 * host ranks only publish (a mixed call runs on the host) -- so a host-only program pays one store
 * per call and a device program nothing more. */
int mi355x_comm_vote(mi355x_comm_t *comm, int device, int *engine);
/* algorithm id of the last collective, coll/tuned numbering (allreduce: 1 linear, 2 nonoverlapping,
 * 3 recursive doubling, 4 ring, 5 segmented ring; reduce: 1 linear, 2 chain, 3 pipeline, 4 binary,
 * 5 binomial; reduce_scatter: 1 non-overlapping, 2 recursive halving, 3 ring) */
int mi355x_comm_last_algorithm(const mi355x_comm_t *comm);
/* Test hook (no reference counterpart): take (acquire = 1) or give back (0) the communicator's
 * pipelined-grid admission token of its GPU outside any call, as a rank inside a pipelined
 * allreduce holds it.  Returns 1 if the token is now held.  Tests kill a holder with SIGKILL and
 * check that the next communicator on that GPU is admitted again (the token is reclaimed from a
 * dead process, coll_comm.cpp). */
int mi355x_debug_pipe_token(mi355x_comm_t *comm, int acquire);
/* Test hook (no GPU needed): the same holder protocol for device uid `dev_uid` on behalf of a
 * communicator named `name` (op 1 take, 0 give back; returns 1 while held).  MI355X_TOKEN_TABLE=/name
 * points a process at a private token table. */
int mi355x_debug_token(uint64_t dev_uid, const char *name, int op);

/* Knobs BLOCKS_PER_CU, PUSH, COPY_BLOCK_KIB, PIPE_WG_PER_CU, PIPE_CHUNK_KIB and PIPE_WT are launch
 * shapes shared by every communicator of the process (setting one through any communicator sets
 * it for all; every rank of a communicator must use the same values); the others belong to the
 * communicator they are set on. */
enum mi355x_knob {
    MI355X_KNOB_ALLREDUCE_ALG = 1,      /* coll_tuned_allreduce_algorithm (0 = decision) */
    MI355X_KNOB_REDUCE_ALG = 2,         /* coll_tuned_reduce_algorithm, used by reduce_scatter_block */
    MI355X_KNOB_REDUCE_SCATTER_ALG = 3, /* coll_tuned_reduce_scatter_algorithm */
    MI355X_KNOB_BLOCKS_PER_CU = 4,      /* grid cap of the coll kernels, 1..1024 (default 1024 = one-shot) */
    MI355X_KNOB_TIMEOUT_S = 5,
    MI355X_KNOB_PUSH = 6,               /* 1: one-phase push data flow (owners write peers' buffers);
                                           single-device use only: across xGMI the remote writes land
                                           behind the owner's L2 (see coll_internal.hpp) */
    MI355X_KNOB_IPC_MAX_BYTES = 7,      /* buffers in allocations of >= this many bytes are never
                                           exported; calls touching one take the staged data flow
                                           (default 2^31: hipIpcOpenMemHandle hangs from 2 GiB) */
    MI355X_KNOB_STAGE_BYTES = 8,        /* size of the per-communicator staging buffer (default 1 GiB) */
    MI355X_KNOB_REDUCE_CHAIN_FANOUT = 10, /* coll_tuned_reduce_algorithm_chain_fanout (default 4) */
    MI355X_KNOB_LL_MAX_BYTES = 9,       /* per-rank message bytes up to which allreduce / allgather /
                                           bcast / reduce take the one-shot low-latency path (0 = never;
                                           default 0, or env MI355X_LL_MAX_BYTES; multi-process
                                           communicators of <= 8 ranks whose LL self-test (device
                                           setup) passed -- otherwise the knob stays 0) */
    MI355X_KNOB_TIME_PHASES = 11,       /* 1: time the two kernels of the direct allreduce with HIP
                                           events on the call's stream (mi355x_comm_phase_ms) */
    MI355X_KNOB_COPY_BLOCK_KIB = 12,    /* bytes per block of the pull-copy kernel, KiB (4..256, default 4) */
    MI355X_KNOB_PIPE = 13,              /* 1: a multi-process ring allreduce runs its reduce and copy
                                           phases in ONE pipelined launch per rank, overlapped chunk by
                                           chunk with device-side ready flags (the segmented ring's
                                           copy/reduce overlap, coll_tuned_allreduce.c:721-831);
                                           0: two phases separated by a host barrier.  Default (environment
                                           MI355X_PIPE=0/1 at creation overrides): 1 from 4 ranks up,
                                           where the one-GPU rehearsal measured it ahead (n = 4: 2.03 vs
                                           2.14 ms, n = 8: 3.50-3.78 vs 4.47), 0 below (n = 2: 1.01 vs 0.93) */
    MI355X_KNOB_PIPE_WG_PER_CU = 14,    /* pipelined allreduce: 256-thread workgroups per CU (1..8, default 2) */
    MI355X_KNOB_PIPE_CHUNK_KIB = 15,    /* pipelined allreduce: chunk size in KiB (0 = auto: ~512 chunks
                                           per ring block, at least 64 KiB) */
    MI355X_KNOB_PIPE_WT = 16,           /* pipelined allreduce: 1 (default) = fold results stored write-
                                           through (system-coherent policy) and pulled with coherent
                                           loads, no per-chunk L2 write-back / invalidate; 0 = fences */
    MI355X_KNOB_ONE_PHASE_MAX_BYTES = 17, /* (per communicator, same value on every rank; env
                                           MI355X_ONE_PHASE_MAX_BYTES at creation) ring-ordered
                                           allreduce (not in place) up to this many bytes
                                           per rank: every rank evaluates every ring block from the n
                                           inputs in one launch (reads n x S, one host barrier and
                                           stream sync fewer than the two phases); default 1 MiB,
                                           0 = always two phases */
    MI355X_KNOB_PIPE_REFUSED = 18,      /* (read-only) calls of this communicator that were to run pipelined
                                           but fell back to two phases because another communicator's
                                           pipelined grid held a GPU (the per-GPU admission token) */
    MI355X_KNOB_SVC_MAX_BYTES = 19,     /* (per communicator, same value on every rank; env MI355X_SVC_MAX_BYTES
                                           at creation) per-rank message bytes up to which allreduce /
                                           reduce / allgather / bcast are served by the resident LL service
                                           (coll_svc.hip: the LL protocol in a kernel that stays resident on a
                                           private HSA queue and waits on a doorbell -- no launch per call).
                                           One service per process and GPU, owned by the first communicator
                                           whose ranks all find it free at creation; reads 0 (and setting it
                                           is ignored) on every other communicator.  MI355X_SVC=0 disables it */
    MI355X_KNOB_SVC_CALLS = 20,         /* (read-only) calls served by the resident service */
    MI355X_KNOB_SVC_LAUNCHES = 21,      /* (read-only) launches of the resident service (it leaves after
                                           MI355X_SVC_IDLE_MS without a call and is relaunched on demand) */
    MI355X_KNOB_SVC_RESIDENT = 22,      /* (read-only) 1 while the service's kernel is resident */
    MI355X_KNOB_SVC_PULL_MAX_BYTES = 23, /* (per communicator, same value on every rank; env
                                           MI355X_SVC_PULL_MAX_BYTES at creation) ring-ordered allreduce,
                                           not in place, above SVC_MAX_BYTES and up to this many bytes per
                                           rank: the resident service evaluates it from the peers' mapped
                                           inputs (buffers 16-B aligned on every rank) instead of a launch
                                           and a host barrier; also the largest block of a
                                           reduce_scatter(_block), not in place, that the service
                                           evaluates from the peers' inputs (any size up to it);
                                           0 = never; reads 0 without a service */
    MI355X_KNOB_SVC_PULL_COPY_MAX_BYTES = 24, /* (per communicator, same value on every rank; env
                                           MI355X_SVC_PULL_COPY_MAX_BYTES at creation) allgather / bcast
                                           above SVC_MAX_BYTES and up to this many bytes per rank (default
                                           1 MiB): the resident service copies from the peers' mapped
                                           buffers instead of a launch and a host barrier; 0 = never */
    MI355X_KNOB_RCACHE_MAX_MAPS = 25,   /* peer-mapping cache: at most this many hipIpc mappings of peers'
                                           allocations stay open; least recently used ones beyond it are
                                           closed (mpool_rgpusm's LRU, mpool_rgpusm_module.c:104-120).  0 =
                                           unlimited (default; env MI355X_RCACHE_MAX_MAPS at creation) */
    MI355X_KNOB_RCACHE_SIZE_LIMIT = 26, /* the same bound in bytes of the mapped allocations
                                           (mpool_rgpusm_rcache_size_limit, mpool_rgpusm_component.c:92-100);
                                           0 = unlimited (default; env MI355X_RCACHE_SIZE_LIMIT) */
    MI355X_KNOB_PEER_MAPS = 27,         /* (read-only) hipIpc mappings of peers' allocations open now */
    MI355X_KNOB_RCACHE_EVICTIONS = 28,  /* (read-only) mappings closed by the cache bounds */
    MI355X_KNOB_FLOWS = 29,             /* (read-only) cross-device flows this communicator may use, a mask
                                           of MI355X_FLOW_*: every default-on flow is self-tested for exact
                                           results on changing data before its first use, the outcome agreed
                                           by every rank, and a flow that failed on any rank stays off on
                                           every rank (the host-synchronised flows take its calls) */
    MI355X_KNOB_FLOWS_FAILED = 30,      /* (read-only) the flows whose self-test failed on some rank */
    MI355X_KNOB_CREATE_US = 31,         /* (read-only) wall time of mi355x_comm_create, microseconds */
    MI355X_KNOB_SELFTEST_US = 32,       /* (read-only) the flow self-tests of the device setup (first device
                                           collective); plus the service flows' self-test at its first claim */
    MI355X_KNOB_SVC_OWNER = 33,         /* (read-only) 1 while this communicator owns its process's
                                           resident service */
    MI355X_KNOB_SVC_CLAIMS = 34,        /* (read-only) times this communicator has taken the service */
    MI355X_KNOB_SVC_IDLE_US = 35,       /* (per communicator, same value on every rank; env MI355X_SVC_IDLE_MS at
                                           creation, default 1000) microseconds the resident service stays
                                           without a call before it leaves (applies from its next launch) */
    MI355X_KNOB_SVC_SHRINK_US = 36,     /* (per communicator; env MI355X_SVC_SHRINK_US, default 100; 0: never)
                                           microseconds without a call after which every workgroup of the
                                           service but the first leaves (applies from its next launch) */
    MI355X_KNOB_SVC_REGROWS = 37,       /* (read-only) calls that relaunched a shrunk service's full grid */
    MI355X_KNOB_DEV_SETUP = 38,         /* (read-only) 1 once the communicator's device-side setup has run: it
                                           is deferred from mi355x_comm_create to the first device-buffer
                                           reduction / allgather / bcast (smcuda's lazy rule,
                                           btl/smcuda/README:36-40); a communicator that only ever sees host
                                           buffers allocates no device memory */
    MI355X_KNOB_SETUP_US = 39,          /* (read-only) wall time of that setup, microseconds (in the call that
                                           triggered it) */
    MI355X_KNOB_SELFTEST = 40,          /* (per communicator, same value on every rank; env MI355X_SELFTEST, default
                                           1) 1: the device setup self-tests the cross-device flows and turns a
                                           flow that failed on any rank off on every rank; 0: trusts them.  Only
                                           a value set before the device setup takes effect. */
    MI355X_KNOB_PIPE_CALLS = 41,        /* (read-only) allreduces served by the pipelined flow */
    MI355X_KNOB_EXPORT_MISMATCHES = 42, /* (read-only) new dmabuf exports of the bounded peer-mapping cache that
                                           named another buffer object (checked, that call staged instead;
                                           env MI355X_EXPORT_CHECK=0 turns the check off) */
    MI355X_KNOB_SELFTEST_REUSED = 43    /* (read-only) flow verdicts this communicator took over from an earlier
                                           communicator of the same processes on the same GPUs (a dup / split):
                                           1 the device setup's (LL, pipelined), 2 also the service's */
};
/* cross-device flows (MI355X_KNOB_FLOWS) */
enum mi355x_flow {
    MI355X_FLOW_SVC_LL = 1,    /* resident service, LL form (granules pushed into the peers) */
    MI355X_FLOW_SVC_PULL = 2,  /* resident service, one-phase ring allreduce from the peers' inputs */
    MI355X_FLOW_SVC_COPY = 4,  /* resident service, allgather / bcast copied from the peers' buffers */
    MI355X_FLOW_SVC_RS = 8,    /* resident service, reduce_scatter(_block) from the peers' inputs */
    MI355X_FLOW_PIPE = 16      /* pipelined allreduce (per-chunk flags written into the peers) */
};
int mi355x_comm_set(mi355x_comm_t *comm, int knob, long value);
/* current value of a knob (LL_MAX_BYTES reads 0 when the device setup's LL self-test failed) */
int mi355x_comm_get(const mi355x_comm_t *comm, int knob, long *value);
/* device time of the last timed direct allreduce: phase 1 (k_fold, the owner's block from every
 * rank) and phase 2 (k_multicopy, the other blocks from their owners); with the pipelined flow
 * phase 1 is the one launch (k_pipe_allreduce) and phase 2 is 0; -1 when not measured */
int mi355x_comm_phase_ms(const mi355x_comm_t *comm, float *phase1_ms, float *phase2_ms);

/* coll/tuned's dynamic rules file (coll_tuned_dynamic_file.c:56-251; MCA
 * coll_tuned_dynamic_rules_filename with coll_tuned_use_dynamic_rules).  Collective ids are
 * coll/tuned's COLLTYPE (coll_tuned.h:41-58); algorithm numbers are coll/tuned's per collective.
 * A communicator with rules picks, per call: rule > forced algorithm (knobs) > fixed decision, as
 * the dec_dynamic functions do (coll_tuned_decision_dynamic.c:59-99).  Rules change the operand
 * order of allreduce / reduce / reduce_scatter(_block) results (reduce chain fan-out included);
 * bcast / allgather rules are read but do not change any result. */
enum mi355x_coll_id {
    MI355X_COLL_ALLGATHER = 0, MI355X_COLL_ALLREDUCE = 2, MI355X_COLL_BCAST = 7, MI355X_COLL_REDUCE = 11,
    MI355X_COLL_REDUCESCATTER = 12, MI355X_COLL_COUNT = 16
};
typedef struct mi355x_rules mi355x_rules_t;
/* returns the number of collectives with rules (>= 0) or a negative status */
int mi355x_rules_load(const char *path, mi355x_rules_t **rules);
int mi355x_rules_destroy(mi355x_rules_t *rules);
/* *alg = 0 when no rule applies; faninout / segsize may be NULL */
int mi355x_rules_decide(const mi355x_rules_t *rules, int coll, int comm_size, size_t msg_bytes, int *alg,
                        int *faninout, int *segsize);
/* the communicator consults `rules` (not owned; NULL = none) from the next call on */
int mi355x_comm_set_rules(mi355x_comm_t *comm, const mi355x_rules_t *rules);

/* MPI_Allreduce.  sbuf == NULL means MPI_IN_PLACE.  Replaces coll_cuda_allreduce.c:30-77 +
 * ompi_coll_tuned_allreduce_intra_dec_fixed (coll_tuned_decision_fixed.c:42-85). */
int mi355x_allreduce(mi355x_comm_t *comm, const void *sbuf, void *rbuf, size_t count, int type, int op,
                     void *stream);
/* MPI_Reduce to `root` (sbuf NULL = MPI_IN_PLACE at the root; rbuf read at the root only).
 * Replaces ompi_coll_tuned_reduce_intra_dec_fixed (coll_tuned_decision_fixed.c:343-446) and the
 * tuned reduce trees (coll_tuned_reduce.c:66-721); MI355X_KNOB_REDUCE_ALG forces one. */
int mi355x_reduce(mi355x_comm_t *comm, const void *sbuf, void *rbuf, size_t count, int type, int op, int root,
                  void *stream);
/* MPI_Reduce_scatter_block: coll_basic_reduce_scatter_block.c:54-111 order. */
int mi355x_reduce_scatter_block(mi355x_comm_t *comm, const void *sbuf, void *rbuf, size_t rcount,
                                int type, int op, void *stream);
/* MPI_Reduce_scatter: ompi_coll_tuned_reduce_scatter_intra_dec_fixed order (decision_fixed.c:456-502). */
int mi355x_reduce_scatter(mi355x_comm_t *comm, const void *sbuf, void *rbuf, const int *rcounts,
                          int type, int op, void *stream);
/* MPI_Allgather of `bytes` contiguous bytes per rank (sbuf NULL = MPI_IN_PLACE). */
int mi355x_allgather(mi355x_comm_t *comm, const void *sbuf, void *rbuf, size_t bytes, void *stream);
/* MPI_Bcast of `bytes` contiguous bytes from `root`. */
int mi355x_bcast(mi355x_comm_t *comm, void *buf, size_t bytes, int root, void *stream);

/* The callers either side of the reduction path, on device buffers (coll_move.cpp).  The
 * reference has no device form of these (coll/cuda wraps only the reductions,
 * coll_cuda_module.c:118-140): tuned / basic run them over the PML.  Here every rank pulls what it
 * receives straight from the owners' memory in one launch.  Counts and displacements are BYTES;
 * NULL sbuf (rbuf for scatter at the root) = MPI_IN_PLACE.  A sender longer than the receiver's
 * count fails with MI355X_ERR_TRUNCATE.
 *   gather(v)   coll_tuned_gather.c / coll_basic_gatherv.c      (rcounts / displs read at the root)
 *   scatter(v)  coll_tuned_scatter.c / coll_basic_scatterv.c    (scounts / displs read at the root)
 *   allgatherv  coll_tuned_allgatherv.c
 *   alltoall(v) coll_tuned_alltoall.c / coll_tuned_alltoallv.c
 *   scan, exscan  coll_basic_scan.c:40-120 / coll_basic_exscan.c:40-110 operand order, bit-exact:
 *               rank r = ((x0 op x1) op ...) op x_r (exscan: up to x_{r-1}; rank 0 untouched). */
int mi355x_gather(mi355x_comm_t *comm, const void *sbuf, void *rbuf, size_t bytes, int root, void *stream);
int mi355x_gatherv(mi355x_comm_t *comm, const void *sbuf, size_t sbytes, void *rbuf, const size_t *rcounts,
                   const size_t *displs, int root, void *stream);
int mi355x_scatter(mi355x_comm_t *comm, const void *sbuf, void *rbuf, size_t bytes, int root, void *stream);
int mi355x_scatterv(mi355x_comm_t *comm, const void *sbuf, const size_t *scounts, const size_t *displs,
                    void *rbuf, size_t rbytes, int root, void *stream);
int mi355x_allgatherv(mi355x_comm_t *comm, const void *sbuf, size_t sbytes, void *rbuf, const size_t *rcounts,
                      const size_t *displs, void *stream);
int mi355x_alltoall(mi355x_comm_t *comm, const void *sbuf, void *rbuf, size_t bytes, void *stream);
int mi355x_alltoallv(mi355x_comm_t *comm, const void *sbuf, const size_t *scounts, const size_t *sdispls,
                     void *rbuf, const size_t *rcounts, const size_t *rdispls, void *stream);
int mi355x_scan(mi355x_comm_t *comm, const void *sbuf, void *rbuf, size_t count, int type, int op, void *stream);
int mi355x_exscan(mi355x_comm_t *comm, const void *sbuf, void *rbuf, size_t count, int type, int op, void *stream);

/* Nonblocking collectives (MPI_Iallreduce, MPI_Ireduce, MPI_Ireduce_scatter_block, MPI_Iallgather,
 * MPI_Ibcast; the coll framework's nonblocking slots, coll.h:241-356, served in the reference by
 * coll/libnbc: nbc_iallreduce.c etc.).  Each call is queued behind the caller's prior work on
 * `stream` and run, in posting order, by the communicator's progress thread; results are
 * identical to the blocking call's.  A blocking collective on the same communicator first waits
 * for every posted one.  Requests: test (non-blocking; *done = 1 once finished, then returns the
 * collective's status), wait (blocks; returns the status), free (only once finished). */
typedef struct mi355x_request mi355x_request_t;
int mi355x_iallreduce(mi355x_comm_t *comm, const void *sbuf, void *rbuf, size_t count, int type, int op,
                      void *stream, mi355x_request_t **req);
int mi355x_ireduce(mi355x_comm_t *comm, const void *sbuf, void *rbuf, size_t count, int type, int op, int root,
                   void *stream, mi355x_request_t **req);
int mi355x_ireduce_scatter_block(mi355x_comm_t *comm, const void *sbuf, void *rbuf, size_t rcount, int type,
                                 int op, void *stream, mi355x_request_t **req);
int mi355x_iallgather(mi355x_comm_t *comm, const void *sbuf, void *rbuf, size_t bytes, void *stream,
                      mi355x_request_t **req);
int mi355x_ibcast(mi355x_comm_t *comm, void *buf, size_t bytes, int root, void *stream, mi355x_request_t **req);
int mi355x_iscan(mi355x_comm_t *comm, const void *sbuf, void *rbuf, size_t count, int type, int op, void *stream,
                 mi355x_request_t **req);
int mi355x_ialltoall(mi355x_comm_t *comm, const void *sbuf, void *rbuf, size_t bytes, void *stream,
                     mi355x_request_t **req);
int mi355x_request_test(mi355x_request_t *req, int *done);
int mi355x_request_wait(mi355x_request_t *req);
int mi355x_request_free(mi355x_request_t *req);

/* ---------------------------------------------------------------- point-to-point */
/* MPI_Send / MPI_Recv / MPI_Isend / MPI_Irecv / MPI_Sendrecv / MPI_Iprobe / MPI_Improbe +
 * MPI_Imrecv between the ranks of a communicator, on device AND host buffers, in ONE matching
 * queue per communicator (ob1's: per-source order, posted receives in posting order,
 * MI355X_ANY_SOURCE; MI355X_ANY_TAG matches tags >= 0 only, pml_ob1_recvfrag.c:487; negative
 * system tags are allowed).  A device payload travels as ob1's RGET over btl/smcuda does: the
 * sender announces its registered buffer (mca_pml_ob1_send_request_start_cuda,
 * pml_ob1_cuda.c:52-100), the receiver matches and pulls it over xGMI (mca_btl_smcuda_get_cuda,
 * btl_smcuda.c:1083-1168), the FIN completes the send.  A host payload -- and a device payload of
 * at most 4 KiB (the sm/smcuda eager limit, btl_sm_component.c:244) -- is copied into the
 * sender's shared-memory arena, as the sm BTL copies fragments; the receiver copies it out (into
 * host memory, or to the device).  Either side may be host or device memory (ob1 decides the
 * convertor per request on each side, pml_ob1_cuda.c:52-100 / pml_ob1_recvreq.c:647-663).
 * `ddt` NULL: `count` contiguous bytes; else `count` instances of the datatype (the GPU
 * convertor on device memory, the host convertor on host memory).  Buffers are read / written
 * once the caller's prior work on `stream` is done.  Completion of a send: messages of at most
 * 4 KiB and buffered sends complete once copied (eager); synchronous sends and larger messages
 * when the receiver has the data (rendezvous).  A receive longer than its buffer gets the first
 * bytes, status.bytes = the message size, status.error = MI355X_ERR_TRUNCATE
 * (pml_ob1_recvreq.h:172-180); the blocking forms then return MI355X_ERR_TRUNCATE.  Requests:
 * mi355x_request_test / wait / free above (they drive progress); mi355x_p2p_progress is the
 * opal_progress hook. */
#define MI355X_ANY_SOURCE (-1)   /* MPI_ANY_SOURCE, mpi.h.in:415 */
#define MI355X_PROC_NULL  (-2)   /* MPI_PROC_NULL,  mpi.h.in:416 */
#define MI355X_ANY_TAG    (-1)   /* MPI_ANY_TAG,    mpi.h.in:418 */
typedef struct mi355x_msg_status {
    int source, tag, error;
    size_t bytes;
} mi355x_status_t;
typedef struct mi355x_ddt mi355x_ddt_t;
int mi355x_isend(mi355x_comm_t *comm, const void *buf, size_t count, const mi355x_ddt_t *ddt, int dest, int tag,
                 void *stream, mi355x_request_t **req);
int mi355x_irecv(mi355x_comm_t *comm, void *buf, size_t count, const mi355x_ddt_t *ddt, int source, int tag,
                 void *stream, mi355x_request_t **req);
int mi355x_send(mi355x_comm_t *comm, const void *buf, size_t count, const mi355x_ddt_t *ddt, int dest, int tag,
                void *stream);
int mi355x_recv(mi355x_comm_t *comm, void *buf, size_t count, const mi355x_ddt_t *ddt, int source, int tag,
                void *stream, mi355x_status_t *status);
int mi355x_sendrecv(mi355x_comm_t *comm, const void *sbuf, size_t scount, const mi355x_ddt_t *sddt, int dest,
                    int stag, void *rbuf, size_t rcount, const mi355x_ddt_t *rddt, int source, int rtag,
                    void *stream, mi355x_status_t *status);
int mi355x_iprobe(mi355x_comm_t *comm, int source, int tag, int *flag, mi355x_status_t *status);
int mi355x_p2p_progress(mi355x_comm_t *comm);
int mi355x_request_get_status(const mi355x_request_t *req, mi355x_status_t *status);
/* send modes: mca_pml_base_send_mode_t (pml.h:78-85), same values */
enum mi355x_send_mode {
    MI355X_SEND_SYNCHRONOUS = 0, MI355X_SEND_COMPLETE = 1, MI355X_SEND_BUFFERED = 2, MI355X_SEND_READY = 3,
    MI355X_SEND_STANDARD = 4
};
/* mi355x_isend / mi355x_send with a send mode (the plain forms are MI355X_SEND_STANDARD):
 * SYNCHRONOUS completes only once the receiver has matched and read the message; BUFFERED
 * completes at once (the payload is copied; MPI_Bsend's attached buffer plays no role). */
int mi355x_isend_mode(mi355x_comm_t *comm, const void *buf, size_t count, const mi355x_ddt_t *ddt, int dest, int tag,
                      int mode, void *stream, mi355x_request_t **req);
int mi355x_send_mode(mi355x_comm_t *comm, const void *buf, size_t count, const mi355x_ddt_t *ddt, int dest, int tag,
                     int mode, void *stream);
/* MPI_Improbe / MPI_Mprobe (mca_pml_ob1_improbe, pml_ob1_iprobe.c:83-134): the first matching
 * message is taken out of the queue (no receive can match it any more) and handed back as *msg;
 * MPI_Imrecv / MPI_Mrecv receive exactly that message (consuming msg). */
typedef struct mi355x_message mi355x_message_t;
int mi355x_improbe(mi355x_comm_t *comm, int source, int tag, int *flag, mi355x_message_t **msg,
                   mi355x_status_t *status);
int mi355x_imrecv(mi355x_comm_t *comm, void *buf, size_t count, const mi355x_ddt_t *ddt, mi355x_message_t *msg,
                  void *stream, mi355x_request_t **req);
/* MPI_Cancel of a receive not matched yet (mca_pml_ob1_recv_request_cancel,
 * pml_ob1_recvreq.c:101-137): it completes with *cancelled = 1; a matched receive or a send is not
 * cancelled (ob1 cancels no send either, pml_ob1_sendreq.c:126-131). */
int mi355x_request_cancel(mi355x_request_t *req);
int mi355x_request_cancelled(const mi355x_request_t *req, int *cancelled);
/* the engine's host-side waits (the buffer-kind vote, and inside collectives the barriers, finish
 * points and completion waits) call this between polls: coll/mi355x passes opal_progress, so
 * requests other ranks depend on keep moving (MPI's progress rule, as ob1's blocking waits) */
int mi355x_set_progress_hook(void (*progress)(void));

/* ---------------------------------------------------------------- GPU convertor */
/* A datatype layout: instance k at base + k*extent; inside it nblk blocks at j*stride; inside a
 * block the runs (disp, len) in order.  The packed stream is that type map in order, as
 * opal_generic_simple_pack produces it (opal/datatype/opal_datatype_pack.c:250-374). */
int mi355x_ddt_create(const int64_t *disp, const int64_t *len, size_t nruns, size_t nblk, int64_t stride,
                      int64_t extent, mi355x_ddt_t **out);
/* MPI_Type_vector over a gap-free type of elem_size bytes (ompi_datatype_create_vector.c:36-65) */
int mi355x_ddt_create_vector(size_t count, size_t blocklen, int64_t stride, size_t elem_size, mi355x_ddt_t **out);
/* MPI_Type_indexed (ompi_datatype_create_indexed.c:32-66, adjacent blocks merged) */
int mi355x_ddt_create_indexed(size_t count, const int *blocklens, const int *disps, size_t elem_size,
                              mi355x_ddt_t **out);
/* compile an optimized opal description (opal_datatype_t::opt_desc, `used` 32-byte ELEM/LOOP/
 * END_LOOP records, opal_datatype_internal.h:148-188); basic_sizes[id] = size of opal basic type id */
int mi355x_ddt_from_opal(const void *desc, uint32_t used, int64_t extent, const uint32_t *basic_sizes,
                         mi355x_ddt_t **out);
int mi355x_ddt_destroy(mi355x_ddt_t *d);
size_t mi355x_ddt_size(const mi355x_ddt_t *d);
int64_t mi355x_ddt_extent(const mi355x_ddt_t *d);
int mi355x_ddt_nruns(const mi355x_ddt_t *d);
/* launch shape of the single-run (row) pack/unpack kernel: 16-B slots per lane for pack and for
 * unpack (2/4/8; 0 keeps), threads per block (256/512/1024; 0 keeps), nontemporal -2 keep,
 * -1 auto (non-temporal above 256 MiB moved), 0..3 mask (1 = loads, 2 = stores) */
int mi355x_ddt_tune(int unroll_pack, int unroll_unpack, int threads, int nontemporal);
/* which pack/unpack kernels may run: 2 (default) the row kernel for every one-run-per-block
 * layout, with the widest slot (16/8/4/2/1 B) its addresses and window allow, and the unit
 * kernel (LDS-staged run tables; 16-B packed slots over 8- or 4-B aligned runs when the packed
 * side is 16-B aligned, else W-byte units) for run lists of up to 4096 runs; 3 as 2 with W-byte
 * units only; 1 the row kernel with 16-B slots only; 0 neither (the general kernel for
 * everything; A/B measurement, tests) */
int mi355x_ddt_tune_rows(int mode);
/* pack packed bytes [pos, pos+bytes) of `count` instances at device `base` into `dst`
 * (replaces opal_convertor_set_position + opal_convertor_pack on a CUDA convertor,
 * opal_convertor.c:223-330 / opal_datatype_cuda.c:93-115).  checksum (may be NULL) receives the
 * window's share of the convertor checksum (opal_uicsum_partial, opal/util/crc.c:921). */
int mi355x_pack(const mi355x_ddt_t *d, size_t count, const void *base, size_t pos, void *dst, size_t bytes,
                uint32_t *checksum, void *stream);
int mi355x_unpack(const mi355x_ddt_t *d, size_t count, void *base, size_t pos, const void *src, size_t bytes,
                  uint32_t *checksum, void *stream);
/* the same windows on HOST memory (ob1's convertor for a host buffer, opal_datatype_pack.c:250-374,
 * opal_datatype_unpack.c:245-…); synchronous, no GPU */
int mi355x_pack_host(const mi355x_ddt_t *d, size_t count, const void *base, size_t pos, void *dst, size_t bytes);
int mi355x_unpack_host(const mi355x_ddt_t *d, size_t count, void *base, size_t pos, const void *src, size_t bytes);
/* opal_convertor_raw (opal_convertor_raw.c:37-…): up to *iov_count memory pieces (offset from the
 * buffer, length) of the type map from packed position *pos onwards; *iov_count = pieces returned,
 * *max_data = their bytes, *pos advanced; returns 1 once the whole message is described, else 0.
 * No GPU. */
int mi355x_ddt_raw(const mi355x_ddt_t *d, size_t count, size_t *pos, int64_t *disp, size_t *len, uint32_t *iov_count,
                   size_t *max_data);

/* Host-only introspection of the schedule compiler: the per-element program the engine runs for
 * a given reference algorithm (layout documented in coll_comm.cpp).  For tests; no GPU needed. */
int mi355x_sched_program(int kind, int n, int alg, int block, int *out, int cap);

#ifdef __cplusplus
}
#endif
#endif /* MI355X_RT_H */
