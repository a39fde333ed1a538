/*
 * coll_mi355x_component.c -- coll/mi355x: device-buffer collectives over the MI355X engine.
 *
 * Component ABI: ompi/mca/coll/coll.h:357-451 (example: coll_cuda_component.c:37-72).  Selection:
 * mca_coll_base_comm_select (coll_base_comm_select.c:114-262) calls collm_comm_query per
 * communicator, then coll_module_enable in ascending priority, then copies every non-NULL
 * function pointer.  See include/coll_mi355x.h for what is intercepted.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "../../../../../include/coll_mi355x.h"
#include "../../../../../include/mi355x_rt.h"

int mca_coll_mi355x_priority = 90;
int mca_coll_mi355x_allreduce_algorithm = 0;
int mca_coll_mi355x_pml_hook = 1;

typedef struct mca_coll_mi355x_module_t {
    mca_coll_base_module_t super;
    mi355x_comm_t *engine;
    /* lower-priority functions snapshotted at enable time (coll_cuda_module.c:126-147) */
    mca_coll_base_module_allreduce_fn_t prev_allreduce;
    mca_coll_base_module_t *prev_allreduce_module;
    mca_coll_base_module_reduce_scatter_fn_t prev_reduce_scatter;
    mca_coll_base_module_t *prev_reduce_scatter_module;
    mca_coll_base_module_reduce_scatter_block_fn_t prev_reduce_scatter_block;
    mca_coll_base_module_t *prev_reduce_scatter_block_module;
    mca_coll_base_module_allgather_fn_t prev_allgather;
    mca_coll_base_module_t *prev_allgather_module;
    mca_coll_base_module_bcast_fn_t prev_bcast;
    mca_coll_base_module_t *prev_bcast_module;
    mca_coll_base_module_reduce_fn_t prev_reduce;
    mca_coll_base_module_t *prev_reduce_module;
    /* the callers either side of the reduction path (coll_move.cpp) */
    mca_coll_base_module_gather_fn_t prev_gather;
    mca_coll_base_module_t *prev_gather_module;
    mca_coll_base_module_gatherv_fn_t prev_gatherv;
    mca_coll_base_module_t *prev_gatherv_module;
    mca_coll_base_module_scatter_fn_t prev_scatter;
    mca_coll_base_module_t *prev_scatter_module;
    mca_coll_base_module_scatterv_fn_t prev_scatterv;
    mca_coll_base_module_t *prev_scatterv_module;
    mca_coll_base_module_allgatherv_fn_t prev_allgatherv;
    mca_coll_base_module_t *prev_allgatherv_module;
    mca_coll_base_module_alltoall_fn_t prev_alltoall;
    mca_coll_base_module_t *prev_alltoall_module;
    mca_coll_base_module_alltoallv_fn_t prev_alltoallv;
    mca_coll_base_module_t *prev_alltoallv_module;
    mca_coll_base_module_scan_fn_t prev_scan;
    mca_coll_base_module_t *prev_scan_module;
    mca_coll_base_module_exscan_fn_t prev_exscan;
    mca_coll_base_module_t *prev_exscan_module;
    /* nonblocking slots: the previous owner (normally coll/libnbc) may be absent */
    mca_coll_base_module_iallreduce_fn_t prev_iallreduce;
    mca_coll_base_module_t *prev_iallreduce_module;
    mca_coll_base_module_ireduce_fn_t prev_ireduce;
    mca_coll_base_module_t *prev_ireduce_module;
    mca_coll_base_module_ireduce_scatter_block_fn_t prev_ireduce_scatter_block;
    mca_coll_base_module_t *prev_ireduce_scatter_block_module;
    mca_coll_base_module_iallgather_fn_t prev_iallgather;
    mca_coll_base_module_t *prev_iallgather_module;
    mca_coll_base_module_ibcast_fn_t prev_ibcast;
    mca_coll_base_module_t *prev_ibcast_module;
    /* GPU-convertor layouts of the derived datatypes seen on this communicator, and the packed
     * staging buffer (device memory; registered once, re-registered when it grows) */
    struct ddt_slot { uint64_t sig; const void *dt; mi355x_ddt_t *d; } ddt_cache[8];
    int ddt_next;
    void *scratch[2];          /* send-side and receive-side staging (device memory) */
    size_t scratch_bytes[2];
    int mixed;                 /* coll_mi355x_mixed_buffers when the module was enabled */
} mca_coll_mi355x_module_t;

static void module_construct(opal_object_t *o)
{
    mca_coll_mi355x_module_t *m = (mca_coll_mi355x_module_t *)o;
    memset((char *)m + sizeof(mca_coll_base_module_t), 0, sizeof(*m) - sizeof(mca_coll_base_module_t));
    m->mixed = mca_coll_mi355x_mixed_buffers;
}

static void release_prev(mca_coll_base_module_t *p)
{
    if (p) mi355x_obj_release(&p->super);
}

static void module_destruct(opal_object_t *o)
{
    mca_coll_mi355x_module_t *m = (mca_coll_mi355x_module_t *)o;
    release_prev(m->prev_allreduce_module);
    release_prev(m->prev_reduce_scatter_module);
    release_prev(m->prev_reduce_scatter_block_module);
    release_prev(m->prev_allgather_module);
    release_prev(m->prev_bcast_module);
    release_prev(m->prev_reduce_module);
    release_prev(m->prev_gather_module);
    release_prev(m->prev_gatherv_module);
    release_prev(m->prev_scatter_module);
    release_prev(m->prev_scatterv_module);
    release_prev(m->prev_allgatherv_module);
    release_prev(m->prev_alltoall_module);
    release_prev(m->prev_alltoallv_module);
    release_prev(m->prev_scan_module);
    release_prev(m->prev_exscan_module);
    release_prev(m->prev_iallreduce_module);
    release_prev(m->prev_ireduce_module);
    release_prev(m->prev_ireduce_scatter_block_module);
    release_prev(m->prev_iallgather_module);
    release_prev(m->prev_ibcast_module);
    for (int i = 0; i < 8; ++i)
        if (m->ddt_cache[i].d) mi355x_ddt_destroy(m->ddt_cache[i].d);
    for (int i = 0; i < 2; ++i)
        if (m->scratch[i]) mi355x_free(m->scratch[i]);
    if (m->engine) mi355x_comm_destroy(m->engine);
}

static opal_class_t mca_coll_mi355x_module_t_class = {
    "mca_coll_mi355x_module_t", &mca_coll_base_module_t_class, module_construct, module_destruct,
    0, 0, NULL, NULL, sizeof(mca_coll_mi355x_module_t)
};

/* ------------------------------------------------------------------ helpers */
static int env_int(const char *name, int dflt)
{
    const char *v = getenv(name);
    return v ? atoi(v) : dflt;
}

static int is_dev(const void *p)
{
    int d = 0;
    if (!p || p == MPI_IN_PLACE) return 0;
    if (mi355x_ptr_is_device(p, &d) != MI355X_SUCCESS) return 0;
    return d;
}

/* The op slot of a datatype the engine can reduce, else -1.  The test is the reference's own: a
 * type predefined as an MPI type (ompi_datatype_is_predefined, ompi_datatype.h:149-152 -- libmpi
 * clears the OPAL flag on the MPI-2 pair types, ompi_datatype_module.c:415-416, 431-432, so that
 * flag would reject every MAXLOC/MINLOC type) whose id maps to an op slot (ompi_op_ddt_map, the
 * lookup ompi_op_reduce makes, op.h:570-574).  The engine moves count x extent bytes: the slot's
 * element is the C layout of the type (pair padding included), so the extent must equal it and
 * the type must start at its lower bound -- NO_GAPS is not required (MPI_DOUBLE_INT is 12 bytes of
 * data in a 16-byte extent, MPI_SHORT_INT 6 in 8). */
static int reducible_type(const struct ompi_datatype_t *dt)
{
    if (!(dt->super.flags & OMPI_DATATYPE_FLAG_PREDEFINED)) return -1;
    if (dt->id < 0 || dt->id >= OMPI_DATATYPE_MPI_MAX_PREDEFINED) return -1;
    const int t = ompi_op_ddt_map[dt->id];
    if (t < 0) return -1;
    const size_t esz = mi355x_type_size(t);
    if (esz == 0 || dt->super.lb != 0 || dt->super.true_lb != 0 || (size_t)(dt->super.ub - dt->super.lb) != esz) return -1;
    return t;
}

/* the op slot the engine would reduce dt as, or -1 (exported for the boundary tests) */
int mca_coll_mi355x_reducible_type(const struct ompi_datatype_t *dt) { return reducible_type(dt); }

/* bytes spanned by `count` instances of dt: true_extent + (count - 1) x extent, the staging size
 * coll/cuda uses (coll_cuda_allreduce.c:44-46) */
static size_t dt_span(const struct ompi_datatype_t *dt, size_t count)
{
    if (count == 0) return 0;
    const ptrdiff_t ext = dt->super.ub - dt->super.lb, text = dt->super.true_ub - dt->super.true_lb;
    return (size_t)(text + (ptrdiff_t)(count - 1) * ext);
}

/* counts are size_t here: a block count times the communicator size (allgather's unpack of n
 * blocks) may exceed INT_MAX; negative int counts are rejected by the callers */
static int contiguous_bytes_n(const struct ompi_datatype_t *dt, size_t count, size_t *bytes)
{
    if (!(dt->super.flags & OPAL_DATATYPE_FLAG_NO_GAPS) || dt->super.true_lb != 0) return 0;
    *bytes = count * dt->super.size;
    return 1;
}

static int contiguous_bytes(const struct ompi_datatype_t *dt, int count, size_t *bytes)
{
    if (count < 0) return 0;
    return contiguous_bytes_n(dt, (size_t)count, bytes);
}

/* ------------------------------------------------------------------ derived datatypes
 * A non-contiguous datatype on device memory moves through the GPU convertor: the layout is
 * compiled once from the datatype's optimized description (opt_desc, the one
 * OPAL_CONVERTOR_PREPARE selects, opal_convertor.c:513), packed into a device staging buffer,
 * moved as bytes by the engine, and unpacked -- the device-side equivalent of the convertor
 * pack/unpack the PML runs per fragment (opal_datatype_pack.c:250-374, _unpack.c:245-...). */

/* sizes of the OPAL basic types by id (opal/datatype/opal_datatype_internal.h:107-131; x86-64:
 * long double is FLOAT16) */
static const uint32_t opal_basic_sizes[25] = {0, 0, 0, 0, 1, 2, 4, 8, 16, 1, 2, 4, 8, 16, 2, 4, 8, 12, 16,
                                              8, 16, 32, 1, 4, 0};

static uint64_t fnv1a(uint64_t h, const void *p, size_t n)
{
    const unsigned char *b = (const unsigned char *)p;
    for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 1099511628211ull;
    return h;
}

/* a new layout of dt (the caller owns it), or NULL when the convertor cannot take it */
static mi355x_ddt_t *ddt_private(const struct ompi_datatype_t *dt)
{
    const dt_type_desc_t *td = dt->super.opt_desc.desc ? &dt->super.opt_desc : &dt->super.desc;
    if (!td->desc || td->used == 0 || dt->super.size == 0) return NULL;
    const int64_t ext = (int64_t)(dt->super.ub - dt->super.lb);
    mi355x_ddt_t *d = NULL;
    if (mi355x_ddt_from_opal(td->desc, td->used, ext, opal_basic_sizes, &d) != MI355X_SUCCESS) return NULL;
    if (mi355x_ddt_size(d) != dt->super.size) {
        mi355x_ddt_destroy(d);
        return NULL;
    }
    return d;
}

/* the layout of dt, or NULL when the convertor cannot take it (the caller then falls back);
 * cached per module (8 entries: valid until the call returns) */
static mi355x_ddt_t *ddt_of(struct mca_coll_mi355x_module_t *m, const struct ompi_datatype_t *dt)
{
    const dt_type_desc_t *td = dt->super.opt_desc.desc ? &dt->super.opt_desc : &dt->super.desc;
    if (!td->desc || td->used == 0 || dt->super.size == 0) return NULL;
    const size_t rec = 32; /* sizeof(dt_elem_desc_t), opal_datatype_internal.h:185-189 */
    uint64_t sig = fnv1a(1469598103934665603ull, td->desc, (size_t)td->used * rec);
    const int64_t ext = (int64_t)(dt->super.ub - dt->super.lb);
    sig = fnv1a(sig, &dt->super.size, sizeof(dt->super.size));
    sig = fnv1a(sig, &ext, sizeof(ext));
    for (int i = 0; i < 8; ++i)
        if (m->ddt_cache[i].d && m->ddt_cache[i].dt == dt && m->ddt_cache[i].sig == sig) return m->ddt_cache[i].d;
    mi355x_ddt_t *d = ddt_private(dt);
    if (!d) return NULL;
    struct ddt_slot *e = &m->ddt_cache[m->ddt_next];
    m->ddt_next = (m->ddt_next + 1) & 7;
    if (e->d) mi355x_ddt_destroy(e->d);
    e->d = d;
    e->dt = dt;
    e->sig = sig;
    return d;
}

static void *scratch_slot(struct mca_coll_mi355x_module_t *m, int slot, size_t bytes)
{
    if (bytes <= m->scratch_bytes[slot]) return m->scratch[slot];
    if (m->scratch[slot]) mi355x_free(m->scratch[slot]);
    m->scratch[slot] = NULL;
    m->scratch_bytes[slot] = 0;
    size_t want = bytes < ((size_t)1 << 20) ? ((size_t)1 << 20) : bytes;
    if (mi355x_malloc(&m->scratch[slot], want) != MI355X_SUCCESS) return NULL;
    m->scratch_bytes[slot] = want;
    return m->scratch[slot];
}

static void *scratch(struct mca_coll_mi355x_module_t *m, size_t bytes) { return scratch_slot(m, 0, bytes); }

/* one side of a convertor move: (buf, count, dt) <-> packed bytes at p */
static int stage(struct mca_coll_mi355x_module_t *m, int pack, void *buf, size_t count, const struct ompi_datatype_t *dt,
                 void *p, size_t bytes)
{
    size_t cb;
    if (contiguous_bytes_n(dt, count, &cb))
        return pack ? mi355x_memcpy_async(p, buf, bytes, NULL) : mi355x_memcpy_async(buf, p, bytes, NULL);
    mi355x_ddt_t *d = ddt_of(m, dt);
    if (!d) return MI355X_ERR_UNSUPPORTED;
    return pack ? mi355x_pack(d, count, buf, 0, p, bytes, NULL, NULL)
                : mi355x_unpack(d, count, buf, 0, p, bytes, NULL, NULL);
}

/* stage() for a buffer that may be host memory: dense host layouts are copied, derived ones go
 * through the host convertor (mi355x_pack_host / mi355x_unpack_host) and a host bounce buffer --
 * the GPU convertor never touches host memory */
static int xstage(struct mca_coll_mi355x_module_t *m, int pack, void *buf, size_t count, const struct ompi_datatype_t *dt,
                  void *p, size_t bytes, int host)
{
    if (!host) return stage(m, pack, buf, count, dt, p, bytes);
    size_t cb;
    if (bytes == 0) return MI355X_SUCCESS;
    if (contiguous_bytes_n(dt, count, &cb)) return pack ? mi355x_memcpy(p, buf, bytes) : mi355x_memcpy(buf, p, bytes);
    mi355x_ddt_t *d = ddt_of(m, dt);
    if (!d) return MI355X_ERR_UNSUPPORTED;
    void *tmp = malloc(bytes);
    if (!tmp) return MI355X_ERR_NOMEM;
    int rc;
    if (pack) {
        rc = mi355x_pack_host(d, count, buf, 0, tmp, bytes);
        if (rc == MI355X_SUCCESS) rc = mi355x_memcpy(p, tmp, bytes);
    } else {
        rc = mi355x_memcpy(tmp, p, bytes);
        if (rc == MI355X_SUCCESS) rc = mi355x_unpack_host(d, count, buf, 0, tmp, bytes);
    }
    free(tmp);
    return rc;
}

static int map_rc(int rc)
{
    switch (rc) {
    case MI355X_SUCCESS: return OMPI_SUCCESS;
    case MI355X_ERR_ARG: return OMPI_ERR_BAD_PARAM;
    case MI355X_ERR_NOMEM: return OMPI_ERR_OUT_OF_RESOURCE;
    case MI355X_ERR_UNSUPPORTED: return OMPI_ERR_NOT_SUPPORTED;
    default:
        fprintf(stderr, "[coll/mi355x] %s\n", mi355x_last_error());
        return OMPI_ERROR;
    }
}

#define MOD(m) ((mca_coll_mi355x_module_t *)(m))

/* ------------------------------------------------------------------ mixed host / device buffers
 * coll/cuda lets ranks mix host and device buffers in one collective: each rank stages its own to
 * the host and runs the host algorithm (coll_cuda_allreduce.c:30-77).  Here the engine runs only
 * if every rank joins it, so for the collectives below every rank votes its buffer kind
 * (mi355x_comm_vote, coll_mi355x_mixed_buffers = 1, the default): a rank with device buffers goes
 * to the engine at once; a rank with host buffers learns whether any peer has device buffers --
 * if so it joins the engine on device copies of its buffers (the staging runs the other way from
 * coll/cuda's), if not every rank takes the previous component's host path.  Ranks with host
 * buffers need contiguous layouts to join (derived host layouts are an error in a mixed call). */
int mca_coll_mi355x_mixed_buffers = 1;
int mca_coll_mi355x_rcache_max_maps = 0;
unsigned long long mca_coll_mi355x_rcache_size_limit = 0;
/* the engine's crossovers and flow parameters (registered in component_register, applied to every
 * communicator's engine in module_enable; defaults = the engine's own) */
int mca_coll_mi355x_pipe_min_ranks = 4;
int mca_coll_mi355x_pipe_chunk_kib = 0;
int mca_coll_mi355x_pipe_wg_per_cu = 2;
int mca_coll_mi355x_pipe_wt = 1;
unsigned long long mca_coll_mi355x_one_phase_max = 1ull << 20;
unsigned long long mca_coll_mi355x_svc_max = 32ull << 10;
unsigned long long mca_coll_mi355x_svc_pull_max = 128ull << 10;
unsigned long long mca_coll_mi355x_svc_copy_max = 1ull << 20;
int mca_coll_mi355x_svc_idle_us = 1000;
int mca_coll_mi355x_svc_shrink_us = 100;
int mca_coll_mi355x_selftest = 1;
int mca_coll_mi355x_timeout_s = 0;  /* 0: the engine's own (MI355X_TIMEOUT_S, else one day) */

/* 1: the call runs in the engine (a rank with host buffers joins on device copies); 0: it runs in
 * the previous component on every rank (a rank with device buffers stages them to the host, as
 * coll/cuda does); < 0: an error (the vote failed).  dev: this rank's buffers are all device
 * memory.  Which side of a call waits for the other's votes is agreed per window of calls
 * (mi355x_comm_vote), so a host-only program pays a store per call, a device program nothing. */
static int route(mca_coll_mi355x_module_t *m, int dev)
{
    if (!m->mixed) return dev;
    int engine = dev;
    const int rc = mi355x_comm_vote(m->engine, dev, &engine);
    if (rc != MI355X_SUCCESS) {
        fprintf(stderr, "[coll/mi355x] %s\n", mi355x_last_error());
        return -1;
    }
    return engine;
}

/* device copy of a host input (scratch slot `slot`), or the buffer itself when it is on the device */
static void *dev_in(mca_coll_mi355x_module_t *m, int slot, const void *buf, size_t bytes, int *rc)
{
    if (is_dev(buf)) return (void *)buf;
    void *d = scratch_slot(m, slot, bytes ? bytes : 1);
    if (!d) {
        *rc = MI355X_ERR_NOMEM;
        return NULL;
    }
    if (bytes && *rc == MI355X_SUCCESS) *rc = mi355x_memcpy(d, buf, bytes);
    return d;
}

/* device stand-in for a host output (contents undefined until the call fills it) */
static void *dev_out(mca_coll_mi355x_module_t *m, int slot, void *buf, size_t bytes, int *rc)
{
    if (is_dev(buf)) return buf;
    void *d = scratch_slot(m, slot, bytes ? bytes : 1);
    if (!d) *rc = MI355X_ERR_NOMEM;
    return d;
}

static int copy_back(void *host, const void *dev, size_t bytes, int rc)
{
    if (rc != MI355X_SUCCESS || host == dev || bytes == 0) return rc;
    return mi355x_memcpy(host, dev, bytes);
}

/* PREV_CALL: the previous component on this rank's own (host) buffers; STAGED_CALL: the same with
 * this rank's device buffers staged through host memory (a device rank in a call that runs on the
 * host) */
#define ROUTE_OR(PREV_CALL, STAGED_CALL)                                               \
    do {                                                                               \
        const int r_ = route(m, dev);                                                  \
        if (r_ < 0) return OMPI_ERROR;                                                 \
        if (r_ == 0) return dev ? (STAGED_CALL) : (PREV_CALL);                         \
    } while (0)

/* ------------------------------------------------------------------ coll/cuda's host staging
 * A reduction the engine declines -- a user-defined MPI_Op, or a type with no engine slot (the x87
 * long double slots the engine has no fold for) -- goes to the lower-priority component, which
 * reads and writes the buffers on the CPU (coll/tuned: opal_datatype_copy_content_same_ddt and
 * ompi_op_reduce on the user's pointers, coll_tuned_allreduce.c:166, 182-185).  Every device
 * buffer of such a call is staged through host memory around it, exactly what coll/cuda does for
 * each call it intercepts (coll_cuda_allreduce.c:43-75, coll_cuda_reduce.c:43-78,
 * coll_cuda_reduce_scatter_block.c:45-83, coll_cuda_scan.c:41-76, coll_cuda_exscan.c:41-76;
 * saved functions coll_cuda_module.c:120-157): the span true_extent + (count - 1) x extent is
 * copied from the type's true lower bound and the host component gets the copy minus true_lb.
 * (coll/cuda copies from the buffer pointer itself and passes copy - true_lb, which is the same
 * thing for every type with true_lb == 0, the predefined ones.)  Nonblocking forms stage at
 * initiation and copy back when the host request completes. */
unsigned long mca_coll_mi355x_staged_calls;  /* calls that went through this staging (tests read it) */

typedef struct {
    char *h;       /* host copy (malloc); NULL: the buffer is not staged */
    char *d;       /* first byte of the device span */
    size_t back;   /* bytes copied back when the call succeeded (0: an input only) */
} hstage_t;

/* stage *arg when it is device memory (span bytes from its true lower bound); *arg becomes the
 * pointer the host component gets.  fill: copy the device contents in. */
static int hstage(hstage_t *s, void **arg, const struct ompi_datatype_t *dt, size_t span, int fill, size_t back)
{
    memset(s, 0, sizeof(*s));
    void *buf = *arg;
    if (!buf || buf == MPI_IN_PLACE || !is_dev(buf)) return OMPI_SUCCESS;
    s->h = (char *)malloc(span ? span : 1);
    if (!s->h) return OMPI_ERR_OUT_OF_RESOURCE;
    s->d = (char *)buf + dt->super.true_lb;
    s->back = back;
    if (fill && span && mi355x_memcpy(s->h, s->d, span) != MI355X_SUCCESS) {
        fprintf(stderr, "[coll/mi355x] staging: %s\n", mi355x_last_error());
        free(s->h);
        s->h = NULL;
        return OMPI_ERROR;
    }
    *arg = s->h - dt->super.true_lb;
    return OMPI_SUCCESS;
}

/* copy the result back (when rc is success) and release the copy; returns the call's status */
static int hunstage(hstage_t *s, int rc)
{
    if (!s->h) return rc;
    if (rc == OMPI_SUCCESS && s->back && mi355x_memcpy(s->d, s->h, s->back) != MI355X_SUCCESS) {
        fprintf(stderr, "[coll/mi355x] staging: %s\n", mi355x_last_error());
        rc = OMPI_ERROR;
    }
    free(s->h);
    s->h = NULL;
    return rc;
}

/* stage the send and receive sides of a reduction; on failure nothing stays staged */
static int hstage2(hstage_t st[2], void **sa, size_t sspan, void **ra, size_t rspan, int rfill, size_t rback,
                   const struct ompi_datatype_t *dt)
{
    int rc = hstage(&st[0], sa, dt, sspan, 1, 0);
    if (rc == OMPI_SUCCESS && (rc = hstage(&st[1], ra, dt, rspan, rfill, rback)) != OMPI_SUCCESS) hunstage(&st[0], rc);
    if (rc == OMPI_SUCCESS && (st[0].h || st[1].h)) __atomic_add_fetch(&mca_coll_mi355x_staged_calls, 1, __ATOMIC_RELAXED);
    return rc;
}

static int hunstage2(hstage_t st[2], int rc)
{
    hunstage(&st[0], rc);
    return hunstage(&st[1], rc);
}

/* the engine reduces (op, type slot t) on the device */
static int engine_op(const struct ompi_op_t *op, int t)
{
    return (op->o_flags & OMPI_OP_FLAGS_INTRINSIC) && t >= 0 && mi355x_comm_op_supported(op->o_f_to_c_index, t);
}

static int staged_allreduce(mca_coll_mi355x_module_t *m, void *sbuf, void *rbuf, int count,
                            struct ompi_datatype_t *dtype, struct ompi_op_t *op, struct ompi_communicator_t *comm)
{
    const size_t span = dt_span(dtype, (size_t)count);
    hstage_t st[2];
    const int rc = hstage2(st, &sbuf, span, &rbuf, span, sbuf == MPI_IN_PLACE, span, dtype);
    if (rc != OMPI_SUCCESS) return rc;
    return hunstage2(st, m->prev_allreduce(sbuf, rbuf, count, dtype, op, comm, m->prev_allreduce_module));
}

/* coll_cuda_reduce.c:43-78; only the root's rbuf is significant */
static int staged_reduce(mca_coll_mi355x_module_t *m, void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                         struct ompi_op_t *op, int root, struct ompi_communicator_t *comm)
{
    const int me = mi355x_comm_rank_of(comm), inplace = (sbuf == MPI_IN_PLACE);
    const size_t span = dt_span(dtype, (size_t)count);
    hstage_t st[2];
    void *ra = me == root ? rbuf : NULL;
    const int rc = hstage2(st, &sbuf, span, &ra, span, inplace, span, dtype);
    if (rc != OMPI_SUCCESS) return rc;
    return hunstage2(st, m->prev_reduce(sbuf, me == root ? ra : rbuf, count, dtype, op, root, comm, m->prev_reduce_module));
}

/* coll_cuda_reduce_scatter_block.c:45-83 (in place: rbuf holds the n blocks) */
static int staged_reduce_scatter_block(mca_coll_mi355x_module_t *m, void *sbuf, void *rbuf, int rcount,
                                       struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                                       struct ompi_communicator_t *comm)
{
    const int inplace = (sbuf == MPI_IN_PLACE);
    const size_t in = dt_span(dtype, (size_t)rcount * (size_t)mi355x_comm_size_of(comm));
    const size_t out = dt_span(dtype, (size_t)rcount);
    hstage_t st[2];
    const int rc = hstage2(st, &sbuf, in, &rbuf, inplace ? in : out, inplace, out, dtype);
    if (rc != OMPI_SUCCESS) return rc;
    return hunstage2(st, m->prev_reduce_scatter_block(sbuf, rbuf, rcount, dtype, op, comm,
                                                      m->prev_reduce_scatter_block_module));
}

/* staged like reduce_scatter_block (in place: rbuf holds every block) */
static int staged_reduce_scatter(mca_coll_mi355x_module_t *m, void *sbuf, void *rbuf, int *rcounts,
                                 struct ompi_datatype_t *dtype, struct ompi_op_t *op, struct ompi_communicator_t *comm)
{
    const int inplace = (sbuf == MPI_IN_PLACE);
    const int n = mi355x_comm_size_of(comm), me = mi355x_comm_rank_of(comm);
    size_t total = 0;
    for (int q = 0; q < n; ++q) total += (size_t)(rcounts[q] > 0 ? rcounts[q] : 0);
    const size_t in = dt_span(dtype, total), out = dt_span(dtype, (size_t)(rcounts[me] > 0 ? rcounts[me] : 0));
    hstage_t st[2];
    const int rc = hstage2(st, &sbuf, in, &rbuf, inplace ? in : out, inplace, out, dtype);
    if (rc != OMPI_SUCCESS) return rc;
    return hunstage2(st, m->prev_reduce_scatter(sbuf, rbuf, rcounts, dtype, op, comm, m->prev_reduce_scatter_module));
}

/* the send and receive sides of a data-movement call staged to the host (coll/cuda's rule applied
 * to the movement collectives): the send span copied in; the receive span copied in too (its gaps
 * keep their bytes) and back after the call.  A side is (buffer, type, span); NULL / MPI_IN_PLACE /
 * host buffers are left alone. */
static int stage_move(hstage_t st[2], void **sa, const struct ompi_datatype_t *sdt, size_t sspan, void **ra,
                      const struct ompi_datatype_t *rdt, size_t rspan)
{
    memset(st, 0, 2 * sizeof(hstage_t));
    int rc = sa ? hstage(&st[0], sa, sdt, sspan, 1, 0) : OMPI_SUCCESS;
    if (rc == OMPI_SUCCESS && ra && (rc = hstage(&st[1], ra, rdt, rspan, 1, rspan)) != OMPI_SUCCESS) hunstage(&st[0], rc);
    if (rc == OMPI_SUCCESS && (st[0].h || st[1].h)) __atomic_add_fetch(&mca_coll_mi355x_staged_calls, 1, __ATOMIC_RELAXED);
    return rc;
}

/* bytes spanned by piece q = counts[q] instances at disps[q] extents (NULL disps: consecutive),
 * over every piece; SIZE_MAX when a displacement is negative (not staged: an error) */
static size_t vspan(const struct ompi_datatype_t *dt, int n, const int *counts, const int *disps)
{
    const ptrdiff_t ext = dt->super.ub - dt->super.lb;
    size_t best = 0, next = 0;
    for (int q = 0; q < n; ++q) {
        const size_t c = counts[q] > 0 ? (size_t)counts[q] : 0;
        const long d = disps ? (long)disps[q] : (long)next;
        if (d < 0) return (size_t)-1;
        next = (size_t)d + c;
        if (c) {
            const size_t e = (size_t)d * (size_t)ext + dt_span(dt, c);
            if (e > best) best = e;
        }
    }
    return best;
}

/* ------------------------------------------------------------------ collectives */
int mca_coll_mi355x_allreduce(void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                              struct ompi_op_t *op, struct ompi_communicator_t *comm,
                              mca_coll_base_module_t *module)
{
    mca_coll_mi355x_module_t *m = MOD(module);
    const int inplace = (sbuf == MPI_IN_PLACE);
    const int t = reducible_type(dtype);
    if (count < 0) return m->prev_allreduce(sbuf, rbuf, count, dtype, op, comm, m->prev_allreduce_module);
    if (!engine_op(op, t)) return staged_allreduce(m, sbuf, rbuf, count, dtype, op, comm);
    const int dev = is_dev(rbuf) && (inplace || is_dev(sbuf));
    ROUTE_OR(m->prev_allreduce(sbuf, rbuf, count, dtype, op, comm, m->prev_allreduce_module),
             staged_allreduce(m, sbuf, rbuf, count, dtype, op, comm));
    if (dev) return map_rc(mi355x_allreduce(m->engine, inplace ? NULL : sbuf, rbuf, (size_t)count, t, op->o_f_to_c_index, NULL));
    const size_t bytes = (size_t)count * mi355x_type_size(t);
    int rc = MI355X_SUCCESS;
    void *rd = inplace ? dev_in(m, 1, rbuf, bytes, &rc) : dev_out(m, 1, rbuf, bytes, &rc);
    const void *sd = inplace ? NULL : dev_in(m, 0, sbuf, bytes, &rc);
    if (rc == MI355X_SUCCESS) rc = mi355x_allreduce(m->engine, sd, rd, (size_t)count, t, op->o_f_to_c_index, NULL);
    return map_rc(copy_back(rbuf, rd, bytes, rc));
}

/* MPI_Reduce: the root's rbuf and every rank's sbuf (MPI_IN_PLACE: the root's rbuf) on the device;
 * a non-root's rbuf is not significant and never looked at */
int mca_coll_mi355x_reduce(void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                           int root, struct ompi_communicator_t *comm, mca_coll_base_module_t *module)
{
    mca_coll_mi355x_module_t *m = MOD(module);
    const int me = mi355x_comm_rank_of(comm);
    const int inplace = (sbuf == MPI_IN_PLACE);
    const int t = reducible_type(dtype);
    if ((inplace && me != root) || count < 0)
        return m->prev_reduce(sbuf, rbuf, count, dtype, op, root, comm, m->prev_reduce_module);
    if (!engine_op(op, t)) return staged_reduce(m, sbuf, rbuf, count, dtype, op, root, comm);
    const int dev = (me != root || is_dev(rbuf)) && (inplace || is_dev(sbuf));
    ROUTE_OR(m->prev_reduce(sbuf, rbuf, count, dtype, op, root, comm, m->prev_reduce_module),
             staged_reduce(m, sbuf, rbuf, count, dtype, op, root, comm));
    if (dev)
        return map_rc(mi355x_reduce(m->engine, inplace ? NULL : sbuf, me == root ? rbuf : NULL, (size_t)count, t,
                                    op->o_f_to_c_index, root, NULL));
    const size_t bytes = (size_t)count * mi355x_type_size(t);
    int rc = MI355X_SUCCESS;
    void *rd = me != root ? NULL : inplace ? dev_in(m, 1, rbuf, bytes, &rc) : dev_out(m, 1, rbuf, bytes, &rc);
    const void *sd = inplace ? NULL : dev_in(m, 0, sbuf, bytes, &rc);
    if (rc == MI355X_SUCCESS) rc = mi355x_reduce(m->engine, sd, rd, (size_t)count, t, op->o_f_to_c_index, root, NULL);
    return map_rc(me == root ? copy_back(rbuf, rd, bytes, rc) : rc);
}

int mca_coll_mi355x_reduce_scatter_block(void *sbuf, void *rbuf, int rcount, struct ompi_datatype_t *dtype,
                                         struct ompi_op_t *op, struct ompi_communicator_t *comm,
                                         mca_coll_base_module_t *module)
{
    mca_coll_mi355x_module_t *m = MOD(module);
    const int inplace = (sbuf == MPI_IN_PLACE);
    const int t = reducible_type(dtype);
    if (rcount < 0)
        return m->prev_reduce_scatter_block(sbuf, rbuf, rcount, dtype, op, comm, m->prev_reduce_scatter_block_module);
    if (!engine_op(op, t)) return staged_reduce_scatter_block(m, sbuf, rbuf, rcount, dtype, op, comm);
    const int dev = is_dev(rbuf) && (inplace || is_dev(sbuf));
    ROUTE_OR(m->prev_reduce_scatter_block(sbuf, rbuf, rcount, dtype, op, comm, m->prev_reduce_scatter_block_module),
             staged_reduce_scatter_block(m, sbuf, rbuf, rcount, dtype, op, comm));
    if (dev)
        return map_rc(mi355x_reduce_scatter_block(m->engine, inplace ? NULL : sbuf, rbuf, (size_t)rcount, t,
                                                  op->o_f_to_c_index, NULL));
    const size_t out = (size_t)rcount * mi355x_type_size(t), in = out * (size_t)mi355x_comm_size_of(comm);
    int rc = MI355X_SUCCESS;
    void *rd = inplace ? dev_in(m, 1, rbuf, in, &rc) : dev_out(m, 1, rbuf, out, &rc);
    const void *sd = inplace ? NULL : dev_in(m, 0, sbuf, in, &rc);
    if (rc == MI355X_SUCCESS)
        rc = mi355x_reduce_scatter_block(m->engine, sd, rd, (size_t)rcount, t, op->o_f_to_c_index, NULL);
    return map_rc(copy_back(rbuf, rd, out, rc));
}

int mca_coll_mi355x_reduce_scatter(void *sbuf, void *rbuf, int *rcounts, struct ompi_datatype_t *dtype,
                                   struct ompi_op_t *op, struct ompi_communicator_t *comm,
                                   mca_coll_base_module_t *module)
{
    mca_coll_mi355x_module_t *m = MOD(module);
    const int inplace = (sbuf == MPI_IN_PLACE);
    const int t = reducible_type(dtype);
    const int n = mi355x_comm_size_of(comm), me = mi355x_comm_rank_of(comm);
    size_t total = 0;
    for (int q = 0; q < n; ++q) total += (size_t)(rcounts[q] > 0 ? rcounts[q] : 0);
    if (!engine_op(op, t)) return staged_reduce_scatter(m, sbuf, rbuf, rcounts, dtype, op, comm);
    const int dev = is_dev(rbuf) && (inplace || is_dev(sbuf));
    ROUTE_OR(m->prev_reduce_scatter(sbuf, rbuf, rcounts, dtype, op, comm, m->prev_reduce_scatter_module),
             staged_reduce_scatter(m, sbuf, rbuf, rcounts, dtype, op, comm));
    if (dev) return map_rc(mi355x_reduce_scatter(m->engine, inplace ? NULL : sbuf, rbuf, rcounts, t, op->o_f_to_c_index, NULL));
    const size_t esz = mi355x_type_size(t), in = total * esz, out = (size_t)(rcounts[me] > 0 ? rcounts[me] : 0) * esz;
    int rc = MI355X_SUCCESS;
    void *rd = inplace ? dev_in(m, 1, rbuf, in, &rc) : dev_out(m, 1, rbuf, out, &rc);
    const void *sd = inplace ? NULL : dev_in(m, 0, sbuf, in, &rc);
    if (rc == MI355X_SUCCESS) rc = mi355x_reduce_scatter(m->engine, sd, rd, rcounts, t, op->o_f_to_c_index, NULL);
    return map_rc(copy_back(rbuf, rd, out, rc));
}

static int staged_allgather(mca_coll_mi355x_module_t *m, void *sbuf, int scount, struct ompi_datatype_t *sdtype,
                            void *rbuf, int rcount, struct ompi_datatype_t *rdtype, struct ompi_communicator_t *comm)
{
    hstage_t st[2];
    void *s = sbuf, *r = rbuf;
    int rc = stage_move(st, &s, sdtype, dt_span(sdtype, (size_t)scount), &r, rdtype,
                        dt_span(rdtype, (size_t)rcount * (size_t)mi355x_comm_size_of(comm)));
    if (rc != OMPI_SUCCESS) return rc;
    return hunstage2(st, m->prev_allgather(s, scount, sdtype, r, rcount, rdtype, comm, m->prev_allgather_module));
}

static int staged_bcast(mca_coll_mi355x_module_t *m, void *buff, int count, struct ompi_datatype_t *datatype, int root,
                        struct ompi_communicator_t *comm)
{
    hstage_t st[2];
    void *b = buff;
    const size_t span = dt_span(datatype, (size_t)count);
    const int me = mi355x_comm_rank_of(comm);
    int rc = me == root ? stage_move(st, &b, datatype, span, NULL, NULL, 0) : stage_move(st, NULL, NULL, 0, &b, datatype, span);
    if (rc != OMPI_SUCCESS) return rc;
    return hunstage2(st, m->prev_bcast(b, count, datatype, root, comm, m->prev_bcast_module));
}

int mca_coll_mi355x_allgather(void *sbuf, int scount, struct ompi_datatype_t *sdtype, void *rbuf, int rcount,
                              struct ompi_datatype_t *rdtype, struct ompi_communicator_t *comm,
                              mca_coll_base_module_t *module)
{
    mca_coll_mi355x_module_t *m = MOD(module);
    const int inplace = (sbuf == MPI_IN_PLACE);
    if (rcount < 0 || (!inplace && scount < 0))
        return m->prev_allgather(sbuf, scount, sdtype, rbuf, rcount, rdtype, comm, m->prev_allgather_module);
    const int dev = is_dev(rbuf) && (inplace || is_dev(sbuf));
    const int n = mi355x_comm_size_of(comm), me = mi355x_comm_rank_of(comm);
    ROUTE_OR(m->prev_allgather(sbuf, scount, sdtype, rbuf, rcount, rdtype, comm, m->prev_allgather_module),
             staged_allgather(m, sbuf, scount, sdtype, rbuf, rcount, rdtype, comm));
    size_t rb = 0, sb = 0;
    if (!dev) {  /* host buffers in a call where peers hold device ones: dense layouts, staged */
        if (!contiguous_bytes(rdtype, rcount, &rb) || (!inplace && (!contiguous_bytes(sdtype, scount, &sb) || sb != rb))) {
            fprintf(stderr, "[coll/mi355x] allgather: host buffers with a derived layout in a call with device peers\n");
            return OMPI_ERR_NOT_SUPPORTED;
        }
        int rc = MI355X_SUCCESS;
        void *rd = inplace ? dev_in(m, 1, rbuf, rb * (size_t)n, &rc) : dev_out(m, 1, rbuf, rb * (size_t)n, &rc);
        const void *sd = inplace ? NULL : dev_in(m, 0, sbuf, rb, &rc);
        if (rc == MI355X_SUCCESS) rc = mi355x_allgather(m->engine, sd, rd, rb, NULL);
        return map_rc(copy_back(rbuf, rd, rb * (size_t)n, rc));
    }
    if (contiguous_bytes(rdtype, rcount, &rb) && (inplace || (contiguous_bytes(sdtype, scount, &sb) && sb == rb)))
        return map_rc(mi355x_allgather(m->engine, inplace ? NULL : sbuf, rbuf, rb, NULL));
    /* derived datatypes: pack my block into the staging buffer, gather packed blocks in place,
     * unpack all n blocks with one launch (block r = instances [r*rcount, (r+1)*rcount)) */
    const size_t blk = (size_t)rcount * rdtype->super.size;
    if (!inplace && (size_t)scount * sdtype->super.size != blk) return OMPI_ERR_BAD_PARAM;
    /* a layout the convertor cannot describe is an error, never a rank-local fallback: the other
     * ranks (whose layouts may differ) are already in the engine */
    if ((!inplace && !contiguous_bytes(sdtype, scount, &sb) && !ddt_of(m, sdtype)) ||
        (!contiguous_bytes(rdtype, rcount, &rb) && !ddt_of(m, rdtype))) {
        fprintf(stderr, "[coll/mi355x] allgather: the GPU convertor cannot describe the datatype\n");
        return OMPI_ERR_NOT_SUPPORTED;
    }
    if (blk == 0) return OMPI_SUCCESS;
    char *st = (char *)scratch(m, blk * (size_t)n);
    if (!st) return OMPI_ERR_OUT_OF_RESOURCE;
    const ptrdiff_t rext = rdtype->super.ub - rdtype->super.lb;
    int rc = inplace ? stage(m, 1, (char *)rbuf + (ptrdiff_t)me * rcount * rext, rcount, rdtype, st + blk * me, blk)
                     : stage(m, 1, sbuf, scount, sdtype, st + blk * me, blk);
    if (rc == MI355X_SUCCESS) rc = mi355x_allgather(m->engine, NULL, st, blk, NULL);
    if (rc == MI355X_SUCCESS) rc = stage(m, 0, rbuf, (size_t)rcount * (size_t)n, rdtype, st, blk * (size_t)n);
    if (rc == MI355X_SUCCESS) rc = mi355x_stream_sync(NULL);
    return map_rc(rc);
}

int mca_coll_mi355x_bcast(void *buff, int count, struct ompi_datatype_t *datatype, int root,
                          struct ompi_communicator_t *comm, mca_coll_base_module_t *module)
{
    mca_coll_mi355x_module_t *m = MOD(module);
    size_t bytes = 0;
    if (count < 0) return m->prev_bcast(buff, count, datatype, root, comm, m->prev_bcast_module);
    const int dev = is_dev(buff);
    ROUTE_OR(m->prev_bcast(buff, count, datatype, root, comm, m->prev_bcast_module),
             staged_bcast(m, buff, count, datatype, root, comm));
    const int me = mi355x_comm_rank_of(comm);
    if (!dev) {  /* host buffer in a call where peers hold device ones: dense layouts, staged */
        if (!contiguous_bytes(datatype, count, &bytes)) {
            fprintf(stderr, "[coll/mi355x] bcast: a host buffer with a derived layout in a call with device peers\n");
            return OMPI_ERR_NOT_SUPPORTED;
        }
        int rc = MI355X_SUCCESS;
        void *bd = me == root ? dev_in(m, 1, buff, bytes, &rc) : dev_out(m, 1, buff, bytes, &rc);
        if (rc == MI355X_SUCCESS) rc = mi355x_bcast(m->engine, bd, bytes, root, NULL);
        return map_rc(me == root ? rc : copy_back(buff, bd, bytes, rc));
    }
    if (contiguous_bytes(datatype, count, &bytes)) return map_rc(mi355x_bcast(m->engine, buff, bytes, root, NULL));
    /* derived datatype: root packs, the packed bytes are broadcast, the others unpack */
    if (!ddt_of(m, datatype)) {  /* see allgather: no rank-local fallback */
        fprintf(stderr, "[coll/mi355x] bcast: the GPU convertor cannot describe datatype %s\n", datatype->name);
        return OMPI_ERR_NOT_SUPPORTED;
    }
    bytes = (size_t)count * datatype->super.size;
    if (bytes == 0) return OMPI_SUCCESS;
    void *st = scratch(m, bytes);
    if (!st) return OMPI_ERR_OUT_OF_RESOURCE;
    int rc = MI355X_SUCCESS;
    if (me == root) rc = stage(m, 1, buff, count, datatype, st, bytes);
    if (rc == MI355X_SUCCESS) rc = mi355x_bcast(m->engine, st, bytes, root, NULL);
    if (rc == MI355X_SUCCESS && me != root) rc = stage(m, 0, buff, count, datatype, st, bytes);
    if (rc == MI355X_SUCCESS) rc = mi355x_stream_sync(NULL);
    return map_rc(rc);
}

/* ------------------------------------------------------------------ gather / scatter / alltoall / scan
 * Which path a call takes may depend only on what MPI requires to agree across ranks (the type
 * SIGNATURES, so the byte counts, and the op) and on where the buffers are: never on a rank-local
 * datatype LAYOUT, which MPI lets differ between ranks (a root may receive into a resized column
 * type while the others send MPI_INT).  So every layout goes to the engine: a dense layout in
 * place, any other through the GPU convertor into a staging buffer -- packed before the call for
 * the bytes a rank sends, unpacked after for the bytes it receives.  A layout the convertor cannot
 * compile is an error, not a silent fallback (the other ranks are already in the engine). */
static int dense(const struct ompi_datatype_t *dt)
{
    return (dt->super.flags & OPAL_DATATYPE_FLAG_NO_GAPS) && dt->super.true_lb == 0 &&
           (size_t)(dt->super.ub - dt->super.lb) == dt->super.size;
}

#define SIDE_MAX 64
/* one rank's send or receive side as the engine sees it: `view` + per-piece byte counts and
 * offsets.  Piece q = cnt[q] instances of dt at base + udisp[q] (bytes). */
typedef struct {
    int n;
    char *base;
    mi355x_ddt_t *d;          /* NULL: dense, view == base */
    int host;                 /* host memory (a rank joining a call whose peers hold device buffers):
                                 the view is a device staging copy, moved by xstage */
    const struct ompi_datatype_t *dt;
    char *view;
    size_t bytes[SIDE_MAX], off[SIDE_MAX], cnt[SIDE_MAX];
    ptrdiff_t udisp[SIDE_MAX];
} side_t;

/* counts/displacements in instances (NULL disps: consecutive pieces of `counts`; NULL counts:
 * every piece `count1` instances).  Returns OMPI_SUCCESS or an error. */
static int side_init(mca_coll_mi355x_module_t *m, side_t *s, int slot, void *buf, const struct ompi_datatype_t *dt,
                     int n, const int *counts, int count1, const int *disps)
{
    if (n > SIDE_MAX) return OMPI_ERR_NOT_SUPPORTED;
    memset(s, 0, sizeof(*s));
    s->n = n;
    s->base = (char *)buf;
    const size_t sz = dt->super.size;
    const ptrdiff_t ext = dt->super.ub - dt->super.lb;
    ptrdiff_t next = 0;
    for (int q = 0; q < n; ++q) {
        const int c = counts ? counts[q] : count1;
        if (c < 0) return OMPI_ERR_BAD_PARAM;
        const ptrdiff_t dq = disps ? (ptrdiff_t)disps[q] : next;
        if (dq < 0) return OMPI_ERR_NOT_SUPPORTED;
        s->cnt[q] = (size_t)c;
        s->bytes[q] = (size_t)c * sz;
        s->udisp[q] = dq * ext;
        next = dq + c;
    }
    s->dt = dt;
    s->host = !is_dev(buf);
    if (dense(dt) && !s->host) {
        s->view = s->base;
        for (int q = 0; q < n; ++q) s->off[q] = (size_t)s->udisp[q];
        return OMPI_SUCCESS;
    }
    s->d = dense(dt) ? NULL : ddt_of(m, dt);
    if (!s->d && !dense(dt)) {
        fprintf(stderr, "[coll/mi355x] the GPU convertor cannot describe datatype %s\n", dt->name);
        return OMPI_ERR_NOT_SUPPORTED;
    }
    size_t total = 0;
    for (int q = 0; q < n; ++q) {
        s->off[q] = total;
        total += s->bytes[q];
    }
    s->view = (char *)scratch_slot(m, slot, total ? total : 1);
    return s->view ? OMPI_SUCCESS : OMPI_ERR_OUT_OF_RESOURCE;
}

/* piece q (or every piece, q < 0): user layout -> view (pack) or view -> user layout (unpack) */
static int side_move(mca_coll_mi355x_module_t *m, side_t *s, int q, int pack)
{
    if (!s->d && !s->host) return MI355X_SUCCESS;
    for (int p = (q < 0 ? 0 : q); p < (q < 0 ? s->n : q + 1); ++p) {
        if (!s->bytes[p]) continue;
        int rc = s->host ? xstage(m, pack, s->base + s->udisp[p], s->cnt[p], s->dt, s->view + s->off[p], s->bytes[p], 1)
                 : pack ? mi355x_pack(s->d, s->cnt[p], s->base + s->udisp[p], 0, s->view + s->off[p], s->bytes[p], NULL, NULL)
                        : mi355x_unpack(s->d, s->cnt[p], s->base + s->udisp[p], 0, s->view + s->off[p], s->bytes[p], NULL, NULL);
        if (rc) return rc;
    }
    return MI355X_SUCCESS;
}

static int finish_unpack(mca_coll_mi355x_module_t *m, side_t *s, int rc)
{
    if (rc == MI355X_SUCCESS && s && (s->d || s->host)) {
        rc = side_move(m, s, -1, 0);
        if (rc == MI355X_SUCCESS) rc = mi355x_stream_sync(NULL);
    }
    return map_rc(rc);
}

int mca_coll_mi355x_gather(void *sbuf, int scount, struct ompi_datatype_t *sdtype, void *rbuf, int rcount,
                           struct ompi_datatype_t *rdtype, int root, struct ompi_communicator_t *comm,
                           mca_coll_base_module_t *module)
{
    mca_coll_mi355x_module_t *m = MOD(module);
    const int n = mi355x_comm_size_of(comm), me = mi355x_comm_rank_of(comm), inplace = (sbuf == MPI_IN_PLACE);
    if (inplace && me != root)
        return m->prev_gather(sbuf, scount, sdtype, rbuf, rcount, rdtype, root, comm, m->prev_gather_module);
    const int dev = (me != root || is_dev(rbuf)) && (inplace || is_dev(sbuf));
    ROUTE_OR(m->prev_gather(sbuf, scount, sdtype, rbuf, rcount, rdtype, root, comm, m->prev_gather_module), ({
                 hstage_t st_[2];
                 void *s_ = sbuf, *r_ = rbuf;
                 int rc_ = stage_move(st_, inplace ? NULL : &s_, sdtype, dt_span(sdtype, (size_t)scount),
                                      me == root ? &r_ : NULL, rdtype, dt_span(rdtype, (size_t)rcount * (size_t)n));
                 rc_ == OMPI_SUCCESS ? hunstage2(st_, m->prev_gather(s_, scount, sdtype, r_, rcount, rdtype, root, comm,
                                                                     m->prev_gather_module)) : rc_;
             }));
    side_t snd, rcv;
    int rc = OMPI_SUCCESS;
    if (!inplace && (rc = side_init(m, &snd, 0, sbuf, sdtype, 1, NULL, scount, NULL))) return rc;
    if (me == root && (rc = side_init(m, &rcv, 1, rbuf, rdtype, n, NULL, rcount, NULL))) return rc;
    const size_t bytes = inplace ? rcv.bytes[me] : snd.bytes[0];
    int erc = inplace ? side_move(m, &rcv, me, 1) : side_move(m, &snd, 0, 1);
    if (erc == MI355X_SUCCESS)
        erc = mi355x_gather(m->engine, inplace ? NULL : snd.view, me == root ? rcv.view : NULL, bytes, root, NULL);
    return finish_unpack(m, me == root ? &rcv : NULL, erc);
}

int mca_coll_mi355x_gatherv(void *sbuf, int scount, struct ompi_datatype_t *sdtype, void *rbuf, int *rcounts,
                            int *disps, struct ompi_datatype_t *rdtype, int root, struct ompi_communicator_t *comm,
                            mca_coll_base_module_t *module)
{
    mca_coll_mi355x_module_t *m = MOD(module);
    const int n = mi355x_comm_size_of(comm), me = mi355x_comm_rank_of(comm), inplace = (sbuf == MPI_IN_PLACE);
    if (n > SIDE_MAX || (inplace && me != root))
        return m->prev_gatherv(sbuf, scount, sdtype, rbuf, rcounts, disps, rdtype, root, comm, m->prev_gatherv_module);
    const int dev = (me != root || is_dev(rbuf)) && (inplace || is_dev(sbuf));
    ROUTE_OR(m->prev_gatherv(sbuf, scount, sdtype, rbuf, rcounts, disps, rdtype, root, comm, m->prev_gatherv_module), ({
                 hstage_t st_[2];
                 void *s_ = sbuf, *r_ = rbuf;
                 const size_t rs_ = me == root ? vspan(rdtype, n, rcounts, disps) : 0;
                 int rc_ = rs_ == (size_t)-1 ? OMPI_ERR_NOT_SUPPORTED
                                             : stage_move(st_, inplace ? NULL : &s_, sdtype, dt_span(sdtype, (size_t)scount),
                                                          me == root ? &r_ : NULL, rdtype, rs_);
                 rc_ == OMPI_SUCCESS ? hunstage2(st_, m->prev_gatherv(s_, scount, sdtype, r_, rcounts, disps, rdtype, root,
                                                                      comm, m->prev_gatherv_module)) : rc_;
             }));
    side_t snd, rcv;
    int rc = OMPI_SUCCESS;
    if (!inplace && (rc = side_init(m, &snd, 0, sbuf, sdtype, 1, NULL, scount, NULL))) return rc;
    if (me == root && (rc = side_init(m, &rcv, 1, rbuf, rdtype, n, rcounts, 0, disps))) return rc;
    int erc = inplace ? side_move(m, &rcv, me, 1) : side_move(m, &snd, 0, 1);
    if (erc == MI355X_SUCCESS)
        erc = mi355x_gatherv(m->engine, inplace ? NULL : snd.view, inplace ? 0 : snd.bytes[0],
                             me == root ? rcv.view : NULL, me == root ? rcv.bytes : NULL,
                             me == root ? rcv.off : NULL, root, NULL);
    return finish_unpack(m, me == root ? &rcv : NULL, erc);
}

int mca_coll_mi355x_scatter(void *sbuf, int scount, struct ompi_datatype_t *sdtype, void *rbuf, int rcount,
                            struct ompi_datatype_t *rdtype, int root, struct ompi_communicator_t *comm,
                            mca_coll_base_module_t *module)
{
    mca_coll_mi355x_module_t *m = MOD(module);
    const int n = mi355x_comm_size_of(comm), me = mi355x_comm_rank_of(comm), inplace = (rbuf == MPI_IN_PLACE);
    if (inplace && me != root)
        return m->prev_scatter(sbuf, scount, sdtype, rbuf, rcount, rdtype, root, comm, m->prev_scatter_module);
    const int dev = (me != root || is_dev(sbuf)) && (inplace || is_dev(rbuf));
    ROUTE_OR(m->prev_scatter(sbuf, scount, sdtype, rbuf, rcount, rdtype, root, comm, m->prev_scatter_module), ({
                 hstage_t st_[2];
                 void *s_ = sbuf, *r_ = rbuf;
                 int rc_ = stage_move(st_, me == root ? &s_ : NULL, sdtype, dt_span(sdtype, (size_t)scount * (size_t)n),
                                      inplace ? NULL : &r_, rdtype, dt_span(rdtype, (size_t)rcount));
                 rc_ == OMPI_SUCCESS ? hunstage2(st_, m->prev_scatter(s_, scount, sdtype, r_, rcount, rdtype, root, comm,
                                                                      m->prev_scatter_module)) : rc_;
             }));
    side_t snd, rcv;
    int rc = OMPI_SUCCESS;
    if (me == root && (rc = side_init(m, &snd, 0, sbuf, sdtype, n, NULL, scount, NULL))) return rc;
    if (!inplace && (rc = side_init(m, &rcv, 1, rbuf, rdtype, 1, NULL, rcount, NULL))) return rc;
    const size_t bytes = me == root ? snd.bytes[0] : rcv.bytes[0];
    int erc = me == root ? side_move(m, &snd, -1, 1) : MI355X_SUCCESS;
    if (erc == MI355X_SUCCESS)
        erc = mi355x_scatter(m->engine, me == root ? snd.view : NULL, inplace ? NULL : rcv.view, bytes, root, NULL);
    return finish_unpack(m, inplace ? NULL : &rcv, erc);
}

int mca_coll_mi355x_scatterv(void *sbuf, int *scounts, int *disps, struct ompi_datatype_t *sdtype, void *rbuf,
                             int rcount, struct ompi_datatype_t *rdtype, int root, struct ompi_communicator_t *comm,
                             mca_coll_base_module_t *module)
{
    mca_coll_mi355x_module_t *m = MOD(module);
    const int n = mi355x_comm_size_of(comm), me = mi355x_comm_rank_of(comm), inplace = (rbuf == MPI_IN_PLACE);
    if (n > SIDE_MAX || (inplace && me != root))
        return m->prev_scatterv(sbuf, scounts, disps, sdtype, rbuf, rcount, rdtype, root, comm,
                                m->prev_scatterv_module);
    const int dev = (me != root || is_dev(sbuf)) && (inplace || is_dev(rbuf));
    ROUTE_OR(m->prev_scatterv(sbuf, scounts, disps, sdtype, rbuf, rcount, rdtype, root, comm, m->prev_scatterv_module), ({
                 hstage_t st_[2];
                 void *s_ = sbuf, *r_ = rbuf;
                 const size_t ss_ = me == root ? vspan(sdtype, n, scounts, disps) : 0;
                 int rc_ = ss_ == (size_t)-1 ? OMPI_ERR_NOT_SUPPORTED
                                             : stage_move(st_, me == root ? &s_ : NULL, sdtype, ss_, inplace ? NULL : &r_,
                                                          rdtype, dt_span(rdtype, (size_t)rcount));
                 rc_ == OMPI_SUCCESS ? hunstage2(st_, m->prev_scatterv(s_, scounts, disps, sdtype, r_, rcount, rdtype, root,
                                                                       comm, m->prev_scatterv_module)) : rc_;
             }));
    side_t snd, rcv;
    int rc = OMPI_SUCCESS;
    if (me == root && (rc = side_init(m, &snd, 0, sbuf, sdtype, n, scounts, 0, disps))) return rc;
    if (!inplace && (rc = side_init(m, &rcv, 1, rbuf, rdtype, 1, NULL, rcount, NULL))) return rc;
    int erc = me == root ? side_move(m, &snd, -1, 1) : MI355X_SUCCESS;
    if (erc == MI355X_SUCCESS)
        erc = mi355x_scatterv(m->engine, me == root ? snd.view : NULL, me == root ? snd.bytes : NULL,
                              me == root ? snd.off : NULL, inplace ? NULL : rcv.view, inplace ? 0 : rcv.bytes[0], root,
                              NULL);
    return finish_unpack(m, inplace ? NULL : &rcv, erc);
}

int mca_coll_mi355x_allgatherv(void *sbuf, int scount, struct ompi_datatype_t *sdtype, void *rbuf, int *rcounts,
                               int *disps, struct ompi_datatype_t *rdtype, struct ompi_communicator_t *comm,
                               mca_coll_base_module_t *module)
{
    mca_coll_mi355x_module_t *m = MOD(module);
    const int n = mi355x_comm_size_of(comm), me = mi355x_comm_rank_of(comm), inplace = (sbuf == MPI_IN_PLACE);
    if (n > SIDE_MAX)
        return m->prev_allgatherv(sbuf, scount, sdtype, rbuf, rcounts, disps, rdtype, comm, m->prev_allgatherv_module);
    const int dev = is_dev(rbuf) && (inplace || is_dev(sbuf));
    ROUTE_OR(m->prev_allgatherv(sbuf, scount, sdtype, rbuf, rcounts, disps, rdtype, comm, m->prev_allgatherv_module), ({
                 hstage_t st_[2];
                 void *s_ = sbuf, *r_ = rbuf;
                 const size_t rs_ = vspan(rdtype, n, rcounts, disps);
                 int rc_ = rs_ == (size_t)-1 ? OMPI_ERR_NOT_SUPPORTED
                                             : stage_move(st_, inplace ? NULL : &s_, sdtype, dt_span(sdtype, (size_t)scount),
                                                          &r_, rdtype, rs_);
                 rc_ == OMPI_SUCCESS ? hunstage2(st_, m->prev_allgatherv(s_, scount, sdtype, r_, rcounts, disps, rdtype, comm,
                                                                         m->prev_allgatherv_module)) : rc_;
             }));
    side_t snd, rcv;
    int rc = OMPI_SUCCESS;
    if (!inplace && (rc = side_init(m, &snd, 0, sbuf, sdtype, 1, NULL, scount, NULL))) return rc;
    if ((rc = side_init(m, &rcv, 1, rbuf, rdtype, n, rcounts, 0, disps))) return rc;
    int erc = inplace ? side_move(m, &rcv, me, 1) : side_move(m, &snd, 0, 1);
    if (erc == MI355X_SUCCESS)
        erc = mi355x_allgatherv(m->engine, inplace ? NULL : snd.view, inplace ? 0 : snd.bytes[0], rcv.view, rcv.bytes,
                                rcv.off, NULL);
    return finish_unpack(m, &rcv, erc);
}

int mca_coll_mi355x_alltoall(void *sbuf, int scount, struct ompi_datatype_t *sdtype, void *rbuf, int rcount,
                             struct ompi_datatype_t *rdtype, struct ompi_communicator_t *comm,
                             mca_coll_base_module_t *module)
{
    mca_coll_mi355x_module_t *m = MOD(module);
    const int n = mi355x_comm_size_of(comm), inplace = (sbuf == MPI_IN_PLACE);
    if (n > SIDE_MAX) return m->prev_alltoall(sbuf, scount, sdtype, rbuf, rcount, rdtype, comm, m->prev_alltoall_module);
    const int dev = is_dev(rbuf) && (inplace || is_dev(sbuf));
    ROUTE_OR(m->prev_alltoall(sbuf, scount, sdtype, rbuf, rcount, rdtype, comm, m->prev_alltoall_module), ({
                 hstage_t st_[2];
                 void *s_ = sbuf, *r_ = rbuf;
                 int rc_ = stage_move(st_, inplace ? NULL : &s_, sdtype, dt_span(sdtype, (size_t)scount * (size_t)n), &r_,
                                      rdtype, dt_span(rdtype, (size_t)rcount * (size_t)n));
                 rc_ == OMPI_SUCCESS ? hunstage2(st_, m->prev_alltoall(s_, scount, sdtype, r_, rcount, rdtype, comm,
                                                                       m->prev_alltoall_module)) : rc_;
             }));
    side_t snd, rcv;
    int rc = OMPI_SUCCESS;
    if (!inplace && (rc = side_init(m, &snd, 0, sbuf, sdtype, n, NULL, scount, NULL))) return rc;
    if ((rc = side_init(m, &rcv, 1, rbuf, rdtype, n, NULL, rcount, NULL))) return rc;
    if (!inplace && snd.bytes[0] != rcv.bytes[0]) return OMPI_ERR_BAD_PARAM;
    int erc = inplace ? side_move(m, &rcv, -1, 1) : side_move(m, &snd, -1, 1);
    if (erc == MI355X_SUCCESS) erc = mi355x_alltoall(m->engine, inplace ? NULL : snd.view, rcv.view, rcv.bytes[0], NULL);
    return finish_unpack(m, &rcv, erc);
}

int mca_coll_mi355x_alltoallv(void *sbuf, int *scounts, int *sdisps, struct ompi_datatype_t *sdtype, void *rbuf,
                              int *rcounts, int *rdisps, struct ompi_datatype_t *rdtype, struct ompi_communicator_t *comm,
                              mca_coll_base_module_t *module)
{
    mca_coll_mi355x_module_t *m = MOD(module);
    const int n = mi355x_comm_size_of(comm), inplace = (sbuf == MPI_IN_PLACE);
    if (n > SIDE_MAX)
        return m->prev_alltoallv(sbuf, scounts, sdisps, sdtype, rbuf, rcounts, rdisps, rdtype, comm,
                                 m->prev_alltoallv_module);
    const int dev = is_dev(rbuf) && (inplace || is_dev(sbuf));
    ROUTE_OR(m->prev_alltoallv(sbuf, scounts, sdisps, sdtype, rbuf, rcounts, rdisps, rdtype, comm,
                               m->prev_alltoallv_module), ({
                 hstage_t st_[2];
                 void *s_ = sbuf, *r_ = rbuf;
                 const size_t ss_ = inplace ? 0 : vspan(sdtype, n, scounts, sdisps), rs_ = vspan(rdtype, n, rcounts, rdisps);
                 int rc_ = (ss_ == (size_t)-1 || rs_ == (size_t)-1)
                               ? OMPI_ERR_NOT_SUPPORTED
                               : stage_move(st_, inplace ? NULL : &s_, sdtype, ss_, &r_, rdtype, rs_);
                 rc_ == OMPI_SUCCESS ? hunstage2(st_, m->prev_alltoallv(s_, scounts, sdisps, sdtype, r_, rcounts, rdisps,
                                                                        rdtype, comm, m->prev_alltoallv_module)) : rc_;
             }));
    side_t snd, rcv;
    int rc = OMPI_SUCCESS;
    if (!inplace && (rc = side_init(m, &snd, 0, sbuf, sdtype, n, scounts, 0, sdisps))) return rc;
    if ((rc = side_init(m, &rcv, 1, rbuf, rdtype, n, rcounts, 0, rdisps))) return rc;
    int erc = inplace ? side_move(m, &rcv, -1, 1) : side_move(m, &snd, -1, 1);
    if (erc == MI355X_SUCCESS)
        erc = mi355x_alltoallv(m->engine, inplace ? NULL : snd.view, inplace ? NULL : snd.bytes,
                               inplace ? NULL : snd.off, rcv.view, rcv.bytes, rcv.off, NULL);
    return finish_unpack(m, &rcv, erc);
}

static int scan_common(mca_coll_mi355x_module_t *m, int exclusive, void *sbuf, void *rbuf, int count,
                       struct ompi_datatype_t *dtype, struct ompi_op_t *op, struct ompi_communicator_t *comm)
{
    const int inplace = (sbuf == MPI_IN_PLACE);
    const int t = reducible_type(dtype);
#define SCAN_PREV(S, R)                                                                              \
    (exclusive ? m->prev_exscan(S, R, count, dtype, op, comm, m->prev_exscan_module)                 \
               : m->prev_scan(S, R, count, dtype, op, comm, m->prev_scan_module))
    if (count < 0) return SCAN_PREV(sbuf, rbuf);
    /* coll_cuda_scan.c:41-76 / coll_cuda_exscan.c:41-76; rbuf is copied in for MPI_IN_PLACE and
     * for exscan (rank 0's rbuf is left as it was) */
#define SCAN_STAGED()                                                                                 \
    ({                                                                                                \
        const size_t span_ = dt_span(dtype, (size_t)count);                                          \
        hstage_t st_[2];                                                                              \
        void *s_ = sbuf, *r_ = rbuf;                                                                  \
        const int rc_ = hstage2(st_, &s_, span_, &r_, span_, inplace || exclusive, span_, dtype);     \
        rc_ != OMPI_SUCCESS ? rc_ : hunstage2(st_, SCAN_PREV(s_, r_));                                \
    })
    if (!engine_op(op, t)) return SCAN_STAGED();
    /* every rank votes its buffer kind, as for allreduce: a rank with host buffers joins the engine
     * on device copies when a peer has device buffers */
    const int dev = is_dev(rbuf) && (inplace || is_dev(sbuf));
    ROUTE_OR(SCAN_PREV(sbuf, rbuf), SCAN_STAGED());
#undef SCAN_STAGED
#undef SCAN_PREV
    if (dev)
        return map_rc((exclusive ? mi355x_exscan : mi355x_scan)(m->engine, inplace ? NULL : sbuf, rbuf, (size_t)count,
                                                                t, op->o_f_to_c_index, NULL));
    const size_t bytes = (size_t)count * mi355x_type_size(t);
    int rc = MI355X_SUCCESS;
    void *rd = (inplace || exclusive) ? dev_in(m, 1, rbuf, bytes, &rc) : dev_out(m, 1, rbuf, bytes, &rc);
    const void *sd = inplace ? NULL : dev_in(m, 0, sbuf, bytes, &rc);
    if (rc == MI355X_SUCCESS)
        rc = (exclusive ? mi355x_exscan : mi355x_scan)(m->engine, sd, rd, (size_t)count, t, op->o_f_to_c_index, NULL);
    return map_rc(copy_back(rbuf, rd, bytes, rc));
}

int mca_coll_mi355x_scan(void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                         struct ompi_communicator_t *comm, mca_coll_base_module_t *module)
{
    return scan_common(MOD(module), 0, sbuf, rbuf, count, dtype, op, comm);
}

int mca_coll_mi355x_exscan(void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                           struct ompi_communicator_t *comm, mca_coll_base_module_t *module)
{
    return scan_common(MOD(module), 1, sbuf, rbuf, count, dtype, op, comm);
}

/* ------------------------------------------------------------------ nonblocking collectives
 * The engine runs a posted collective on the communicator's progress thread (mi355x_i*); the
 * component hands MPI an ompi_request_t subclass -- as coll/libnbc does
 * (coll_libnbc_component.c:300-333, coll_libnbc.h:120-135) -- and completes it from an
 * opal_progress callback (libnbc: ompi_coll_libnbc_progress, :239-268) when the engine request
 * has finished.  MPI_Wait / MPI_Test then find it complete and call req_free. */
typedef struct mi355x_nbreq_t {
    ompi_request_t super;
    mi355x_request_t *eng;
    int p2p;                       /* 0 collective, 1 send, 2 receive (status filled at completion) */
    struct mi355x_nbreq_t *next;   /* active list */
    /* derived datatypes (iallgather / ibcast): the packed bytes travel through `stage` (owned by
     * the request); at completion they are unpacked into (ubuf, ucount, ud) -- ud NULL: copied --
     * before MPI sees the request complete, then stage and ud are released */
    void *stage;
    size_t stage_bytes;
    void *ubuf;
    size_t ucount;
    mi355x_ddt_t *ud;
    mi355x_ddt_t *pd;              /* layout of the initiation-time pack (kept until completion) */
    int uhost;                     /* ubuf is host memory: copied (ud NULL) or host-unpacked (ud) */
    /* persistent point-to-point (pml_isend_init / pml_irecv_init): 1 send, 2 receive, 0 none; the
     * arguments each MPI_Start posts */
    int pers;
    void *pbuf;
    size_t pcount;
    struct ompi_datatype_t *pdt;
    int ppeer, ptag, pmode;
    int free_called;               /* MPI_Request_free while active: released at completion */
    /* a declined nonblocking reduction: the lower-priority component's request on host copies of
     * the device buffers (coll/cuda's staging, copied back when it completes) */
    ompi_request_t *inner;
    hstage_t hs[2];
} mi355x_nbreq_t;

static pthread_mutex_t nb_lock = PTHREAD_MUTEX_INITIALIZER;
static mi355x_nbreq_t *nb_active;
static int nb_registered;

/* MPI_Request_free.  A collective must be complete (libnbc likewise); a point-to-point request
 * may be freed while active -- it is released once it completes (ob1's req_free_called,
 * pml_ob1_sendreq.c:97-122) */
static int nbreq_free(ompi_request_t **rp)
{
    mi355x_nbreq_t *r = (mi355x_nbreq_t *)*rp;
    if (true != r->super.req_complete && r->inner) return MPI_ERR_REQUEST;
    if (true != r->super.req_complete && r->eng) {
        if (!r->p2p) return MPI_ERR_REQUEST;
        pthread_mutex_lock(&nb_lock);
        const int active = r->eng != NULL;
        if (active) r->free_called = 1;
        pthread_mutex_unlock(&nb_lock);
        if (active) {
            *rp = &ompi_request_null.request;
            return OMPI_SUCCESS;
        }
    }
    mi355x_ompi_request_fini(&r->super);
    mi355x_obj_release(&r->super.super.super.super);
    *rp = &ompi_request_null.request;
    return OMPI_SUCCESS;
}

/* MPI_Cancel: a receive not matched yet completes as cancelled (ob1,
 * pml_ob1_recvreq.c:101-137); sends and collectives are not cancelled (ob1's send cancel and
 * libnbc's do nothing) */
static int nbreq_cancel(ompi_request_t *q, int flag)
{
    (void)flag;
    mi355x_nbreq_t *r = (mi355x_nbreq_t *)q;
    if (r->p2p == 2 && r->eng) (void)mi355x_request_cancel(r->eng);
    return OMPI_SUCCESS;
}

static void nbreq_construct(opal_object_t *o)
{
    mi355x_nbreq_t *r = (mi355x_nbreq_t *)o;
    r->super.req_type = OMPI_REQUEST_COLL;
    r->super.req_status._cancelled = 0;
    r->super.req_free = nbreq_free;
    r->super.req_cancel = nbreq_cancel;
    r->eng = NULL;
    r->next = NULL;
    r->stage = NULL;
    r->stage_bytes = 0;
    r->ubuf = NULL;
    r->ucount = 0;
    r->ud = NULL;
    r->pd = NULL;
    r->uhost = 0;
    r->pers = 0;
    r->pbuf = NULL;
    r->pcount = 0;
    r->pdt = NULL;
    r->ppeer = r->ptag = r->pmode = 0;
    r->free_called = 0;
    r->inner = NULL;
    memset(r->hs, 0, sizeof(r->hs));
}

/* completion-time unpack of a derived-datatype nonblocking collective (local work only) */
static int nb_finish_stage(mi355x_nbreq_t *r, int rc)
{
    if (!r->stage) return rc;
    if (rc == MI355X_SUCCESS && r->ubuf && r->uhost && r->ud) {  /* host layout: host convertor */
        void *tmp = malloc(r->stage_bytes ? r->stage_bytes : 1);
        rc = tmp ? mi355x_memcpy(tmp, r->stage, r->stage_bytes) : MI355X_ERR_NOMEM;
        if (rc == MI355X_SUCCESS) rc = mi355x_unpack_host(r->ud, r->ucount, r->ubuf, 0, tmp, r->stage_bytes);
        free(tmp);
    } else if (rc == MI355X_SUCCESS && r->ubuf) {
        rc = r->ud ? mi355x_unpack(r->ud, r->ucount, r->ubuf, 0, r->stage, r->stage_bytes, NULL, NULL)
                   : mi355x_memcpy_async(r->ubuf, r->stage, r->stage_bytes, NULL);
        if (rc == MI355X_SUCCESS) rc = mi355x_stream_sync(NULL);
    } else {
        (void)mi355x_stream_sync(NULL);
    }
    mi355x_free(r->stage);
    r->stage = NULL;
    if (r->ud) mi355x_ddt_destroy(r->ud);
    if (r->pd) mi355x_ddt_destroy(r->pd);
    r->ud = r->pd = NULL;
    return rc;
}

static opal_class_t mi355x_nbreq_t_class = {"mca_coll_mi355x_request_t", &ompi_request_t_class, nbreq_construct,
                                            NULL, 0, 0, NULL, NULL, sizeof(mi355x_nbreq_t)};

/* opal_progress callback: complete the requests whose engine call has finished */
static int nb_progress(void)
{
    if (!__atomic_load_n(&nb_active, __ATOMIC_ACQUIRE)) return 0;  /* (every opal_progress call lands here) */
    if (pthread_mutex_trylock(&nb_lock)) return 0;
    int completed = 0;
    for (mi355x_nbreq_t **p = &nb_active; *p;) {
        mi355x_nbreq_t *r = *p;
        if (r->inner) {  /* a staged host request: done when the lower-priority request is */
            if (true != r->inner->req_complete) {
                p = &r->next;
                continue;
            }
            *p = r->next;
            ompi_request_t *in = r->inner;
            int rc = in->req_status.MPI_ERROR;
            r->inner = NULL;
            if (in != &ompi_request_null.request && in->req_free) in->req_free(&in);
            rc = hunstage2(r->hs, rc);
            r->super.req_status.MPI_ERROR = rc;
            mi355x_ompi_request_complete(&r->super, true);
            completed++;
            continue;
        }
        int done = 0;
        const int rc0 = mi355x_request_test(r->eng, &done);
        if (!done) {
            p = &r->next;
            continue;
        }
        *p = r->next;
        const int rc = nb_finish_stage(r, rc0);
        if (r->p2p == 2) {  /* MPI_Status of a receive (pml_ob1_recvreq.h:172-180 for truncation) */
            mi355x_status_t st;
            int cancelled = 0;
            memset(&st, 0, sizeof(st));
            mi355x_request_get_status(r->eng, &st);
            mi355x_request_cancelled(r->eng, &cancelled);
            r->super.req_status.MPI_SOURCE = st.source;
            r->super.req_status.MPI_TAG = st.tag;
            r->super.req_status._ucount = st.bytes;
            r->super.req_status._cancelled = cancelled;
        }
        if (rc == MI355X_ERR_TRUNCATE) {
            r->super.req_status.MPI_ERROR = MPI_ERR_TRUNCATE;
        } else {
            if (rc != MI355X_SUCCESS) fprintf(stderr, "[coll/mi355x] %s\n", mi355x_last_error());
            r->super.req_status.MPI_ERROR = (rc == MI355X_SUCCESS) ? 0 : MPI_ERR_INTERN;
        }
        mi355x_request_free(r->eng);
        r->eng = NULL;
        mi355x_ompi_request_complete(&r->super, true);
        if (r->free_called) {  /* freed by the application while active */
            mi355x_ompi_request_fini(&r->super);
            mi355x_obj_release(&r->super.super.super.super);
        }
        completed++;
    }
    pthread_mutex_unlock(&nb_lock);
    return completed;
}

/* wrap an engine request into an active MPI request (OMPI_REQUEST_INIT + ACTIVE, coll_libnbc.h:
 * 126-131) */
struct nb_stage {
    void *stage;
    size_t bytes;
    void *ubuf;       /* NULL: nothing to unpack on this rank */
    size_t ucount;
    mi355x_ddt_t *ud; /* owned by the request; NULL with ubuf set: a plain copy */
    mi355x_ddt_t *pd; /* layout of the initiation-time pack, owned by the request */
    int uhost;        /* ubuf is host memory (the host convertor unpacks a derived layout) */
};

static void nb_stage_release(struct nb_stage *st)
{
    if (!st) return;
    (void)mi355x_stream_sync(NULL);
    if (st->stage) mi355x_free(st->stage);
    if (st->ud) mi355x_ddt_destroy(st->ud);
    if (st->pd) mi355x_ddt_destroy(st->pd);
}

/* put r on the active list (completed by nb_progress) */
static void nb_activate(mi355x_nbreq_t *r)
{
    pthread_mutex_lock(&nb_lock);
    r->next = nb_active;
    nb_active = r;
    if (!nb_registered) {
        opal_progress_register(nb_progress);
        nb_registered = 1;
    }
    pthread_mutex_unlock(&nb_lock);
}

static int nb_start_full(mi355x_request_t *eng, struct ompi_communicator_t *comm, ompi_request_t **request, int p2p,
                         struct nb_stage *st)
{
    mi355x_nbreq_t *r = (mi355x_nbreq_t *)mi355x_obj_new(&mi355x_nbreq_t_class);
    if (!r) {
        mi355x_request_wait(eng);
        mi355x_request_free(eng);
        nb_stage_release(st);
        return OMPI_ERR_OUT_OF_RESOURCE;
    }
    r->p2p = p2p;
    if (st) {
        r->stage = st->stage;
        r->stage_bytes = st->bytes;
        r->ubuf = st->ubuf;
        r->ucount = st->ucount;
        r->ud = st->ud;
        r->pd = st->pd;
        r->uhost = st->uhost;
    }
    if (p2p) r->super.req_type = OMPI_REQUEST_PML;
    r->super.req_complete = false;
    r->super.req_persistent = false;
    r->super.req_state = OMPI_REQUEST_ACTIVE;
    r->super.req_status.MPI_ERROR = 0;
    r->super.req_mpi_object.comm = comm;
    r->eng = eng;
    nb_activate(r);
    *request = &r->super;
    return OMPI_SUCCESS;
}

static int nb_start_kind(mi355x_request_t *eng, struct ompi_communicator_t *comm, ompi_request_t **request, int p2p)
{
    return nb_start_full(eng, comm, request, p2p, NULL);
}

static int nb_start(mi355x_request_t *eng, struct ompi_communicator_t *comm, ompi_request_t **request)
{
    return nb_start_kind(eng, comm, request, 0);
}

#define NB_FALLBACK(FN, ...)                                                          \
    do {                                                                              \
        if (!m->prev_##FN) return OMPI_ERR_NOT_SUPPORTED;                             \
        return m->prev_##FN(__VA_ARGS__, m->prev_##FN##_module);                      \
    } while (0)

/* hand the lower-priority component's request to MPI: as it is when nothing was staged, else
 * wrapped so that the staged results are copied back when it completes (nb_progress) */
static int nb_staged_start(struct ompi_communicator_t *comm, ompi_request_t **request, hstage_t st[2],
                           ompi_request_t *inner, int rc)
{
    if (!st[0].h && !st[1].h) {
        if (rc == OMPI_SUCCESS) *request = inner;
        return rc;
    }
    if (rc != OMPI_SUCCESS) return hunstage2(st, rc);
    mi355x_nbreq_t *r = (mi355x_nbreq_t *)mi355x_obj_new(&mi355x_nbreq_t_class);
    if (!r) {  /* cannot wrap: finish the call here (the staged copies must outlive it) */
        while (true != inner->req_complete) opal_progress();
        const int err = inner->req_status.MPI_ERROR;
        if (inner != &ompi_request_null.request && inner->req_free) inner->req_free(&inner);
        return hunstage2(st, err) == OMPI_SUCCESS ? OMPI_ERR_OUT_OF_RESOURCE : OMPI_ERROR;
    }
    r->inner = inner;
    r->hs[0] = st[0];
    r->hs[1] = st[1];
    r->super.req_complete = false;
    r->super.req_persistent = false;
    r->super.req_state = OMPI_REQUEST_ACTIVE;
    r->super.req_status.MPI_ERROR = 0;
    r->super.req_mpi_object.comm = comm;
    nb_activate(r);
    *request = &r->super;
    return OMPI_SUCCESS;
}

/* A nonblocking initiation may not wait for its peers (a vote would: MPI lets a rank start the
 * call, then block in point-to-point its peer needs before that peer starts it), so with mixed
 * buffers allowed the path depends only on what every rank shares -- the op and the type: every
 * rank enters the engine, and a rank whose buffers are host memory joins on device copies made at
 * initiation (its input) and copied back at completion (its output).  With
 * coll_mi355x_mixed_buffers = 0 every rank must use one kind, and host buffers go to the
 * lower-priority component as before. */
static int nb_host_join(mca_coll_mi355x_module_t *m, void *sbuf, void *rbuf, int inplace, size_t in_bytes,
                        size_t out_bytes, int rsig, void **sd, void **rd, struct nb_stage *st)
{
    const int rh = rsig && !is_dev(rbuf), sh = !inplace && !is_dev(sbuf);
    memset(st, 0, sizeof(*st));
    *sd = inplace ? NULL : sbuf;
    *rd = rsig ? rbuf : NULL;
    const size_t rspan = inplace ? in_bytes : out_bytes;
    const size_t a = (rh ? rspan : 0) + (sh ? in_bytes : 0);
    if (mi355x_malloc(&st->stage, a ? a : 1) != MI355X_SUCCESS) return MI355X_ERR_NOMEM;
    int rc = MI355X_SUCCESS;
    if (rh) {
        *rd = st->stage;
        st->bytes = out_bytes;
        st->ubuf = rbuf;
        st->uhost = 1;
        if (inplace && in_bytes) rc = mi355x_memcpy(st->stage, rbuf, in_bytes);
    }
    if (sh && rc == MI355X_SUCCESS) {
        *sd = (char *)st->stage + (rh ? rspan : 0);
        if (in_bytes) rc = mi355x_memcpy(*sd, sbuf, in_bytes);
    }
    if (rc != MI355X_SUCCESS) {
        mi355x_free(st->stage);
        st->stage = NULL;
    }
    return rc;
}

/* the declined / host-buffer form of a nonblocking reduction: device buffers staged to the host */
#define NB_STAGED(FN, SSPAN, RSPAN, RFILL, RBACK, DT, ...)                                       \
    do {                                                                                          \
        if (!m->prev_##FN) return OMPI_ERR_NOT_SUPPORTED;                                         \
        hstage_t st_[2];                                                                          \
        int rc_ = hstage2(st_, &sbuf, (SSPAN), &rbuf, (RSPAN), (RFILL), (RBACK), (DT));           \
        if (rc_ != OMPI_SUCCESS) return rc_;                                                      \
        ompi_request_t *in_ = NULL;                                                               \
        rc_ = m->prev_##FN(__VA_ARGS__, &in_, m->prev_##FN##_module);                             \
        return nb_staged_start(comm, request, st_, in_, rc_);                                     \
    } while (0)

int mca_coll_mi355x_iallreduce(void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                               struct ompi_communicator_t *comm, ompi_request_t **request,
                               mca_coll_base_module_t *module)
{
    mca_coll_mi355x_module_t *m = MOD(module);
    const int inplace = (sbuf == MPI_IN_PLACE);
    const int t = reducible_type(dtype);
    if (count < 0) NB_FALLBACK(iallreduce, sbuf, rbuf, count, dtype, op, comm, request);
    const int dev = is_dev(rbuf) && (inplace || is_dev(sbuf));
    if (!engine_op(op, t) || (!dev && !m->mixed)) {
        const size_t span = dt_span(dtype, (size_t)count);
        NB_STAGED(iallreduce, span, span, inplace, span, dtype, sbuf, rbuf, count, dtype, op, comm);
    }
    mi355x_request_t *eng = NULL;
    if (!dev) {  /* host buffers: join the engine on device copies (nb_host_join) */
        const size_t bytes = (size_t)count * mi355x_type_size(t);
        struct nb_stage st;
        void *sd, *rd;
        int rc = nb_host_join(m, sbuf, rbuf, inplace, bytes, bytes, 1, &sd, &rd, &st);
        if (rc == MI355X_SUCCESS) rc = mi355x_iallreduce(m->engine, sd, rd, (size_t)count, t, op->o_f_to_c_index, NULL, &eng);
        if (rc != MI355X_SUCCESS) {
            nb_stage_release(&st);
            return map_rc(rc);
        }
        return nb_start_full(eng, comm, request, 0, &st);
    }
    int rc = mi355x_iallreduce(m->engine, inplace ? NULL : sbuf, rbuf, (size_t)count, t, op->o_f_to_c_index, NULL, &eng);
    return rc ? map_rc(rc) : nb_start(eng, comm, request);
}

int mca_coll_mi355x_ireduce(void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                            int root, struct ompi_communicator_t *comm, ompi_request_t **request,
                            mca_coll_base_module_t *module)
{
    mca_coll_mi355x_module_t *m = MOD(module);
    const int me = mi355x_comm_rank_of(comm);
    const int inplace = (sbuf == MPI_IN_PLACE);
    const int t = reducible_type(dtype);
    if (count < 0 || (inplace && me != root)) NB_FALLBACK(ireduce, sbuf, rbuf, count, dtype, op, root, comm, request);
    const int dev = (me != root || is_dev(rbuf)) && (inplace || is_dev(sbuf));
    if (!engine_op(op, t) || (!dev && !m->mixed)) {
        const size_t span = dt_span(dtype, (size_t)count);
        if (me != root) rbuf = NULL;  /* not significant off the root: never staged */
        NB_STAGED(ireduce, span, span, inplace, span, dtype, sbuf, rbuf, count, dtype, op, root, comm);
    }
    mi355x_request_t *eng = NULL;
    if (!dev) {  /* host buffers: join the engine on device copies (nb_host_join) */
        const size_t bytes = (size_t)count * mi355x_type_size(t);
        struct nb_stage st;
        void *sd, *rd;
        int rc = nb_host_join(m, sbuf, rbuf, inplace, bytes, bytes, me == root, &sd, &rd, &st);
        if (rc == MI355X_SUCCESS)
            rc = mi355x_ireduce(m->engine, sd, rd, (size_t)count, t, op->o_f_to_c_index, root, NULL, &eng);
        if (rc != MI355X_SUCCESS) {
            nb_stage_release(&st);
            return map_rc(rc);
        }
        return nb_start_full(eng, comm, request, 0, &st);
    }
    int rc = mi355x_ireduce(m->engine, inplace ? NULL : sbuf, me == root ? rbuf : NULL, (size_t)count, t,
                            op->o_f_to_c_index, root, NULL, &eng);
    return rc ? map_rc(rc) : nb_start(eng, comm, request);
}

int mca_coll_mi355x_ireduce_scatter_block(void *sbuf, void *rbuf, int rcount, struct ompi_datatype_t *dtype,
                                          struct ompi_op_t *op, struct ompi_communicator_t *comm,
                                          ompi_request_t **request, mca_coll_base_module_t *module)
{
    mca_coll_mi355x_module_t *m = MOD(module);
    const int inplace = (sbuf == MPI_IN_PLACE);
    const int t = reducible_type(dtype);
    if (rcount < 0) NB_FALLBACK(ireduce_scatter_block, sbuf, rbuf, rcount, dtype, op, comm, request);
    const int dev = is_dev(rbuf) && (inplace || is_dev(sbuf));
    if (!engine_op(op, t) || (!dev && !m->mixed)) {
        const size_t in = dt_span(dtype, (size_t)rcount * (size_t)mi355x_comm_size_of(comm));
        const size_t out = dt_span(dtype, (size_t)rcount);
        NB_STAGED(ireduce_scatter_block, in, inplace ? in : out, inplace, out, dtype, sbuf, rbuf, rcount, dtype, op,
                  comm);
    }
    mi355x_request_t *eng = NULL;
    if (!dev) {  /* host buffers: join the engine on device copies (nb_host_join) */
        const size_t out = (size_t)rcount * mi355x_type_size(t), in = out * (size_t)mi355x_comm_size_of(comm);
        struct nb_stage st;
        void *sd, *rd;
        int rc = nb_host_join(m, sbuf, rbuf, inplace, in, out, 1, &sd, &rd, &st);
        if (rc == MI355X_SUCCESS)
            rc = mi355x_ireduce_scatter_block(m->engine, sd, rd, (size_t)rcount, t, op->o_f_to_c_index, NULL, &eng);
        if (rc != MI355X_SUCCESS) {
            nb_stage_release(&st);
            return map_rc(rc);
        }
        return nb_start_full(eng, comm, request, 0, &st);
    }
    int rc = mi355x_ireduce_scatter_block(m->engine, inplace ? NULL : sbuf, rbuf, (size_t)rcount, t,
                                          op->o_f_to_c_index, NULL, &eng);
    return rc ? map_rc(rc) : nb_start(eng, comm, request);
}

/* the (count, dt) side of a staged nonblocking move: pack it into `p` now (local work), or set up
 * the completion-time unpack into `st` (the request then owns a private layout of dt) */
static int nb_stage_side(int pack, void *buf, size_t count, const struct ompi_datatype_t *dt, void *p, size_t bytes,
                         struct nb_stage *st)
{
    size_t cb;
    if (contiguous_bytes_n(dt, count, &cb)) {
        if (pack) return mi355x_memcpy_async(p, buf, bytes, NULL);
        st->ubuf = buf;
        return MI355X_SUCCESS;
    }
    mi355x_ddt_t *d = ddt_private(dt);
    if (!d) return MI355X_ERR_UNSUPPORTED;
    if (pack) {
        st->pd = d;  /* the pack kernel reads its run tables until it finishes: released at completion */
        return mi355x_pack(d, count, buf, 0, p, bytes, NULL, NULL);
    }
    st->ubuf = buf;
    st->ucount = count;
    st->ud = d;
    return MI355X_SUCCESS;
}

/* Contiguous layouts go straight to the engine.  Derived layouts -- on any rank, whatever the
 * others use (MPI lets layouts differ; only the type signatures match) -- also stay in the
 * engine: my block is packed into a per-request staging buffer at initiation, the engine gathers
 * the packed blocks in place, and the completion unpacks them into rbuf (all local work, so the
 * call stays nonblocking); rank-local fallbacks to libnbc would leave the ranks in different
 * components. */
int mca_coll_mi355x_iallgather(void *sbuf, int scount, struct ompi_datatype_t *sdtype, void *rbuf, int rcount,
                               struct ompi_datatype_t *rdtype, struct ompi_communicator_t *comm,
                               ompi_request_t **request, mca_coll_base_module_t *module)
{
    mca_coll_mi355x_module_t *m = MOD(module);
    const int inplace = (sbuf == MPI_IN_PLACE);
    size_t rb = 0, sb = 0;
    if (rcount < 0 || (!inplace && scount < 0))
        NB_FALLBACK(iallgather, sbuf, scount, sdtype, rbuf, rcount, rdtype, comm, request);
    const int rh = !is_dev(rbuf), sh = !inplace && !is_dev(sbuf);
    if ((rh || sh) && !m->mixed) {  /* a host side, one kind per call: device sides staged to the host */
        if (!m->prev_iallgather) return OMPI_ERR_NOT_SUPPORTED;
        const size_t n = (size_t)mi355x_comm_size_of(comm);
        hstage_t st[2];
        int rc = hstage(&st[0], &sbuf, sdtype, inplace ? 0 : dt_span(sdtype, (size_t)scount), 1, 0);
        if (rc != OMPI_SUCCESS) return rc;
        const size_t rspan = dt_span(rdtype, (size_t)rcount * n);
        if ((rc = hstage(&st[1], &rbuf, rdtype, rspan, inplace, rspan)) != OMPI_SUCCESS) return hunstage(&st[0], rc);
        if (st[0].h || st[1].h) __atomic_add_fetch(&mca_coll_mi355x_staged_calls, 1, __ATOMIC_RELAXED);
        ompi_request_t *inner = NULL;
        rc = m->prev_iallgather(sbuf, scount, sdtype, rbuf, rcount, rdtype, comm, &inner, m->prev_iallgather_module);
        return nb_staged_start(comm, request, st, inner, rc);
    }
    mi355x_request_t *eng = NULL;
    if (!rh && !sh && contiguous_bytes(rdtype, rcount, &rb) &&
        (inplace || (contiguous_bytes(sdtype, scount, &sb) && sb == rb))) {
        int rc = mi355x_iallgather(m->engine, inplace ? NULL : sbuf, rbuf, rb, NULL, &eng);
        return rc ? map_rc(rc) : nb_start(eng, comm, request);
    }
    /* derived layouts or host sides (a host rank joins the engine, nb_host_join): my block packed
     * into the per-request staging buffer now, the n blocks moved out of it at completion */
    const int n = mi355x_comm_size_of(comm), me = mi355x_comm_rank_of(comm);
    const size_t blk = (size_t)rcount * rdtype->super.size;
    if (!inplace && (size_t)scount * sdtype->super.size != blk) return OMPI_ERR_BAD_PARAM;
    struct nb_stage st = {NULL, blk * (size_t)n, NULL, 0, NULL, NULL, 0};
    if (mi355x_malloc(&st.stage, st.bytes ? st.bytes : 1) != MI355X_SUCCESS) return OMPI_ERR_OUT_OF_RESOURCE;
    const ptrdiff_t rext = rdtype->super.ub - rdtype->super.lb;
    int rc;
    if (inplace && rh)
        rc = xstage(m, 1, (char *)rbuf + (ptrdiff_t)me * rcount * rext, rcount, rdtype, (char *)st.stage + blk * me, blk, 1);
    else if (sh)
        rc = xstage(m, 1, sbuf, scount, sdtype, (char *)st.stage + blk * me, blk, 1);
    else
        rc = inplace ? nb_stage_side(1, (char *)rbuf + (ptrdiff_t)me * rcount * rext, rcount, rdtype,
                                     (char *)st.stage + blk * me, blk, &st)
                     : nb_stage_side(1, sbuf, scount, sdtype, (char *)st.stage + blk * me, blk, &st);
    if (rc == MI355X_SUCCESS && rh) {
        st.ubuf = rbuf;
        st.ucount = (size_t)rcount * (size_t)n;
        st.uhost = 1;
        if (!contiguous_bytes_n(rdtype, st.ucount, &rb) && !(st.ud = ddt_private(rdtype))) rc = MI355X_ERR_UNSUPPORTED;
    } else if (rc == MI355X_SUCCESS) {
        rc = nb_stage_side(0, rbuf, (size_t)rcount * (size_t)n, rdtype, st.stage, st.bytes, &st);
    }
    if (rc == MI355X_SUCCESS) rc = mi355x_iallgather(m->engine, NULL, st.stage, blk, NULL, &eng);
    if (rc != MI355X_SUCCESS) {
        if (rc == MI355X_ERR_UNSUPPORTED)
            fprintf(stderr, "[coll/mi355x] iallgather: the GPU convertor cannot describe the datatype\n");
        nb_stage_release(&st);
        return map_rc(rc);
    }
    return nb_start_full(eng, comm, request, 0, &st);
}

/* derived layouts as in iallgather: the root packs at initiation, the others unpack at completion */
int mca_coll_mi355x_ibcast(void *buff, int count, struct ompi_datatype_t *datatype, int root,
                           struct ompi_communicator_t *comm, ompi_request_t **request, mca_coll_base_module_t *module)
{
    mca_coll_mi355x_module_t *m = MOD(module);
    size_t bytes = 0;
    const int host = !is_dev(buff);
    if (count < 0 || (host && !m->mixed)) NB_FALLBACK(ibcast, buff, count, datatype, root, comm, request);
    mi355x_request_t *eng = NULL;
    if (!host && contiguous_bytes(datatype, count, &bytes)) {
        int rc = mi355x_ibcast(m->engine, buff, bytes, root, NULL, &eng);
        return rc ? map_rc(rc) : nb_start(eng, comm, request);
    }
    const int me = mi355x_comm_rank_of(comm);
    struct nb_stage st = {NULL, (size_t)count * datatype->super.size, NULL, 0, NULL, NULL, 0};
    if (mi355x_malloc(&st.stage, st.bytes ? st.bytes : 1) != MI355X_SUCCESS) return OMPI_ERR_OUT_OF_RESOURCE;
    int rc = MI355X_SUCCESS;
    if (!host) {
        rc = nb_stage_side(me == root, buff, count, datatype, st.stage, st.bytes, &st);
    } else if (me == root) {  /* a host rank joining the engine (nb_host_join): packed / copied now */
        rc = xstage(m, 1, buff, (size_t)count, datatype, st.stage, st.bytes, 1);
    } else {                  /* ... or moved out of the staging buffer at completion */
        st.ubuf = buff;
        st.ucount = (size_t)count;
        st.uhost = 1;
        if (!contiguous_bytes(datatype, count, &bytes) && !(st.ud = ddt_private(datatype))) rc = MI355X_ERR_UNSUPPORTED;
    }
    if (rc == MI355X_SUCCESS) rc = mi355x_ibcast(m->engine, st.stage, st.bytes, root, NULL, &eng);
    if (rc != MI355X_SUCCESS) {
        if (rc == MI355X_ERR_UNSUPPORTED)
            fprintf(stderr, "[coll/mi355x] ibcast: the GPU convertor cannot describe datatype %s\n", datatype->name);
        nb_stage_release(&st);
        return map_rc(rc);
    }
    return nb_start_full(eng, comm, request, 0, &st);
}

/* ------------------------------------------------------------------ point-to-point (PML hook)
 * ob1 matches every message of a communicator in ONE queue whatever the buffer kind, deciding per
 * request on each side how the bytes move (pml_ob1_cuda.c:52-100, pml_ob1_recvreq.c:647-663): a
 * device send can meet a host receive, MPI_ANY_SOURCE sees every sender, and messages between a
 * pair never overtake each other.  coll/mi355x owns an engine per communicator whose point-to-
 * point does exactly that device-natively (device payloads pulled over xGMI, host payloads through
 * a shared-memory arena, one match queue; engine p2p.cpp), so on those communicators EVERY
 * point-to-point call goes to the engine -- host or device buffer, any send mode, persistent and
 * matched-probe requests included -- and routing never depends on a buffer's kind.  Communicators
 * without the engine keep the selected PML.  The hook is installed the way pml/v parasites the
 * selected PML (pml_v_component.c:110-131): once the PML is selected (coll components are queried
 * after it, ompi_mpi_init.c:610-660) its table `mca_pml` is saved and the entries are replaced. */
static mca_pml_base_module_t host_pml;
static int pml_hooked;

static mca_coll_mi355x_module_t *engine_module(struct ompi_communicator_t *comm)
{
    if (!comm || comm->c_coll.coll_allreduce != mca_coll_mi355x_allreduce || !comm->c_coll.coll_allreduce_module)
        return NULL;
    mca_coll_mi355x_module_t *m = MOD(comm->c_coll.coll_allreduce_module);
    return m->engine ? m : NULL;
}

/* `count` instances of dt as the engine's (count, layout): contiguous -> bytes and no layout.
 * Fails (MPI_ERR_TYPE) only for a layout the convertor cannot describe (more than 2^20 runs). */
static int p2p_layout(mca_coll_mi355x_module_t *m, struct ompi_datatype_t *dt, size_t count, size_t *ecount,
                      mi355x_ddt_t **d)
{
    size_t b;
    if (count <= (size_t)0x7fffffff && contiguous_bytes(dt, (int)count, &b)) {
        *ecount = b;
        *d = NULL;
        return OMPI_SUCCESS;
    }
    *d = ddt_of(m, dt);
    *ecount = count;
    if (*d) return OMPI_SUCCESS;
    fprintf(stderr, "[coll/mi355x] point-to-point: the convertor cannot describe datatype %s\n", dt->name);
    return MPI_ERR_TYPE;
}

static void status_from(ompi_status_public_t *status, const mi355x_status_t *st, int rc)
{
    if (!status) return;  /* MPI_STATUS_IGNORE is NULL */
    status->MPI_SOURCE = st->source;
    status->MPI_TAG = st->tag;
    status->_ucount = st->bytes;
    status->MPI_ERROR = rc == MI355X_ERR_TRUNCATE ? MPI_ERR_TRUNCATE : (rc ? MPI_ERR_INTERN : 0);
}

int mca_coll_mi355x_pml_isend(void *buf, size_t count, struct ompi_datatype_t *dt, int dst, int tag,
                              mca_pml_base_send_mode_t mode, struct ompi_communicator_t *comm,
                              ompi_request_t **request)
{
    mca_coll_mi355x_module_t *m = engine_module(comm);
    if (!m) return host_pml.pml_isend(buf, count, dt, dst, tag, mode, comm, request);
    size_t ec = 0;
    mi355x_ddt_t *d = NULL;
    int rc = p2p_layout(m, dt, count, &ec, &d);
    if (rc) return rc;
    mi355x_request_t *eng = NULL;
    rc = mi355x_isend_mode(m->engine, buf, ec, d, dst, tag, (int)mode, NULL, &eng);
    return rc ? map_rc(rc) : nb_start_kind(eng, comm, request, 1);
}

/* synchronous sends complete once the receiver has the data; buffered and small sends once the
 * payload is copied (ob1's eager protocol); larger standard sends are rendezvous (engine p2p.cpp) */
int mca_coll_mi355x_pml_send(void *buf, size_t count, struct ompi_datatype_t *dt, int dst, int tag,
                             mca_pml_base_send_mode_t mode, struct ompi_communicator_t *comm)
{
    mca_coll_mi355x_module_t *m = engine_module(comm);
    if (!m) return host_pml.pml_send(buf, count, dt, dst, tag, mode, comm);
    size_t ec = 0;
    mi355x_ddt_t *d = NULL;
    int rc = p2p_layout(m, dt, count, &ec, &d);
    if (rc) return rc;
    return map_rc(mi355x_send_mode(m->engine, buf, ec, d, dst, tag, (int)mode, NULL));
}

int mca_coll_mi355x_pml_irecv(void *buf, size_t count, struct ompi_datatype_t *dt, int src, int tag,
                              struct ompi_communicator_t *comm, ompi_request_t **request)
{
    mca_coll_mi355x_module_t *m = engine_module(comm);
    if (!m) return host_pml.pml_irecv(buf, count, dt, src, tag, comm, request);
    size_t ec = 0;
    mi355x_ddt_t *d = NULL;
    int rc = p2p_layout(m, dt, count, &ec, &d);
    if (rc) return rc;
    mi355x_request_t *eng = NULL;
    rc = mi355x_irecv(m->engine, buf, ec, d, src, tag, NULL, &eng);
    return rc ? map_rc(rc) : nb_start_kind(eng, comm, request, 2);
}

int mca_coll_mi355x_pml_recv(void *buf, size_t count, struct ompi_datatype_t *dt, int src, int tag,
                             struct ompi_communicator_t *comm, ompi_status_public_t *status)
{
    mca_coll_mi355x_module_t *m = engine_module(comm);
    if (!m) return host_pml.pml_recv(buf, count, dt, src, tag, comm, status);
    size_t ec = 0;
    mi355x_ddt_t *d = NULL;
    int rc = p2p_layout(m, dt, count, &ec, &d);
    if (rc) return rc;
    mi355x_status_t st;
    memset(&st, 0, sizeof(st));
    rc = mi355x_recv(m->engine, buf, ec, d, src, tag, NULL, &st);
    status_from(status, &st, rc);
    if (rc == MI355X_ERR_TRUNCATE) return MPI_ERR_TRUNCATE;
    return map_rc(rc);
}

/* every message of an engine communicator is in the engine's queue */
int mca_coll_mi355x_pml_iprobe(int src, int tag, struct ompi_communicator_t *comm, int *matched,
                               ompi_status_public_t *status)
{
    mca_coll_mi355x_module_t *m = engine_module(comm);
    if (!m) return host_pml.pml_iprobe(src, tag, comm, matched, status);
    mi355x_status_t st;
    int flag = 0;
    memset(&st, 0, sizeof(st));
    const int rc = mi355x_iprobe(m->engine, src, tag, &flag, &st);
    if (rc != MI355X_SUCCESS) return map_rc(rc);
    *matched = flag;
    if (flag) status_from(status, &st, 0);
    else opal_progress();  /* ob1's iprobe progresses when nothing matched (pml_ob1_iprobe.c:46-50) */
    return OMPI_SUCCESS;
}

int mca_coll_mi355x_pml_probe(int src, int tag, struct ompi_communicator_t *comm, ompi_status_public_t *status)
{
    if (!engine_module(comm)) return host_pml.pml_probe(src, tag, comm, status);
    for (;;) {
        int matched = 0;
        const int rc = mca_coll_mi355x_pml_iprobe(src, tag, comm, &matched, status);
        if (rc != OMPI_SUCCESS || matched) return rc;
    }
}

/* ---- matched probe (MPI_Improbe / MPI_Mprobe + MPI_Imrecv / MPI_Mrecv): the message leaves the
 * queue at the probe and travels in an ompi_message_t, as ob1 does (pml_ob1_iprobe.c:83-134);
 * req_ptr holds the engine's message */
int mca_coll_mi355x_pml_improbe(int src, int tag, struct ompi_communicator_t *comm, int *matched,
                                struct ompi_message_t **message, ompi_status_public_t *status)
{
    mca_coll_mi355x_module_t *m = engine_module(comm);
    if (!m) return host_pml.pml_improbe(src, tag, comm, matched, message, status);
    mi355x_status_t st;
    mi355x_message_t *em = NULL;
    int flag = 0;
    memset(&st, 0, sizeof(st));
    const int rc = mi355x_improbe(m->engine, src, tag, &flag, &em, &st);
    if (rc != MI355X_SUCCESS) return map_rc(rc);
    *matched = flag && em;
    if (!*matched) {
        *message = &ompi_message_null.message;
        opal_progress();
        return OMPI_SUCCESS;
    }
    ompi_message_t *msg = (ompi_message_t *)mi355x_obj_new(&ompi_message_t_class);
    if (!msg) return OMPI_ERR_OUT_OF_RESOURCE;  /* (the engine message stays out of the queue) */
    msg->m_f_to_c_index = MPI_UNDEFINED;
    msg->comm = comm;
    msg->req_ptr = em;
    msg->peer = st.source;
    msg->count = st.bytes;
    *message = msg;
    status_from(status, &st, 0);
    return OMPI_SUCCESS;
}

int mca_coll_mi355x_pml_mprobe(int src, int tag, struct ompi_communicator_t *comm, struct ompi_message_t **message,
                               ompi_status_public_t *status)
{
    if (!engine_module(comm)) return host_pml.pml_mprobe(src, tag, comm, message, status);
    for (;;) {
        int matched = 0;
        const int rc = mca_coll_mi355x_pml_improbe(src, tag, comm, &matched, message, status);
        if (rc != OMPI_SUCCESS || matched) return rc;
    }
}

/* the engine message of an ompi_message_t from our improbe, or NULL (another PML's) */
static mi355x_message_t *engine_message(struct ompi_message_t *msg, mca_coll_mi355x_module_t **mm)
{
    if (!msg || msg == &ompi_message_null.message) return NULL;
    *mm = engine_module(msg->comm);
    return *mm ? (mi355x_message_t *)msg->req_ptr : NULL;
}

int mca_coll_mi355x_pml_imrecv(void *buf, size_t count, struct ompi_datatype_t *dt, struct ompi_message_t **message,
                               ompi_request_t **request)
{
    mca_coll_mi355x_module_t *m = NULL;
    mi355x_message_t *em = engine_message(*message, &m);
    if (!em) return host_pml.pml_imrecv(buf, count, dt, message, request);
    size_t ec = 0;
    mi355x_ddt_t *d = NULL;
    int rc = p2p_layout(m, dt, count, &ec, &d);
    if (rc) return rc;
    struct ompi_communicator_t *comm = (*message)->comm;
    mi355x_request_t *eng = NULL;
    rc = mi355x_imrecv(m->engine, buf, ec, d, em, NULL, &eng);
    if (rc) return map_rc(rc);
    mi355x_obj_release(&(*message)->super.super);   /* ob1: ompi_message_return */
    *message = &ompi_message_null.message;
    return nb_start_kind(eng, comm, request, 2);
}

int mca_coll_mi355x_pml_mrecv(void *buf, size_t count, struct ompi_datatype_t *dt, struct ompi_message_t **message,
                              ompi_status_public_t *status)
{
    mca_coll_mi355x_module_t *m = NULL;
    mi355x_message_t *em = engine_message(*message, &m);
    if (!em) return host_pml.pml_mrecv(buf, count, dt, message, status);
    size_t ec = 0;
    mi355x_ddt_t *d = NULL;
    int rc = p2p_layout(m, dt, count, &ec, &d);
    if (rc) return rc;
    mi355x_request_t *eng = NULL;
    rc = mi355x_imrecv(m->engine, buf, ec, d, em, NULL, &eng);
    if (rc) return map_rc(rc);
    mi355x_obj_release(&(*message)->super.super);
    *message = &ompi_message_null.message;
    rc = mi355x_request_wait(eng);
    mi355x_status_t st;
    memset(&st, 0, sizeof(st));
    mi355x_request_get_status(eng, &st);
    if (rc != MI355X_ERR_TIMEOUT) mi355x_request_free(eng);
    status_from(status, &st, rc);
    if (rc == MI355X_ERR_TRUNCATE) return MPI_ERR_TRUNCATE;
    return map_rc(rc);
}

/* ---- persistent requests (MPI_Send_init / MPI_Recv_init / MPI_Start): the arguments are kept in
 * the request and every MPI_Start posts them to the engine (ob1: mca_pml_ob1_start,
 * pml_ob1_start.c:29-…); completion leaves the request INACTIVE for the next start (the MPI
 * layer's wait does that, req_wait.c:59-63) */
static int pers_init(int kind, void *buf, size_t count, struct ompi_datatype_t *dt, int peer, int tag, int mode,
                     struct ompi_communicator_t *comm, ompi_request_t **request)
{
    mi355x_nbreq_t *r = (mi355x_nbreq_t *)mi355x_obj_new(&mi355x_nbreq_t_class);
    if (!r) return OMPI_ERR_OUT_OF_RESOURCE;
    r->p2p = kind;
    r->pers = kind;
    r->pbuf = buf;
    r->pcount = count;
    r->pdt = dt;
    r->ppeer = peer;
    r->ptag = tag;
    r->pmode = mode;
    r->super.req_type = OMPI_REQUEST_PML;
    r->super.req_complete = false;    /* OMPI_REQUEST_INIT(req, persistent), request.h:139-144 */
    r->super.req_state = OMPI_REQUEST_INACTIVE;
    r->super.req_persistent = true;
    r->super.req_mpi_object.comm = comm;
    *request = &r->super;
    return OMPI_SUCCESS;
}

int mca_coll_mi355x_pml_isend_init(void *buf, size_t count, struct ompi_datatype_t *dt, int dst, int tag,
                                   mca_pml_base_send_mode_t mode, struct ompi_communicator_t *comm,
                                   ompi_request_t **request)
{
    if (!engine_module(comm)) return host_pml.pml_isend_init(buf, count, dt, dst, tag, mode, comm, request);
    return pers_init(1, buf, count, dt, dst, tag, (int)mode, comm, request);
}

int mca_coll_mi355x_pml_irecv_init(void *buf, size_t count, struct ompi_datatype_t *dt, int src, int tag,
                                   struct ompi_communicator_t *comm, ompi_request_t **request)
{
    if (!engine_module(comm)) return host_pml.pml_irecv_init(buf, count, dt, src, tag, comm, request);
    return pers_init(2, buf, count, dt, src, tag, 0, comm, request);
}

static int pers_start(mi355x_nbreq_t *r)
{
    if (r->eng) return MPI_ERR_REQUEST;  /* still in flight: MPI forbids a second start */
    struct ompi_communicator_t *comm = r->super.req_mpi_object.comm;
    mca_coll_mi355x_module_t *m = engine_module(comm);
    if (!m) return OMPI_ERROR;
    size_t ec = 0;
    mi355x_ddt_t *d = NULL;
    int rc = p2p_layout(m, r->pdt, r->pcount, &ec, &d);
    if (rc) return rc;
    mi355x_request_t *eng = NULL;
    rc = r->pers == 1 ? mi355x_isend_mode(m->engine, r->pbuf, ec, d, r->ppeer, r->ptag, r->pmode, NULL, &eng)
                      : mi355x_irecv(m->engine, r->pbuf, ec, d, r->ppeer, r->ptag, NULL, &eng);
    if (rc) return map_rc(rc);
    memset(&r->super.req_status, 0, sizeof(r->super.req_status));
    r->super.req_complete = false;
    r->super.req_state = OMPI_REQUEST_ACTIVE;
    r->eng = eng;
    nb_activate(r);
    return OMPI_SUCCESS;
}

int mca_coll_mi355x_pml_start(size_t count, ompi_request_t **requests)
{
    for (size_t i = 0; i < count; ++i) {
        ompi_request_t *q = requests[i];
        if (!q || q->req_type != OMPI_REQUEST_PML) continue;
        int rc;
        if (q->req_free == nbreq_free && ((mi355x_nbreq_t *)q)->pers) rc = pers_start((mi355x_nbreq_t *)q);
        else rc = host_pml.pml_start ? host_pml.pml_start(1, &requests[i]) : OMPI_ERR_NOT_SUPPORTED;
        if (rc != OMPI_SUCCESS) return rc;
    }
    return OMPI_SUCCESS;
}

/* install / remove the hook (idempotent) */
#define HOOK(F)                                                                 \
    do {                                                                        \
        if (mca_pml.pml_##F) mca_pml.pml_##F = mca_coll_mi355x_pml_##F;         \
    } while (0)
#define UNHOOK(F)                                                               \
    do {                                                                        \
        if (mca_pml.pml_##F == mca_coll_mi355x_pml_##F) mca_pml.pml_##F = host_pml.pml_##F; \
    } while (0)

static void pml_hook_install(void)
{
    if (pml_hooked || mca_coll_mi355x_pml_hook == 0) return;
    if (!mca_pml.pml_isend || !mca_pml.pml_irecv || !mca_pml.pml_send || !mca_pml.pml_recv) return;  /* no PML */
    host_pml = mca_pml;
    HOOK(isend);
    HOOK(send);
    HOOK(irecv);
    HOOK(recv);
    HOOK(iprobe);
    HOOK(probe);
    HOOK(improbe);
    HOOK(mprobe);
    HOOK(imrecv);
    HOOK(mrecv);
    HOOK(isend_init);
    HOOK(irecv_init);
    HOOK(start);
    pml_hooked = 1;
}

static void pml_hook_remove(void)
{
    if (!pml_hooked) return;
    UNHOOK(isend);
    UNHOOK(send);
    UNHOOK(irecv);
    UNHOOK(recv);
    UNHOOK(iprobe);
    UNHOOK(probe);
    UNHOOK(improbe);
    UNHOOK(mprobe);
    UNHOOK(imrecv);
    UNHOOK(mrecv);
    UNHOOK(isend_init);
    UNHOOK(irecv_init);
    UNHOOK(start);
    pml_hooked = 0;
}

/* ------------------------------------------------------------------ module / component */
#define SNAP(FN)                                                                \
    do {                                                                        \
        m->prev_##FN = comm->c_coll.coll_##FN;                                  \
        m->prev_##FN##_module = comm->c_coll.coll_##FN##_module;                \
        if (!m->prev_##FN || !m->prev_##FN##_module) return OMPI_ERROR;         \
        mi355x_obj_retain(&m->prev_##FN##_module->super);                       \
    } while (0)

/* coll/tuned's own tuning, honoured so that a job tuned for the reference keeps its choices:
 * with coll_tuned_use_dynamic_rules set (coll_tuned_component.c:151-167), the forced algorithms
 * (coll_tuned_{allreduce,reduce,reduce_scatter}_algorithm, reduce_algorithm_chain_fanout;
 * coll_tuned_allreduce.c:949-1005 and siblings) and the rules file
 * coll_tuned_dynamic_rules_filename (read once per process, like
 * mca_coll_tuned_component.all_base_rules, coll_tuned_component.c:213-229).  The values are read
 * from coll/tuned's own registered variables through the MCA variable system (mca_base_var_find +
 * mca_base_var_get_value, as tuned_open reads coll_base_verbose, coll_tuned_component.c:200-209),
 * so every source opal knows -- command line, environment, openmpi-mca-params.conf,
 * mca_base_param_files -- reaches the engine exactly as it reaches coll/tuned.  Only when no
 * variable system or no coll/tuned registration is present does the component read
 * OMPI_MCA_coll_tuned_<name> from the environment itself. */
static mi355x_rules_t *tuned_rules;
static int tuned_rules_read;

/* pointer to coll/tuned's storage of variable `name`, or NULL */
static const void *tuned_var(const char *name)
{
    if (!mca_base_var_find || !mca_base_var_get_value) return NULL;
    const int idx = mca_base_var_find("ompi", "coll", "tuned", name);
    if (idx < 0) return NULL;
    const void *storage = NULL;
    if (mca_base_var_get_value(idx, &storage, NULL, NULL) != OMPI_SUCCESS) return NULL;
    return storage;
}

static int tuned_int(const char *name, int is_bool)
{
    const void *p = tuned_var(name);
    if (p) return is_bool ? (int)*(const bool *)p : *(const int *)p;
    char env[96];
    snprintf(env, sizeof(env), "OMPI_MCA_coll_tuned_%s", name);
    return env_int(env, 0);
}

static const char *tuned_string(const char *name)
{
    const void *p = tuned_var(name);
    if (p) return *(char *const *)p;
    char env[96];
    snprintf(env, sizeof(env), "OMPI_MCA_coll_tuned_%s", name);
    return getenv(env);
}

static void apply_tuned_params(mca_coll_mi355x_module_t *m)
{
    if (!tuned_int("use_dynamic_rules", 1)) return;
    const int ar = tuned_int("allreduce_algorithm", 0);
    const int red = tuned_int("reduce_algorithm", 0);
    const int fo = tuned_int("reduce_algorithm_chain_fanout", 0);
    const int rs = tuned_int("reduce_scatter_algorithm", 0);
    if (ar && !mca_coll_mi355x_allreduce_algorithm) mi355x_comm_set(m->engine, MI355X_KNOB_ALLREDUCE_ALG, ar);
    if (red) mi355x_comm_set(m->engine, MI355X_KNOB_REDUCE_ALG, red);
    if (fo) mi355x_comm_set(m->engine, MI355X_KNOB_REDUCE_CHAIN_FANOUT, fo);
    if (rs) mi355x_comm_set(m->engine, MI355X_KNOB_REDUCE_SCATTER_ALG, rs);
    const char *file = tuned_string("dynamic_rules_filename");
    if (file && *file && !tuned_rules_read) {
        tuned_rules_read = 1;
        if (mi355x_rules_load(file, &tuned_rules) < 0) {
            fprintf(stderr, "[coll/mi355x] %s -- ignoring the rules file\n", mi355x_last_error());
            tuned_rules = NULL;
        }
    }
    if (tuned_rules) mi355x_comm_set_rules(m->engine, tuned_rules);
}

#define SNAP_OPT(FN)                                                            \
    do {                                                                        \
        m->prev_##FN = comm->c_coll.coll_##FN;                                  \
        m->prev_##FN##_module = comm->c_coll.coll_##FN##_module;                \
        if (m->prev_##FN##_module) mi355x_obj_retain(&m->prev_##FN##_module->super); \
    } while (0)

/* The engine's crossovers as MCA variables, applied to each communicator's engine the way
 * coll/tuned applies its forced-algorithm variables per communicator (coll_tuned_module.c:178-226).
 * They are set before the engine's device-side setup runs (it waits for the first device-buffer
 * collective), so the ones that size that setup -- the service limits -- take effect in it.  Every
 * rank of a communicator must see the same values (as for coll/tuned's variables). */
static int set_knob(mca_coll_mi355x_module_t *m, int knob, long v, const char *name)
{
    if (mi355x_comm_set(m->engine, knob, v) == MI355X_SUCCESS) return OMPI_SUCCESS;
    fprintf(stderr, "[coll/mi355x] coll_mi355x_%s = %ld rejected: %s\n", name, v, mi355x_last_error());
    return OMPI_ERR_BAD_PARAM;
}

static int apply_engine_params(mca_coll_mi355x_module_t *m, struct ompi_communicator_t *comm)
{
    const int n = mi355x_comm_size_of(comm);
    int rc = OMPI_SUCCESS;
#define KNOB(K, V, NAME) if (rc == OMPI_SUCCESS) rc = set_knob(m, MI355X_KNOB_##K, (long)(V), NAME)
    KNOB(SELFTEST, mca_coll_mi355x_selftest != 0, "selftest");
    KNOB(PIPE, mca_coll_mi355x_pipe_min_ranks > 0 && n >= mca_coll_mi355x_pipe_min_ranks, "pipe_min_ranks");
    KNOB(PIPE_CHUNK_KIB, mca_coll_mi355x_pipe_chunk_kib, "pipe_chunk_kib");
    KNOB(PIPE_WG_PER_CU, mca_coll_mi355x_pipe_wg_per_cu, "pipe_wg_per_cu");
    KNOB(PIPE_WT, mca_coll_mi355x_pipe_wt != 0, "pipe_wt");
    KNOB(ONE_PHASE_MAX_BYTES, mca_coll_mi355x_one_phase_max, "one_phase_max");
    KNOB(SVC_MAX_BYTES, mca_coll_mi355x_svc_max, "svc_max");
    KNOB(SVC_PULL_MAX_BYTES, mca_coll_mi355x_svc_pull_max, "svc_pull_max");
    KNOB(SVC_PULL_COPY_MAX_BYTES, mca_coll_mi355x_svc_copy_max, "svc_copy_max");
    KNOB(SVC_IDLE_US, mca_coll_mi355x_svc_idle_us, "svc_idle_us");
    KNOB(SVC_SHRINK_US, mca_coll_mi355x_svc_shrink_us, "svc_shrink_us");
    if (mca_coll_mi355x_timeout_s > 0) KNOB(TIMEOUT_S, mca_coll_mi355x_timeout_s, "timeout_s");
#undef KNOB
    return rc;
}

/* the engine of a communicator this component serves, or NULL (tools and tests) */
struct mi355x_comm *mca_coll_mi355x_engine_of(struct ompi_communicator_t *comm)
{
    if (!comm || comm->c_coll.coll_allreduce != mca_coll_mi355x_allreduce || !comm->c_coll.coll_allreduce_module)
        return NULL;
    return MOD(comm->c_coll.coll_allreduce_module)->engine;
}

/* coll_module_enable (coll.h:176-178): runs after every lower-priority module is installed */
static int module_enable(mca_coll_base_module_t *module, struct ompi_communicator_t *comm)
{
    mca_coll_mi355x_module_t *m = MOD(module);
    SNAP(allreduce);
    SNAP(reduce_scatter);
    SNAP(reduce_scatter_block);
    SNAP(allgather);
    SNAP(bcast);
    SNAP(reduce);
    SNAP(gather);
    SNAP(gatherv);
    SNAP(scatter);
    SNAP(scatterv);
    SNAP(allgatherv);
    SNAP(alltoall);
    SNAP(alltoallv);
    SNAP(scan);
    SNAP(exscan);
    SNAP_OPT(iallreduce);
    SNAP_OPT(ireduce);
    SNAP_OPT(ireduce_scatter_block);
    SNAP_OPT(iallgather);
    SNAP_OPT(ibcast);
    /* Node-unique rendezvous key, picked by rank 0 and broadcast with the lower-priority bcast
     * just snapshotted (the communicator is p2p-capable during enable, coll.h:125-127).  Neither
     * the job id nor the context id would do: MPI_Comm_split allocates ONE cid for every color
     * group of the parent (ompi_comm_nextcid over the parent, comm.c:610), so sibling groups on
     * one node share (jobid, cid). */
    char key[64];
    memset(key, 0, sizeof(key));
    if (mi355x_comm_rank_of(comm) == 0) {
        static unsigned counter;
        unsigned rnd = 0;
        FILE *ur = fopen("/dev/urandom", "rb");
        if (!ur || fread(&rnd, sizeof(rnd), 1, ur) != 1) rnd = (unsigned)time(NULL) ^ (unsigned)(uintptr_t)&rnd;
        if (ur) fclose(ur);
        snprintf(key, sizeof(key), "ompi_%d_%u_%08x", (int)getpid(), __atomic_add_fetch(&counter, 1, __ATOMIC_RELAXED),
                 rnd);
    }
    int rc = m->prev_bcast(key, (int)sizeof(key), MPI_BYTE, 0, comm, m->prev_bcast_module);
    if (rc != OMPI_SUCCESS) return rc;
    key[sizeof(key) - 1] = 0;
    /* the GPU this process selected before the communicator was created (hipSetDevice), never a
     * device derived from the local rank: the engine must run where the application's buffers are */
    int dev = 0;
    if (mi355x_get_device(&dev) != MI355X_SUCCESS) return OMPI_ERROR;
    rc = mi355x_comm_create(key, mi355x_comm_rank_of(comm), mi355x_comm_size_of(comm), dev, &m->engine);
    if (rc != MI355X_SUCCESS) return map_rc(rc);
    if (mca_coll_mi355x_allreduce_algorithm)
        mi355x_comm_set(m->engine, MI355X_KNOB_ALLREDUCE_ALG, mca_coll_mi355x_allreduce_algorithm);
    /* the peer-mapping cache bounds (mpool_rgpusm_rcache_size_limit's role) */
    if (mca_coll_mi355x_rcache_max_maps > 0)
        mi355x_comm_set(m->engine, MI355X_KNOB_RCACHE_MAX_MAPS, mca_coll_mi355x_rcache_max_maps);
    if (mca_coll_mi355x_rcache_size_limit > 0)
        mi355x_comm_set(m->engine, MI355X_KNOB_RCACHE_SIZE_LIMIT, (long)mca_coll_mi355x_rcache_size_limit);
    apply_tuned_params(m);
    return apply_engine_params(m, comm);
}

/* an int parameter: through the MCA variable system when libopen-pal provides it (in-tree build,
 * coll_cuda_component.c:77-90), else OMPI_MCA_coll_mi355x_<name> from the environment */
static void register_int(const char *name, const char *desc, mca_base_var_info_lvl_t lvl, int *storage)
{
    if (mca_base_component_var_register) {
        (void)mca_base_component_var_register(&mca_coll_mi355x_component.collm_version, name, desc,
                                              MCA_BASE_VAR_TYPE_INT, NULL, 0, 0, lvl, MCA_BASE_VAR_SCOPE_READONLY,
                                              storage);
        return;
    }
    char env[96];
    snprintf(env, sizeof(env), "OMPI_MCA_coll_mi355x_%s", name);
    *storage = env_int(env, *storage);
}

/* an unsigned long long parameter (a byte count), the same two sources */
static void register_ull(const char *name, const char *desc, mca_base_var_info_lvl_t lvl, unsigned long long *storage)
{
    if (mca_base_component_var_register) {
        (void)mca_base_component_var_register(&mca_coll_mi355x_component.collm_version, name, desc,
                                              MCA_BASE_VAR_TYPE_UNSIGNED_LONG_LONG, NULL, 0, 0, lvl,
                                              MCA_BASE_VAR_SCOPE_READONLY, storage);
        return;
    }
    char env[96];
    snprintf(env, sizeof(env), "OMPI_MCA_coll_mi355x_%s", name);
    const char *v = getenv(env);
    if (v) *storage = strtoull(v, NULL, 10);
}

static int component_register(void)
{
    register_int("priority", "Priority of the mi355x coll component (device-buffer collectives over xGMI)",
                 OPAL_INFO_LVL_6, &mca_coll_mi355x_priority);
    register_int("allreduce_algorithm",
                 "Allreduce algorithm forced on the engine, in coll_tuned's numbering "
                 "(coll_tuned_allreduce.c:38-47); 0 = coll_tuned's fixed decision", OPAL_INFO_LVL_5, &mca_coll_mi355x_allreduce_algorithm);
    register_int("pml_hook", "Route device-buffer point-to-point on engine communicators through the engine",
                 OPAL_INFO_LVL_5, &mca_coll_mi355x_pml_hook);
    register_int("mixed_buffers", "Let ranks mix host and device buffers in one allreduce / reduce / reduce_scatter(_block) / "
                 "allgather / bcast (every rank votes its buffer kind; 0: every rank must use the same kind)",
                 OPAL_INFO_LVL_5, &mca_coll_mi355x_mixed_buffers);
    register_int("rcache_max_maps", "Most mappings of peers' device allocations kept open per communicator; the least "
                 "recently used beyond it are closed (0 = unlimited)", OPAL_INFO_LVL_9, &mca_coll_mi355x_rcache_max_maps);
    register_ull("rcache_size_limit", "The same bound in bytes of mapped peer allocations, as mpool_rgpusm_rcache_size_limit "
                 "(0 = unlimited)", OPAL_INFO_LVL_9, &mca_coll_mi355x_rcache_size_limit);
    /* the engine's crossovers, in the manner of coll/tuned's knobs (coll_tuned_component.c:115-170,
     * coll_tuned_allreduce.c:949-1005); the defaults were chosen where the ranks shared one GPU */
    register_int("pipe_min_ranks", "Communicators of at least this many ranks run large allreduces through the "
                 "pipelined copy||reduce flow (one persistent launch, per-chunk flags); 0 = never", OPAL_INFO_LVL_5,
                 &mca_coll_mi355x_pipe_min_ranks);
    register_int("pipe_chunk_kib", "Chunk size of the pipelined allreduce in KiB (0 = about 512 chunks per ring block)",
                 OPAL_INFO_LVL_6, &mca_coll_mi355x_pipe_chunk_kib);
    register_int("pipe_wg_per_cu", "Workgroups per CU of the pipelined allreduce (1..8)", OPAL_INFO_LVL_6,
                 &mca_coll_mi355x_pipe_wg_per_cu);
    register_int("pipe_wt", "Pipelined allreduce: 1 = fold results stored write-through with system-scope ready flags, "
                 "0 = stored and released by the producer's fence", OPAL_INFO_LVL_9, &mca_coll_mi355x_pipe_wt);
    register_ull("one_phase_max", "Per-rank message bytes up to which an allreduce runs the one-launch ring-ordered flow "
                 "instead of the two-phase one", OPAL_INFO_LVL_6, &mca_coll_mi355x_one_phase_max);
    register_ull("svc_max", "Per-rank message bytes up to which small allreduce / reduce / allgather / bcast / "
                 "reduce_scatter_block calls go to the resident LL service in its LL form (svc_max, svc_pull_max and "
                 "svc_copy_max all 0: no service)", OPAL_INFO_LVL_5,
                 &mca_coll_mi355x_svc_max);
    register_ull("svc_pull_max", "Per-rank bytes up to which the service serves allreduce in its pull form (above "
                 "svc_max)", OPAL_INFO_LVL_6, &mca_coll_mi355x_svc_pull_max);
    register_ull("svc_copy_max", "Per-rank bytes up to which the service copies allgather / bcast (above svc_max)",
                 OPAL_INFO_LVL_6, &mca_coll_mi355x_svc_copy_max);
    register_int("svc_idle_us", "Idle time after which the resident service's kernel leaves the GPU, microseconds "
                 "(100 .. 60000000)", OPAL_INFO_LVL_6, &mca_coll_mi355x_svc_idle_us);
    register_int("svc_shrink_us", "Idle time after which the resident service shrinks to one workgroup, microseconds "
                 "(0 = never)", OPAL_INFO_LVL_6, &mca_coll_mi355x_svc_shrink_us);
    register_int("selftest", "Run the cross-device flows' self-tests at a communicator's first device-buffer collective "
                 "(a flow that fails on any rank is turned off on every rank); 0 = trust every flow", OPAL_INFO_LVL_9,
                 &mca_coll_mi355x_selftest);
    register_int("timeout_s", "Bound of every wait of the engine, seconds (0 = the engine's own: MI355X_TIMEOUT_S, "
                 "else one day -- MPI's waits are unbounded; a rank whose process is gone is noticed without it)",
                 OPAL_INFO_LVL_9, &mca_coll_mi355x_timeout_s);
    return OMPI_SUCCESS;
}
static int component_open(void) { return OMPI_SUCCESS; }
static int component_close(void)
{
    pml_hook_remove();
    if (tuned_rules) mi355x_rules_destroy(tuned_rules);
    tuned_rules = NULL;
    tuned_rules_read = 0;
    return OMPI_SUCCESS;
}

static int component_init_query(bool enable_progress_threads, bool enable_mpi_threads)
{
    (void)enable_progress_threads;
    (void)enable_mpi_threads;
    int n = 0;
    if (mi355x_device_count(&n) != MI355X_SUCCESS || n < 1) return OMPI_ERR_NOT_SUPPORTED;
    pml_hook_install();  /* the PML is selected by now (ompi_mpi_init.c:610 before :660) */
    mi355x_set_progress_hook(opal_progress);  /* the engine's host-side waits keep MPI progressing */
    return OMPI_SUCCESS;
}

/* collm_comm_query (coll.h:137-139); declines like coll/tuned for inter/size-1 communicators
 * (coll_tuned_module.c:63-75) and when the job spans several nodes */
static mca_coll_base_module_t *component_comm_query(struct ompi_communicator_t *comm, int *priority)
{
    if ((comm->c_flags & OMPI_COMM_INTER) || mi355x_comm_size_of(comm) < 2) return NULL;
    if (mca_coll_mi355x_priority <= 0) return NULL;
    const int wsize = env_int("OMPI_COMM_WORLD_SIZE", -1), lsize = env_int("OMPI_COMM_WORLD_LOCAL_SIZE", -2);
    if (wsize != lsize) return NULL;
    mca_coll_mi355x_module_t *m = (mca_coll_mi355x_module_t *)mi355x_obj_new(&mca_coll_mi355x_module_t_class);
    if (!m) return NULL;
    m->super.coll_module_enable = module_enable;
    m->super.coll_allreduce = mca_coll_mi355x_allreduce;
    m->super.coll_reduce_scatter = mca_coll_mi355x_reduce_scatter;
    m->super.coll_reduce_scatter_block = mca_coll_mi355x_reduce_scatter_block;
    m->super.coll_allgather = mca_coll_mi355x_allgather;
    m->super.coll_bcast = mca_coll_mi355x_bcast;
    m->super.coll_reduce = mca_coll_mi355x_reduce;
    m->super.coll_gather = mca_coll_mi355x_gather;
    m->super.coll_gatherv = mca_coll_mi355x_gatherv;
    m->super.coll_scatter = mca_coll_mi355x_scatter;
    m->super.coll_scatterv = mca_coll_mi355x_scatterv;
    m->super.coll_allgatherv = mca_coll_mi355x_allgatherv;
    m->super.coll_alltoall = mca_coll_mi355x_alltoall;
    m->super.coll_alltoallv = mca_coll_mi355x_alltoallv;
    m->super.coll_scan = mca_coll_mi355x_scan;
    m->super.coll_exscan = mca_coll_mi355x_exscan;
    m->super.coll_iallreduce = mca_coll_mi355x_iallreduce;
    m->super.coll_ireduce = mca_coll_mi355x_ireduce;
    m->super.coll_ireduce_scatter_block = mca_coll_mi355x_ireduce_scatter_block;
    m->super.coll_iallgather = mca_coll_mi355x_iallgather;
    m->super.coll_ibcast = mca_coll_mi355x_ibcast;
    m->super.ft_event = NULL;
    *priority = mca_coll_mi355x_priority > 100 ? 100 : mca_coll_mi355x_priority;
    return &m->super;
}

mca_coll_base_component_t mca_coll_mi355x_component = {
    .collm_version = {
        MCA_COLL_BASE_VERSION_2_0_0,
        "mi355x", 1, 0, 0,
        component_open, component_close, NULL, component_register, {0}
    },
    .collm_data = {0, {0}},
    .collm_init_query = component_init_query,
    .collm_comm_query = component_comm_query,
};
