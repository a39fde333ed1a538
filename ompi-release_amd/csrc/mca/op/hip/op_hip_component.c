/*
 * op_hip_component.c -- op/hip: MI355X reduction kernels behind the op framework tables.
 *
 * Component / module ABI: ompi/mca/op/op.h:253-373.  Selection: ompi_op_base_op_select
 * (ompi/mca/op/base/op_base_op_select.c:88-204) calls opc_op_query once per intrinsic MPI_Op at
 * MPI_Init (op.c:427-433), then opm_enable, then copies every non-NULL slot of the module over
 * the op's tables in ascending priority.  See include/op_hip.h for the per-call behaviour.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>

#include "../../../../../include/mi355x_rt.h"
#include "../../../../../include/op_hip.h"

int mca_op_hip_priority = 50;

/* module = the base module + what this component needs per MPI_Op */
typedef struct mca_op_hip_module_t {
    ompi_op_base_module_t super;
    int op;                                            /* MI355X_OP_* == o_f_to_c_index */
    ompi_op_base_handler_fn_t prev2[OMPI_OP_BASE_TYPE_MAX];        /* slot owners before us */
    ompi_op_base_module_t *prev2_mod[OMPI_OP_BASE_TYPE_MAX];
    ompi_op_base_3buff_handler_fn_t prev3[OMPI_OP_BASE_TYPE_MAX];
    ompi_op_base_module_t *prev3_mod[OMPI_OP_BASE_TYPE_MAX];
    pthread_mutex_t lock;                              /* guards the staging buffers */
    void *dscratch;                                    /* device staging */
    size_t dscratch_bytes;
} mca_op_hip_module_t;

static void module_construct(opal_object_t *o)
{
    mca_op_hip_module_t *m = (mca_op_hip_module_t *)o;
    m->op = 0;
    memset(m->prev2, 0, sizeof(m->prev2));
    memset(m->prev2_mod, 0, sizeof(m->prev2_mod));
    memset(m->prev3, 0, sizeof(m->prev3));
    memset(m->prev3_mod, 0, sizeof(m->prev3_mod));
    pthread_mutex_init(&m->lock, NULL);
    m->dscratch = NULL;
    m->dscratch_bytes = 0;
}

static void module_destruct(opal_object_t *o)
{
    mca_op_hip_module_t *m = (mca_op_hip_module_t *)o;
    for (int t = 0; t < OMPI_OP_BASE_TYPE_MAX; ++t) {
        if (m->prev2_mod[t]) mi355x_obj_release(&m->prev2_mod[t]->super);
        if (m->prev3_mod[t]) mi355x_obj_release(&m->prev3_mod[t]->super);
    }
    if (m->dscratch) mi355x_free(m->dscratch);
    pthread_mutex_destroy(&m->lock);
}

/* OBJ_CLASS_INSTANCE(mca_op_hip_module_t, ompi_op_base_module_t, ...) (opal_object.h:221) */
static opal_class_t mca_op_hip_module_t_class = {
    "mca_op_hip_module_t", &ompi_op_base_module_t_class, module_construct, module_destruct,
    0, 0, NULL, NULL, sizeof(mca_op_hip_module_t)
};

static void die(const char *what)
{
    fprintf(stderr, "[op/hip] fatal: %s: %s\n", what, mi355x_last_error());
    abort();
}

/* x87 long double slots: MAX/MIN (and MAXLOC/MINLOC on MPI_LONG_DOUBLE_INT) compare and select on
 * the 80-bit encoding, SUM/PROD (real and complex) run the x87 add / multiply restated in integer
 * arithmetic (f80_arith.hpp) -- every slot has a GPU kernel; the staging below stays for a runtime
 * without one */
static int x87_type(int t)
{
    return t == MI355X_T_LONG_DOUBLE || t == MI355X_T_C_LONG_DOUBLE_COMPLEX || t == MI355X_T_LONG_DOUBLE_INT;
}

static int is_dev(const void *p)
{
    int d = 0;
    if (mi355x_ptr_is_device(p, &d) != MI355X_SUCCESS) die("pointer query");
    return d;
}

static void *scratch(mca_op_hip_module_t *m, size_t bytes)
{
    if (m->dscratch_bytes < bytes) {
        if (m->dscratch) mi355x_free(m->dscratch);
        m->dscratch = NULL;
        m->dscratch_bytes = 0;
        if (mi355x_malloc(&m->dscratch, bytes) != MI355X_SUCCESS) die("scratch allocation");
        m->dscratch_bytes = bytes;
    }
    return m->dscratch;
}

/* run the saved lower-priority function on host copies of device operands */
static void staged_host2(mca_op_hip_module_t *m, int t, void *in, void *inout, int *count,
                         struct ompi_datatype_t **dtype, int din, int dio)
{
    size_t bytes = (size_t)*count * mi355x_type_size(t);
    void *hin = in, *hio = inout;
    if (din) { hin = malloc(bytes); if (!hin || mi355x_memcpy(hin, in, bytes)) die("stage in"); }
    if (dio) { hio = malloc(bytes); if (!hio || mi355x_memcpy(hio, inout, bytes)) die("stage inout"); }
    m->prev2[t](hin, hio, count, dtype, m->prev2_mod[t]);
    if (dio) { if (mi355x_memcpy(inout, hio, bytes)) die("unstage inout"); free(hio); }
    if (din) free(hin);
}

void mca_op_hip_2buff(void *in, void *inout, int *count, struct ompi_datatype_t **dtype,
                      struct ompi_op_base_module_1_0_0_t *module)
{
    mca_op_hip_module_t *m = (mca_op_hip_module_t *)module;
    const int t = ompi_op_ddt_map[(*dtype)->id];
    if (*count <= 0) return;
    const int din = is_dev(in), dio = is_dev(inout);
    if (!din && !dio) {                                   /* host buffers: the base loop */
        m->prev2[t](in, inout, count, dtype, m->prev2_mod[t]);
        return;
    }
    if (!mi355x_op_supported(m->op, t)) {  /* an x87 arithmetic slot */
        staged_host2(m, t, in, inout, count, dtype, din, dio);
        return;
    }
    if (din && dio) {  /* all-device: no shared state, concurrent callers do not serialise */
        if (mi355x_op_reduce(m->op, t, in, inout, (size_t)*count, NULL) || mi355x_stream_sync(NULL))
            die("mi355x_op_reduce");
        return;
    }
    const size_t bytes = (size_t)*count * mi355x_type_size(t);
    pthread_mutex_lock(&m->lock);  /* guards the staging buffer */
    const void *src = in;
    void *dst = inout;
    if (!din) {                                           /* stage the host operand */
        src = scratch(m, bytes);
        if (mi355x_memcpy((void *)src, in, bytes)) die("stage in");
    } else if (!dio) {
        dst = scratch(m, bytes);
        if (mi355x_memcpy(dst, inout, bytes)) die("stage inout");
    }
    if (mi355x_op_reduce(m->op, t, src, dst, (size_t)*count, NULL) || mi355x_stream_sync(NULL))
        die("mi355x_op_reduce");
    if (dst != inout && mi355x_memcpy(inout, dst, bytes)) die("unstage inout");
    pthread_mutex_unlock(&m->lock);
}

void mca_op_hip_3buff(void *in1, void *in2, void *out, int *count, struct ompi_datatype_t **dtype,
                      struct ompi_op_base_module_1_0_0_t *module)
{
    mca_op_hip_module_t *m = (mca_op_hip_module_t *)module;
    const int t = ompi_op_ddt_map[(*dtype)->id];
    if (*count <= 0) return;
    const int d1 = is_dev(in1), d2 = is_dev(in2), dout = is_dev(out);
    if (!d1 && !d2 && !dout) {
        m->prev3[t](in1, in2, out, count, dtype, m->prev3_mod[t]);
        return;
    }
    const size_t bytes = (size_t)*count * mi355x_type_size(t);
    if (!mi355x_op_supported(m->op, t)) {  /* an x87 arithmetic slot */
        void *h1 = malloc(bytes), *h2 = malloc(bytes), *ho = malloc(bytes);
        if (!h1 || !h2 || !ho || mi355x_memcpy(h1, in1, bytes) || mi355x_memcpy(h2, in2, bytes)) die("stage");
        m->prev3[t](h1, h2, ho, count, dtype, m->prev3_mod[t]);
        if (mi355x_memcpy(out, ho, bytes)) die("unstage");
        free(h1); free(h2); free(ho);
        return;
    }
    if (d1 && d2 && dout) {  /* all-device: lock-free */
        if (mi355x_op_reduce_3buff(m->op, t, in1, in2, out, (size_t)*count, NULL) || mi355x_stream_sync(NULL))
            die("mi355x_op_reduce_3buff");
        return;
    }
    pthread_mutex_lock(&m->lock);  /* guards the staging buffer */
    /* stage host operands into one scratch of up to three slices */
    char *s = NULL;
    const void *a = in1, *b = in2;
    void *o = out;
    if (!d1 || !d2 || !dout) s = (char *)scratch(m, 3 * bytes);
    if (!d1) { if (mi355x_memcpy(s, in1, bytes)) die("stage in1"); a = s; }
    if (!d2) { if (mi355x_memcpy(s + bytes, in2, bytes)) die("stage in2"); b = s + bytes; }
    if (!dout) o = s + 2 * bytes;
    if (mi355x_op_reduce_3buff(m->op, t, a, b, o, (size_t)*count, NULL) || mi355x_stream_sync(NULL))
        die("mi355x_op_reduce_3buff");
    if (o != out && mi355x_memcpy(out, o, bytes)) die("unstage out");
    pthread_mutex_unlock(&m->lock);
}

/* opm_enable (op.h:343-345), called before the slot copy (op_base_op_select.c:141-142) */
static int module_enable(struct ompi_op_base_module_1_0_0_t *module, struct ompi_op_t *op)
{
    mca_op_hip_module_t *m = (mca_op_hip_module_t *)module;
    for (int t = 0; t < OMPI_OP_BASE_TYPE_MAX; ++t) {
        /* keep the reference NULL pattern (sanity check :185-201): only slots the op has */
        if (NULL == op->o_func.intrinsic.fns[t] || NULL == op->o_3buff_intrinsic.fns[t]) {
            m->super.opm_fns[t] = NULL;
            m->super.opm_3buff_fns[t] = NULL;
            continue;
        }
        if (NULL == m->super.opm_fns[t]) continue;
        m->prev2[t] = op->o_func.intrinsic.fns[t];
        m->prev2_mod[t] = op->o_func.intrinsic.modules[t];
        m->prev3[t] = op->o_3buff_intrinsic.fns[t];
        m->prev3_mod[t] = op->o_3buff_intrinsic.modules[t];
        if (m->prev2_mod[t]) mi355x_obj_retain(&m->prev2_mod[t]->super);
        if (m->prev3_mod[t]) mi355x_obj_retain(&m->prev3_mod[t]->super);
        /* op_base_op_select.c:162-168 releases the 2-buff slot's module (now this one) when it
         * installs a 3-buff function: one extra reference per dual slot keeps the count equal
         * to the number of table slots holding this module (else double free at op.c:476-487). */
        mi355x_obj_retain(&m->super.super);
    }
    m->super.opm_op = op;
    return OMPI_SUCCESS;
}

/* op_hip_priority: through the MCA variable system when libopen-pal provides it (in-tree build;
 * the same call coll_cuda_component.c:77-82 makes), else OMPI_MCA_op_hip_priority */
static int component_register(void)
{
    if (mca_base_component_var_register) {
        (void)mca_base_component_var_register(&mca_op_hip_component.opc_version, "priority",
                                              "Priority of the hip op component (MI355X reduction kernels)",
                                              MCA_BASE_VAR_TYPE_INT, NULL, 0, 0, OPAL_INFO_LVL_6,
                                              MCA_BASE_VAR_SCOPE_READONLY, &mca_op_hip_priority);
        return OMPI_SUCCESS;
    }
    const char *v = getenv("OMPI_MCA_op_hip_priority");
    if (v) mca_op_hip_priority = atoi(v);
    return OMPI_SUCCESS;
}

static int component_open(void) { return OMPI_SUCCESS; }
static int component_close(void) { return OMPI_SUCCESS; }

static int component_init_query(bool enable_progress_threads, bool enable_mpi_threads)
{
    (void)enable_progress_threads;
    (void)enable_mpi_threads;
    int n = 0;
    if (mi355x_device_count(&n) != MI355X_SUCCESS || n < 1) return OMPI_ERR_NOT_SUPPORTED;
    return OMPI_SUCCESS;
}

static struct ompi_op_base_module_1_0_0_t *component_op_query(struct ompi_op_t *op, int *priority)
{
    const int code = op->o_f_to_c_index;
    int any = 0;
    for (int t = 0; t < OMPI_OP_BASE_TYPE_MAX && !any; ++t) any = mi355x_op_supported(code, t);
    if (!any) return NULL;
    mca_op_hip_module_t *m = (mca_op_hip_module_t *)mi355x_obj_new(&mca_op_hip_module_t_class);
    if (!m) return NULL;
    m->op = code;
    m->super.opm_enable = module_enable;
    for (int t = 0; t < OMPI_OP_BASE_TYPE_MAX; ++t) {
        if (mi355x_op_supported(code, t) || (x87_type(t) && (code == MI355X_OP_SUM || code == MI355X_OP_PROD))) {
            m->super.opm_fns[t] = mca_op_hip_2buff;
            m->super.opm_3buff_fns[t] = mca_op_hip_3buff;
        }
    }
    *priority = mca_op_hip_priority;
    return &m->super;
}

ompi_op_base_component_t mca_op_hip_component = {
    .opc_version = {
        OMPI_OP_BASE_VERSION_1_0_0,
        "hip", 1, 0, 0,
        component_open, component_close, NULL, component_register, {0}
    },
    .opc_data = {0, {0}},
    .opc_init_query = component_init_query,
    .opc_op_query = component_op_query,
};
