/*
 * ompi_mini.c -- "mini Open MPI": the few pieces of libmpi / libopen-pal that the op/hip and
 * coll/mi355x components link against, restated so the components can be loaded, selected and
 * called exactly as Open MPI 1.8.5 would, without a built Open MPI (none can be built here,
 * SURVEY.md §0).  This is the host side the tests and examples drive; it contains no reduction
 * arithmetic of its own (the "base" op functions are supplied by whoever sets up the harness).
 *
 * Restated behaviour (file:line of the reference):
 *   opal_class_initialize            opal/class/opal_object.c:73-150 (construct/destruct arrays)
 *   ompi_op_base_module_t class ctor ompi/mca/op/base/op_base_frame.c:43-62 (zeroes the tables)
 *   mca_coll_base_module_t class ctor ompi/mca/coll/base/coll_base_frame.c:45-52
 *   ompi_op_ddt_map                  ompi/op/op.c:125-215 (C types)
 *   op selection                     ompi/mca/op/base/op_base_op_select.c:88-204, including the
 *                                    2-buff/3-buff module release at :162-168
 *   ompi_op_reduce / 3buff dispatch  ompi/op/op.h:540-636
 *   op destruction                   ompi/op/op.c:476-487
 *   coll selection                   ompi/mca/coll/base/coll_base_comm_select.c:114-262
 */
#define _GNU_SOURCE /* RTLD_DEFAULT */
#include "ompi_mini.h"

#include <dlfcn.h>
#include <fcntl.h>
#include <stdarg.h>
#include <sched.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <unistd.h>

static void chan_release(ompi_communicator_t *c);

/* ------------------------------------------------------------------ opal objects */
void opal_class_initialize(opal_class_t *cls)
{
    if (cls->cls_initialized) return;
    int depth = 0, nc = 0, nd = 0;
    for (opal_class_t *c = cls; c; c = c->cls_parent) {
        depth++;
        if (c->cls_construct) nc++;
        if (c->cls_destruct) nd++;
    }
    cls->cls_depth = depth;
    opal_construct_t *ca = calloc((size_t)nc + 1, sizeof(*ca));
    opal_destruct_t *da = calloc((size_t)nd + 1, sizeof(*da));
    /* constructors run base -> derived, destructors derived -> base */
    int i = nc;
    for (opal_class_t *c = cls; c; c = c->cls_parent)
        if (c->cls_construct) ca[--i] = c->cls_construct;
    int j = 0;
    for (opal_class_t *c = cls; c; c = c->cls_parent)
        if (c->cls_destruct) da[j++] = c->cls_destruct;
    cls->cls_construct_array = ca;
    cls->cls_destruct_array = da;
    cls->cls_initialized = 1;
}

static opal_class_t opal_object_t_class = {"opal_object_t", NULL, NULL, NULL, 0, 0, NULL, NULL,
                                           sizeof(opal_object_t)};

static void op_module_construct(opal_object_t *o)
{
    ompi_op_base_module_t *m = (ompi_op_base_module_t *)o;
    m->opm_enable = NULL;
    m->opm_op = NULL;
    memset(m->opm_fns, 0, sizeof(m->opm_fns));
    memset(m->opm_3buff_fns, 0, sizeof(m->opm_3buff_fns));
}
opal_class_t ompi_op_base_module_t_class = {"ompi_op_base_module_t", &opal_object_t_class, op_module_construct,
                                            NULL, 0, 0, NULL, NULL, sizeof(ompi_op_base_module_t)};

static void coll_module_construct(opal_object_t *o)
{
    mca_coll_base_module_t *m = (mca_coll_base_module_t *)o;
    memset((char *)m + sizeof(opal_object_t), 0, sizeof(*m) - sizeof(opal_object_t));
}
opal_class_t mca_coll_base_module_t_class = {"mca_coll_base_module_t", &opal_object_t_class, coll_module_construct,
                                             NULL, 0, 0, NULL, NULL, sizeof(mca_coll_base_module_t)};

/* ------------------------------------------------------------------ datatypes / ddt map */
int ompi_op_ddt_map[OMPI_DATATYPE_MPI_MAX_PREDEFINED];

/* The predefined types as libmpi leaves them after ompi_datatype_init.  The basic C types are
 * OPAL basic types (OPAL_DATATYPE_FLAG_BASIC, opal_datatype.h:78-82) that are also MPI-predefined
 * (OMPI_DATATYPE_INIT_PREDEFINED_BASIC_TYPE, ompi_datatype_internal.h:406-414).  The MPI-2 pair
 * types are built as a contiguous block or a struct, committed, and then have the OPAL predefined
 * flag cleared and the MPI one set (DECLARE_MPI2_COMPOSED_{STRUCT,BLOCK}_DDT,
 * ompi_datatype_module.c:391-437, instantiated :471-509): their size, bounds and contiguity are
 * what opal_datatype_add computes for the x86-64 C struct -- MPI_DOUBLE_INT / MPI_LONG_INT are 12
 * bytes in a 16-byte extent, MPI_SHORT_INT 6 bytes with a hole at 2..4 in 8, MPI_LONG_DOUBLE_INT
 * 20 in 32 -- and their description is the two (or one block of two) basic elements.
 * tests/test_boundary.py checks every pair row against oracle/opal_types.py's restatement. */
#define F_BASIC (OPAL_DATATYPE_FLAG_PREDEFINED | OPAL_DATATYPE_FLAG_CONTIGUOUS | OPAL_DATATYPE_FLAG_NO_GAPS | \
                 OPAL_DATATYPE_FLAG_DATA | OPAL_DATATYPE_FLAG_COMMITTED | OMPI_DATATYPE_FLAG_PREDEFINED)
#define F_PAIR (OPAL_DATATYPE_FLAG_DATA | OPAL_DATATYPE_FLAG_COMMITTED | OMPI_DATATYPE_FLAG_PREDEFINED | \
                OMPI_DATATYPE_FLAG_DATA_C)
#define F_CNG (OPAL_DATATYPE_FLAG_CONTIGUOUS | OPAL_DATATYPE_FLAG_NO_GAPS)
enum { O_INT2 = 5, O_INT4 = 6, O_INT8 = 7, O_FLOAT4 = 15, O_FLOAT8 = 16, O_FLOAT16 = 18 }; /* opal_datatype_internal.h:107-131 */
static const struct mini_predef {
    int id, slot;
    size_t size;
    ptrdiff_t ext, true_ub;
    uint16_t flags;
    const char *name;
    int ne;                                                    /* description elements (pair types) */
    struct { uint16_t type; uint32_t count; int64_t ext, disp; } e[2];
} predefined[] = {
    {0x01, MI355X_T_INT8, 1, 1, 1, F_BASIC, "MPI_INT8_T", 0, {{0}}},
    {0x02, MI355X_T_UINT8, 1, 1, 1, F_BASIC, "MPI_UINT8_T", 0, {{0}}},
    {0x03, MI355X_T_INT16, 2, 2, 2, F_BASIC, "MPI_INT16_T", 0, {{0}}},
    {0x04, MI355X_T_UINT16, 2, 2, 2, F_BASIC, "MPI_UINT16_T", 0, {{0}}},
    {0x05, MI355X_T_INT32, 4, 4, 4, F_BASIC, "MPI_INT32_T", 0, {{0}}},
    {0x06, MI355X_T_UINT32, 4, 4, 4, F_BASIC, "MPI_UINT32_T", 0, {{0}}},
    {0x07, MI355X_T_INT64, 8, 8, 8, F_BASIC, "MPI_INT64_T", 0, {{0}}},
    {0x08, MI355X_T_UINT64, 8, 8, 8, F_BASIC, "MPI_UINT64_T", 0, {{0}}},
    {0x09, MI355X_T_FLOAT, 4, 4, 4, F_BASIC, "MPI_FLOAT", 0, {{0}}},
    {0x0A, MI355X_T_DOUBLE, 8, 8, 8, F_BASIC, "MPI_DOUBLE", 0, {{0}}},
    {0x0B, MI355X_T_LONG_DOUBLE, 16, 16, 16, F_BASIC, "MPI_LONG_DOUBLE", 0, {{0}}},
    {0x11, MI355X_T_BOOL, 1, 1, 1, F_BASIC, "MPI_CXX_BOOL", 0, {{0}}},
    {0x13, MI355X_T_UINT8, 1, 1, 1, F_BASIC, "MPI_CHARACTER", 0, {{0}}},
    {0x1A, MI355X_T_2INT, 8, 8, 8, F_PAIR | F_CNG | OMPI_DATATYPE_FLAG_DATA_INT, "MPI_2INT", 1,
     {{O_INT4, 2, 4, 0}}},
    {0x20, MI355X_T_FLOAT_INT, 8, 8, 8, F_PAIR | F_CNG, "MPI_FLOAT_INT", 2, {{O_FLOAT4, 1, 4, 0}, {O_INT4, 1, 4, 4}}},
    {0x21, MI355X_T_DOUBLE_INT, 12, 16, 12, F_PAIR | OPAL_DATATYPE_FLAG_CONTIGUOUS, "MPI_DOUBLE_INT", 2,
     {{O_FLOAT8, 1, 8, 0}, {O_INT4, 1, 4, 8}}},
    {0x22, MI355X_T_LONG_DOUBLE_INT, 20, 32, 20, F_PAIR | OPAL_DATATYPE_FLAG_CONTIGUOUS, "MPI_LONG_DOUBLE_INT", 2,
     {{O_FLOAT16, 1, 16, 0}, {O_INT4, 1, 4, 16}}},
    {0x23, MI355X_T_LONG_INT, 12, 16, 12, F_PAIR | OPAL_DATATYPE_FLAG_CONTIGUOUS | OMPI_DATATYPE_FLAG_DATA_INT,
     "MPI_LONG_INT", 2, {{O_INT8, 1, 8, 0}, {O_INT4, 1, 4, 8}}},
    {0x24, MI355X_T_SHORT_INT, 6, 8, 8, F_PAIR | OMPI_DATATYPE_FLAG_DATA_INT, "MPI_SHORT_INT", 2,
     {{O_INT2, 1, 2, 0}, {O_INT4, 1, 4, 4}}},
    {0x27, MI355X_T_BOOL, 1, 1, 1, F_BASIC, "MPI_C_BOOL", 0, {{0}}},
    {0x29, MI355X_T_C_FLOAT_COMPLEX, 8, 8, 8, F_BASIC, "MPI_C_FLOAT_COMPLEX", 0, {{0}}},
    {0x2A, MI355X_T_C_DOUBLE_COMPLEX, 16, 16, 16, F_BASIC, "MPI_C_DOUBLE_COMPLEX", 0, {{0}}},
    {0x2B, MI355X_T_C_LONG_DOUBLE_COMPLEX, 32, 32, 32, F_BASIC, "MPI_C_LONG_DOUBLE_COMPLEX", 0, {{0}}},
};
static ompi_datatype_t *dt_objs[OMPI_DATATYPE_MPI_MAX_PREDEFINED];

static opal_class_t ompi_datatype_t_class = {"ompi_datatype_t", &opal_object_t_class, NULL, NULL, 0, 0, NULL, NULL,
                                             sizeof(ompi_datatype_t)};

ompi_predefined_datatype_t ompi_mpi_byte;  /* MPI_BYTE (mpi.h.in:913) */

/* a committed description (dt_elem_desc_t records of 32 bytes, opal_datatype_internal.h:148-188):
 * the elements as opal_datatype_add appends them (:276-350), then the END_LOOP that
 * opal_datatype_commit adds (opal_datatype_optimize.c:255-282) */
static void put16(unsigned char *p, uint16_t v) { memcpy(p, &v, 2); }
static void put32(unsigned char *p, uint32_t v) { memcpy(p, &v, 4); }
static void put64(unsigned char *p, int64_t v) { memcpy(p, &v, 8); }
static void pair_desc(ompi_datatype_t *d, const struct mini_predef *p)
{
    const uint32_t used = (uint32_t)p->ne + 1;
    unsigned char *r = calloc(used, 32);
    for (int i = 0; i < p->ne; ++i) {
        unsigned char *e = r + 32 * i;
        /* the added basic type's flags less COMMITTED (opal_datatype_add.c:283-290) */
        put16(e, OPAL_DATATYPE_FLAG_PREDEFINED | OPAL_DATATYPE_FLAG_CONTIGUOUS | OPAL_DATATYPE_FLAG_NO_GAPS |
                     OPAL_DATATYPE_FLAG_DATA);
        put16(e + 2, p->e[i].type);
        put32(e + 4, p->e[i].count);
        put32(e + 8, 1);
        put64(e + 16, p->e[i].ext);
        put64(e + 24, p->e[i].disp);
    }
    unsigned char *end = r + 32 * p->ne;
    put16(end + 2, 1);  /* OPAL_DATATYPE_END_LOOP */
    put32(end + 4, (uint32_t)p->ne);
    put64(end + 16, (int64_t)p->size);
    put64(end + 24, p->e[0].disp);
    d->super.desc.desc = (dt_elem_desc_t *)r;
    d->super.desc.used = (uint32_t)p->ne;  /* the END_LOOP sits at desc[used] (opal_datatype_optimize.c:257) */
    d->super.desc.length = used;
    d->super.opt_desc = d->super.desc;
}

void mini_init(void)
{
    static int done = 0;
    if (done) return;
    done = 1;
    mini_pml_install_stub();
    /* MPI_REQUEST_NULL (ompi_request_init, request.c:108-150): complete, inactive, index 0 */
    ompi_request_null.request.req_type = OMPI_REQUEST_NULL;
    ompi_request_null.request.req_complete = true;
    ompi_request_null.request.req_state = OMPI_REQUEST_INACTIVE;
    ompi_request_null.request.req_f_to_c_index = 0;
    for (int i = 0; i < OMPI_DATATYPE_MPI_MAX_PREDEFINED; ++i) ompi_op_ddt_map[i] = -1;
    for (size_t k = 0; k < sizeof(predefined) / sizeof(predefined[0]); ++k) {
        ompi_op_ddt_map[predefined[k].id] = predefined[k].slot;
        ompi_datatype_t *d = (ompi_datatype_t *)mi355x_obj_new(&ompi_datatype_t_class);
        memset((char *)d + sizeof(opal_object_t), 0, sizeof(*d) - sizeof(opal_object_t));
        d->super.flags = predefined[k].flags;
        d->super.id = (uint16_t)predefined[k].id;
        d->super.size = predefined[k].size;
        d->super.ub = predefined[k].ext;
        d->super.true_ub = predefined[k].true_ub;
        d->id = predefined[k].id;
        if (predefined[k].ne) pair_desc(d, &predefined[k]);
        snprintf(d->name, sizeof(d->name), "%s", predefined[k].name);
        dt_objs[predefined[k].id] = d;
    }
    ompi_datatype_t *b = &ompi_mpi_byte.dt;
    b->super.super.obj_class = &ompi_datatype_t_class;
    b->super.super.obj_reference_count = 1;
    b->super.flags = F_BASIC;
    b->super.id = 4; /* OPAL_DATATYPE_UINT1 */
    b->super.size = 1;
    b->super.true_ub = b->super.ub = 1;
    b->id = OMPI_DATATYPE_MPI_BYTE;
    snprintf(b->name, sizeof(b->name), "MPI_BYTE");
}

ompi_datatype_t *mini_datatype(int id)
{
    mini_init();
    return (id >= 0 && id < OMPI_DATATYPE_MPI_MAX_PREDEFINED) ? dt_objs[id] : NULL;
}

/* a committed derived datatype from its optimized description (records of 32 bytes,
 * opal_datatype_internal.h:148-188) and bounds -- what ompi_datatype_create_* + commit leave in
 * opal_datatype_t (opal_datatype.h:103-131) */
ompi_datatype_t *mini_datatype_create_raw(const void *desc, uint32_t used, size_t size, ptrdiff_t lb, ptrdiff_t ub,
                                          ptrdiff_t true_lb, ptrdiff_t true_ub, uint16_t flags)
{
    mini_init();
    ompi_datatype_t *d = (ompi_datatype_t *)mi355x_obj_new(&ompi_datatype_t_class);
    memset((char *)d + sizeof(opal_object_t), 0, sizeof(*d) - sizeof(opal_object_t));
    d->super.flags = flags;
    d->super.id = 0; /* OPAL_DATATYPE_LOOP: not a predefined id */
    d->super.size = size;
    d->super.lb = lb;
    d->super.ub = ub;
    d->super.true_lb = true_lb;
    d->super.true_ub = true_ub;
    void *copy = malloc((size_t)used * 32);
    memcpy(copy, desc, (size_t)used * 32);
    d->super.opt_desc.desc = (dt_elem_desc_t *)copy;
    d->super.opt_desc.used = used;
    d->super.opt_desc.length = used;
    d->super.desc = d->super.opt_desc;
    d->id = -1;
    snprintf(d->name, sizeof(d->name), "derived");
    return d;
}

void mini_datatype_destroy(ompi_datatype_t *d)
{
    if (!d) return;
    free(d->super.opt_desc.desc);
    d->super.opt_desc.desc = NULL;
    d->super.desc.desc = NULL;
    mi355x_obj_release(&d->super.super);
}

/* the committed datatype's opal fields, for tests: flags, size, lb, ub, true_lb, true_ub, desc.used,
 * and its description records (desc.used + 1 with the trailing END_LOOP) */
void mini_datatype_fields(const ompi_datatype_t *d, int64_t out[7])
{
    out[0] = d->super.flags;
    out[1] = (int64_t)d->super.size;
    out[2] = d->super.lb;
    out[3] = d->super.ub;
    out[4] = d->super.true_lb;
    out[5] = d->super.true_ub;
    out[6] = d->super.desc.used;
}
const void *mini_datatype_desc(const ompi_datatype_t *d) { return d->super.desc.desc; }

int mini_datatype_id_for_slot(int slot)
{
    mini_init();
    for (size_t k = 0; k < sizeof(predefined) / sizeof(predefined[0]); ++k)
        if (predefined[k].slot == slot) return predefined[k].id;
    return -1;
}

/* ------------------------------------------------------------------ ops */
static ompi_op_base_handler_fn_t base2[MI355X_OP_MAX_][OMPI_OP_BASE_TYPE_MAX];
static ompi_op_base_3buff_handler_fn_t base3[MI355X_OP_MAX_][OMPI_OP_BASE_TYPE_MAX];

void mini_set_base_function(int op, int slot, void *fn2, void *fn3)
{
    base2[op][slot] = (ompi_op_base_handler_fn_t)fn2;
    base3[op][slot] = (ompi_op_base_3buff_handler_fn_t)fn3;
}

static opal_class_t ompi_op_t_class = {"ompi_op_t", &opal_object_t_class, NULL, NULL, 0, 0, NULL, NULL,
                                       sizeof(ompi_op_t)};

ompi_op_t *mini_op_create(int code)
{
    mini_init();
    ompi_op_t *op = (ompi_op_t *)mi355x_obj_new(&ompi_op_t_class);
    memset((char *)op + sizeof(opal_object_t), 0, sizeof(*op) - sizeof(opal_object_t));
    snprintf(op->o_name, sizeof(op->o_name), "MPI_OP_%d", code);
    op->op_type = code;
    op->o_f_to_c_index = code;
    op->o_flags = OMPI_OP_FLAGS_INTRINSIC | OMPI_OP_FLAGS_COMMUTE;
    return op;
}

/* ompi_op_base_op_select (op_base_op_select.c:88-204) over an explicit component list sorted by
 * ascending priority by the caller's query results.  Returns OMPI_SUCCESS or an error. */
int mini_op_select(ompi_op_t *op, ompi_op_base_component_t **comps, int ncomp)
{
    ompi_op_base_module_t *basemod = (ompi_op_base_module_t *)mi355x_obj_new(&ompi_op_base_module_t_class);
    for (int i = 0; i < OMPI_OP_BASE_TYPE_MAX; ++i) {
        op->o_func.intrinsic.fns[i] = base2[op->o_f_to_c_index][i];
        op->o_func.intrinsic.modules[i] = basemod;
        mi355x_obj_retain(&basemod->super);
        op->o_3buff_intrinsic.fns[i] = base3[op->o_f_to_c_index][i];
        op->o_3buff_intrinsic.modules[i] = basemod;
        mi355x_obj_retain(&basemod->super);
    }
    mi355x_obj_release(&basemod->super);
    /* query, keep the modules, sort by ascending priority (check_components :227-263) */
    ompi_op_base_module_t *mods[16];
    int prios[16], nm = 0;
    for (int c = 0; c < ncomp && nm < 16; ++c) {
        int prio = 0;
        ompi_op_base_module_t *m = comps[c]->opc_op_query(op, &prio);
        if (!m) continue;
        if (prio > 100) prio = 100;
        int k = nm++;
        while (k > 0 && prios[k - 1] > prio) { mods[k] = mods[k - 1]; prios[k] = prios[k - 1]; --k; }
        mods[k] = m;
        prios[k] = prio;
    }
    for (int k = 0; k < nm; ++k) {
        ompi_op_base_module_t *m = mods[k];
        if (m->opm_enable && OMPI_SUCCESS != m->opm_enable(m, op)) {
            mi355x_obj_release(&m->super);
            continue;
        }
        for (int i = 0; i < OMPI_OP_BASE_TYPE_MAX; ++i) {
            if (m->opm_fns[i]) {
                mi355x_obj_release(&op->o_func.intrinsic.modules[i]->super);
                op->o_func.intrinsic.fns[i] = m->opm_fns[i];
                op->o_func.intrinsic.modules[i] = m;
                mi355x_obj_retain(&m->super);
            }
            if (m->opm_3buff_fns[i]) {
                /* op_base_op_select.c:162-168 releases the 2-buff slot's module here */
                mi355x_obj_release(&op->o_func.intrinsic.modules[i]->super);
                op->o_3buff_intrinsic.fns[i] = m->opm_3buff_fns[i];
                op->o_3buff_intrinsic.modules[i] = m;
                mi355x_obj_retain(&m->super);
            }
        }
        mi355x_obj_release(&m->super);
    }
    for (int i = 0; i < OMPI_OP_BASE_TYPE_MAX; ++i) {
        const int want = base2[op->o_f_to_c_index][i] != NULL;
        if (want != (op->o_func.intrinsic.fns[i] != NULL)) return OMPI_ERR_NOT_FOUND;
    }
    return OMPI_SUCCESS;
}

void mini_op_reduce(ompi_op_t *op, void *source, void *target, int count, ompi_datatype_t *dtype)
{
    const int t = ompi_op_ddt_map[dtype->id];
    op->o_func.intrinsic.fns[t](source, target, &count, &dtype, op->o_func.intrinsic.modules[t]);
}

void mini_op_reduce_3buff(ompi_op_t *op, void *s1, void *s2, void *target, int count, ompi_datatype_t *dtype)
{
    const int t = ompi_op_ddt_map[dtype->id];
    op->o_3buff_intrinsic.fns[t](s1, s2, target, &count, &dtype, op->o_3buff_intrinsic.modules[t]);
}

void *mini_op_fn2(ompi_op_t *op, int slot) { return (void *)op->o_func.intrinsic.fns[slot]; }
void *mini_op_module2(ompi_op_t *op, int slot) { return op->o_func.intrinsic.modules[slot]; }
void *mini_op_module3(ompi_op_t *op, int slot) { return op->o_3buff_intrinsic.modules[slot]; }
int mini_obj_refcount(void *obj) { return ((opal_object_t *)obj)->obj_reference_count; }

/* ompi_op_destruct (op.c:476-487): release every slot's module, 2-buff then 3-buff */
void mini_op_destroy(ompi_op_t *op)
{
    for (int i = 0; i < OMPI_OP_BASE_TYPE_MAX; ++i) {
        if (op->o_func.intrinsic.modules[i]) mi355x_obj_release(&op->o_func.intrinsic.modules[i]->super);
        if (op->o_3buff_intrinsic.modules[i]) mi355x_obj_release(&op->o_3buff_intrinsic.modules[i]->super);
    }
    free(op);
}

/* ------------------------------------------------------------------ communicators */
static opal_class_t comm_class = {"ompi_communicator_t", &opal_object_t_class, NULL, NULL, 0, 0, NULL, NULL,
                                  sizeof(ompi_communicator_t)};
static opal_class_t group_class = {"ompi_group_t", &opal_object_t_class, NULL, NULL, 0, 0, NULL, NULL,
                                   sizeof(ompi_group_t)};

ompi_communicator_t *mini_comm_create(int rank, int size, unsigned cid)
{
    mini_init();
    ompi_communicator_t *c = (ompi_communicator_t *)mi355x_obj_new(&comm_class);
    memset((char *)c + sizeof(opal_object_t), 0, sizeof(*c) - sizeof(opal_object_t));
    ompi_group_t *g = (ompi_group_t *)mi355x_obj_new(&group_class);
    memset((char *)g + sizeof(opal_object_t), 0, sizeof(*g) - sizeof(opal_object_t));
    g->grp_proc_count = size;
    g->grp_my_rank = rank;
    c->c_local_group = g;
    c->c_remote_group = g;
    c->c_my_rank = rank;
    c->c_contextid = cid;
    snprintf(c->c_name, sizeof(c->c_name), "mini_comm_%u", cid);
    return c;
}

/* install a lower-priority module's functions (what coll/basic + tuned would have done) */
void mini_comm_install(ompi_communicator_t *c, mca_coll_base_module_t *m)
{
#define INST(FN)                                                                 \
    if (m->coll_##FN) {                                                          \
        if (c->c_coll.coll_##FN##_module) mi355x_obj_release(&c->c_coll.coll_##FN##_module->super); \
        c->c_coll.coll_##FN = m->coll_##FN;                                      \
        c->c_coll.coll_##FN##_module = m;                                        \
        mi355x_obj_retain(&m->super);                                            \
    }
    INST(allgather)
    INST(allreduce)
    INST(bcast)
    INST(reduce)
    INST(reduce_scatter)
    INST(reduce_scatter_block)
    INST(iallgather)
    INST(iallreduce)
    INST(ibcast)
    INST(ireduce)
    INST(ireduce_scatter_block)
    INST(gather)
    INST(gatherv)
    INST(scatter)
    INST(scatterv)
    INST(allgatherv)
    INST(alltoall)
    INST(alltoallv)
    INST(scan)
    INST(exscan)
#undef INST
}

/* mca_coll_base_comm_select for one extra component (coll_base_comm_select.c:114-262): query,
 * enable, copy non-NULL functions.  Returns the priority, or < 0 when the component declined. */
/* mca_coll_base_find_available (coll_base_find_available.c:108-160) -> collm_init_query, and
 * mca_base_component_close -> mca_close_component, for one component */
int mini_coll_init(mca_coll_base_component_t *comp)
{
    return comp->collm_init_query ? comp->collm_init_query(false, false) : OMPI_SUCCESS;
}
int mini_coll_close(mca_coll_base_component_t *comp)
{
    return comp->collm_version.mca_close_component ? comp->collm_version.mca_close_component() : OMPI_SUCCESS;
}

int mini_coll_select(ompi_communicator_t *c, mca_coll_base_component_t *comp)
{
    int prio = 0;
    mca_coll_base_module_t *m = comp->collm_comm_query(c, &prio);
    if (!m) return -1;
    if (m->coll_module_enable && OMPI_SUCCESS != m->coll_module_enable(m, c)) {
        mi355x_obj_release(&m->super);
        return -2;
    }
    mini_comm_install(c, m);
    mi355x_obj_release(&m->super);
    return prio;
}

mca_coll_base_module_t *mini_coll_module_new(void)
{
    mini_init();
    return (mca_coll_base_module_t *)mi355x_obj_new(&mca_coll_base_module_t_class);
}

void mini_comm_destroy(ompi_communicator_t *c)
{
#define REL(FN) if (c->c_coll.coll_##FN##_module) mi355x_obj_release(&c->c_coll.coll_##FN##_module->super);
    REL(allgather)
    REL(allreduce)
    REL(bcast)
    REL(reduce)
    REL(reduce_scatter)
    REL(reduce_scatter_block)
    REL(iallgather)
    REL(iallreduce)
    REL(ibcast)
    REL(ireduce)
    REL(ireduce_scatter_block)
    REL(gather)
    REL(gatherv)
    REL(scatter)
    REL(scatterv)
    REL(allgatherv)
    REL(alltoall)
    REL(alltoallv)
    REL(scan)
    REL(exscan)
#undef REL
    chan_release(c);
    mi355x_obj_release(&c->c_local_group->super);
    free(c);
}

/* ---- requests + progress (ompi/request/request.c, req_wait.c; opal/runtime/opal_progress.c) ---- */
static void request_construct(opal_object_t *o)  /* ompi_request_construct, request.c:52-65 */
{
    ompi_request_t *req = (ompi_request_t *)o;
    req->req_state = OMPI_REQUEST_INVALID;
    req->req_complete = false;
    req->req_persistent = false;
    req->req_free = NULL;
    req->req_cancel = NULL;
    req->req_complete_cb = NULL;
    req->req_complete_cb_data = NULL;
    req->req_f_to_c_index = MPI_UNDEFINED;
    req->req_mpi_object.comm = NULL;
}
opal_class_t ompi_request_t_class = {"ompi_request_t", &opal_object_t_class, request_construct, NULL, 0, 0,
                                     NULL, NULL, sizeof(ompi_request_t)};
size_t ompi_request_waiting = 0, ompi_request_completed = 0, ompi_request_failed = 0;
opal_condition_t ompi_request_cond;
ompi_predefined_request_t ompi_request_null;
struct opal_pointer_array_t { int unused; } ompi_request_f_to_c_table;
int opal_pointer_array_set_item(struct opal_pointer_array_t *array, int index, void *value)
{
    (void)array; (void)index; (void)value;
    return 0;
}

static opal_progress_callback_t progress_cbs[16];
static int progress_n;
int opal_progress_register(opal_progress_callback_t cb)
{
    for (int i = 0; i < progress_n; ++i)
        if (progress_cbs[i] == cb) return 0;
    if (progress_n == 16) return -1;
    progress_cbs[progress_n++] = cb;
    return 0;
}
int opal_progress_unregister(opal_progress_callback_t cb)
{
    for (int i = 0; i < progress_n; ++i)
        if (progress_cbs[i] == cb) {
            progress_cbs[i] = progress_cbs[--progress_n];
            return 0;
        }
    return -1;
}
int mini_progress(void)  /* opal_progress: run every registered callback */
{
    int events = 0;
    for (int i = 0; i < progress_n; ++i) events += progress_cbs[i]();
    return events;
}
int mini_progress_callbacks(void) { return progress_n; }
void opal_progress(void) { (void)mini_progress(); }
/* MPI_Wait (ompi_request_default_wait, req_wait.c:33-76): progress until complete, copy the status
 * out (not MPI_ERROR), then a persistent request goes INACTIVE (:59-63) and any other is freed
 * unless it failed; *req becomes MPI_REQUEST_NULL */
int mini_wait_status(ompi_request_t **req, ompi_status_public_t *st)
{
    ompi_request_t *r = *req;
    if (r == &ompi_request_null.request) return 0;
    while (!r->req_complete) mini_progress();
    if (st) {
        st->MPI_SOURCE = r->req_status.MPI_SOURCE;
        st->MPI_TAG = r->req_status.MPI_TAG;
        st->_ucount = r->req_status._ucount;
        st->_cancelled = r->req_status._cancelled;
        st->MPI_ERROR = r->req_status.MPI_ERROR;  /* (MPI_Wait returns it; kept here for the tests) */
    }
    if (r->req_persistent) {
        if (r->req_state == OMPI_REQUEST_INACTIVE) return 0;
        r->req_state = OMPI_REQUEST_INACTIVE;
        return r->req_status.MPI_ERROR;
    }
    if (r->req_status.MPI_ERROR != 0) return r->req_status.MPI_ERROR;
    return r->req_free(req);
}
int mini_wait(ompi_request_t **req) { return mini_wait_status(req, NULL); }
/* MPI_Test (ompi_request_default_test, req_test.c:30-90): one progress pass; complete -> as wait */
int mini_test(ompi_request_t **req, int *flag, ompi_status_public_t *st)
{
    ompi_request_t *r = *req;
    *flag = 0;
    if (r == &ompi_request_null.request) {
        *flag = 1;
        return 0;
    }
    if (!r->req_complete) mini_progress();
    if (!r->req_complete) return 0;
    *flag = 1;
    return mini_wait_status(req, st);
}
/* MPI_Request_free (ompi/mpi/c/request_free.c:54-60 -> req_free) */
int mini_request_free(ompi_request_t **req) { return (*req)->req_free(req); }
/* MPI_Cancel (ompi/mpi/c/cancel.c -> ompi_request_cancel, request.h:353-360) */
int mini_cancel(ompi_request_t *r) { return r->req_cancel ? r->req_cancel(r, r->req_complete) : 0; }
/* MPI_Start (ompi/mpi/c/start.c:66-72: a PML request -> MCA_PML_CALL(start(1, request))) */
int mini_start(ompi_request_t **req) { return mca_pml.pml_start(1, req); }

/* MPI_MESSAGE_NULL (message.c) and the message class; the PML allocates messages */
opal_class_t ompi_message_t_class = {"ompi_message_t", &opal_object_t_class, NULL, NULL, 0, 0, NULL, NULL,
                                     sizeof(ompi_message_t)};
ompi_predefined_message_t ompi_message_null;
int mini_message_is_null(ompi_message_t *m) { return m == &ompi_message_null.message; }
int mini_request_is_null(ompi_request_t *r) { return r == &ompi_request_null.request; }

/* ---- the PML slot (ompi/mca/pml/pml.h:497-558): `mca_pml` is the selected PML's table and
 * MCA_PML_CALL(x) is mca_pml.pml_x.  The harness's "selected PML" is a stub (no transport):
 * it counts calls and returns the stub marker -- what a host-buffer message would hand to ob1. */
mca_pml_base_module_t mca_pml;
static int pml_stub_calls[16];
static int pst_isend(void *b, size_t n, struct ompi_datatype_t *d, int dst, int tag, mca_pml_base_send_mode_t m,
                     struct ompi_communicator_t *c, struct ompi_request_t **req)
{ (void)b; (void)n; (void)d; (void)dst; (void)tag; (void)m; (void)c; *req = &ompi_request_null.request; pml_stub_calls[0]++; return 77; }
static int pst_send(void *b, size_t n, struct ompi_datatype_t *d, int dst, int tag, mca_pml_base_send_mode_t m,
                    struct ompi_communicator_t *c)
{ (void)b; (void)n; (void)d; (void)dst; (void)tag; (void)m; (void)c; pml_stub_calls[1]++; return 77; }
static int pst_irecv(void *b, size_t n, struct ompi_datatype_t *d, int src, int tag, struct ompi_communicator_t *c,
                     struct ompi_request_t **req)
{ (void)b; (void)n; (void)d; (void)src; (void)tag; (void)c; *req = &ompi_request_null.request; pml_stub_calls[2]++; return 77; }
static int pst_recv(void *b, size_t n, struct ompi_datatype_t *d, int src, int tag, struct ompi_communicator_t *c,
                    ompi_status_public_t *st)
{ (void)b; (void)n; (void)d; (void)src; (void)tag; (void)c; (void)st; pml_stub_calls[3]++; return 77; }
static int pst_iprobe(int src, int tag, struct ompi_communicator_t *c, int *matched, ompi_status_public_t *st)
{ (void)src; (void)tag; (void)c; (void)st; *matched = 0; pml_stub_calls[4]++; return 0; }
static int pst_probe(int src, int tag, struct ompi_communicator_t *c, ompi_status_public_t *st)
{ (void)src; (void)tag; (void)c; (void)st; pml_stub_calls[5]++; return 77; }
static int pst_isend_init(void *b, size_t n, struct ompi_datatype_t *d, int dst, int tag, mca_pml_base_send_mode_t m,
                          struct ompi_communicator_t *c, struct ompi_request_t **req)
{ (void)b; (void)n; (void)d; (void)dst; (void)tag; (void)m; (void)c; *req = &ompi_request_null.request; pml_stub_calls[6]++; return 77; }
static int pst_irecv_init(void *b, size_t n, struct ompi_datatype_t *d, int src, int tag, struct ompi_communicator_t *c,
                          struct ompi_request_t **req)
{ (void)b; (void)n; (void)d; (void)src; (void)tag; (void)c; *req = &ompi_request_null.request; pml_stub_calls[7]++; return 77; }
static int pst_start(size_t n, struct ompi_request_t **reqs) { (void)n; (void)reqs; pml_stub_calls[8]++; return 77; }
static int pst_improbe(int src, int tag, struct ompi_communicator_t *c, int *matched, struct ompi_message_t **msg,
                       ompi_status_public_t *st)
{ (void)src; (void)tag; (void)c; (void)st; *matched = 0; *msg = &ompi_message_null.message; pml_stub_calls[9]++; return 0; }
static int pst_mprobe(int src, int tag, struct ompi_communicator_t *c, struct ompi_message_t **msg, ompi_status_public_t *st)
{ (void)src; (void)tag; (void)c; (void)msg; (void)st; pml_stub_calls[10]++; return 77; }
static int pst_imrecv(void *b, size_t n, struct ompi_datatype_t *d, struct ompi_message_t **msg, struct ompi_request_t **req)
{ (void)b; (void)n; (void)d; (void)msg; *req = &ompi_request_null.request; pml_stub_calls[11]++; return 77; }
static int pst_mrecv(void *b, size_t n, struct ompi_datatype_t *d, struct ompi_message_t **msg, ompi_status_public_t *st)
{ (void)b; (void)n; (void)d; (void)msg; (void)st; pml_stub_calls[12]++; return 77; }

void mini_pml_install_stub(void)
{
    memset(&mca_pml, 0, sizeof(mca_pml));
    mca_pml.pml_isend = pst_isend;
    mca_pml.pml_send = pst_send;
    mca_pml.pml_irecv = pst_irecv;
    mca_pml.pml_recv = pst_recv;
    mca_pml.pml_iprobe = pst_iprobe;
    mca_pml.pml_probe = pst_probe;
    mca_pml.pml_isend_init = pst_isend_init;
    mca_pml.pml_irecv_init = pst_irecv_init;
    mca_pml.pml_start = pst_start;
    mca_pml.pml_improbe = pst_improbe;
    mca_pml.pml_mprobe = pst_mprobe;
    mca_pml.pml_imrecv = pst_imrecv;
    mca_pml.pml_mrecv = pst_mrecv;
    mca_pml.pml_max_tag = 0x7fffffff;
}
int mini_pml_stub_calls(int which) { return (which >= 0 && which < 16) ? pml_stub_calls[which] : -1; }
void *mini_pml_fn(int which)
{
    switch (which) {
    case 0: return (void *)mca_pml.pml_isend;
    case 1: return (void *)mca_pml.pml_send;
    case 2: return (void *)mca_pml.pml_irecv;
    case 3: return (void *)mca_pml.pml_recv;
    case 4: return (void *)mca_pml.pml_iprobe;
    case 5: return (void *)mca_pml.pml_probe;
    case 6: return (void *)mca_pml.pml_isend_init;
    case 7: return (void *)mca_pml.pml_irecv_init;
    case 8: return (void *)mca_pml.pml_start;
    case 9: return (void *)mca_pml.pml_improbe;
    case 10: return (void *)mca_pml.pml_mprobe;
    case 11: return (void *)mca_pml.pml_imrecv;
    case 12: return (void *)mca_pml.pml_mrecv;
    default: return NULL;
    }
}
/* MPI_Send / MPI_Recv / MPI_Isend / MPI_Irecv / MPI_Iprobe as the bindings call them
 * (ompi/mpi/c/send.c:75, recv.c:69, isend.c:76, irecv.c:69, iprobe.c:67): MCA_PML_CALL(...) */
int mini_send(void *b, int n, ompi_datatype_t *d, int dst, int tag, ompi_communicator_t *c)
{
    return mca_pml.pml_send(b, (size_t)n, d, dst, tag, MCA_PML_BASE_SEND_STANDARD, c);
}
int mini_ssend(void *b, int n, ompi_datatype_t *d, int dst, int tag, ompi_communicator_t *c)
{
    return mca_pml.pml_send(b, (size_t)n, d, dst, tag, MCA_PML_BASE_SEND_SYNCHRONOUS, c);
}
int mini_recv(void *b, int n, ompi_datatype_t *d, int src, int tag, ompi_communicator_t *c, ompi_status_public_t *st)
{
    return mca_pml.pml_recv(b, (size_t)n, d, src, tag, c, st);
}
int mini_isend(void *b, int n, ompi_datatype_t *d, int dst, int tag, ompi_communicator_t *c, ompi_request_t **req)
{
    return mca_pml.pml_isend(b, (size_t)n, d, dst, tag, MCA_PML_BASE_SEND_STANDARD, c, req);
}
int mini_irecv(void *b, int n, ompi_datatype_t *d, int src, int tag, ompi_communicator_t *c, ompi_request_t **req)
{
    return mca_pml.pml_irecv(b, (size_t)n, d, src, tag, c, req);
}
int mini_iprobe(int src, int tag, ompi_communicator_t *c, int *flag, ompi_status_public_t *st)
{
    return mca_pml.pml_iprobe(src, tag, c, flag, st);
}
/* any send mode: MPI_Bsend (bsend.c: MCA_PML_BASE_SEND_BUFFERED), MPI_Rsend (READY), MPI_Ssend */
int mini_send_mode(void *b, int n, ompi_datatype_t *d, int dst, int tag, int mode, ompi_communicator_t *c)
{
    return mca_pml.pml_send(b, (size_t)n, d, dst, tag, (mca_pml_base_send_mode_t)mode, c);
}
int mini_isend_mode(void *b, int n, ompi_datatype_t *d, int dst, int tag, int mode, ompi_communicator_t *c,
                    ompi_request_t **req)
{
    return mca_pml.pml_isend(b, (size_t)n, d, dst, tag, (mca_pml_base_send_mode_t)mode, c, req);
}
int mini_probe(int src, int tag, ompi_communicator_t *c, ompi_status_public_t *st)
{
    return mca_pml.pml_probe(src, tag, c, st);
}
/* MPI_Send_init / MPI_Recv_init (send_init.c:74-77, recv_init.c:66-67) */
int mini_send_init(void *b, int n, ompi_datatype_t *d, int dst, int tag, int mode, ompi_communicator_t *c,
                   ompi_request_t **req)
{
    return mca_pml.pml_isend_init(b, (size_t)n, d, dst, tag, (mca_pml_base_send_mode_t)mode, c, req);
}
int mini_recv_init(void *b, int n, ompi_datatype_t *d, int src, int tag, ompi_communicator_t *c, ompi_request_t **req)
{
    return mca_pml.pml_irecv_init(b, (size_t)n, d, src, tag, c, req);
}
/* MPI_Improbe / MPI_Mprobe / MPI_Imrecv / MPI_Mrecv (improbe.c:73, mprobe.c:72, imrecv.c:69, mrecv.c:71) */
int mini_improbe(int src, int tag, ompi_communicator_t *c, int *flag, ompi_message_t **msg, ompi_status_public_t *st)
{
    return mca_pml.pml_improbe(src, tag, c, flag, msg, st);
}
int mini_mprobe(int src, int tag, ompi_communicator_t *c, ompi_message_t **msg, ompi_status_public_t *st)
{
    return mca_pml.pml_mprobe(src, tag, c, msg, st);
}
int mini_imrecv(void *b, int n, ompi_datatype_t *d, ompi_message_t **msg, ompi_request_t **req)
{
    return mca_pml.pml_imrecv(b, (size_t)n, d, msg, req);
}
int mini_mrecv(void *b, int n, ompi_datatype_t *d, ompi_message_t **msg, ompi_status_public_t *st)
{
    return mca_pml.pml_mrecv(b, (size_t)n, d, msg, st);
}
int mini_request_complete(ompi_request_t *r) { return r->req_complete ? 1 : 0; }

/* C-callable MPI-style entry points through the communicator's installed functions */
int mini_allreduce(ompi_communicator_t *c, void *s, void *r, int n, ompi_datatype_t *d, ompi_op_t *op)
{
    return c->c_coll.coll_allreduce(s, r, n, d, op, c, c->c_coll.coll_allreduce_module);
}
int mini_iallreduce(ompi_communicator_t *c, void *s, void *r, int n, ompi_datatype_t *d, ompi_op_t *op,
                    ompi_request_t **req)
{
    return c->c_coll.coll_iallreduce(s, r, n, d, op, c, req, c->c_coll.coll_iallreduce_module);
}
int mini_ireduce(ompi_communicator_t *c, void *s, void *r, int n, ompi_datatype_t *d, ompi_op_t *op, int root,
                 ompi_request_t **req)
{
    return c->c_coll.coll_ireduce(s, r, n, d, op, root, c, req, c->c_coll.coll_ireduce_module);
}
int mini_ireduce_scatter_block(ompi_communicator_t *c, void *s, void *r, int n, ompi_datatype_t *d, ompi_op_t *op,
                               ompi_request_t **req)
{
    return c->c_coll.coll_ireduce_scatter_block(s, r, n, d, op, c, req, c->c_coll.coll_ireduce_scatter_block_module);
}
int mini_iallgather(ompi_communicator_t *c, void *s, int sc, ompi_datatype_t *sd, void *r, int rc, ompi_datatype_t *rd,
                    ompi_request_t **req)
{
    return c->c_coll.coll_iallgather(s, sc, sd, r, rc, rd, c, req, c->c_coll.coll_iallgather_module);
}
int mini_ibcast(ompi_communicator_t *c, void *b, int n, ompi_datatype_t *d, int root, ompi_request_t **req)
{
    return c->c_coll.coll_ibcast(b, n, d, root, c, req, c->c_coll.coll_ibcast_module);
}
int mini_reduce(ompi_communicator_t *c, void *s, void *r, int n, ompi_datatype_t *d, ompi_op_t *op, int root)
{
    return c->c_coll.coll_reduce(s, r, n, d, op, root, c, c->c_coll.coll_reduce_module);
}
int mini_reduce_scatter_block(ompi_communicator_t *c, void *s, void *r, int n, ompi_datatype_t *d, ompi_op_t *op)
{
    return c->c_coll.coll_reduce_scatter_block(s, r, n, d, op, c, c->c_coll.coll_reduce_scatter_block_module);
}
int mini_reduce_scatter(ompi_communicator_t *c, void *s, void *r, int *rc, ompi_datatype_t *d, ompi_op_t *op)
{
    return c->c_coll.coll_reduce_scatter(s, r, rc, d, op, c, c->c_coll.coll_reduce_scatter_module);
}
int mini_allgather(ompi_communicator_t *c, void *s, int sc, ompi_datatype_t *sd, void *r, int rc, ompi_datatype_t *rd)
{
    return c->c_coll.coll_allgather(s, sc, sd, r, rc, rd, c, c->c_coll.coll_allgather_module);
}
int mini_bcast(ompi_communicator_t *c, void *b, int n, ompi_datatype_t *d, int root)
{
    return c->c_coll.coll_bcast(b, n, d, root, c, c->c_coll.coll_bcast_module);
}
int mini_gather(ompi_communicator_t *c, void *s, int sc, ompi_datatype_t *sd, void *r, int rc, ompi_datatype_t *rd,
                int root)
{
    return c->c_coll.coll_gather(s, sc, sd, r, rc, rd, root, c, c->c_coll.coll_gather_module);
}
int mini_gatherv(ompi_communicator_t *c, void *s, int sc, ompi_datatype_t *sd, void *r, int *rc, int *dp,
                 ompi_datatype_t *rd, int root)
{
    return c->c_coll.coll_gatherv(s, sc, sd, r, rc, dp, rd, root, c, c->c_coll.coll_gatherv_module);
}
int mini_scatter(ompi_communicator_t *c, void *s, int sc, ompi_datatype_t *sd, void *r, int rc, ompi_datatype_t *rd,
                 int root)
{
    return c->c_coll.coll_scatter(s, sc, sd, r, rc, rd, root, c, c->c_coll.coll_scatter_module);
}
int mini_scatterv(ompi_communicator_t *c, void *s, int *sc, int *dp, ompi_datatype_t *sd, void *r, int rc,
                  ompi_datatype_t *rd, int root)
{
    return c->c_coll.coll_scatterv(s, sc, dp, sd, r, rc, rd, root, c, c->c_coll.coll_scatterv_module);
}
int mini_allgatherv(ompi_communicator_t *c, void *s, int sc, ompi_datatype_t *sd, void *r, int *rc, int *dp,
                    ompi_datatype_t *rd)
{
    return c->c_coll.coll_allgatherv(s, sc, sd, r, rc, dp, rd, c, c->c_coll.coll_allgatherv_module);
}
int mini_alltoall(ompi_communicator_t *c, void *s, int sc, ompi_datatype_t *sd, void *r, int rc, ompi_datatype_t *rd)
{
    return c->c_coll.coll_alltoall(s, sc, sd, r, rc, rd, c, c->c_coll.coll_alltoall_module);
}
int mini_alltoallv(ompi_communicator_t *c, void *s, int *sc, int *sdp, ompi_datatype_t *sd, void *r, int *rc,
                   int *rdp, ompi_datatype_t *rd)
{
    return c->c_coll.coll_alltoallv(s, sc, sdp, sd, r, rc, rdp, rd, c, c->c_coll.coll_alltoallv_module);
}
int mini_scan(ompi_communicator_t *c, void *s, void *r, int n, ompi_datatype_t *d, ompi_op_t *op)
{
    return c->c_coll.coll_scan(s, r, n, d, op, c, c->c_coll.coll_scan_module);
}
int mini_exscan(ompi_communicator_t *c, void *s, void *r, int n, ompi_datatype_t *d, ompi_op_t *op)
{
    return c->c_coll.coll_exscan(s, r, n, d, op, c, c->c_coll.coll_exscan_module);
}

void *mini_comm_fn(ompi_communicator_t *c, int which)
{
    switch (which) {
    case 0: return (void *)c->c_coll.coll_allreduce;
    case 1: return (void *)c->c_coll.coll_reduce_scatter_block;
    case 2: return (void *)c->c_coll.coll_reduce_scatter;
    case 3: return (void *)c->c_coll.coll_allgather;
    case 4: return (void *)c->c_coll.coll_bcast;
    case 5: return (void *)c->c_coll.coll_reduce;
    case 6: return (void *)c->c_coll.coll_iallreduce;
    case 7: return (void *)c->c_coll.coll_ireduce;
    case 8: return (void *)c->c_coll.coll_ireduce_scatter_block;
    case 9: return (void *)c->c_coll.coll_iallgather;
    case 10: return (void *)c->c_coll.coll_ibcast;
    case 11: return (void *)c->c_coll.coll_gather;
    case 12: return (void *)c->c_coll.coll_gatherv;
    case 13: return (void *)c->c_coll.coll_scatter;
    case 14: return (void *)c->c_coll.coll_scatterv;
    case 15: return (void *)c->c_coll.coll_allgatherv;
    case 16: return (void *)c->c_coll.coll_alltoall;
    case 17: return (void *)c->c_coll.coll_alltoallv;
    case 18: return (void *)c->c_coll.coll_scan;
    case 19: return (void *)c->c_coll.coll_exscan;
    default: return NULL;
    }
}

/* ------------------------------------------------------------------ host channel
 * What ob1 + the sm BTL give coll/basic and coll/tuned in a real job: a way for the ranks of ONE
 * communicator to move host bytes.  The harness stands it in with one POSIX shm segment per
 * communicator, named by the test (each group of a split gets its own, as each group's PML
 * traffic is its own): a small bcast area (what coll/mi355x's module_enable uses to agree on its
 * rendezvous key), a barrier, and one data slot per rank through which the host module below
 * moves and reduces buffers of any size in slot-sized pieces. */
#define MINI_CHAN_MAX 64
#define MINI_CHAN_BYTES 4096
#define MINI_SLOT_BYTES ((size_t)128 << 10)
struct mini_chan {
    _Atomic uint64_t gen;                 /* number of the last bcast the root published */
    _Atomic uint64_t ack[MINI_CHAN_MAX];  /* per rank: last bcast it has copied out */
    _Atomic uint64_t bar[MINI_CHAN_MAX];  /* per rank: last barrier it has reached */
    uint64_t len;
    char data[MINI_CHAN_BYTES];
    /* followed by comm size x MINI_SLOT_BYTES of per-rank data slots */
};
static struct {
    ompi_communicator_t *comm;
    struct mini_chan *ch;
    uint64_t calls, bars;
    size_t map_bytes;
    char name[128];
} chans[64];

static struct mini_chan *chan_of(ompi_communicator_t *c, uint64_t **calls)
{
    for (int i = 0; i < 64; ++i)
        if (chans[i].comm == c) {
            if (calls) *calls = &chans[i].calls;
            return chans[i].ch;
        }
    return NULL;
}

static int chan_index(ompi_communicator_t *c)
{
    for (int i = 0; i < 64; ++i)
        if (chans[i].comm == c) return i;
    return -1;
}

static char *chan_slot(struct mini_chan *ch, int q)
{
    return (char *)ch + sizeof(struct mini_chan) + (size_t)q * MINI_SLOT_BYTES;
}

int mini_comm_set_channel(ompi_communicator_t *c, const char *name)
{
    int slot = -1;
    for (int i = 0; i < 64 && slot < 0; ++i)
        if (!chans[i].comm) slot = i;
    const int n = c->c_local_group->grp_proc_count;
    if (slot < 0 || n > MINI_CHAN_MAX) return OMPI_ERR_OUT_OF_RESOURCE;
    char shm[112];
    snprintf(shm, sizeof(shm), "/mini_chan_%s", name);
    const size_t bytes = sizeof(struct mini_chan) + (size_t)n * MINI_SLOT_BYTES;
    /* every rank creates-or-opens; a fresh object is zero-filled by ftruncate */
    const int fd = shm_open(shm, O_CREAT | O_RDWR, 0600);
    if (fd < 0) return OMPI_ERROR;
    if (ftruncate(fd, (off_t)bytes) != 0) {
        close(fd);
        return OMPI_ERROR;
    }
    void *m = mmap(NULL, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (m == MAP_FAILED) return OMPI_ERROR;
    chans[slot].comm = c;
    chans[slot].ch = (struct mini_chan *)m;
    chans[slot].calls = 0;
    chans[slot].bars = 0;
    chans[slot].map_bytes = bytes;
    snprintf(chans[slot].name, sizeof(chans[slot].name), "%s", shm);
    return OMPI_SUCCESS;
}

static void chan_release(ompi_communicator_t *c)
{
    for (int i = 0; i < 64; ++i)
        if (chans[i].comm == c) {
            munmap(chans[i].ch, chans[i].map_bytes);
            if (c->c_my_rank == 0) shm_unlink(chans[i].name);
            chans[i].comm = NULL;
        }
}

/* every rank of the communicator reaches barrier number k before any leaves it */
static void chan_barrier(ompi_communicator_t *c, int ci)
{
    struct mini_chan *ch = chans[ci].ch;
    const int n = c->c_local_group->grp_proc_count;
    const uint64_t k = ++chans[ci].bars;
    atomic_store_explicit(&ch->bar[c->c_my_rank], k, memory_order_release);
    for (int q = 0; q < n; ++q)
        while (atomic_load_explicit(&ch->bar[q], memory_order_acquire) < k) sched_yield();
}

/* linear bcast of <= 4 KiB of host memory: the root waits until every rank acknowledged the
 * previous call, writes, publishes the call number; the others wait for it and copy; every rank
 * (the root too) acknowledges the call */
static int chan_bcast(ompi_communicator_t *c, struct mini_chan *ch, uint64_t *calls, void *buf, size_t bytes,
                      int root)
{
    if (bytes > MINI_CHAN_BYTES) return OMPI_ERR_NOT_SUPPORTED;
    const int n = c->c_local_group->grp_proc_count, me = c->c_my_rank;
    const uint64_t k = ++*calls;
    if (me == root) {
        for (int q = 0; q < n; ++q)
            while (q != root && atomic_load_explicit(&ch->ack[q], memory_order_acquire) + 1 < k) sched_yield();
        memcpy(ch->data, buf, bytes);
        ch->len = bytes;
        atomic_store_explicit(&ch->gen, k, memory_order_release);
        atomic_store_explicit(&ch->ack[me], k, memory_order_release);  /* every rank acks every call */
        return OMPI_SUCCESS;
    }
    while (atomic_load_explicit(&ch->gen, memory_order_acquire) < k) sched_yield();
    memcpy(buf, ch->data, bytes < ch->len ? bytes : ch->len);
    atomic_store_explicit(&ch->ack[me], k, memory_order_release);
    return OMPI_SUCCESS;
}

/* ------------------------------------------------------------------ device-buffer guard
 * A host component (coll/basic, coll/tuned, libnbc) reads and writes its buffers with the CPU:
 * handed hipMalloc memory it faults.  The harness's lower-priority modules check every buffer
 * pointer they are given instead, so a test sees the fault as a failed call: the pointer is
 * reported, counted, and the call returns MINI_ERR_DEVICE_BUFFER.  The query is the engine's own
 * (resolved at run time: libmi355x_rt is loaded before any component). */
#define MINI_ERR_DEVICE_BUFFER 78
static int device_hits;
static int on_device(const void *p)
{
    static int (*is_dev)(const void *, int *);
    static int looked;
    if (!looked) {
        is_dev = (int (*)(const void *, int *))dlsym(RTLD_DEFAULT, "mi355x_ptr_is_device");
        looked = 1;
    }
    int d = 0;
    if (!p || p == MPI_IN_PLACE || !is_dev || is_dev(p, &d) != 0) return 0;
    return d;
}
static int guard(const char *fn, int n, ...)
{
    va_list ap;
    va_start(ap, n);
    int bad = 0;
    for (int i = 0; i < n; ++i) {
        const void *p = va_arg(ap, const void *);
        if (on_device(p)) {
            fprintf(stderr, "[mini] %s: device buffer %p handed to a host component\n", fn, p);
            bad = 1;
        }
    }
    va_end(ap);
    if (bad) device_hits++;
    return bad;
}
int mini_device_hits(void) { return device_hits; }

/* a stub "lower-priority" module for tests: records which function ran and returns `marker`
 * (bcast on a communicator with a host channel really broadcasts host buffers) */
static int stub_calls[16];
static int stub_marker = 77;
static int st_allreduce(void *s, void *r, int n, struct ompi_datatype_t *d, struct ompi_op_t *o,
                        struct ompi_communicator_t *c, mca_coll_base_module_t *m)
{ if (guard("st_allreduce", 2, s, r)) return MINI_ERR_DEVICE_BUFFER; (void)s; (void)r; (void)n; (void)d; (void)o; (void)c; (void)m; stub_calls[0]++; return stub_marker; }
static int st_rsb(void *s, void *r, int n, struct ompi_datatype_t *d, struct ompi_op_t *o,
                  struct ompi_communicator_t *c, mca_coll_base_module_t *m)
{ if (guard("st_rsb", 2, s, r)) return MINI_ERR_DEVICE_BUFFER; (void)s; (void)r; (void)n; (void)d; (void)o; (void)c; (void)m; stub_calls[1]++; return stub_marker; }
static int st_rs(void *s, void *r, int *n, struct ompi_datatype_t *d, struct ompi_op_t *o,
                 struct ompi_communicator_t *c, mca_coll_base_module_t *m)
{ if (guard("st_rs", 2, s, r)) return MINI_ERR_DEVICE_BUFFER; (void)s; (void)r; (void)n; (void)d; (void)o; (void)c; (void)m; stub_calls[2]++; return stub_marker; }
static int st_allgather(void *s, int sc, struct ompi_datatype_t *sd, void *r, int rc, struct ompi_datatype_t *rd,
                        struct ompi_communicator_t *c, mca_coll_base_module_t *m)
{ if (guard("st_allgather", 2, s, r)) return MINI_ERR_DEVICE_BUFFER; (void)s; (void)sc; (void)sd; (void)r; (void)rc; (void)rd; (void)c; (void)m; stub_calls[3]++; return stub_marker; }
static int st_bcast(void *b, int n, struct ompi_datatype_t *d, int root, struct ompi_communicator_t *c,
                    mca_coll_base_module_t *m)
{
    (void)m;
    if (guard("st_bcast", 1, b)) return MINI_ERR_DEVICE_BUFFER;
    stub_calls[4]++;
    uint64_t *calls = NULL;
    struct mini_chan *ch = chan_of(c, &calls);
    if (!ch || n < 0 || !(d->super.flags & OPAL_DATATYPE_FLAG_NO_GAPS)) return stub_marker;
    return chan_bcast(c, ch, calls, b, (size_t)n * d->super.size, root);
}
static int st_reduce(void *s, void *r, int n, struct ompi_datatype_t *d, struct ompi_op_t *o, int root,
                     struct ompi_communicator_t *c, mca_coll_base_module_t *m)
{ if (guard("st_reduce", 2, s, r)) return MINI_ERR_DEVICE_BUFFER; (void)s; (void)r; (void)n; (void)d; (void)o; (void)root; (void)c; (void)m; stub_calls[5]++; return stub_marker; }

static int st_iallreduce(void *s, void *r, int n, struct ompi_datatype_t *d, struct ompi_op_t *o,
                         struct ompi_communicator_t *c, ompi_request_t **req, mca_coll_base_module_t *m)
{ if (guard("st_iallreduce", 2, s, r)) return MINI_ERR_DEVICE_BUFFER; (void)s; (void)r; (void)n; (void)d; (void)o; (void)c; (void)m; *req = &ompi_request_null.request; stub_calls[6]++; return stub_marker; }

static int st_gather(void *s, int sc, struct ompi_datatype_t *sd, void *r, int rc, struct ompi_datatype_t *rd,
                     int root, struct ompi_communicator_t *c, mca_coll_base_module_t *m)
{ if (guard("st_gather", 2, s, r)) return MINI_ERR_DEVICE_BUFFER; (void)s; (void)sc; (void)sd; (void)r; (void)rc; (void)rd; (void)root; (void)c; (void)m; stub_calls[7]++; return stub_marker; }
static int st_alltoall(void *s, int sc, struct ompi_datatype_t *sd, void *r, int rc, struct ompi_datatype_t *rd,
                       struct ompi_communicator_t *c, mca_coll_base_module_t *m)
{ if (guard("st_alltoall", 2, s, r)) return MINI_ERR_DEVICE_BUFFER; (void)s; (void)sc; (void)sd; (void)r; (void)rc; (void)rd; (void)c; (void)m; stub_calls[8]++; return stub_marker; }
static int st_scan(void *s, void *r, int n, struct ompi_datatype_t *d, struct ompi_op_t *o,
                   struct ompi_communicator_t *c, mca_coll_base_module_t *m)
{ if (guard("st_scan", 2, s, r)) return MINI_ERR_DEVICE_BUFFER; (void)s; (void)r; (void)n; (void)d; (void)o; (void)c; (void)m; stub_calls[9]++; return stub_marker; }
static int st_gatherv(void *s, int sc, struct ompi_datatype_t *sd, void *r, int *rc, int *dp,
                      struct ompi_datatype_t *rd, int root, struct ompi_communicator_t *c, mca_coll_base_module_t *m)
{ if (guard("st_gatherv", 2, s, r)) return MINI_ERR_DEVICE_BUFFER; (void)s; (void)sc; (void)sd; (void)r; (void)rc; (void)dp; (void)rd; (void)root; (void)c; (void)m; stub_calls[10]++; return stub_marker; }
static int st_scatterv(void *s, int *sc, int *dp, struct ompi_datatype_t *sd, void *r, int rc,
                       struct ompi_datatype_t *rd, int root, struct ompi_communicator_t *c, mca_coll_base_module_t *m)
{ if (guard("st_scatterv", 2, s, r)) return MINI_ERR_DEVICE_BUFFER; (void)s; (void)sc; (void)dp; (void)sd; (void)r; (void)rc; (void)rd; (void)root; (void)c; (void)m; stub_calls[11]++; return stub_marker; }
static int st_allgatherv(void *s, int sc, struct ompi_datatype_t *sd, void *r, int *rc, int *dp,
                         struct ompi_datatype_t *rd, struct ompi_communicator_t *c, mca_coll_base_module_t *m)
{ if (guard("st_allgatherv", 2, s, r)) return MINI_ERR_DEVICE_BUFFER; (void)s; (void)sc; (void)sd; (void)r; (void)rc; (void)dp; (void)rd; (void)c; (void)m; stub_calls[12]++; return stub_marker; }
static int st_alltoallv(void *s, int *sc, int *sdp, struct ompi_datatype_t *sd, void *r, int *rc, int *rdp,
                        struct ompi_datatype_t *rd, struct ompi_communicator_t *c, mca_coll_base_module_t *m)
{ if (guard("st_alltoallv", 2, s, r)) return MINI_ERR_DEVICE_BUFFER; (void)s; (void)sc; (void)sdp; (void)sd; (void)r; (void)rc; (void)rdp; (void)rd; (void)c; (void)m; stub_calls[13]++; return stub_marker; }

mca_coll_base_module_t *mini_stub_module(void)
{
    mca_coll_base_module_t *m = mini_coll_module_new();
    m->coll_allreduce = st_allreduce;
    m->coll_reduce_scatter_block = st_rsb;
    m->coll_reduce_scatter = st_rs;
    m->coll_allgather = st_allgather;
    m->coll_bcast = st_bcast;
    m->coll_reduce = st_reduce;
    m->coll_iallreduce = st_iallreduce;
    m->coll_gather = st_gather;
    m->coll_scatter = st_gather;
    m->coll_alltoall = st_alltoall;
    m->coll_scan = st_scan;
    m->coll_exscan = st_scan;
    m->coll_gatherv = st_gatherv;
    m->coll_scatterv = st_scatterv;
    m->coll_allgatherv = st_allgatherv;
    m->coll_alltoallv = st_alltoallv;
    return m;
}
int mini_stub_calls(int which) { return (which >= 0 && which < 16) ? stub_calls[which] : -1; }
int mini_stub_marker(void) { return stub_marker; }

/* ------------------------------------------------------------------ host module
 * The lower-priority module the engine's declined calls land on, doing what coll/basic over ob1 +
 * sm does with host buffers: the data really moves (through the communicator's host channel, in
 * slot-sized pieces) and is reduced on the CPU by ompi_op_reduce (op.h:540-636) -- an intrinsic
 * op through its selected slot functions (op/hip's, which hand host buffers to the base loops), a
 * user op through its C function.  Orders are coll/basic's: reduce and allreduce linear,
 * rbuf = r[n-1], then r[i] op rbuf for i = n-2..0 (coll_basic_reduce.c:215-250); scan and exscan
 * the rank-order chain p[k] = p[k-1] op r[k] (coll_basic_scan.c:84-110, coll_basic_exscan.c:
 * 63-104).  Types: any with true_lb == 0 (instances extent apart, true_ub bytes each).  Nonblocking
 * forms are queued and run in order from an opal_progress callback, so their requests complete
 * only under MPI_Wait / MPI_Test, as libnbc's do.  Every buffer passes the device guard. */
static int host_calls[16];

static void host_op_reduce(ompi_op_t *op, void *in, void *inout, int count, ompi_datatype_t *dt)
{
    if (count <= 0) return;
    if (op->o_flags & OMPI_OP_FLAGS_INTRINSIC) {
        const int t = ompi_op_ddt_map[dt->id];
        op->o_func.intrinsic.fns[t](in, inout, &count, &dt, op->o_func.intrinsic.modules[t]);
    } else {
        ((void (*)(void *, void *, int *, ompi_datatype_t **))op->o_func.c_fn)(in, inout, &count, &dt);
    }
}

static size_t span_of(const ompi_datatype_t *dt, size_t k)
{
    return k ? (size_t)(dt->super.true_ub + (ptrdiff_t)(k - 1) * (dt->super.ub - dt->super.lb)) : 0;
}

/* Reduce the ranks' `total`-instance contributions (src; NULL: contributes nothing -- never
 * happens in MPI, every rank contributes) over instances [lo, lo + cnt) into dst (cnt instances;
 * NULL: this rank only contributes).  chain < 0: linear order over all ranks; chain >= 0: the
 * scan chain over ranks 0..chain. */
static int host_reduce(ompi_communicator_t *c, const char *src, size_t total, size_t lo, size_t cnt, int chain,
                       char *dst, ompi_datatype_t *dt, ompi_op_t *op)
{
    const int ci = chan_index(c);
    if (ci < 0) return stub_marker;  /* no channel: the bare stub's answer */
    if (dt->super.true_lb != 0) return OMPI_ERR_NOT_SUPPORTED;
    struct mini_chan *ch = chans[ci].ch;
    const int n = c->c_local_group->grp_proc_count, me = c->c_my_rank;
    const size_t ext = (size_t)(dt->super.ub - dt->super.lb);
    const size_t per = ext ? MINI_SLOT_BYTES / ext : 0;
    if (per == 0) return OMPI_ERR_NOT_SUPPORTED;
    /* the operands of every ompi_op_reduce are private heap buffers of the message's size, as in
     * coll/basic: the result buffer, and a receive buffer each peer's piece lands in first
     * (coll_basic_reduce.c:204-250: free_buffer = malloc(true_extent + (count - 1) x extent), the
     * PML receives into it, then ompi_op_reduce(op, inbuf, rbuf, ...)) -- never the shared segment */
    const size_t piece = span_of(dt, total < per ? total : per) + 1;
    char *acc = malloc(piece), *tmp = malloc(piece), *inb = malloc(piece);
    if (!acc || !tmp || !inb) {
        free(acc);
        free(tmp);
        free(inb);
        return OMPI_ERR_OUT_OF_RESOURCE;
    }
    for (size_t c0 = 0; c0 < total || (total == 0 && c0 == 0); c0 += per) {
        if (total == 0) break;
        const size_t k = total - c0 < per ? total - c0 : per;
        memcpy(chan_slot(ch, me), src + c0 * ext, span_of(dt, k));
        chan_barrier(c, ci);
        const size_t a = c0 > lo ? c0 : lo, b = (c0 + k < lo + cnt) ? c0 + k : lo + cnt;
        if (dst && a < b) {
            const size_t off = (a - c0) * ext, m = b - a, bytes = span_of(dt, m);
            if (chain < 0) {
                memcpy(acc, chan_slot(ch, n - 1) + off, bytes);
                for (int i = n - 2; i >= 0; --i) {
                    memcpy(inb, chan_slot(ch, i) + off, bytes);
                    host_op_reduce(op, inb, acc, (int)m, dt);
                }
            } else {
                memcpy(acc, chan_slot(ch, 0) + off, bytes);
                for (int q = 1; q <= chain; ++q) {
                    memcpy(tmp, chan_slot(ch, q) + off, bytes);
                    host_op_reduce(op, acc, tmp, (int)m, dt);
                    char *sw = acc;
                    acc = tmp;
                    tmp = sw;
                }
            }
            memcpy(dst + (a - lo) * ext, acc, bytes);
        }
        chan_barrier(c, ci);
    }
    free(acc);
    free(tmp);
    free(inb);
    return OMPI_SUCCESS;
}

/* root's `total` instances to every rank, slot-sized pieces through the root's slot */
static int host_bcast(ompi_communicator_t *c, char *buf, size_t total, ompi_datatype_t *dt, int root)
{
    const int ci = chan_index(c);
    if (ci < 0) return stub_marker;
    if (dt->super.true_lb != 0 || !(dt->super.flags & OPAL_DATATYPE_FLAG_CONTIGUOUS)) return OMPI_ERR_NOT_SUPPORTED;
    struct mini_chan *ch = chans[ci].ch;
    const size_t ext = (size_t)(dt->super.ub - dt->super.lb), per = ext ? MINI_SLOT_BYTES / ext : 0;
    if (per == 0) return OMPI_ERR_NOT_SUPPORTED;
    for (size_t c0 = 0; c0 < total; c0 += per) {
        const size_t k = total - c0 < per ? total - c0 : per;
        if (c->c_my_rank == root) memcpy(chan_slot(ch, root), buf + c0 * ext, span_of(dt, k));
        chan_barrier(c, ci);
        if (c->c_my_rank != root) memcpy(buf + c0 * ext, chan_slot(ch, root), span_of(dt, k));
        chan_barrier(c, ci);
    }
    return OMPI_SUCCESS;
}

static int h_allreduce(void *s, void *r, int n, struct ompi_datatype_t *d, struct ompi_op_t *o,
                       struct ompi_communicator_t *c, mca_coll_base_module_t *m)
{
    (void)m;
    host_calls[0]++;
    if (guard("allreduce", 2, s, r)) return MINI_ERR_DEVICE_BUFFER;
    if (n < 0) return OMPI_ERR_BAD_PARAM;
    const char *src = s == MPI_IN_PLACE ? (const char *)r : (const char *)s;
    char *copy = NULL;
    if (s == MPI_IN_PLACE) {  /* rbuf is both the contribution and the result */
        copy = malloc(span_of(d, (size_t)n) + 1);
        if (!copy) return OMPI_ERR_OUT_OF_RESOURCE;
        memcpy(copy, r, span_of(d, (size_t)n));
        src = copy;
    }
    const int rc = host_reduce(c, src, (size_t)n, 0, (size_t)n, -1, (char *)r, d, o);
    free(copy);
    return rc;
}

static int h_reduce(void *s, void *r, int n, struct ompi_datatype_t *d, struct ompi_op_t *o, int root,
                    struct ompi_communicator_t *c, mca_coll_base_module_t *m)
{
    (void)m;
    host_calls[5]++;
    const int me = c->c_my_rank;
    if (guard("reduce", 2, s, me == root ? r : NULL)) return MINI_ERR_DEVICE_BUFFER;
    if (n < 0) return OMPI_ERR_BAD_PARAM;
    const char *src = s == MPI_IN_PLACE ? (const char *)r : (const char *)s;
    char *copy = NULL;
    if (s == MPI_IN_PLACE) {
        copy = malloc(span_of(d, (size_t)n) + 1);
        if (!copy) return OMPI_ERR_OUT_OF_RESOURCE;
        memcpy(copy, r, span_of(d, (size_t)n));
        src = copy;
    }
    const int rc = host_reduce(c, src, (size_t)n, 0, (size_t)n, -1, me == root ? (char *)r : NULL, d, o);
    free(copy);
    return rc;
}

/* reduce_scatter(_block): my block of the linear reduction (coll/basic reduces to 0 and scatters) */
static int h_rs_common(void *s, void *r, const int *counts, int rcount, struct ompi_datatype_t *d, struct ompi_op_t *o,
                       struct ompi_communicator_t *c)
{
    const int n = c->c_local_group->grp_proc_count, me = c->c_my_rank;
    size_t total = 0, lo = 0;
    for (int q = 0; q < n; ++q) {
        const int k = counts ? counts[q] : rcount;
        if (k < 0) return OMPI_ERR_BAD_PARAM;
        if (q < me) lo += (size_t)k;
        total += (size_t)k;
    }
    const size_t mine = (size_t)(counts ? counts[me] : rcount);
    const char *src = s == MPI_IN_PLACE ? (const char *)r : (const char *)s;
    char *copy = NULL;
    if (s == MPI_IN_PLACE) {
        copy = malloc(span_of(d, total) + 1);
        if (!copy) return OMPI_ERR_OUT_OF_RESOURCE;
        memcpy(copy, r, span_of(d, total));
        src = copy;
    }
    const int rc = host_reduce(c, src, total, lo, mine, -1, (char *)r, d, o);
    free(copy);
    return rc;
}

static int h_rsb(void *s, void *r, int n, struct ompi_datatype_t *d, struct ompi_op_t *o,
                 struct ompi_communicator_t *c, mca_coll_base_module_t *m)
{
    (void)m;
    host_calls[1]++;
    if (guard("reduce_scatter_block", 2, s, r)) return MINI_ERR_DEVICE_BUFFER;
    return h_rs_common(s, r, NULL, n, d, o, c);
}

static int h_rs(void *s, void *r, int *counts, struct ompi_datatype_t *d, struct ompi_op_t *o,
                struct ompi_communicator_t *c, mca_coll_base_module_t *m)
{
    (void)m;
    host_calls[2]++;
    if (guard("reduce_scatter", 2, s, r)) return MINI_ERR_DEVICE_BUFFER;
    return h_rs_common(s, r, counts, 0, d, o, c);
}

static int h_scan_common(int exclusive, void *s, void *r, int n, struct ompi_datatype_t *d, struct ompi_op_t *o,
                         struct ompi_communicator_t *c)
{
    if (n < 0) return OMPI_ERR_BAD_PARAM;
    const int me = c->c_my_rank;
    const char *src = s == MPI_IN_PLACE ? (const char *)r : (const char *)s;
    char *copy = NULL;
    if (s == MPI_IN_PLACE) {
        copy = malloc(span_of(d, (size_t)n) + 1);
        if (!copy) return OMPI_ERR_OUT_OF_RESOURCE;
        memcpy(copy, r, span_of(d, (size_t)n));
        src = copy;
    }
    const int last = exclusive ? me - 1 : me;  /* exscan: rank 0's rbuf is left alone */
    const int rc = host_reduce(c, src, (size_t)n, 0, (size_t)n, last < 0 ? 0 : last, last < 0 ? NULL : (char *)r, d, o);
    free(copy);
    return rc;
}

static int h_scan(void *s, void *r, int n, struct ompi_datatype_t *d, struct ompi_op_t *o,
                  struct ompi_communicator_t *c, mca_coll_base_module_t *m)
{
    (void)m;
    host_calls[9]++;
    if (guard("scan", 2, s, r)) return MINI_ERR_DEVICE_BUFFER;
    return h_scan_common(0, s, r, n, d, o, c);
}

static int h_exscan(void *s, void *r, int n, struct ompi_datatype_t *d, struct ompi_op_t *o,
                    struct ompi_communicator_t *c, mca_coll_base_module_t *m)
{
    (void)m;
    host_calls[10]++;
    if (guard("exscan", 2, s, r)) return MINI_ERR_DEVICE_BUFFER;
    return h_scan_common(1, s, r, n, d, o, c);
}

static int h_bcast(void *b, int n, struct ompi_datatype_t *d, int root, struct ompi_communicator_t *c,
                   mca_coll_base_module_t *m)
{
    (void)m;
    host_calls[4]++;
    if (guard("bcast", 1, b)) return MINI_ERR_DEVICE_BUFFER;
    if (n < 0) return OMPI_ERR_BAD_PARAM;
    return host_bcast(c, (char *)b, (size_t)n, d, root);
}

/* allgather as n bcasts of the ranks' blocks (coll/basic: gather to 0 + bcast) */
static int h_allgather(void *s, int sc, struct ompi_datatype_t *sd, void *r, int rc, struct ompi_datatype_t *rd,
                       struct ompi_communicator_t *c, mca_coll_base_module_t *m)
{
    (void)m;
    host_calls[3]++;
    if (guard("allgather", 2, s, r)) return MINI_ERR_DEVICE_BUFFER;
    if (rc < 0) return OMPI_ERR_BAD_PARAM;
    const int n = c->c_local_group->grp_proc_count, me = c->c_my_rank;
    const size_t ext = (size_t)(rd->super.ub - rd->super.lb);
    if (s != MPI_IN_PLACE) {
        if ((size_t)sc * sd->super.size != (size_t)rc * rd->super.size || !(sd->super.flags & OPAL_DATATYPE_FLAG_NO_GAPS) ||
            !(rd->super.flags & OPAL_DATATYPE_FLAG_NO_GAPS))
            return OMPI_ERR_NOT_SUPPORTED;
        memcpy((char *)r + (size_t)me * rc * ext, s, (size_t)rc * rd->super.size);
    }
    for (int q = 0; q < n; ++q) {
        const int e = host_bcast(c, (char *)r + (size_t)q * rc * ext, (size_t)rc, rd, q);
        if (e) return e;
    }
    return OMPI_SUCCESS;
}

/* dense layouts only (the host module's gather / alltoall move bytes) */
static int h_dense(const struct ompi_datatype_t *d)
{
    return (d->super.flags & OPAL_DATATYPE_FLAG_NO_GAPS) && d->super.true_lb == 0 &&
           (size_t)(d->super.ub - d->super.lb) == d->super.size;
}

/* MPI_Gather: rank q's block broadcast by q through its slot, kept by the root (coll/basic's linear
 * gather moves the same bytes, coll_basic_gather.c:40-110) */
static int h_gather(void *s, int sc, struct ompi_datatype_t *sd, void *r, int rc, struct ompi_datatype_t *rd, int root,
                    struct ompi_communicator_t *c, mca_coll_base_module_t *m)
{
    (void)m;
    const int n = c->c_local_group->grp_proc_count, me = c->c_my_rank;
    if (chan_index(c) < 0) return stub_marker;
    if (guard("gather", 2, s == MPI_IN_PLACE ? NULL : s, me == root ? r : NULL)) return MINI_ERR_DEVICE_BUFFER;
    if ((s != MPI_IN_PLACE && !h_dense(sd)) || (me == root && !h_dense(rd))) return OMPI_ERR_NOT_SUPPORTED;
    const size_t blk = me == root ? (size_t)rc * rd->super.size : (size_t)sc * sd->super.size;
    ompi_datatype_t *bytes = (ompi_datatype_t *)&ompi_mpi_byte;
    char *tmp = malloc(blk + 1);
    if (!tmp) return OMPI_ERR_OUT_OF_RESOURCE;
    if (me == root && s != MPI_IN_PLACE) memcpy((char *)r + (size_t)root * blk, s, blk);
    int e = OMPI_SUCCESS;
    for (int q = 0; q < n && e == OMPI_SUCCESS; ++q) {
        if (q == root) continue;
        char *b = me == q ? (char *)s : me == root ? (char *)r + (size_t)q * blk : tmp;
        e = host_bcast(c, b, blk, bytes, q);
    }
    free(tmp);
    return e;
}

/* MPI_Alltoall: each rank's n blocks broadcast by it; every rank keeps its own block */
static int h_alltoall(void *s, int sc, struct ompi_datatype_t *sd, void *r, int rc, struct ompi_datatype_t *rd,
                      struct ompi_communicator_t *c, mca_coll_base_module_t *m)
{
    (void)m;
    (void)sc;
    (void)sd;
    const int n = c->c_local_group->grp_proc_count, me = c->c_my_rank;
    if (chan_index(c) < 0) return stub_marker;
    if (guard("alltoall", 2, s == MPI_IN_PLACE ? NULL : s, r)) return MINI_ERR_DEVICE_BUFFER;
    if ((s != MPI_IN_PLACE && !h_dense(sd)) || !h_dense(rd)) return OMPI_ERR_NOT_SUPPORTED;
    const size_t blk = (size_t)rc * rd->super.size, all = blk * (size_t)n;
    ompi_datatype_t *bytes = (ompi_datatype_t *)&ompi_mpi_byte;
    char *mine = malloc(all + 1), *tmp = malloc(all + 1);
    if (!mine || !tmp) {
        free(mine);
        free(tmp);
        return OMPI_ERR_OUT_OF_RESOURCE;
    }
    memcpy(mine, s == MPI_IN_PLACE ? r : s, all);
    int e = OMPI_SUCCESS;
    for (int q = 0; q < n && e == OMPI_SUCCESS; ++q) {
        if (me == q) memcpy(tmp, mine, all);
        e = host_bcast(c, tmp, all, bytes, q);
        if (e == OMPI_SUCCESS) memcpy((char *)r + (size_t)q * blk, tmp + (size_t)me * blk, blk);
    }
    free(mine);
    free(tmp);
    return e;
}

/* ---- nonblocking: queued, run in posting order from the progress callback */
typedef struct mini_hreq {
    ompi_request_t super;
    int kind;  /* 0 allreduce, 1 reduce, 2 rsb, 3 allgather, 4 bcast */
    void *s, *r;
    int n, n2, root;
    struct ompi_datatype_t *d, *d2;
    struct ompi_op_t *o;
    struct ompi_communicator_t *c;
    struct mini_hreq *next;
} mini_hreq_t;
static mini_hreq_t *hq_head, *hq_tail;
static int hq_running, hq_registered;

static int hreq_free(ompi_request_t **rp)
{
    mini_hreq_t *q = (mini_hreq_t *)*rp;
    if (!q->super.req_complete) return MPI_ERR_REQUEST;
    mi355x_obj_release(&q->super.super.super.super);
    *rp = &ompi_request_null.request;
    return OMPI_SUCCESS;
}
static opal_class_t mini_hreq_t_class = {"mini_hreq_t", &ompi_request_t_class, NULL, NULL, 0, 0, NULL, NULL,
                                         sizeof(mini_hreq_t)};

static int hq_progress(void)
{
    if (hq_running || !hq_head) return 0;
    hq_running = 1;
    int done = 0;
    while (hq_head) {
        mini_hreq_t *q = hq_head;
        hq_head = q->next;
        if (!hq_head) hq_tail = NULL;
        int rc;
        switch (q->kind) {
        case 0: rc = h_allreduce(q->s, q->r, q->n, q->d, q->o, q->c, NULL); break;
        case 1: rc = h_reduce(q->s, q->r, q->n, q->d, q->o, q->root, q->c, NULL); break;
        case 2: rc = h_rsb(q->s, q->r, q->n, q->d, q->o, q->c, NULL); break;
        case 3: rc = h_allgather(q->s, q->n, q->d, q->r, q->n2, q->d2, q->c, NULL); break;
        default: rc = h_bcast(q->r, q->n, q->d, q->root, q->c, NULL); break;
        }
        q->super.req_status.MPI_ERROR = rc;
        q->super.req_complete = true;
        q->super.req_state = OMPI_REQUEST_INACTIVE;
        done++;
    }
    hq_running = 0;
    return done;
}

static int hq_post(mini_hreq_t proto, ompi_request_t **req)
{
    mini_hreq_t *q = (mini_hreq_t *)mi355x_obj_new(&mini_hreq_t_class);
    if (!q) return OMPI_ERR_OUT_OF_RESOURCE;
    const ompi_request_t base = q->super;
    *q = proto;
    q->super = base;
    q->super.req_type = OMPI_REQUEST_COLL;
    q->super.req_free = hreq_free;
    q->super.req_complete = false;
    q->super.req_state = OMPI_REQUEST_ACTIVE;
    q->super.req_status.MPI_ERROR = 0;
    q->next = NULL;
    if (hq_tail) hq_tail->next = q;
    else hq_head = q;
    hq_tail = q;
    if (!hq_registered) {
        opal_progress_register(hq_progress);
        hq_registered = 1;
    }
    *req = &q->super;
    return OMPI_SUCCESS;
}

static int h_iallreduce(void *s, void *r, int n, struct ompi_datatype_t *d, struct ompi_op_t *o,
                        struct ompi_communicator_t *c, ompi_request_t **req, mca_coll_base_module_t *m)
{
    (void)m;
    host_calls[6]++;
    if (guard("iallreduce", 2, s, r)) return MINI_ERR_DEVICE_BUFFER;
    return hq_post((mini_hreq_t){.kind = 0, .s = s, .r = r, .n = n, .d = d, .o = o, .c = c}, req);
}
static int h_ireduce(void *s, void *r, int n, struct ompi_datatype_t *d, struct ompi_op_t *o, int root,
                     struct ompi_communicator_t *c, ompi_request_t **req, mca_coll_base_module_t *m)
{
    (void)m;
    host_calls[11]++;
    if (guard("ireduce", 2, s, c->c_my_rank == root ? r : NULL)) return MINI_ERR_DEVICE_BUFFER;
    return hq_post((mini_hreq_t){.kind = 1, .s = s, .r = r, .n = n, .root = root, .d = d, .o = o, .c = c}, req);
}
static int h_irsb(void *s, void *r, int n, struct ompi_datatype_t *d, struct ompi_op_t *o,
                  struct ompi_communicator_t *c, ompi_request_t **req, mca_coll_base_module_t *m)
{
    (void)m;
    host_calls[12]++;
    if (guard("ireduce_scatter_block", 2, s, r)) return MINI_ERR_DEVICE_BUFFER;
    return hq_post((mini_hreq_t){.kind = 2, .s = s, .r = r, .n = n, .d = d, .o = o, .c = c}, req);
}
static int h_iallgather(void *s, int sc, struct ompi_datatype_t *sd, void *r, int rc, struct ompi_datatype_t *rd,
                        struct ompi_communicator_t *c, ompi_request_t **req, mca_coll_base_module_t *m)
{
    (void)m;
    host_calls[13]++;
    if (guard("iallgather", 2, s, r)) return MINI_ERR_DEVICE_BUFFER;
    return hq_post((mini_hreq_t){.kind = 3, .s = s, .r = r, .n = sc, .n2 = rc, .d = sd, .d2 = rd, .c = c}, req);
}
static int h_ibcast(void *b, int n, struct ompi_datatype_t *d, int root, struct ompi_communicator_t *c,
                    ompi_request_t **req, mca_coll_base_module_t *m)
{
    (void)m;
    host_calls[14]++;
    if (guard("ibcast", 1, b)) return MINI_ERR_DEVICE_BUFFER;
    return hq_post((mini_hreq_t){.kind = 4, .r = b, .n = n, .root = root, .d = d, .c = c}, req);
}

/* the host module: real host collectives for the reduction slots and bcast / allgather (the stub's
 * counting functions for the rest) */
mca_coll_base_module_t *mini_host_module(void)
{
    mca_coll_base_module_t *m = mini_stub_module();
    m->coll_allreduce = h_allreduce;
    m->coll_reduce = h_reduce;
    m->coll_reduce_scatter_block = h_rsb;
    m->coll_reduce_scatter = h_rs;
    m->coll_scan = h_scan;
    m->coll_exscan = h_exscan;
    m->coll_bcast = h_bcast;
    m->coll_allgather = h_allgather;
    m->coll_gather = h_gather;
    m->coll_alltoall = h_alltoall;
    m->coll_iallreduce = h_iallreduce;
    m->coll_ireduce = h_ireduce;
    m->coll_ireduce_scatter_block = h_irsb;
    m->coll_iallgather = h_iallgather;
    m->coll_ibcast = h_ibcast;
    return m;
}
int mini_host_calls(int which) { return (which >= 0 && which < 16) ? host_calls[which] : -1; }

/* MPI_Op_create (ompi_op_create_user, op.c:351-400): not intrinsic, commutative or not, the C
 * function in o_func.c_fn; its f2c index lies past the predefined ops */
ompi_op_t *mini_op_create_user(void *fn, int commute)
{
    mini_init();
    ompi_op_t *op = (ompi_op_t *)mi355x_obj_new(&ompi_op_t_class);
    memset((char *)op + sizeof(opal_object_t), 0, sizeof(*op) - sizeof(opal_object_t));
    snprintf(op->o_name, sizeof(op->o_name), "user op");
    op->op_type = MI355X_OP_MAX_;
    op->o_f_to_c_index = 100;
    op->o_flags = commute ? OMPI_OP_FLAGS_COMMUTE : 0;
    op->o_func.c_fn = fn;
    return op;
}

/* layout facts for tests/test_boundary.py */
size_t mini_offsetof(int which)
{
    switch (which) {
    case 0: return offsetof(ompi_op_t, o_f_to_c_index);
    case 1: return offsetof(ompi_op_t, o_func);
    case 2: return offsetof(ompi_op_t, o_3buff_intrinsic);
    case 3: return offsetof(ompi_op_base_module_t, opm_fns);
    case 4: return offsetof(ompi_op_base_module_t, opm_3buff_fns);
    case 5: return offsetof(ompi_datatype_t, id);
    case 6: return offsetof(opal_datatype_t, size);
    case 7: return offsetof(ompi_communicator_t, c_my_rank);
    case 8: return offsetof(ompi_communicator_t, c_local_group);
    case 9: return offsetof(ompi_communicator_t, c_coll);
    case 10: return offsetof(mca_coll_base_module_t, coll_allreduce);
    case 11: return offsetof(mca_coll_base_module_t, ft_event);
    case 12: return sizeof(mca_base_component_t);
    case 13: return sizeof(opal_datatype_t);
    case 14: return sizeof(ompi_datatype_t);
    case 15: return offsetof(ompi_communicator_t, c_contextid);
    case 16: return sizeof(mca_coll_base_comm_coll_t);
    case 17: return offsetof(mca_coll_base_module_t, coll_iallreduce);
    case 18: return sizeof(ompi_request_t);
    case 19: return offsetof(ompi_request_t, req_status);
    case 20: return offsetof(ompi_request_t, req_free);
    case 21: return offsetof(mca_coll_base_comm_coll_t, coll_iallreduce);
    case 22: return sizeof(ompi_predefined_request_t);
    case 23: return offsetof(mca_coll_base_module_t, coll_scan);
    case 24: return offsetof(mca_coll_base_comm_coll_t, coll_scatterv);
    case 25: return offsetof(mca_coll_base_comm_coll_t, coll_gather);
    case 26: return offsetof(mca_pml_base_module_t, pml_irecv);
    case 27: return offsetof(mca_pml_base_module_t, pml_isend);
    case 28: return offsetof(mca_pml_base_module_t, pml_probe);
    case 29: return offsetof(mca_pml_base_module_t, pml_max_tag);
    case 30: return sizeof(mca_pml_base_module_t);
    case 31: return sizeof(ompi_status_public_t);
    default: return (size_t)-1;
    }
}

/* ------------------------------------------------------------------ MCA variable system
 * mca_base_component_var_register (opal/mca/base/mca_base_var.c): full name
 * <framework>_<component>_<name>, value from OMPI_MCA_<full name> in the environment (the
 * highest-priority source the harness has), else the storage's current value as the default. */
#define MINI_MAX_VARS 64
static struct {
    char name[160], desc[160], type_name[32], comp_name[64], var_name[64];
    int type, lvl;
    void *storage;
} mini_vars[MINI_MAX_VARS];
static int mini_nvars;

int mca_base_component_var_register(const mca_base_component_t *component, const char *variable_name,
                                    const char *description, mca_base_var_type_t type,
                                    mca_base_var_enum_t *enumerator, int bind, mca_base_var_flag_t flags,
                                    mca_base_var_info_lvl_t info_lvl, mca_base_var_scope_t scope, void *storage)
{
    (void)enumerator; (void)bind; (void)flags; (void)scope;
    if (!component || !variable_name || !storage) return -1;
    if (type != MCA_BASE_VAR_TYPE_INT && type != MCA_BASE_VAR_TYPE_BOOL && type != MCA_BASE_VAR_TYPE_STRING &&
        type != MCA_BASE_VAR_TYPE_UNSIGNED_LONG_LONG)
        return -1;
    char full[160], env[200];
    snprintf(full, sizeof(full), "%s_%s_%s", component->mca_type_name, component->mca_component_name, variable_name);
    int idx = -1;
    for (int i = 0; i < mini_nvars; ++i)
        if (!strcmp(mini_vars[i].name, full)) idx = i;
    if (idx < 0) {
        if (mini_nvars == MINI_MAX_VARS) return -1;
        idx = mini_nvars++;
    }
    snprintf(mini_vars[idx].name, sizeof(mini_vars[idx].name), "%s", full);
    snprintf(mini_vars[idx].desc, sizeof(mini_vars[idx].desc), "%s", description ? description : "");
    mini_vars[idx].type = type;
    mini_vars[idx].lvl = info_lvl;
    mini_vars[idx].storage = storage;
    snprintf(mini_vars[idx].type_name, sizeof(mini_vars[idx].type_name), "%s", component->mca_type_name);
    snprintf(mini_vars[idx].comp_name, sizeof(mini_vars[idx].comp_name), "%s", component->mca_component_name);
    snprintf(mini_vars[idx].var_name, sizeof(mini_vars[idx].var_name), "%s", variable_name);
    snprintf(env, sizeof(env), "OMPI_MCA_%s", full);
    const char *v = getenv(env);
    if (v) {
        if (type == MCA_BASE_VAR_TYPE_INT) *(int *)storage = atoi(v);
        else if (type == MCA_BASE_VAR_TYPE_BOOL) *(bool *)storage = atoi(v) != 0;
        else if (type == MCA_BASE_VAR_TYPE_UNSIGNED_LONG_LONG) *(unsigned long long *)storage = strtoull(v, NULL, 10);
        else *(char **)storage = strdup(v);
    }
    return idx;
}
/* mca_base_var_find / mca_base_var_get_value (mca_base_var.c:816-820, :421-455): the index of a
 * registered variable, and a pointer to its storage */
int mca_base_var_find(const char *project_name, const char *type_name, const char *component_name,
                      const char *param_name)
{
    (void)project_name;
    for (int i = 0; i < mini_nvars; ++i)
        if (!strcmp(mini_vars[i].type_name, type_name) && !strcmp(mini_vars[i].comp_name, component_name) &&
            !strcmp(mini_vars[i].var_name, param_name))
            return i;
    return OMPI_ERR_NOT_FOUND;
}
int mca_base_var_get_value(int vari, const void *value, mca_base_var_source_t *source, const char **source_file)
{
    if (vari < 0 || vari >= mini_nvars) return OMPI_ERR_BAD_PARAM;
    if (value) *(void **)value = mini_vars[vari].storage;
    if (source) *source = MCA_BASE_VAR_SOURCE_FILE;
    if (source_file) *source_file = "mini-mca-params.conf";
    return OMPI_SUCCESS;
}
/* coll/tuned as the variable system knows it after tuned_register (coll_tuned_component.c:151-167
 * and the forced-algorithm registrations, coll_tuned_allreduce.c:949-1005): values as if they came
 * from openmpi-mca-params.conf -- nothing in the environment */
static mca_base_component_t mini_tuned_version = {2, 0, 0, "coll", 2, 0, 0, "tuned", 1, 8, 5, NULL, NULL, NULL, NULL, {0}};
static bool tuned_use_dynamic_rules;
static int tuned_allreduce_alg, tuned_reduce_alg, tuned_chain_fanout, tuned_rs_alg;
static char *tuned_rules_file;
int mini_tuned_register(int use_dynamic_rules, int allreduce_alg, int reduce_alg, int chain_fanout, int rs_alg,
                        const char *rules_file)
{
    tuned_use_dynamic_rules = use_dynamic_rules != 0;
    tuned_allreduce_alg = allreduce_alg;
    tuned_reduce_alg = reduce_alg;
    tuned_chain_fanout = chain_fanout;
    tuned_rs_alg = rs_alg;
    free(tuned_rules_file);
    tuned_rules_file = rules_file ? strdup(rules_file) : NULL;
    const mca_base_component_t *c = &mini_tuned_version;
    int rc = 0;
    rc |= mca_base_component_var_register(c, "use_dynamic_rules", "", MCA_BASE_VAR_TYPE_BOOL, NULL, 0, 0,
                                          OPAL_INFO_LVL_6, MCA_BASE_VAR_SCOPE_READONLY, &tuned_use_dynamic_rules) < 0;
    rc |= mca_base_component_var_register(c, "dynamic_rules_filename", "", MCA_BASE_VAR_TYPE_STRING, NULL, 0, 0,
                                          OPAL_INFO_LVL_6, MCA_BASE_VAR_SCOPE_READONLY, &tuned_rules_file) < 0;
    rc |= mca_base_component_var_register(c, "allreduce_algorithm", "", MCA_BASE_VAR_TYPE_INT, NULL, 0, 0,
                                          OPAL_INFO_LVL_5, MCA_BASE_VAR_SCOPE_READONLY, &tuned_allreduce_alg) < 0;
    rc |= mca_base_component_var_register(c, "reduce_algorithm", "", MCA_BASE_VAR_TYPE_INT, NULL, 0, 0,
                                          OPAL_INFO_LVL_5, MCA_BASE_VAR_SCOPE_READONLY, &tuned_reduce_alg) < 0;
    rc |= mca_base_component_var_register(c, "reduce_algorithm_chain_fanout", "", MCA_BASE_VAR_TYPE_INT, NULL, 0, 0,
                                          OPAL_INFO_LVL_5, MCA_BASE_VAR_SCOPE_READONLY, &tuned_chain_fanout) < 0;
    rc |= mca_base_component_var_register(c, "reduce_scatter_algorithm", "", MCA_BASE_VAR_TYPE_INT, NULL, 0, 0,
                                          OPAL_INFO_LVL_5, MCA_BASE_VAR_SCOPE_READONLY, &tuned_rs_alg) < 0;
    return rc ? -1 : 0;
}
int mini_var_count(void) { return mini_nvars; }
const char *mini_var_name(int i) { return (i >= 0 && i < mini_nvars) ? mini_vars[i].name : NULL; }
int mini_var_int(int i)
{
    if (i < 0 || i >= mini_nvars) return -1;
    if (mini_vars[i].type == MCA_BASE_VAR_TYPE_BOOL) return *(bool *)mini_vars[i].storage;
    if (mini_vars[i].type == MCA_BASE_VAR_TYPE_STRING) return *(char **)mini_vars[i].storage != NULL;
    if (mini_vars[i].type == MCA_BASE_VAR_TYPE_UNSIGNED_LONG_LONG) return (int)*(unsigned long long *)mini_vars[i].storage;
    return *(int *)mini_vars[i].storage;
}
int mini_component_register(const mca_base_component_t *c)
{
    return c->mca_register_component_params ? c->mca_register_component_params() : OMPI_SUCCESS;
}
