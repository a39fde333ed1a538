/*
 * ompi_abi.h -- the subset of the Open MPI 1.8.5 binary interface that the op/hip and
 * coll/mi355x MCA components touch, restated from the reference headers (layouts, not code).
 *
 * Configure profile this is pinned to (the one the SURVEY's reference build uses):
 *   x86-64 Linux, LP64, OPAL_ENABLE_DEBUG = 0, POSIX threads, OPAL_MAX_OBJECT_NAME = 64,
 *   OMPI_WANT_PERUSE defined (the field is present whenever the macro is defined,
 *   communicator.h:147-152), Fortran bindings disabled.
 * Every struct cites its reference definition; tests/test_boundary.py checks the offsets the
 * components depend on against the values derived from those definitions.  Components include
 * this header instead of the reference tree's headers when built out of tree;
 * the symbols they need at run time (opal_class_initialize, the module classes,
 * ompi_op_ddt_map) come from libmpi / libopen-pal, or from libompi_mini in the test harness.
 */
#ifndef MI355X_OMPI_ABI_H
#define MI355X_OMPI_ABI_H

#include <pthread.h>
#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------ constants */
#define OMPI_SUCCESS 0                 /* opal/include/opal/constants.h:29 */
#define OMPI_ERROR (-1)                /* :31 */
#define OMPI_ERR_OUT_OF_RESOURCE (-2)  /* :32 */
#define OMPI_ERR_BAD_PARAM (-5)        /* :35 */
#define OMPI_ERR_NOT_SUPPORTED (-8)    /* :38 */
#define OMPI_ERR_NOT_FOUND (-13)       /* :43 */
#define MPI_MAX_OBJECT_NAME 64         /* ompi/include/mpi.h.in:421 (= OPAL_MAX_OBJECT_NAME) */
#define MPI_IN_PLACE ((void *)1)       /* mpi.h.in:435 */
#define OMPI_COMM_INTER 0x00000001     /* ompi/communicator/communicator.h:45 */
#define OMPI_OP_FLAGS_INTRINSIC 0x0001 /* ompi/op/op.h:91 */
#define OMPI_OP_FLAGS_COMMUTE 0x0040   /* ompi/op/op.h:109 */
#define OMPI_OP_BASE_TYPE_MAX 39       /* ompi/mca/op/op.h:182 */
#define OMPI_DATATYPE_MPI_MAX_PREDEFINED 0x30 /* ompi/datatype/ompi_datatype_internal.h:79 */

/* ------------------------------------------------------------------ opal objects */
/* opal/class/opal_object.h:140-197 (non-debug) */
typedef struct opal_object_t opal_object_t;
typedef struct opal_class_t opal_class_t;
typedef void (*opal_construct_t)(opal_object_t *);
typedef void (*opal_destruct_t)(opal_object_t *);

struct opal_class_t {
    const char *cls_name;
    opal_class_t *cls_parent;
    opal_construct_t cls_construct;
    opal_destruct_t cls_destruct;
    int cls_initialized;
    int cls_depth;
    opal_construct_t *cls_construct_array;
    opal_destruct_t *cls_destruct_array;
    size_t cls_sizeof;
};

struct opal_object_t {
    opal_class_t *obj_class;
    volatile int32_t obj_reference_count;
};

/* provided by libopen-pal (opal/class/opal_object.c) or by the harness */
void opal_class_initialize(opal_class_t *cls);

/* OBJ_NEW / OBJ_RETAIN / OBJ_RELEASE semantics of opal_object.h:250-330, 440-503 */
static inline opal_object_t *mi355x_obj_new(opal_class_t *cls)
{
    opal_object_t *o = (opal_object_t *)malloc(cls->cls_sizeof);
    if (0 == cls->cls_initialized) opal_class_initialize(cls);
    if (o) {
        o->obj_class = cls;
        o->obj_reference_count = 1;
        for (opal_construct_t *c = cls->cls_construct_array; c && *c; ++c) (*c)(o);
    }
    return o;
}
static inline void mi355x_obj_retain(opal_object_t *o)
{
    __atomic_add_fetch(&o->obj_reference_count, 1, __ATOMIC_ACQ_REL);
}
static inline int mi355x_obj_release(opal_object_t *o)  /* returns 1 if freed */
{
    if (0 == __atomic_sub_fetch(&o->obj_reference_count, 1, __ATOMIC_ACQ_REL)) {
        for (opal_destruct_t *d = o->obj_class->cls_destruct_array; d && *d; ++d) (*d)(o);
        free(o);
        return 1;
    }
    return 0;
}

/* ------------------------------------------------------------------ MCA component base */
/* opal/mca/mca.h:230-296 */
typedef int (*mca_base_open_component_fn_t)(void);
typedef int (*mca_base_close_component_fn_t)(void);
typedef int (*mca_base_query_component_fn_t)(void **module, int *priority);
typedef int (*mca_base_register_component_params_fn_t)(void);

typedef struct mca_base_component_2_0_0_t {
    int mca_major_version;
    int mca_minor_version;
    int mca_release_version;
    char mca_type_name[32];
    int mca_type_major_version;
    int mca_type_minor_version;
    int mca_type_release_version;
    char mca_component_name[64];
    int mca_component_major_version;
    int mca_component_minor_version;
    int mca_component_release_version;
    mca_base_open_component_fn_t mca_open_component;
    mca_base_close_component_fn_t mca_close_component;
    mca_base_query_component_fn_t mca_query_component;
    mca_base_register_component_params_fn_t mca_register_component_params;
    char reserved[32];
} mca_base_component_t;

typedef struct mca_base_component_data_2_0_0_t {
    uint32_t param_field;
    char reserved[32];
} mca_base_component_data_t;

#define MCA_BASE_VERSION_2_0_0 2, 0, 0   /* opal/mca/mca.h:312 */

/* ------------------------------------------------------------------ MCA variables */
/* opal/mca/base/mca_base_var.h:74-160, :401-406.  Declared weak: a component built into an Open
 * MPI tree binds libopen-pal's definition (parameters then appear in ompi_info and are read from
 * openmpi-mca-params.conf / the command line / the environment); loaded anywhere without it the
 * address is NULL and the component reads OMPI_MCA_<framework>_<component>_<name> itself. */
typedef enum {
    MCA_BASE_VAR_TYPE_INT,
    MCA_BASE_VAR_TYPE_UNSIGNED_INT,
    MCA_BASE_VAR_TYPE_UNSIGNED_LONG,
    MCA_BASE_VAR_TYPE_UNSIGNED_LONG_LONG,
    MCA_BASE_VAR_TYPE_SIZE_T,
    MCA_BASE_VAR_TYPE_STRING,
    MCA_BASE_VAR_TYPE_BOOL,
    MCA_BASE_VAR_TYPE_DOUBLE,
    MCA_BASE_VAR_TYPE_MAX
} mca_base_var_type_t;
typedef enum {
    MCA_BASE_VAR_SCOPE_CONSTANT,
    MCA_BASE_VAR_SCOPE_READONLY,
    MCA_BASE_VAR_SCOPE_LOCAL,
    MCA_BASE_VAR_SCOPE_GROUP,
    MCA_BASE_VAR_SCOPE_GROUP_EQ,
    MCA_BASE_VAR_SCOPE_ALL,
    MCA_BASE_VAR_SCOPE_ALL_EQ,
    MCA_BASE_VAR_SCOPE_MAX
} mca_base_var_scope_t;
typedef enum {
    OPAL_INFO_LVL_1, OPAL_INFO_LVL_2, OPAL_INFO_LVL_3, OPAL_INFO_LVL_4, OPAL_INFO_LVL_5,
    OPAL_INFO_LVL_6, OPAL_INFO_LVL_7, OPAL_INFO_LVL_8, OPAL_INFO_LVL_9, OPAL_INFO_LVL_MAX
} mca_base_var_info_lvl_t;
typedef int mca_base_var_flag_t;                       /* enum of flag bits, :165-180 */
typedef struct mca_base_var_enum_t mca_base_var_enum_t;  /* opaque here */
extern int mca_base_component_var_register(const mca_base_component_t *component, const char *variable_name,
                                           const char *description, mca_base_var_type_t type,
                                           mca_base_var_enum_t *enumerator, int bind, mca_base_var_flag_t flags,
                                           mca_base_var_info_lvl_t info_lvl, mca_base_var_scope_t scope,
                                           void *storage) __attribute__((weak));
/* reading another component's variable (mca_base_var.h:96-115, :559-562; mca_base_var.c:421-455):
 * find its index by (project, framework, component, name), then get a pointer to its storage
 * (int *, bool * or char ** by the variable's type).  Weak like the registration above. */
typedef enum {
    MCA_BASE_VAR_SOURCE_DEFAULT,
    MCA_BASE_VAR_SOURCE_COMMAND_LINE,
    MCA_BASE_VAR_SOURCE_ENV,
    MCA_BASE_VAR_SOURCE_FILE,
    MCA_BASE_VAR_SOURCE_SET,
    MCA_BASE_VAR_SOURCE_OVERRIDE,
    MCA_BASE_VAR_SOURCE_MAX
} mca_base_var_source_t;
extern int mca_base_var_find(const char *project_name, const char *type_name, const char *component_name,
                             const char *param_name) __attribute__((weak));
extern int mca_base_var_get_value(int vari, const void *value, mca_base_var_source_t *source,
                                  const char **source_file) __attribute__((weak));

/* ------------------------------------------------------------------ datatypes */
/* opal/datatype/opal_datatype.h:103-131, opal_datatype_internal.h:148-188 */
typedef struct dt_elem_desc dt_elem_desc_t;
typedef struct dt_type_desc {
    uint32_t length;
    uint32_t used;
    dt_elem_desc_t *desc;
} dt_type_desc_t;

typedef struct opal_datatype_t {
    opal_object_t super;
    uint16_t flags;
    uint16_t id;
    uint32_t bdt_used;
    size_t size;
    ptrdiff_t true_lb;
    ptrdiff_t true_ub;
    ptrdiff_t lb;
    ptrdiff_t ub;
    size_t nbElems;
    uint32_t align;
    char name[64];
    dt_type_desc_t desc;
    dt_type_desc_t opt_desc;
    uint32_t btypes[47];      /* OPAL_DATATYPE_MAX_SUPPORTED */
} opal_datatype_t;

#define OPAL_DATATYPE_FLAG_PREDEFINED 0x0002  /* opal/datatype/opal_datatype.h:66 */
#define OPAL_DATATYPE_FLAG_CONTIGUOUS 0x0010  /* :69 */
#define OPAL_DATATYPE_FLAG_NO_GAPS 0x0020     /* :70, contiguous and extent == size */
#define OPAL_DATATYPE_FLAG_COMMITTED 0x0004   /* :67 */
#define OPAL_DATATYPE_FLAG_DATA 0x0100        /* :73 */
/* predefined as an MPI type, not necessarily as an OPAL type: libmpi clears the OPAL flag and sets
 * this one on the MPI-2 pair types (ompi/datatype/ompi_datatype.h:51-52, ompi_datatype_module.c:
 * 415-416, 431-432); ompi_datatype_is_predefined tests it (ompi_datatype.h:149-152) */
#define OMPI_DATATYPE_FLAG_PREDEFINED 0x0200
#define OMPI_DATATYPE_FLAG_DATA_INT 0x1000    /* ompi_datatype.h:54 */
#define OMPI_DATATYPE_FLAG_DATA_FLOAT 0x2000  /* :55 */
#define OMPI_DATATYPE_FLAG_DATA_C 0x4000      /* :59 */

/* ompi/datatype/ompi_datatype.h:73-88 */
typedef struct ompi_datatype_t {
    opal_datatype_t super;
    int32_t id;
    int32_t d_f_to_c_index;
    void *d_keyhash;
    void *args;
    void *packed_description;
    char name[MPI_MAX_OBJECT_NAME];
} ompi_datatype_t;

/* ompi/op/op.c:98: datatype id -> OMPI_OP_BASE_TYPE_* slot (-1: not reducible) */
extern int ompi_op_ddt_map[OMPI_DATATYPE_MPI_MAX_PREDEFINED];

/* predefined datatype objects are padded to 512 bytes (ompi/datatype/ompi_datatype.h:103-110);
 * MPI_BYTE is &ompi_mpi_byte (mpi.h.in:913, OMPI_PREDEFINED_GLOBAL), id OMPI_DATATYPE_MPI_BYTE
 * = OMPI_DATATYPE_MPI_UINT8_T when char is 1 byte (ompi_datatype_internal.h:122) */
#define PREDEFINED_DATATYPE_PAD 512
typedef struct ompi_predefined_datatype_t {
    ompi_datatype_t dt;
    char padding[PREDEFINED_DATATYPE_PAD - sizeof(ompi_datatype_t)];
} ompi_predefined_datatype_t;
extern ompi_predefined_datatype_t ompi_mpi_byte;
#define MPI_BYTE (&ompi_mpi_byte.dt)
#define OMPI_DATATYPE_MPI_BYTE 0x02

/* ------------------------------------------------------------------ op framework */
struct ompi_op_base_module_1_0_0_t;
struct ompi_op_t;

/* ompi/mca/op/op.h:253-266 */
typedef void (*ompi_op_base_handler_fn_t)(void *, void *, int *, struct ompi_datatype_t **,
                                          struct ompi_op_base_module_1_0_0_t *);
typedef void (*ompi_op_base_3buff_handler_fn_t)(void *, void *, void *, int *,
                                                struct ompi_datatype_t **,
                                                struct ompi_op_base_module_1_0_0_t *);
typedef int (*ompi_op_base_component_init_query_fn_t)(bool enable_progress_threads,
                                                      bool enable_mpi_threads);
typedef struct ompi_op_base_module_1_0_0_t *(*ompi_op_base_component_op_query_fn_t)(
    struct ompi_op_t *op, int *priority);
typedef int (*ompi_op_base_module_enable_fn_t)(struct ompi_op_base_module_1_0_0_t *module,
                                               struct ompi_op_t *op);

/* op.h:326-336 */
typedef struct ompi_op_base_component_1_0_0_t {
    mca_base_component_t opc_version;
    mca_base_component_data_t opc_data;
    ompi_op_base_component_init_query_fn_t opc_init_query;
    ompi_op_base_component_op_query_fn_t opc_op_query;
} ompi_op_base_component_t;

/* op.h:357-373 */
typedef struct ompi_op_base_module_1_0_0_t {
    opal_object_t super;
    ompi_op_base_module_enable_fn_t opm_enable;
    struct ompi_op_t *opm_op;
    ompi_op_base_handler_fn_t opm_fns[OMPI_OP_BASE_TYPE_MAX];
    ompi_op_base_3buff_handler_fn_t opm_3buff_fns[OMPI_OP_BASE_TYPE_MAX];
} ompi_op_base_module_t;

/* class object of ompi_op_base_module_t (op_base_frame.c:43-62), exported by libmpi */
extern opal_class_t ompi_op_base_module_t_class;

/* op.h:388-403 */
typedef struct ompi_op_base_op_fns_1_0_0_t {
    ompi_op_base_handler_fn_t fns[OMPI_OP_BASE_TYPE_MAX];
    ompi_op_base_module_t *modules[OMPI_OP_BASE_TYPE_MAX];
} ompi_op_base_op_fns_t;
typedef struct ompi_op_base_op_3buff_fns_1_0_0_t {
    ompi_op_base_3buff_handler_fn_t fns[OMPI_OP_BASE_TYPE_MAX];
    ompi_op_base_module_t *modules[OMPI_OP_BASE_TYPE_MAX];
} ompi_op_base_op_3buff_fns_t;

#define OMPI_OP_BASE_VERSION_1_0_0 MCA_BASE_VERSION_2_0_0, "op", 1, 0, 0  /* op.h:412-414 */

/* ompi/op/op.h:138-188 */
typedef struct ompi_op_t {
    opal_object_t super;
    char o_name[MPI_MAX_OBJECT_NAME];
    int op_type;                     /* enum ompi_op_type */
    uint32_t o_flags;
    int o_f_to_c_index;
    union {
        ompi_op_base_op_fns_t intrinsic;
        void *c_fn;
        void *fort_fn;
        struct { void *user_fn; void *intercept_fn; } cxx_data;
        struct { void *intercept_fn; void *jnienv, *object; int baseType; } java_data;
    } o_func;
    ompi_op_base_op_3buff_fns_t o_3buff_intrinsic;
} ompi_op_t;

/* ------------------------------------------------------------------ communicators */
/* opal/threads/mutex_unix.h:50-64 (non-debug, POSIX threads) */
typedef struct opal_mutex_t {
    opal_object_t super;
    pthread_mutex_t m_lock_pthread;
    int32_t m_lock_atomic;           /* opal_atomic_lock_t */
} opal_mutex_t;

/* ompi/group/group.h:81-98 (prefix used by the components) */
typedef struct ompi_group_t {
    opal_object_t super;
    int grp_proc_count;
    int grp_my_rank;
    int grp_f_to_c_index;
    struct ompi_proc_t **grp_proc_pointers;
    uint32_t grp_flags;
    struct ompi_group_t *grp_parent_group_ptr;
} ompi_group_t;

/* ---- requests (the nonblocking collective slots hand one back) ------------------------------ */
/* opal/class/opal_list.h:100-116 (non-debug) */
typedef struct opal_list_item_t {
    opal_object_t super;
    volatile struct opal_list_item_t *opal_list_next;
    volatile struct opal_list_item_t *opal_list_prev;
    int32_t item_free;
} opal_list_item_t;

/* ompi/class/ompi_free_list.h:62-67 */
typedef struct ompi_free_list_item_t {
    opal_list_item_t super;
    struct mca_mpool_base_registration_t *registration;
    void *ptr;
} ompi_free_list_item_t;

/* ompi/include/mpi.h.in:344-356 */
typedef struct ompi_status_public_t {
    int MPI_SOURCE;
    int MPI_TAG;
    int MPI_ERROR;
    int _cancelled;
    size_t _ucount;
} ompi_status_public_t;

/* ompi/request/request_dbg.h:25-50 */
typedef enum {
    OMPI_REQUEST_PML, OMPI_REQUEST_IO, OMPI_REQUEST_GEN, OMPI_REQUEST_WIN, OMPI_REQUEST_COLL,
    OMPI_REQUEST_NULL, OMPI_REQUEST_NOOP, OMPI_REQUEST_COMM, OMPI_REQUEST_MAX
} ompi_request_type_t;
typedef enum {
    OMPI_REQUEST_INVALID, OMPI_REQUEST_INACTIVE, OMPI_REQUEST_ACTIVE, OMPI_REQUEST_CANCELLED
} ompi_request_state_t;

struct ompi_request_t;
/* ompi/request/request.h:58-78 */
typedef int (*ompi_request_free_fn_t)(struct ompi_request_t **rptr);
typedef int (*ompi_request_cancel_fn_t)(struct ompi_request_t *request, int flag);
typedef int (*ompi_request_complete_fn_t)(struct ompi_request_t *request);
typedef union ompi_mpi_object_t {
    struct ompi_communicator_t *comm;
    struct ompi_file_t *file;
    struct ompi_win_t *win;
} ompi_mpi_object_t;

/* ompi/request/request.h:98-110 */
typedef struct ompi_request_t {
    ompi_free_list_item_t super;
    ompi_request_type_t req_type;
    ompi_status_public_t req_status;
    volatile bool req_complete;
    volatile ompi_request_state_t req_state;
    bool req_persistent;
    int req_f_to_c_index;
    ompi_request_free_fn_t req_free;
    ompi_request_cancel_fn_t req_cancel;
    ompi_request_complete_fn_t req_complete_cb;
    void *req_complete_cb_data;
    ompi_mpi_object_t req_mpi_object;
} ompi_request_t;

/* request.h:122-127: MPI_REQUEST_NULL is &ompi_request_null.request */
typedef struct ompi_predefined_request_t {
    ompi_request_t request;
    char padding[sizeof(void *) * 32 - sizeof(ompi_request_t)];
} ompi_predefined_request_t;

/* ompi/message/message.h:21-29: the handle MPI_Mprobe / MPI_Improbe hand back (the PML allocates it
 * and frees it in mrecv / imrecv, pml_ob1_iprobe.c:83-134); opal_free_list_item_t is
 * { opal_list_item_t super; } (opal/class/opal_free_list.h:47-50) */
typedef struct ompi_message_t {
    opal_list_item_t super;
    int m_f_to_c_index;
    struct ompi_communicator_t *comm;
    void *req_ptr;
    int peer;
    size_t count;
} ompi_message_t;
typedef struct ompi_predefined_message_t {  /* message.h:40-45 */
    ompi_message_t message;
    char padding[sizeof(void *) * 32 - sizeof(ompi_message_t)];
} ompi_predefined_message_t;
extern opal_class_t ompi_message_t_class;              /* message.h:31 */
extern ompi_predefined_message_t ompi_message_null;    /* MPI_MESSAGE_NULL, mpi.h.in:739,886 */

/* opal/threads/condition.h:46-50 */
typedef struct opal_condition_t {
    opal_object_t super;
    volatile int c_waiting;
    volatile int c_signaled;
} opal_condition_t;

#define MPI_UNDEFINED (-32766)  /* mpi.h.in:423 */
#define MPI_ERR_TYPE 3          /* mpi.h.in:535 */
#define MPI_ERR_REQUEST 7       /* mpi.h.in:539 */
#define MPI_ERR_INTERN 17       /* mpi.h.in:549 */

/* exported by libmpi (request.c) / libopen-pal (opal_progress.c), or by the harness */
extern opal_class_t ompi_request_t_class;
extern size_t ompi_request_waiting;
extern size_t ompi_request_completed;
extern size_t ompi_request_failed;
extern opal_condition_t ompi_request_cond;
extern ompi_predefined_request_t ompi_request_null;
struct opal_pointer_array_t;
extern struct opal_pointer_array_t ompi_request_f_to_c_table;
int opal_pointer_array_set_item(struct opal_pointer_array_t *array, int index, void *value);
typedef int (*opal_progress_callback_t)(void);
void opal_progress(void);  /* opal/runtime/opal_progress.h:63 */
int opal_progress_register(opal_progress_callback_t cb);
int opal_progress_unregister(opal_progress_callback_t cb);

/* OMPI_REQUEST_FINI (request.h:161-169) */
static inline void mi355x_ompi_request_fini(ompi_request_t *request)
{
    request->req_state = OMPI_REQUEST_INVALID;
    if (MPI_UNDEFINED != request->req_f_to_c_index) {
        opal_pointer_array_set_item(&ompi_request_f_to_c_table, request->req_f_to_c_index, NULL);
        request->req_f_to_c_index = MPI_UNDEFINED;
    }
}

/* ompi_request_complete (request.h:397-416; opal_condition_broadcast, condition.h:138-142, is
 * `c_signaled = c_waiting`), restated because it is static inline in the reference */
static inline int mi355x_ompi_request_complete(ompi_request_t *request, bool with_signal)
{
    ompi_request_complete_fn_t tmp = request->req_complete_cb;
    if (NULL != tmp) {
        request->req_complete_cb = NULL;
        tmp(request);
    }
    ompi_request_completed++;
    request->req_complete = true;
    if (0 != request->req_status.MPI_ERROR) ompi_request_failed++;
    if (with_signal && ompi_request_waiting) ompi_request_cond.c_signaled = ompi_request_cond.c_waiting;
    return OMPI_SUCCESS;
}

struct ompi_communicator_t;
struct mca_coll_base_module_2_0_0_t;
typedef struct mca_coll_base_module_2_0_0_t mca_coll_base_module_t;

/* ompi/mca/coll/coll.h:181-239 */
typedef int (*mca_coll_base_module_allgather_fn_t)(void *sbuf, int scount, struct ompi_datatype_t *sdtype,
                                                   void *rbuf, int rcount, struct ompi_datatype_t *rdtype,
                                                   struct ompi_communicator_t *comm, mca_coll_base_module_t *module);
typedef int (*mca_coll_base_module_allreduce_fn_t)(void *sbuf, void *rbuf, int count,
                                                   struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                                                   struct ompi_communicator_t *comm, mca_coll_base_module_t *module);
typedef int (*mca_coll_base_module_bcast_fn_t)(void *buff, int count, struct ompi_datatype_t *datatype, int root,
                                               struct ompi_communicator_t *comm, mca_coll_base_module_t *module);
typedef int (*mca_coll_base_module_reduce_fn_t)(void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                                                struct ompi_op_t *op, int root, struct ompi_communicator_t *comm,
                                                mca_coll_base_module_t *module);
typedef int (*mca_coll_base_module_reduce_scatter_fn_t)(void *sbuf, void *rbuf, int *rcounts,
                                                        struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                                                        struct ompi_communicator_t *comm, mca_coll_base_module_t *module);
typedef int (*mca_coll_base_module_reduce_scatter_block_fn_t)(void *sbuf, void *rbuf, int rcount,
                                                              struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                                                              struct ompi_communicator_t *comm,
                                                              mca_coll_base_module_t *module);
/* coll.h:185-238: the blocking slots of the reduction path's callers that coll/mi355x fills */
typedef int (*mca_coll_base_module_allgatherv_fn_t)(void *sbuf, int scount, struct ompi_datatype_t *sdtype,
                                                    void *rbuf, int *rcounts, int *disps,
                                                    struct ompi_datatype_t *rdtype, struct ompi_communicator_t *comm,
                                                    mca_coll_base_module_t *module);
typedef int (*mca_coll_base_module_alltoall_fn_t)(void *sbuf, int scount, struct ompi_datatype_t *sdtype, void *rbuf,
                                                  int rcount, struct ompi_datatype_t *rdtype,
                                                  struct ompi_communicator_t *comm, mca_coll_base_module_t *module);
typedef int (*mca_coll_base_module_alltoallv_fn_t)(void *sbuf, int *scounts, int *sdisps,
                                                   struct ompi_datatype_t *sdtype, void *rbuf, int *rcounts,
                                                   int *rdisps, struct ompi_datatype_t *rdtype,
                                                   struct ompi_communicator_t *comm, mca_coll_base_module_t *module);
typedef int (*mca_coll_base_module_exscan_fn_t)(void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                                                struct ompi_op_t *op, struct ompi_communicator_t *comm,
                                                mca_coll_base_module_t *module);
typedef mca_coll_base_module_exscan_fn_t mca_coll_base_module_scan_fn_t;
typedef int (*mca_coll_base_module_gather_fn_t)(void *sbuf, int scount, struct ompi_datatype_t *sdtype, void *rbuf,
                                                int rcount, struct ompi_datatype_t *rdtype, int root,
                                                struct ompi_communicator_t *comm, mca_coll_base_module_t *module);
typedef mca_coll_base_module_gather_fn_t mca_coll_base_module_scatter_fn_t;
typedef int (*mca_coll_base_module_gatherv_fn_t)(void *sbuf, int scount, struct ompi_datatype_t *sdtype, void *rbuf,
                                                 int *rcounts, int *disps, struct ompi_datatype_t *rdtype, int root,
                                                 struct ompi_communicator_t *comm, mca_coll_base_module_t *module);
typedef int (*mca_coll_base_module_scatterv_fn_t)(void *sbuf, int *scounts, int *disps,
                                                  struct ompi_datatype_t *sdtype, void *rbuf, int rcount,
                                                  struct ompi_datatype_t *rdtype, int root,
                                                  struct ompi_communicator_t *comm, mca_coll_base_module_t *module);

/* coll.h:241-356 (the nonblocking slots coll/mi355x provides) */
typedef int (*mca_coll_base_module_iallgather_fn_t)(void *sbuf, int scount, struct ompi_datatype_t *sdtype,
                                                    void *rbuf, int rcount, struct ompi_datatype_t *rdtype,
                                                    struct ompi_communicator_t *comm, ompi_request_t **request,
                                                    mca_coll_base_module_t *module);
typedef int (*mca_coll_base_module_iallreduce_fn_t)(void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                                                    struct ompi_op_t *op, struct ompi_communicator_t *comm,
                                                    ompi_request_t **request, mca_coll_base_module_t *module);
typedef int (*mca_coll_base_module_ibcast_fn_t)(void *buff, int count, struct ompi_datatype_t *datatype, int root,
                                                struct ompi_communicator_t *comm, ompi_request_t **request,
                                                mca_coll_base_module_t *module);
typedef int (*mca_coll_base_module_ireduce_fn_t)(void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                                                 struct ompi_op_t *op, int root, struct ompi_communicator_t *comm,
                                                 ompi_request_t **request, mca_coll_base_module_t *module);
typedef int (*mca_coll_base_module_ireduce_scatter_block_fn_t)(void *sbuf, void *rbuf, int rcount,
                                                               struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                                                               struct ompi_communicator_t *comm,
                                                               ompi_request_t **request,
                                                               mca_coll_base_module_t *module);
typedef int (*mca_coll_base_module_enable_fn_t)(mca_coll_base_module_t *module, struct ompi_communicator_t *comm);
typedef int (*mca_coll_base_module_ft_event_fn_t)(int state);
typedef void (*mca_coll_base_any_fn_t)(void);   /* slots the components never call */

/* coll.h:390-451: 17 blocking, 17 nonblocking, 10 neighborhood function pointers */
struct mca_coll_base_module_2_0_0_t {
    opal_object_t super;
    mca_coll_base_module_enable_fn_t coll_module_enable;
    mca_coll_base_module_allgather_fn_t coll_allgather;
    mca_coll_base_module_allgatherv_fn_t coll_allgatherv;
    mca_coll_base_module_allreduce_fn_t coll_allreduce;
    mca_coll_base_module_alltoall_fn_t coll_alltoall;
    mca_coll_base_module_alltoallv_fn_t coll_alltoallv;
    mca_coll_base_any_fn_t coll_alltoallw;
    mca_coll_base_any_fn_t coll_barrier;
    mca_coll_base_module_bcast_fn_t coll_bcast;
    mca_coll_base_module_exscan_fn_t coll_exscan;
    mca_coll_base_module_gather_fn_t coll_gather;
    mca_coll_base_module_gatherv_fn_t coll_gatherv;
    mca_coll_base_module_reduce_fn_t coll_reduce;
    mca_coll_base_module_reduce_scatter_fn_t coll_reduce_scatter;
    mca_coll_base_module_reduce_scatter_block_fn_t coll_reduce_scatter_block;
    mca_coll_base_module_scan_fn_t coll_scan;
    mca_coll_base_module_scatter_fn_t coll_scatter;
    mca_coll_base_module_scatterv_fn_t coll_scatterv;
    /* coll.h:418-434 */
    mca_coll_base_module_iallgather_fn_t coll_iallgather;
    mca_coll_base_any_fn_t coll_iallgatherv;
    mca_coll_base_module_iallreduce_fn_t coll_iallreduce;
    mca_coll_base_any_fn_t coll_ialltoall, coll_ialltoallv, coll_ialltoallw, coll_ibarrier;
    mca_coll_base_module_ibcast_fn_t coll_ibcast;
    mca_coll_base_any_fn_t coll_iexscan, coll_igather, coll_igatherv;
    mca_coll_base_module_ireduce_fn_t coll_ireduce;
    mca_coll_base_any_fn_t coll_ireduce_scatter;
    mca_coll_base_module_ireduce_scatter_block_fn_t coll_ireduce_scatter_block;
    mca_coll_base_any_fn_t coll_iscan, coll_iscatter, coll_iscatterv;
    mca_coll_base_any_fn_t coll_neighbor[10];
    mca_coll_base_module_ft_event_fn_t ft_event;
};

/* class object of mca_coll_base_module_t (coll_base_frame.c:45-62), exported by libmpi */
extern opal_class_t mca_coll_base_module_t_class;

/* coll.h:469-566: (fn, module) pairs in the order of the module struct */
typedef struct mca_coll_base_comm_coll_t {
    mca_coll_base_module_allgather_fn_t coll_allgather;
    mca_coll_base_module_t *coll_allgather_module;
    mca_coll_base_module_allgatherv_fn_t coll_allgatherv;
    mca_coll_base_module_t *coll_allgatherv_module;
    mca_coll_base_module_allreduce_fn_t coll_allreduce;
    mca_coll_base_module_t *coll_allreduce_module;
    mca_coll_base_module_alltoall_fn_t coll_alltoall;
    mca_coll_base_module_t *coll_alltoall_module;
    mca_coll_base_module_alltoallv_fn_t coll_alltoallv;
    mca_coll_base_module_t *coll_alltoallv_module;
    struct { mca_coll_base_any_fn_t fn; mca_coll_base_module_t *module; } coll_aw_bar[2]; /* alltoallw, barrier */
    mca_coll_base_module_bcast_fn_t coll_bcast;
    mca_coll_base_module_t *coll_bcast_module;
    mca_coll_base_module_exscan_fn_t coll_exscan;
    mca_coll_base_module_t *coll_exscan_module;
    mca_coll_base_module_gather_fn_t coll_gather;
    mca_coll_base_module_t *coll_gather_module;
    mca_coll_base_module_gatherv_fn_t coll_gatherv;
    mca_coll_base_module_t *coll_gatherv_module;
    mca_coll_base_module_reduce_fn_t coll_reduce;
    mca_coll_base_module_t *coll_reduce_module;
    mca_coll_base_module_reduce_scatter_fn_t coll_reduce_scatter;
    mca_coll_base_module_t *coll_reduce_scatter_module;
    mca_coll_base_module_reduce_scatter_block_fn_t coll_reduce_scatter_block;
    mca_coll_base_module_t *coll_reduce_scatter_block_module;
    mca_coll_base_module_scan_fn_t coll_scan;
    mca_coll_base_module_t *coll_scan_module;
    mca_coll_base_module_scatter_fn_t coll_scatter;
    mca_coll_base_module_t *coll_scatter_module;
    mca_coll_base_module_scatterv_fn_t coll_scatterv;
    mca_coll_base_module_t *coll_scatterv_module;
    /* coll.h:505-540 */
    mca_coll_base_module_iallgather_fn_t coll_iallgather;
    mca_coll_base_module_t *coll_iallgather_module;
    struct { mca_coll_base_any_fn_t fn; mca_coll_base_module_t *module; } coll_iallgatherv_pair;
    mca_coll_base_module_iallreduce_fn_t coll_iallreduce;
    mca_coll_base_module_t *coll_iallreduce_module;
    struct { mca_coll_base_any_fn_t fn; mca_coll_base_module_t *module; } coll_ia2a[4];  /* ialltoall(v,w), ibarrier */
    mca_coll_base_module_ibcast_fn_t coll_ibcast;
    mca_coll_base_module_t *coll_ibcast_module;
    struct { mca_coll_base_any_fn_t fn; mca_coll_base_module_t *module; } coll_iegg[3];  /* iexscan, igather(v) */
    mca_coll_base_module_ireduce_fn_t coll_ireduce;
    mca_coll_base_module_t *coll_ireduce_module;
    struct { mca_coll_base_any_fn_t fn; mca_coll_base_module_t *module; } coll_ireduce_scatter_pair;
    mca_coll_base_module_ireduce_scatter_block_fn_t coll_ireduce_scatter_block;
    mca_coll_base_module_t *coll_ireduce_scatter_block_module;
    struct { mca_coll_base_any_fn_t fn; mca_coll_base_module_t *module; } coll_isss[3];  /* iscan, iscatter(v) */
    struct { mca_coll_base_any_fn_t fn; mca_coll_base_module_t *module; } coll_neighbor[10];
} mca_coll_base_comm_coll_t;

/* ompi/communicator/communicator.h:111-166 */
typedef struct ompi_communicator_t {
    opal_object_t c_base;
    opal_mutex_t c_lock;
    char c_name[MPI_MAX_OBJECT_NAME];
    uint32_t c_contextid;
    int c_my_rank;
    uint32_t c_flags;
    int c_id_available;
    int c_id_start_index;
    ompi_group_t *c_local_group;
    ompi_group_t *c_remote_group;
    struct ompi_communicator_t *c_local_comm;
    void *c_keyhash;
    int c_cube_dim;
    void *c_topo;
    int c_f_to_c_index;
    void **c_peruse_handles;
    void *error_handler;
    int errhandler_type;
    void *c_pml_comm;
    mca_coll_base_comm_coll_t c_coll;
} ompi_communicator_t;

static inline int mi355x_comm_rank_of(const ompi_communicator_t *c) { return c->c_my_rank; }
static inline int mi355x_comm_size_of(const ompi_communicator_t *c) { return c->c_local_group->grp_proc_count; }

/* coll.h:105-139, 357-367 */
typedef int (*mca_coll_base_component_init_query_fn_t)(bool enable_progress_threads, bool enable_mpi_threads);
typedef mca_coll_base_module_t *(*mca_coll_base_component_comm_query_fn_t)(struct ompi_communicator_t *comm,
                                                                           int *priority);
typedef struct mca_coll_base_component_2_0_0_t {
    mca_base_component_t collm_version;
    mca_base_component_data_t collm_data;
    mca_coll_base_component_init_query_fn_t collm_init_query;
    mca_coll_base_component_comm_query_fn_t collm_comm_query;
} mca_coll_base_component_t;

#define MCA_COLL_BASE_VERSION_2_0_0 MCA_BASE_VERSION_2_0_0, "coll", 2, 0, 0  /* coll.h:576-578 */

/* ------------------------------------------------------------------ point-to-point (PML) */
#define MPI_ANY_SOURCE (-1)     /* mpi.h.in:415 */
#define MPI_PROC_NULL (-2)      /* mpi.h.in:416 */
#define MPI_ANY_TAG (-1)        /* mpi.h.in:418 */
#define MPI_ERR_TRUNCATE 15     /* mpi.h.in:547 */

/* ompi/mca/pml/pml.h:77-84 */
typedef enum {
    MCA_PML_BASE_SEND_SYNCHRONOUS,
    MCA_PML_BASE_SEND_COMPLETE,
    MCA_PML_BASE_SEND_BUFFERED,
    MCA_PML_BASE_SEND_READY,
    MCA_PML_BASE_SEND_STANDARD,
    MCA_PML_BASE_SEND_SIZE
} mca_pml_base_send_mode_t;

struct ompi_proc_t;
struct ompi_message_t;
/* the module's function types (pml.h:146-470) */
typedef int (*mca_pml_base_module_add_procs_fn_t)(struct ompi_proc_t **procs, size_t nprocs);
typedef int (*mca_pml_base_module_del_procs_fn_t)(struct ompi_proc_t **procs, size_t nprocs);
typedef int (*mca_pml_base_module_enable_fn_t)(bool enable);
typedef int (*mca_pml_base_module_progress_fn_t)(void);
typedef int (*mca_pml_base_module_add_comm_fn_t)(struct ompi_communicator_t *comm);
typedef int (*mca_pml_base_module_del_comm_fn_t)(struct ompi_communicator_t *comm);
typedef int (*mca_pml_base_module_irecv_init_fn_t)(void *buf, size_t count, struct ompi_datatype_t *datatype, int src,
                                                   int tag, struct ompi_communicator_t *comm,
                                                   struct ompi_request_t **request);
typedef int (*mca_pml_base_module_irecv_fn_t)(void *buf, size_t count, struct ompi_datatype_t *datatype, int src, int tag,
                                              struct ompi_communicator_t *comm, struct ompi_request_t **request);
typedef int (*mca_pml_base_module_recv_fn_t)(void *buf, size_t count, struct ompi_datatype_t *datatype, int src, int tag,
                                             struct ompi_communicator_t *comm, ompi_status_public_t *status);
typedef int (*mca_pml_base_module_isend_init_fn_t)(void *buf, size_t count, struct ompi_datatype_t *datatype, int dst,
                                                   int tag, mca_pml_base_send_mode_t mode,
                                                   struct ompi_communicator_t *comm, struct ompi_request_t **request);
typedef int (*mca_pml_base_module_isend_fn_t)(void *buf, size_t count, struct ompi_datatype_t *datatype, int dst, int tag,
                                              mca_pml_base_send_mode_t mode, struct ompi_communicator_t *comm,
                                              struct ompi_request_t **request);
typedef int (*mca_pml_base_module_send_fn_t)(void *buf, size_t count, struct ompi_datatype_t *datatype, int dst, int tag,
                                             mca_pml_base_send_mode_t mode, struct ompi_communicator_t *comm);
typedef int (*mca_pml_base_module_iprobe_fn_t)(int src, int tag, struct ompi_communicator_t *comm, int *matched,
                                               ompi_status_public_t *status);
typedef int (*mca_pml_base_module_probe_fn_t)(int src, int tag, struct ompi_communicator_t *comm,
                                              ompi_status_public_t *status);
typedef int (*mca_pml_base_module_start_fn_t)(size_t count, struct ompi_request_t **requests);
typedef int (*mca_pml_base_module_improbe_fn_t)(int src, int tag, struct ompi_communicator_t *comm, int *matched,
                                                struct ompi_message_t **message, ompi_status_public_t *status);
typedef int (*mca_pml_base_module_mprobe_fn_t)(int src, int tag, struct ompi_communicator_t *comm,
                                               struct ompi_message_t **message, ompi_status_public_t *status);
typedef int (*mca_pml_base_module_imrecv_fn_t)(void *buf, size_t count, struct ompi_datatype_t *datatype,
                                               struct ompi_message_t **message, struct ompi_request_t **request);
typedef int (*mca_pml_base_module_mrecv_fn_t)(void *buf, size_t count, struct ompi_datatype_t *datatype,
                                              struct ompi_message_t **message, ompi_status_public_t *status);
typedef int (*mca_pml_base_module_dump_fn_t)(struct ompi_communicator_t *comm, int verbose);
typedef int (*mca_pml_base_module_ft_event_fn_t)(int status);

/* ompi/mca/pml/pml.h:497-528: the selected PML's function table, the global `mca_pml`
 * (pml.h:558) that MCA_PML_CALL dispatches through */
typedef struct mca_pml_base_module_1_0_0_t {
    mca_pml_base_module_add_procs_fn_t pml_add_procs;
    mca_pml_base_module_del_procs_fn_t pml_del_procs;
    mca_pml_base_module_enable_fn_t pml_enable;
    mca_pml_base_module_progress_fn_t pml_progress;
    mca_pml_base_module_add_comm_fn_t pml_add_comm;
    mca_pml_base_module_del_comm_fn_t pml_del_comm;
    mca_pml_base_module_irecv_init_fn_t pml_irecv_init;
    mca_pml_base_module_irecv_fn_t pml_irecv;
    mca_pml_base_module_recv_fn_t pml_recv;
    mca_pml_base_module_isend_init_fn_t pml_isend_init;
    mca_pml_base_module_isend_fn_t pml_isend;
    mca_pml_base_module_send_fn_t pml_send;
    mca_pml_base_module_iprobe_fn_t pml_iprobe;
    mca_pml_base_module_probe_fn_t pml_probe;
    mca_pml_base_module_start_fn_t pml_start;
    mca_pml_base_module_improbe_fn_t pml_improbe;
    mca_pml_base_module_mprobe_fn_t pml_mprobe;
    mca_pml_base_module_imrecv_fn_t pml_imrecv;
    mca_pml_base_module_mrecv_fn_t pml_mrecv;
    mca_pml_base_module_dump_fn_t pml_dump;
    mca_pml_base_module_ft_event_fn_t pml_ft_event;
    uint32_t pml_max_contextid;
    int pml_max_tag;
} mca_pml_base_module_t;
extern mca_pml_base_module_t mca_pml;

#ifdef __cplusplus
}
#endif
#endif /* MI355X_OMPI_ABI_H */
