/*
 * mi355x_types.h -- reduction-op and element-type codes shared by every layer of the
 * MI355X collective-reduction path (op/hip, coll/mi355x, libmi355x_rt, and the oracle).
 *
 * The numeric values are the Open MPI 1.8.5 op-framework ABI, restated (not copied):
 *   element types : OMPI_OP_BASE_TYPE_*     ompi/mca/op/op.h:103-194
 *   operations    : OMPI_OP_BASE_FORTRAN_*  ompi/mca/op/op.h:201-235
 * so an op-module slot index `opm_fns[type]` and an `o_f_to_c_index` op index can be passed
 * straight through the C ABI without translation.
 */
#ifndef MI355X_TYPES_H
#define MI355X_TYPES_H

#ifdef __cplusplus
extern "C" {
#endif

/* Element types: the slot index of ompi_op_base_module_t::opm_fns[] (op.h:103-194). */
enum mi355x_type {
    MI355X_T_INT8 = 0,
    MI355X_T_UINT8,
    MI355X_T_INT16,
    MI355X_T_UINT16,
    MI355X_T_INT32,
    MI355X_T_UINT32,
    MI355X_T_INT64,
    MI355X_T_UINT64,
    /* Fortran integers (op.h:123-129) */
    MI355X_T_F_INTEGER,
    MI355X_T_F_INTEGER1,
    MI355X_T_F_INTEGER2,
    MI355X_T_F_INTEGER4,
    MI355X_T_F_INTEGER8,
    MI355X_T_F_INTEGER16,
    /* floating point (op.h:131-141) */
    MI355X_T_FLOAT,
    MI355X_T_DOUBLE,
    MI355X_T_F_REAL,
    MI355X_T_F_REAL2,
    MI355X_T_F_REAL4,
    MI355X_T_F_REAL8,
    MI355X_T_F_REAL16,
    MI355X_T_F_DOUBLE_PRECISION,
    MI355X_T_LONG_DOUBLE,
    /* logical (op.h:143-146) */
    MI355X_T_F_LOGICAL,
    MI355X_T_BOOL,
    /* complex (op.h:148-156) */
    MI355X_T_C_FLOAT_COMPLEX,
    MI355X_T_C_DOUBLE_COMPLEX,
    MI355X_T_C_LONG_DOUBLE_COMPLEX,
    /* byte (op.h:158-159) */
    MI355X_T_BYTE,
    /* pair types for MAXLOC/MINLOC (op.h:161-177) */
    MI355X_T_F_2REAL,
    MI355X_T_F_2DOUBLE_PRECISION,
    MI355X_T_F_2INTEGER,
    MI355X_T_FLOAT_INT,
    MI355X_T_DOUBLE_INT,
    MI355X_T_LONG_INT,
    MI355X_T_2INT,
    MI355X_T_SHORT_INT,
    MI355X_T_LONG_DOUBLE_INT,
    /* wchar (op.h:179-180) -- no op table row uses it */
    MI355X_T_WCHAR,
    MI355X_T_MAX /* == OMPI_OP_BASE_TYPE_MAX == 39 */
};

/* Operations: the o_f_to_c_index of the predefined MPI_Op (op.h:201-235). */
enum mi355x_op {
    MI355X_OP_NULL = 0,
    MI355X_OP_MAX,
    MI355X_OP_MIN,
    MI355X_OP_SUM,
    MI355X_OP_PROD,
    MI355X_OP_LAND,
    MI355X_OP_BAND,
    MI355X_OP_LOR,
    MI355X_OP_BOR,
    MI355X_OP_LXOR,
    MI355X_OP_BXOR,
    MI355X_OP_MAXLOC,
    MI355X_OP_MINLOC,
    MI355X_OP_REPLACE,
    MI355X_OP_NO_OP,
    MI355X_OP_MAX_ /* == OMPI_OP_BASE_FORTRAN_OP_MAX == 15 */
};

/* Error codes returned by every mi355x_* entry point (0 == success, OMPI_SUCCESS). */
enum mi355x_status {
    MI355X_SUCCESS = 0,
    MI355X_ERR_ARG = -1,        /* bad argument (NULL pointer, negative count, bad enum) */
    MI355X_ERR_UNSUPPORTED = -2,/* (op,type) slot is NULL in the reference table or has no GPU form */
    MI355X_ERR_HIP = -3,        /* a HIP runtime call failed; see mi355x_last_error() */
    MI355X_ERR_NOMEM = -4,
    MI355X_ERR_PEER = -5,       /* peer unreachable / IPC open failed */
    MI355X_ERR_TIMEOUT = -6,    /* a cross-rank wait exceeded its bound */
    MI355X_ERR_TRUNCATE = -7    /* message longer than the receive buffer (MPI_ERR_TRUNCATE) */
};

#ifdef __cplusplus
}
#endif
#endif /* MI355X_TYPES_H */
