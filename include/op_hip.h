/*
 * op_hip.h -- the op/hip MCA component (lib/mca_op_hip.so).
 *
 * Plugs into the op framework's per-MPI_Op function tables (ompi/mca/op/op.h:326-373): for
 * every intrinsic MPI_Op it returns a module whose opm_fns[] / opm_3buff_fns[] slots run the
 * CDNA4 kernels of libmi355x_rt on device buffers.  The functions below have exactly the
 * reference op-table signatures (op.h:253-266) and replace, slot by slot,
 * ompi_op_base_2buff_<op>_<type> / ompi_op_base_3buff_<op>_<type>
 * (ompi/mca/op/base/op_base_functions.c:39-683) once installed by ompi_op_base_op_select
 * (op_base_op_select.c:88-204).
 *
 * Behaviour per call (synchronous, like the reference loops -- the caller reuses the result
 * immediately, coll_tuned_allreduce.c:491-496):
 *   - every operand in host memory      -> the lower-priority function that was installed in the
 *                                          slot before op/hip (op/base's CPU loop), unchanged;
 *   - any operand in device memory      -> HIP kernel on the null stream, then stream sync; a
 *                                          host operand is staged through device scratch;
 *   - x87 long double slots on device   -> staged to the host and run by the lower-priority
 *                                          function (CDNA4 has no 80-bit format);
 *   - a HIP failure                     -> abort(), as opal_cuda_memcpy does
 *                                          (opal/datatype/opal_datatype_cuda.c:106-111); the
 *                                          op ABI has no error return (op.h:519-520).
 */
#ifndef MI355X_OP_HIP_H
#define MI355X_OP_HIP_H

#include "ompi_abi.h"

#ifdef __cplusplus
extern "C" {
#endif

/* the component symbol the MCA loader looks up (opal/mca/base/mca_base_component_find.c:619-631) */
extern ompi_op_base_component_t mca_op_hip_component;

/* 2-buff and 3-buff entry points installed in every supported slot (the element type comes from
 * ompi_op_ddt_map[(*dtype)->id], the MPI_Op from the module) */
void mca_op_hip_2buff(void *in, void *inout, int *count, struct ompi_datatype_t **dtype,
                      struct ompi_op_base_module_1_0_0_t *module);
void mca_op_hip_3buff(void *in1, void *in2, void *out, int *count, struct ompi_datatype_t **dtype,
                      struct ompi_op_base_module_1_0_0_t *module);

/* MCA parameters (environment: OMPI_MCA_op_hip_<name>) */
extern int mca_op_hip_priority;      /* default 50 (op/base is 0) */

#ifdef __cplusplus
}
#endif
#endif
