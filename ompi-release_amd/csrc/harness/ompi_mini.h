/* ompi_mini.h -- API of the mini-Open-MPI host harness (see ompi_mini.c). */
#ifndef MI355X_OMPI_MINI_H
#define MI355X_OMPI_MINI_H

#include "../../../include/mi355x_types.h"
#include "../../../include/ompi_abi.h"

#ifdef __cplusplus
extern "C" {
#endif

void mini_init(void);
ompi_datatype_t *mini_datatype(int id);
int mini_datatype_id_for_slot(int slot);
void mini_datatype_fields(const ompi_datatype_t *d, int64_t out[7]);
const void *mini_datatype_desc(const ompi_datatype_t *d);
ompi_datatype_t *mini_datatype_create_raw(const void *desc, uint32_t used, size_t size, ptrdiff_t lb, ptrdiff_t ub,
                                          ptrdiff_t true_lb, ptrdiff_t true_ub, uint16_t flags);
void mini_datatype_destroy(ompi_datatype_t *d);
void mini_set_base_function(int op, int slot, void *fn2, void *fn3);
ompi_op_t *mini_op_create(int code);
int mini_op_select(ompi_op_t *op, ompi_op_base_component_t **comps, int ncomp);
void mini_op_reduce(ompi_op_t *op, void *source, void *target, int count, ompi_datatype_t *dtype);
void mini_op_reduce_3buff(ompi_op_t *op, void *s1, void *s2, void *target, int count, ompi_datatype_t *dtype);
void *mini_op_fn2(ompi_op_t *op, int slot);
void *mini_op_module2(ompi_op_t *op, int slot);
void *mini_op_module3(ompi_op_t *op, int slot);
int mini_obj_refcount(void *obj);
void mini_op_destroy(ompi_op_t *op);
ompi_communicator_t *mini_comm_create(int rank, int size, unsigned cid);
void mini_comm_install(ompi_communicator_t *c, mca_coll_base_module_t *m);
int mini_coll_select(ompi_communicator_t *c, mca_coll_base_component_t *comp);
mca_coll_base_module_t *mini_coll_module_new(void);
void mini_comm_destroy(ompi_communicator_t *c);
int mini_comm_set_channel(ompi_communicator_t *c, const char *name);  /* host bcast for the stub module */
int mini_allreduce(ompi_communicator_t *c, void *s, void *r, int n, ompi_datatype_t *d, ompi_op_t *op);
int mini_reduce_scatter_block(ompi_communicator_t *c, void *s, void *r, int n, ompi_datatype_t *d, ompi_op_t *op);
int mini_reduce_scatter(ompi_communicator_t *c, void *s, void *r, int *rc, ompi_datatype_t *d, ompi_op_t *op);
int mini_allgather(ompi_communicator_t *c, void *s, int sc, ompi_datatype_t *sd, void *r, int rc, ompi_datatype_t *rd);
int mini_bcast(ompi_communicator_t *c, void *b, int n, ompi_datatype_t *d, int root);
void *mini_comm_fn(ompi_communicator_t *c, int which);
mca_coll_base_module_t *mini_stub_module(void);
int mini_stub_calls(int which);
int mini_stub_marker(void);
mca_coll_base_module_t *mini_host_module(void);  /* real host collectives over the channel */
int mini_host_calls(int which);
int mini_device_hits(void);  /* device buffers the host modules were handed */
ompi_op_t *mini_op_create_user(void *fn, int commute);
size_t mini_offsetof(int which);
/* the PML slot: a counting stub as the selected PML, and the bindings' MCA_PML_CALL paths */
int mini_var_count(void);
const char *mini_var_name(int i);
int mini_var_int(int i);
int mini_component_register(const mca_base_component_t *c);
int mini_coll_init(mca_coll_base_component_t *comp);
int mini_coll_close(mca_coll_base_component_t *comp);
void mini_pml_install_stub(void);
int mini_pml_stub_calls(int which);
void *mini_pml_fn(int which);
int mini_send(void *b, int n, ompi_datatype_t *d, int dst, int tag, ompi_communicator_t *c);
int mini_ssend(void *b, int n, ompi_datatype_t *d, int dst, int tag, ompi_communicator_t *c);
int mini_recv(void *b, int n, ompi_datatype_t *d, int src, int tag, ompi_communicator_t *c, ompi_status_public_t *st);
int mini_isend(void *b, int n, ompi_datatype_t *d, int dst, int tag, ompi_communicator_t *c, ompi_request_t **req);
int mini_irecv(void *b, int n, ompi_datatype_t *d, int src, int tag, ompi_communicator_t *c, ompi_request_t **req);
int mini_iprobe(int src, int tag, ompi_communicator_t *c, int *flag, ompi_status_public_t *st);
int mini_wait_status(ompi_request_t **req, ompi_status_public_t *st);
int mini_wait(ompi_request_t **req);
int mini_test(ompi_request_t **req, int *flag, ompi_status_public_t *st);
int mini_request_free(ompi_request_t **req);
int mini_cancel(ompi_request_t *r);
int mini_start(ompi_request_t **req);
int mini_message_is_null(ompi_message_t *m);
int mini_send_mode(void *b, int n, ompi_datatype_t *d, int dst, int tag, int mode, ompi_communicator_t *c);
int mini_isend_mode(void *b, int n, ompi_datatype_t *d, int dst, int tag, int mode, ompi_communicator_t *c,
                    ompi_request_t **req);
int mini_probe(int src, int tag, ompi_communicator_t *c, ompi_status_public_t *st);
int mini_send_init(void *b, int n, ompi_datatype_t *d, int dst, int tag, int mode, ompi_communicator_t *c,
                   ompi_request_t **req);
int mini_recv_init(void *b, int n, ompi_datatype_t *d, int src, int tag, ompi_communicator_t *c, ompi_request_t **req);
int mini_improbe(int src, int tag, ompi_communicator_t *c, int *flag, ompi_message_t **msg, ompi_status_public_t *st);
int mini_mprobe(int src, int tag, ompi_communicator_t *c, ompi_message_t **msg, ompi_status_public_t *st);
int mini_imrecv(void *b, int n, ompi_datatype_t *d, ompi_message_t **msg, ompi_request_t **req);
int mini_mrecv(void *b, int n, ompi_datatype_t *d, ompi_message_t **msg, ompi_status_public_t *st);

#ifdef __cplusplus
}
#endif
#endif
