"""ctypes view of the mini-Open-MPI harness (libompi_mini.so) and the two MCA component DSOs.

Load order mirrors Open MPI: libmi355x_rt and libompi_mini are global (they play libmpi /
libopen-pal), then the component DSOs are dlopen'ed and their component symbols looked up by the
MCA naming rule (opal/mca/base/mca_base_component_find.c:619-631).
"""
from __future__ import annotations

import ctypes

from conftest import load_pkg

_h = None


class Mini:
    def __init__(self):
        pkg = load_pkg()
        pkg.rt()  # RTLD_GLOBAL
        lib_dir = pkg.LIB_DIR
        self.pkg = pkg
        self.lib = ctypes.CDLL(str(lib_dir / "libompi_mini.so"), mode=ctypes.RTLD_GLOBAL)
        self.op_hip = ctypes.CDLL(str(lib_dir / "mca_op_hip.so"))
        self.coll = ctypes.CDLL(str(lib_dir / "mca_coll_mi355x.so"))
        L = self.lib
        vp, i = ctypes.c_void_p, ctypes.c_int
        L.mini_datatype.restype = vp
        L.mini_datatype.argtypes = [i]
        L.mini_datatype_id_for_slot.argtypes = [i]
        L.mini_set_base_function.argtypes = [i, i, vp, vp]
        L.mini_op_create.restype = vp
        L.mini_op_create.argtypes = [i]
        L.mini_op_select.argtypes = [vp, ctypes.POINTER(vp), i]
        L.mini_op_reduce.argtypes = [vp, vp, vp, i, vp]
        L.mini_op_reduce_3buff.argtypes = [vp, vp, vp, vp, i, vp]
        for f in ("mini_op_fn2", "mini_op_module2", "mini_op_module3"):
            getattr(L, f).restype = vp
            getattr(L, f).argtypes = [vp, i]
        L.mini_obj_refcount.argtypes = [vp]
        L.mini_op_destroy.argtypes = [vp]
        L.mini_comm_create.restype = vp
        L.mini_comm_create.argtypes = [i, i, ctypes.c_uint]
        L.mini_comm_install.argtypes = [vp, vp]
        L.mini_comm_set_channel.argtypes = [vp, ctypes.c_char_p]
        L.mini_coll_select.argtypes = [vp, vp]
        L.mini_coll_init.argtypes = [vp]
        L.mini_var_name.restype = ctypes.c_char_p
        L.mini_var_name.argtypes = [i]
        L.mini_var_int.argtypes = [i]
        L.mini_component_register.argtypes = [vp]
        L.mini_coll_close.argtypes = [vp]
        L.mini_pml_fn.restype = vp
        L.mini_pml_fn.argtypes = [i]
        L.mini_pml_stub_calls.argtypes = [i]
        L.mini_send.argtypes = [vp, i, vp, i, i, vp]
        L.mini_ssend.argtypes = [vp, i, vp, i, i, vp]
        L.mini_recv.argtypes = [vp, i, vp, i, i, vp, vp]
        L.mini_isend.argtypes = [vp, i, vp, i, i, vp, ctypes.POINTER(vp)]
        L.mini_irecv.argtypes = [vp, i, vp, i, i, vp, ctypes.POINTER(vp)]
        L.mini_iprobe.argtypes = [i, i, vp, ctypes.POINTER(i), vp]
        L.mini_wait_status.argtypes = [ctypes.POINTER(vp), vp]
        L.mini_send_mode.argtypes = [vp, i, vp, i, i, i, vp]
        L.mini_isend_mode.argtypes = [vp, i, vp, i, i, i, vp, ctypes.POINTER(vp)]
        L.mini_probe.argtypes = [i, i, vp, vp]
        L.mini_send_init.argtypes = [vp, i, vp, i, i, i, vp, ctypes.POINTER(vp)]
        L.mini_recv_init.argtypes = [vp, i, vp, i, i, vp, ctypes.POINTER(vp)]
        L.mini_start.argtypes = [ctypes.POINTER(vp)]
        L.mini_request_free.argtypes = [ctypes.POINTER(vp)]
        L.mini_cancel.argtypes = [vp]
        L.mini_test.argtypes = [ctypes.POINTER(vp), ctypes.POINTER(i), vp]
        L.mini_improbe.argtypes = [i, i, vp, ctypes.POINTER(i), ctypes.POINTER(vp), vp]
        L.mini_mprobe.argtypes = [i, i, vp, ctypes.POINTER(vp), vp]
        L.mini_imrecv.argtypes = [vp, i, vp, ctypes.POINTER(vp), ctypes.POINTER(vp)]
        L.mini_mrecv.argtypes = [vp, i, vp, ctypes.POINTER(vp), vp]
        L.mini_message_is_null.argtypes = [vp]
        L.mini_coll_module_new.restype = vp
        L.mini_comm_destroy.argtypes = [vp]
        L.mini_allreduce.argtypes = [vp, vp, vp, i, vp, vp]
        L.mini_reduce_scatter_block.argtypes = [vp, vp, vp, i, vp, vp]
        L.mini_reduce.argtypes = [vp, vp, vp, i, vp, vp, i]
        P = ctypes.POINTER(vp)
        L.mini_iallreduce.argtypes = [vp, vp, vp, i, vp, vp, P]
        L.mini_ireduce.argtypes = [vp, vp, vp, i, vp, vp, i, P]
        L.mini_ireduce_scatter_block.argtypes = [vp, vp, vp, i, vp, vp, P]
        L.mini_iallgather.argtypes = [vp, vp, i, vp, vp, i, vp, P]
        L.mini_ibcast.argtypes = [vp, vp, i, vp, i, P]
        L.mini_wait.argtypes = [P]
        L.mini_request_is_null.argtypes = [vp]
        L.mini_request_complete.argtypes = [vp]
        L.mini_reduce_scatter.argtypes = [vp, vp, vp, ctypes.POINTER(i), vp, vp]
        L.mini_allgather.argtypes = [vp, vp, i, vp, vp, i, vp]
        L.mini_bcast.argtypes = [vp, vp, i, vp, i]
        IP = ctypes.POINTER(i)
        L.mini_gather.argtypes = [vp, vp, i, vp, vp, i, vp, i]
        L.mini_scatter.argtypes = [vp, vp, i, vp, vp, i, vp, i]
        L.mini_gatherv.argtypes = [vp, vp, i, vp, vp, IP, IP, vp, i]
        L.mini_scatterv.argtypes = [vp, vp, IP, IP, vp, vp, i, vp, i]
        L.mini_allgatherv.argtypes = [vp, vp, i, vp, vp, IP, IP, vp]
        L.mini_alltoall.argtypes = [vp, vp, i, vp, vp, i, vp]
        L.mini_alltoallv.argtypes = [vp, vp, IP, IP, vp, vp, IP, IP, vp]
        L.mini_scan.argtypes = [vp, vp, vp, i, vp, vp]
        L.mini_exscan.argtypes = [vp, vp, vp, i, vp, vp]
        L.mini_comm_fn.restype = vp
        L.mini_comm_fn.argtypes = [vp, i]
        L.mini_stub_module.restype = vp
        L.mini_stub_calls.argtypes = [i]
        L.mini_offsetof.restype = ctypes.c_size_t
        L.mini_offsetof.argtypes = [i]
        L.mini_datatype_create_raw.restype = vp
        L.mini_datatype_create_raw.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_size_t] + \
            [ctypes.c_ssize_t] * 4 + [ctypes.c_uint16]
        L.mini_datatype_destroy.argtypes = [vp]
        L.mini_init()

    def addr(self, lib, sym):
        return ctypes.cast(getattr(lib, sym), ctypes.c_void_p).value

    def component_ptr(self, lib, sym):
        return ctypes.addressof(ctypes.c_char.in_dll(lib, sym))

    def dtype_for_slot(self, slot):
        did = self.lib.mini_datatype_id_for_slot(slot)
        return None if did < 0 else self.lib.mini_datatype(did)

    def derived(self, desc, used, size, lb, ub):
        """a committed derived datatype (not predefined, with gaps) from an opal description"""
        return self.lib.mini_datatype_create_raw(desc, used, size, lb, ub, lb, ub, 0)

    def install_oracle_base(self, oracle):
        """op/base's CPU loops in the harness = the oracle's reference-signature thunks"""
        for op in range(15):
            for ty in range(39):
                if oracle.oracle_has_op(op, ty):
                    self.lib.mini_set_base_function(op, ty, oracle.oracle_ompi_fn2(op, ty), oracle.oracle_ompi_fn3(op, ty))

    def select_op(self, code, with_hip=True):
        op = self.lib.mini_op_create(code)
        comps = (ctypes.c_void_p * 1)(self.component_ptr(self.op_hip, "mca_op_hip_component"))
        rc = self.lib.mini_op_select(op, comps, 1 if with_hip else 0)
        assert rc == 0, rc
        return op


def mini() -> Mini:
    global _h
    if _h is None:
        _h = Mini()
    return _h
