"""Host-side (Python) view of the MI355X collective-reduction path.

The product is native: ``lib/libmi355x_rt.so`` (HIP kernels behind a C ABI, include/mi355x_rt.h)
plus the two Open MPI components ``lib/mca_op_hip.so`` and ``lib/mca_coll_mi355x.so`` written in
C.  This module is the thin ctypes binding used by the tests, ``bench.py`` and
``__graft_entry__.py``; it mirrors the reference's op vocabulary (ompi/mca/op/op.h:103-235) so a
test reads like the reference's own.  It has no compute path of its own: every reduction goes
through the HIP library, and loading fails loudly when the library is missing.

Import it with :func:`load` (the directory name is not a valid Python identifier)::

    import importlib.util, pathlib
    spec = importlib.util.spec_from_file_location("ompi_release_amd", ".../ompi-release_amd/__init__.py")
"""
from __future__ import annotations

import ctypes
import os
import pathlib

PKG_DIR = pathlib.Path(__file__).resolve().parent
# MI355X_LIB_DIR selects another build of the same libraries (the host-sanitizer build in
# lib_san, csrc/Makefile.san, loaded by tools/san_boundary.sh)
LIB_DIR = pathlib.Path(os.environ["MI355X_LIB_DIR"]) if os.environ.get("MI355X_LIB_DIR") else PKG_DIR / "lib"
REPO_DIR = PKG_DIR.parent

# ---------------------------------------------------------------- reference enums (op.h)
TYPES = [
    "INT8", "UINT8", "INT16", "UINT16", "INT32", "UINT32", "INT64", "UINT64",
    "F_INTEGER", "F_INTEGER1", "F_INTEGER2", "F_INTEGER4", "F_INTEGER8", "F_INTEGER16",
    "FLOAT", "DOUBLE", "F_REAL", "F_REAL2", "F_REAL4", "F_REAL8", "F_REAL16",
    "F_DOUBLE_PRECISION", "LONG_DOUBLE", "F_LOGICAL", "BOOL",
    "C_FLOAT_COMPLEX", "C_DOUBLE_COMPLEX", "C_LONG_DOUBLE_COMPLEX", "BYTE",
    "F_2REAL", "F_2DOUBLE_PRECISION", "F_2INTEGER",
    "FLOAT_INT", "DOUBLE_INT", "LONG_INT", "2INT", "SHORT_INT", "LONG_DOUBLE_INT", "WCHAR",
]
T = {name: i for i, name in enumerate(TYPES)}
OPS = ["NULL", "MAX", "MIN", "SUM", "PROD", "LAND", "BAND", "LOR", "BOR", "LXOR", "BXOR",
       "MAXLOC", "MINLOC", "REPLACE", "NO_OP"]
OP = {name: i for i, name in enumerate(OPS)}

MI355X_SUCCESS = 0


class MI355XError(RuntimeError):
    pass


_rt = None


def lib_path(name: str = "libmi355x_rt.so") -> pathlib.Path:
    return LIB_DIR / name


def rt() -> ctypes.CDLL:
    """Load libmi355x_rt.so (RTLD_GLOBAL so the MCA component DSOs resolve against it)."""
    global _rt
    if _rt is None:
        p = lib_path()
        if not p.exists():
            raise MI355XError(f"{p} is missing: run __graft_entry__.build() (make -C ompi-release_amd/csrc)")
        lib = ctypes.CDLL(str(p), mode=ctypes.RTLD_GLOBAL)
        _declare(lib)
        _rt = lib
    return _rt


class MsgStatus(ctypes.Structure):
    """mi355x_status_t: MPI_Status of a device point-to-point receive"""
    _fields_ = [("source", ctypes.c_int), ("tag", ctypes.c_int), ("error", ctypes.c_int),
                ("bytes", ctypes.c_size_t)]

    def as_tuple(self) -> tuple[int, int, int, int]:
        return self.source, self.tag, self.error, self.bytes


class TruncateError(MI355XError):
    """a receive longer than its buffer (MPI_ERR_TRUNCATE); .status holds the message's status"""

    def __init__(self, msg: str, status: tuple[int, int, int, int]):
        super().__init__(msg)
        self.status = status


ANY_SOURCE, PROC_NULL, ANY_TAG = -1, -2, -1
ERR_TRUNCATE = -7


def _declare(lib: ctypes.CDLL) -> None:
    c = ctypes
    vp, sz, i = c.c_void_p, c.c_size_t, c.c_int
    sigs = {
        "mi355x_last_error": (c.c_char_p, []),
        "mi355x_version": (i, []),
        "mi355x_device_count": (i, [c.POINTER(i)]),
        "mi355x_set_device": (i, [i]),
        "mi355x_get_device": (i, [c.POINTER(i)]),
        "mi355x_stream_create": (i, [c.POINTER(vp)]),
        "mi355x_stream_destroy": (i, [vp]),
        "mi355x_stream_sync": (i, [vp]),
        "mi355x_device_sync": (i, []),
        "mi355x_malloc": (i, [c.POINTER(vp), sz]),
        "mi355x_free": (i, [vp]),
        "mi355x_memcpy": (i, [vp, vp, sz]),
        "mi355x_memcpy_async": (i, [vp, vp, sz, vp]),
        "mi355x_memset_async": (i, [vp, i, sz, vp]),
        "mi355x_ptr_is_device": (i, [vp, c.POINTER(i)]),
        "mi355x_event_create": (i, [c.POINTER(vp)]),
        "mi355x_event_destroy": (i, [vp]),
        "mi355x_event_record": (i, [vp, vp]),
        "mi355x_event_elapsed_ms": (i, [vp, vp, c.POINTER(c.c_float)]),
        "mi355x_op_supported": (i, [i, i]),
        "mi355x_comm_op_supported": (i, [i, i]),
        "mi355x_type_size": (sz, [i]),
        "mi355x_op_reduce": (i, [i, i, vp, vp, sz, vp]),
        "mi355x_op_reduce_3buff": (i, [i, i, vp, vp, vp, sz, vp]),
        "mi355x_op_tune": (i, [i, i, i]),
        "mi355x_op_get_tune": (i, [c.POINTER(i), c.POINTER(i), c.POINTER(i)]),
        "mi355x_op_set_mode": (i, [i]),
        "mi355x_op_get_mode": (i, []),
        "mi355x_op_set_threads": (i, [i]),
        "mi355x_comm_create": (i, [c.c_char_p, i, i, i, c.POINTER(vp)]),
        "mi355x_comm_create_loopback": (i, [i, i, c.POINTER(vp)]),
        "mi355x_comm_destroy": (i, [vp]),
        "mi355x_comm_rank": (i, [vp]),
        "mi355x_comm_size": (i, [vp]),
        "mi355x_comm_barrier": (i, [vp]),
        "mi355x_comm_last_algorithm": (i, [vp]),
        "mi355x_debug_pipe_token": (i, [vp, i]),
        "mi355x_debug_token": (i, [c.c_uint64, c.c_char_p, i]),
        "mi355x_comm_set": (i, [vp, i, c.c_long]),
        "mi355x_comm_phase_ms": (i, [vp, c.POINTER(c.c_float), c.POINTER(c.c_float)]),
        "mi355x_comm_get": (i, [vp, i, c.POINTER(c.c_long)]),
        "mi355x_allreduce": (i, [vp, vp, vp, sz, i, i, vp]),
        "mi355x_reduce_scatter_block": (i, [vp, vp, vp, sz, i, i, vp]),
        "mi355x_reduce": (i, [vp, vp, vp, sz, i, i, i, vp]),
        "mi355x_iallreduce": (i, [vp, vp, vp, sz, i, i, vp, c.POINTER(vp)]),
        "mi355x_ireduce": (i, [vp, vp, vp, sz, i, i, i, vp, c.POINTER(vp)]),
        "mi355x_ireduce_scatter_block": (i, [vp, vp, vp, sz, i, i, vp, c.POINTER(vp)]),
        "mi355x_iallgather": (i, [vp, vp, vp, sz, vp, c.POINTER(vp)]),
        "mi355x_ibcast": (i, [vp, vp, sz, i, vp, c.POINTER(vp)]),
        "mi355x_request_test": (i, [vp, c.POINTER(i)]),
        "mi355x_request_wait": (i, [vp]),
        "mi355x_request_free": (i, [vp]),
        "mi355x_reduce_scatter": (i, [vp, vp, vp, c.POINTER(i), i, i, vp]),
        "mi355x_allgather": (i, [vp, vp, vp, sz, vp]),
        "mi355x_bcast": (i, [vp, vp, sz, i, vp]),
        "mi355x_sched_program": (i, [i, i, i, i, c.POINTER(i), i]),
        "mi355x_rules_load": (i, [c.c_char_p, c.POINTER(vp)]),
        "mi355x_rules_destroy": (i, [vp]),
        "mi355x_rules_decide": (i, [vp, i, i, sz, c.POINTER(i), c.POINTER(i), c.POINTER(i)]),
        "mi355x_comm_set_rules": (i, [vp, vp]),
        "mi355x_ddt_create": (i, [c.POINTER(c.c_int64), c.POINTER(c.c_int64), sz, sz, c.c_int64, c.c_int64, c.POINTER(vp)]),
        "mi355x_ddt_create_vector": (i, [sz, sz, c.c_int64, sz, c.POINTER(vp)]),
        "mi355x_ddt_create_indexed": (i, [sz, c.POINTER(i), c.POINTER(i), sz, c.POINTER(vp)]),
        "mi355x_ddt_from_opal": (i, [vp, c.c_uint32, c.c_int64, c.POINTER(c.c_uint32), c.POINTER(vp)]),
        "mi355x_ddt_destroy": (i, [vp]),
        "mi355x_ddt_size": (sz, [vp]),
        "mi355x_ddt_extent": (c.c_int64, [vp]),
        "mi355x_ddt_nruns": (i, [vp]),
        "mi355x_ddt_tune": (i, [i, i, i, i]),
        "mi355x_ddt_tune_rows": (i, [i]),
        "mi355x_comm_vote": (i, [vp, i, c.POINTER(i)]),
        "mi355x_gather": (i, [vp, vp, vp, sz, i, vp]),
        "mi355x_gatherv": (i, [vp, vp, sz, vp, c.POINTER(sz), c.POINTER(sz), i, vp]),
        "mi355x_scatter": (i, [vp, vp, vp, sz, i, vp]),
        "mi355x_scatterv": (i, [vp, vp, c.POINTER(sz), c.POINTER(sz), vp, sz, i, vp]),
        "mi355x_allgatherv": (i, [vp, vp, sz, vp, c.POINTER(sz), c.POINTER(sz), vp]),
        "mi355x_alltoall": (i, [vp, vp, vp, sz, vp]),
        "mi355x_alltoallv": (i, [vp, vp, c.POINTER(sz), c.POINTER(sz), vp, c.POINTER(sz), c.POINTER(sz), vp]),
        "mi355x_scan": (i, [vp, vp, vp, sz, i, i, vp]),
        "mi355x_exscan": (i, [vp, vp, vp, sz, i, i, vp]),
        "mi355x_iscan": (i, [vp, vp, vp, sz, i, i, vp, c.POINTER(vp)]),
        "mi355x_ialltoall": (i, [vp, vp, vp, sz, vp, c.POINTER(vp)]),
        "mi355x_isend": (i, [vp, vp, sz, vp, i, i, vp, c.POINTER(vp)]),
        "mi355x_irecv": (i, [vp, vp, sz, vp, i, i, vp, c.POINTER(vp)]),
        "mi355x_send": (i, [vp, vp, sz, vp, i, i, vp]),
        "mi355x_recv": (i, [vp, vp, sz, vp, i, i, vp, c.POINTER(MsgStatus)]),
        "mi355x_sendrecv": (i, [vp, vp, sz, vp, i, i, vp, sz, vp, i, i, vp, c.POINTER(MsgStatus)]),
        "mi355x_iprobe": (i, [vp, i, i, c.POINTER(i), c.POINTER(MsgStatus)]),
        "mi355x_p2p_progress": (i, [vp]),
        "mi355x_request_get_status": (i, [vp, c.POINTER(MsgStatus)]),
        "mi355x_isend_mode": (i, [vp, vp, sz, vp, i, i, i, vp, c.POINTER(vp)]),
        "mi355x_send_mode": (i, [vp, vp, sz, vp, i, i, i, vp]),
        "mi355x_improbe": (i, [vp, i, i, c.POINTER(i), c.POINTER(vp), c.POINTER(MsgStatus)]),
        "mi355x_imrecv": (i, [vp, vp, sz, vp, vp, vp, c.POINTER(vp)]),
        "mi355x_request_cancel": (i, [vp]),
        "mi355x_request_cancelled": (i, [vp, c.POINTER(i)]),
        "mi355x_set_progress_hook": (i, [vp]),
        "mi355x_pack_host": (i, [vp, sz, vp, sz, vp, sz]),
        "mi355x_unpack_host": (i, [vp, sz, vp, sz, vp, sz]),
        "mi355x_ddt_raw": (i, [vp, sz, c.POINTER(sz), c.POINTER(c.c_int64), c.POINTER(sz), c.POINTER(c.c_uint32),
                               c.POINTER(sz)]),
        "mi355x_pack": (i, [vp, sz, vp, sz, vp, sz, c.POINTER(c.c_uint32), vp]),
        "mi355x_unpack": (i, [vp, sz, vp, sz, vp, sz, c.POINTER(c.c_uint32), vp]),
    }
    for name, (res, args) in sigs.items():
        fn = getattr(lib, name, None)
        if fn is None:
            continue  # optional symbols are checked by tests/test_boundary.py
        fn.restype = res
        fn.argtypes = args


def check(rc: int, what: str = "") -> None:
    if rc != MI355X_SUCCESS:
        msg = rt().mi355x_last_error().decode(errors="replace")
        raise MI355XError(f"{what} failed ({rc}): {msg}")


def op_reduce(op: int, ty: int, src: int, inout: int, count: int, stream: int | None = None) -> None:
    """2-buff reduction on device pointers (MPI_Reduce_local semantics)."""
    check(rt().mi355x_op_reduce(op, ty, src, inout, count, stream), "mi355x_op_reduce")


def op_reduce_3buff(op: int, ty: int, in1: int, in2: int, out: int, count: int,
                    stream: int | None = None) -> None:
    check(rt().mi355x_op_reduce_3buff(op, ty, in1, in2, out, count, stream), "mi355x_op_reduce_3buff")


def op_supported(op: int, ty: int) -> bool:
    return bool(rt().mi355x_op_supported(op, ty))


def comm_op_supported(op: int, ty: int) -> bool:
    """the collective engine folds (op, ty) on the device (op/hip's slots less the 32-byte pairs)"""
    return bool(rt().mi355x_comm_op_supported(op, ty))


def type_size(ty: int) -> int:
    return int(rt().mi355x_type_size(ty))


def set_threads(threads: int) -> None:
    check(rt().mi355x_op_set_threads(threads), "mi355x_op_set_threads")


def tune(unroll: int = 0, blocks_per_cu: int = 0, nontemporal: int = -2) -> None:
    check(rt().mi355x_op_tune(unroll, blocks_per_cu, nontemporal), "mi355x_op_tune")


def set_mode(mode: int) -> None:
    check(rt().mi355x_op_set_mode(mode), "mi355x_op_set_mode")


def get_mode() -> int:
    return int(rt().mi355x_op_get_mode())


def get_tune() -> tuple[int, int, int]:
    a, b, c = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    check(rt().mi355x_op_get_tune(ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)))
    return a.value, b.value, c.value


# ---------------------------------------------------------------- coll/mi355x engine
KNOB = {"ALLREDUCE_ALG": 1, "REDUCE_ALG": 2, "REDUCE_SCATTER_ALG": 3, "BLOCKS_PER_CU": 4, "TIMEOUT_S": 5,
        "PUSH": 6, "IPC_MAX_BYTES": 7, "STAGE_BYTES": 8,
        "LL_MAX_BYTES": 9, "REDUCE_CHAIN_FANOUT": 10, "TIME_PHASES": 11,
        "COPY_BLOCK_KIB": 12, "PIPE": 13, "PIPE_WG_PER_CU": 14, "PIPE_CHUNK_KIB": 15, "PIPE_WT": 16,
        "ONE_PHASE_MAX_BYTES": 17, "PIPE_REFUSED": 18, "SVC_MAX_BYTES": 19, "SVC_CALLS": 20,
        "SVC_LAUNCHES": 21, "SVC_RESIDENT": 22, "SVC_PULL_MAX_BYTES": 23,
        "SVC_PULL_COPY_MAX_BYTES": 24, "RCACHE_MAX_MAPS": 25, "RCACHE_SIZE_LIMIT": 26, "PEER_MAPS": 27,
        "RCACHE_EVICTIONS": 28, "FLOWS": 29, "FLOWS_FAILED": 30, "CREATE_US": 31, "SELFTEST_US": 32,
        "SVC_OWNER": 33, "SVC_CLAIMS": 34, "SVC_IDLE_US": 35,
        "SVC_SHRINK_US": 36, "SVC_REGROWS": 37, "DEV_SETUP": 38, "SETUP_US": 39, "SELFTEST": 40,
        "PIPE_CALLS": 41, "EXPORT_MISMATCHES": 42, "SELFTEST_REUSED": 43}
FLOW = {"SVC_LL": 1, "SVC_PULL": 2, "SVC_COPY": 4, "SVC_RS": 8, "PIPE": 16}
# coll/tuned COLLTYPE ids (coll_tuned.h:41-58)
COLL = {"ALLGATHER": 0, "ALLREDUCE": 2, "BCAST": 7, "REDUCE": 11, "REDUCESCATTER": 12}
AR_ALG = {"DECISION": 0, "LINEAR": 1, "NONOVERLAPPING": 2, "RECURSIVE_DOUBLING": 3, "RING": 4,
          "RING_SEGMENTED": 5}


class Comm:
    """A coll/mi355x communicator handle (multi-process via a node-local key, or one loopback
    rank).  Methods mirror the MPI calls; buffers are device pointers (ints)."""

    def __init__(self, handle: int):
        self.h = ctypes.c_void_p(handle)

    @classmethod
    def create(cls, key: str, rank: int, size: int, device: int) -> "Comm":
        h = ctypes.c_void_p()
        check(rt().mi355x_comm_create(key.encode(), rank, size, device, ctypes.byref(h)), "mi355x_comm_create")
        return cls(h.value)

    @classmethod
    def loopback(cls, size: int, device: int = 0) -> list["Comm"]:
        arr = (ctypes.c_void_p * size)()
        check(rt().mi355x_comm_create_loopback(size, device, arr), "mi355x_comm_create_loopback")
        return [cls(arr[i]) for i in range(size)]

    def destroy(self) -> None:
        if self.h:
            rt().mi355x_comm_destroy(self.h)
            self.h = ctypes.c_void_p()

    @property
    def rank(self) -> int:
        return rt().mi355x_comm_rank(self.h)

    @property
    def size(self) -> int:
        return rt().mi355x_comm_size(self.h)

    def barrier(self) -> None:
        check(rt().mi355x_comm_barrier(self.h), "mi355x_comm_barrier")

    def vote(self, device: bool) -> bool:
        """mi355x_comm_vote: this rank's buffer kind for one collective; True if the call runs in the engine"""
        anyd = ctypes.c_int(0)
        check(rt().mi355x_comm_vote(self.h, 1 if device else 0, ctypes.byref(anyd)), "mi355x_comm_vote")
        return bool(anyd.value)

    def last_algorithm(self) -> int:
        return rt().mi355x_comm_last_algorithm(self.h)

    def debug_pipe_token(self, acquire: bool) -> bool:
        """test hook: hold (or give back) this communicator's pipelined-grid token of its GPU"""
        rc = rt().mi355x_debug_pipe_token(self.h, 1 if acquire else 0)
        if rc < 0:
            check(rc, "mi355x_debug_pipe_token")
        return rc == 1

    def phase_ms(self) -> tuple[float, float]:
        """device ms of the last timed direct allreduce's two kernels (knob TIME_PHASES)"""
        a, b = ctypes.c_float(), ctypes.c_float()
        check(rt().mi355x_comm_phase_ms(self.h, ctypes.byref(a), ctypes.byref(b)), "mi355x_comm_phase_ms")
        return a.value, b.value

    def get(self, knob: str) -> int:
        v = ctypes.c_long()
        check(rt().mi355x_comm_get(self.h, KNOB[knob], ctypes.byref(v)), "mi355x_comm_get")
        return v.value

    def set(self, knob: str, value: int) -> None:
        check(rt().mi355x_comm_set(self.h, KNOB[knob], value), "mi355x_comm_set")

    def allreduce(self, sbuf, rbuf, count, ty, op, stream=None) -> None:
        check(rt().mi355x_allreduce(self.h, sbuf, rbuf, count, ty, op, stream), "mi355x_allreduce")

    def set_rules(self, rules) -> None:
        check(rt().mi355x_comm_set_rules(self.h, rules.h if rules else None), "mi355x_comm_set_rules")

    def _post(self, fn, *args) -> Request:
        h = ctypes.c_void_p()
        check(getattr(rt(), fn)(self.h, *args, ctypes.byref(h)), fn)
        return Request(h.value)

    def iallreduce(self, sbuf, rbuf, count, ty, op, stream=None) -> Request:
        return self._post("mi355x_iallreduce", sbuf, rbuf, count, ty, op, stream)

    def ireduce(self, sbuf, rbuf, count, ty, op, root, stream=None) -> Request:
        return self._post("mi355x_ireduce", sbuf, rbuf, count, ty, op, root, stream)

    def ireduce_scatter_block(self, sbuf, rbuf, rcount, ty, op, stream=None) -> Request:
        return self._post("mi355x_ireduce_scatter_block", sbuf, rbuf, rcount, ty, op, stream)

    def iallgather(self, sbuf, rbuf, nbytes, stream=None) -> Request:
        return self._post("mi355x_iallgather", sbuf, rbuf, nbytes, stream)

    def ibcast(self, buf, nbytes, root, stream=None) -> Request:
        return self._post("mi355x_ibcast", buf, nbytes, root, stream)

    def reduce(self, sbuf, rbuf, count, ty, op, root, stream=None) -> None:
        check(rt().mi355x_reduce(self.h, sbuf, rbuf, count, ty, op, root, stream), "mi355x_reduce")

    def reduce_scatter_block(self, sbuf, rbuf, rcount, ty, op, stream=None) -> None:
        check(rt().mi355x_reduce_scatter_block(self.h, sbuf, rbuf, rcount, ty, op, stream),
              "mi355x_reduce_scatter_block")

    def reduce_scatter(self, sbuf, rbuf, rcounts, ty, op, stream=None) -> None:
        arr = (ctypes.c_int * len(rcounts))(*rcounts)
        check(rt().mi355x_reduce_scatter(self.h, sbuf, rbuf, arr, ty, op, stream), "mi355x_reduce_scatter")

    def allgather(self, sbuf, rbuf, nbytes, stream=None) -> None:
        check(rt().mi355x_allgather(self.h, sbuf, rbuf, nbytes, stream), "mi355x_allgather")

    def bcast(self, buf, nbytes, root, stream=None) -> None:
        check(rt().mi355x_bcast(self.h, buf, nbytes, root, stream), "mi355x_bcast")

    # ---- gather / scatter / allgatherv / alltoall(v) (bytes) and scan / exscan (elements)
    @staticmethod
    def _sizes(v):
        return None if v is None else (ctypes.c_size_t * len(v))(*v)

    def gather(self, sbuf, rbuf, nbytes, root, stream=None) -> None:
        check(rt().mi355x_gather(self.h, sbuf, rbuf, nbytes, root, stream), "mi355x_gather")

    def gatherv(self, sbuf, sbytes, rbuf, rcounts, displs, root, stream=None) -> None:
        check(rt().mi355x_gatherv(self.h, sbuf, sbytes, rbuf, self._sizes(rcounts), self._sizes(displs), root,
                                  stream), "mi355x_gatherv")

    def scatter(self, sbuf, rbuf, nbytes, root, stream=None) -> None:
        check(rt().mi355x_scatter(self.h, sbuf, rbuf, nbytes, root, stream), "mi355x_scatter")

    def scatterv(self, sbuf, scounts, displs, rbuf, rbytes, root, stream=None) -> None:
        check(rt().mi355x_scatterv(self.h, sbuf, self._sizes(scounts), self._sizes(displs), rbuf, rbytes, root,
                                   stream), "mi355x_scatterv")

    def allgatherv(self, sbuf, sbytes, rbuf, rcounts, displs, stream=None) -> None:
        check(rt().mi355x_allgatherv(self.h, sbuf, sbytes, rbuf, self._sizes(rcounts), self._sizes(displs),
                                     stream), "mi355x_allgatherv")

    def alltoall(self, sbuf, rbuf, nbytes, stream=None) -> None:
        check(rt().mi355x_alltoall(self.h, sbuf, rbuf, nbytes, stream), "mi355x_alltoall")

    def alltoallv(self, sbuf, scounts, sdispls, rbuf, rcounts, rdispls, stream=None) -> None:
        check(rt().mi355x_alltoallv(self.h, sbuf, self._sizes(scounts), self._sizes(sdispls), rbuf,
                                    self._sizes(rcounts), self._sizes(rdispls), stream), "mi355x_alltoallv")

    def scan(self, sbuf, rbuf, count, ty, op, stream=None) -> None:
        check(rt().mi355x_scan(self.h, sbuf, rbuf, count, ty, op, stream), "mi355x_scan")

    def exscan(self, sbuf, rbuf, count, ty, op, stream=None) -> None:
        check(rt().mi355x_exscan(self.h, sbuf, rbuf, count, ty, op, stream), "mi355x_exscan")

    def iscan(self, sbuf, rbuf, count, ty, op, stream=None) -> Request:
        return self._post("mi355x_iscan", sbuf, rbuf, count, ty, op, stream)

    def ialltoall(self, sbuf, rbuf, nbytes, stream=None) -> Request:
        return self._post("mi355x_ialltoall", sbuf, rbuf, nbytes, stream)

    # ---- point-to-point, device or host buffers (count = bytes when ddt is None, else datatype
    #      instances); mode: SEND_MODE (mca_pml_base_send_mode_t)
    def isend(self, buf, count, dest, tag, ddt=None, stream=None, mode=None) -> Request:
        if mode is not None:
            return self._post("mi355x_isend_mode", buf, count, ddt.h if ddt else None, dest, tag, SEND_MODE[mode],
                              stream)
        return self._post("mi355x_isend", buf, count, ddt.h if ddt else None, dest, tag, stream)

    def improbe(self, source, tag):
        """(Message, status tuple) of the first matching message, taken out of the queue, or None"""
        flag, st, msg = ctypes.c_int(0), MsgStatus(), ctypes.c_void_p()
        check(rt().mi355x_improbe(self.h, source, tag, ctypes.byref(flag), ctypes.byref(msg), ctypes.byref(st)),
              "mi355x_improbe")
        return (msg.value, st.as_tuple()) if flag.value else None

    def imrecv(self, buf, count, msg, ddt=None, stream=None) -> Request:
        h = ctypes.c_void_p()
        check(rt().mi355x_imrecv(self.h, buf, count, ddt.h if ddt else None, msg, stream, ctypes.byref(h)),
              "mi355x_imrecv")
        return Request(h.value)

    def irecv(self, buf, count, source, tag, ddt=None, stream=None) -> Request:
        return self._post("mi355x_irecv", buf, count, ddt.h if ddt else None, source, tag, stream)

    def send(self, buf, count, dest, tag, ddt=None, stream=None, mode=None) -> None:
        if mode is not None:
            check(rt().mi355x_send_mode(self.h, buf, count, ddt.h if ddt else None, dest, tag, SEND_MODE[mode], stream),
                  "mi355x_send_mode")
            return
        check(rt().mi355x_send(self.h, buf, count, ddt.h if ddt else None, dest, tag, stream), "mi355x_send")

    def recv(self, buf, count, source, tag, ddt=None, stream=None) -> tuple[int, int, int, int]:
        st = MsgStatus()
        rc = rt().mi355x_recv(self.h, buf, count, ddt.h if ddt else None, source, tag, stream, ctypes.byref(st))
        _check_p2p(rc, "mi355x_recv", st)
        return st.as_tuple()

    def sendrecv(self, sbuf, scount, dest, stag, rbuf, rcount, source, rtag, sddt=None, rddt=None,
                 stream=None) -> tuple[int, int, int, int]:
        st = MsgStatus()
        rc = rt().mi355x_sendrecv(self.h, sbuf, scount, sddt.h if sddt else None, dest, stag, rbuf, rcount,
                                  rddt.h if rddt else None, source, rtag, stream, ctypes.byref(st))
        _check_p2p(rc, "mi355x_sendrecv", st)
        return st.as_tuple()

    def iprobe(self, source, tag):
        """status tuple of the first matching unreceived message, or None"""
        flag, st = ctypes.c_int(0), MsgStatus()
        check(rt().mi355x_iprobe(self.h, source, tag, ctypes.byref(flag), ctypes.byref(st)), "mi355x_iprobe")
        return st.as_tuple() if flag.value else None

    def progress(self) -> None:
        check(rt().mi355x_p2p_progress(self.h), "mi355x_p2p_progress")


def _check_p2p(rc: int, what: str, st: "MsgStatus") -> None:
    if rc == ERR_TRUNCATE:
        raise TruncateError(rt().mi355x_last_error().decode(errors="replace"), st.as_tuple())
    check(rc, what)


# mca_pml_base_send_mode_t (pml.h:78-85)
SEND_MODE = {"SYNCHRONOUS": 0, "COMPLETE": 1, "BUFFERED": 2, "READY": 3, "STANDARD": 4}


class Rules:
    """coll/tuned dynamic rules (mi355x_rules_t), loaded from a coll_tuned_dynamic_rules_filename file."""

    def __init__(self, path: str):
        h = ctypes.c_void_p()
        n = rt().mi355x_rules_load(str(path).encode(), ctypes.byref(h))
        if n < 0:
            check(n, "mi355x_rules_load")
        self.h = h
        self.ncoll = n

    def decide(self, coll: int, comm_size: int, msg_bytes: int) -> tuple[int, int, int]:
        a, f, g = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        check(rt().mi355x_rules_decide(self.h, coll, comm_size, msg_bytes, ctypes.byref(a), ctypes.byref(f),
                                       ctypes.byref(g)), "mi355x_rules_decide")
        return a.value, f.value, g.value

    def destroy(self) -> None:
        if self.h:
            rt().mi355x_rules_destroy(self.h)
            self.h = ctypes.c_void_p()


class Request:
    """A posted nonblocking collective or point-to-point call (mi355x_request_t)."""

    def __init__(self, h: int):
        self.h = ctypes.c_void_p(h)

    def test(self) -> bool:
        done = ctypes.c_int(0)
        rc = rt().mi355x_request_test(self.h, ctypes.byref(done))
        if rc == ERR_TRUNCATE:
            return True   # complete; wait() reports the truncation
        check(rc, "mi355x_request_test")
        return bool(done.value)

    def cancel(self) -> None:
        check(rt().mi355x_request_cancel(self.h), "mi355x_request_cancel")

    def cancelled(self) -> bool:
        f = ctypes.c_int(0)
        check(rt().mi355x_request_cancelled(self.h, ctypes.byref(f)), "mi355x_request_cancelled")
        return bool(f.value)

    def wait(self):
        """wait, free; returns the receive status tuple (source, tag, error, bytes)"""
        st = MsgStatus()
        try:
            rc = rt().mi355x_request_wait(self.h)
            rt().mi355x_request_get_status(self.h, ctypes.byref(st))
            _check_p2p(rc, "mi355x_request_wait", st)
        finally:
            rt().mi355x_request_free(self.h)
            self.h = ctypes.c_void_p()
        return st.as_tuple()


class Ddt:
    """A GPU-convertor datatype layout (mi355x_ddt_t)."""

    def __init__(self, h):
        self.h = h

    @classmethod
    def vector(cls, count, blocklen, stride, elem_size):
        h = ctypes.c_void_p()
        check(rt().mi355x_ddt_create_vector(count, blocklen, stride, elem_size, ctypes.byref(h)), "ddt vector")
        return cls(h)

    @classmethod
    def indexed(cls, blocklens, disps, elem_size):
        n = len(blocklens)
        h = ctypes.c_void_p()
        check(rt().mi355x_ddt_create_indexed(n, (ctypes.c_int * n)(*blocklens), (ctypes.c_int * n)(*disps),
                                             elem_size, ctypes.byref(h)), "ddt indexed")
        return cls(h)

    @classmethod
    def runs(cls, disps, lens, nblk=1, stride=0, extent=0):
        n = len(disps)
        h = ctypes.c_void_p()
        check(rt().mi355x_ddt_create((ctypes.c_int64 * n)(*disps), (ctypes.c_int64 * n)(*lens), n, nblk, stride,
                                     extent, ctypes.byref(h)), "ddt create")
        return cls(h)

    @classmethod
    def from_opal(cls, desc_bytes: bytes, used: int, extent: int, basic_sizes):
        h = ctypes.c_void_p()
        buf = ctypes.create_string_buffer(desc_bytes, len(desc_bytes))
        bs = (ctypes.c_uint32 * len(basic_sizes))(*basic_sizes)
        check(rt().mi355x_ddt_from_opal(buf, used, extent, bs, ctypes.byref(h)), "ddt from opal")
        return cls(h)

    @property
    def size(self):
        return int(rt().mi355x_ddt_size(self.h))

    @property
    def extent(self):
        return int(rt().mi355x_ddt_extent(self.h))

    @property
    def nruns(self):
        return int(rt().mi355x_ddt_nruns(self.h))

    def pack(self, count, base, pos, dst, nbytes, stream=None, checksum=False):
        cs = ctypes.c_uint32()
        check(rt().mi355x_pack(self.h, count, base, pos, dst, nbytes, ctypes.byref(cs) if checksum else None, stream),
              "mi355x_pack")
        return cs.value if checksum else None

    def unpack(self, count, base, pos, src, nbytes, stream=None, checksum=False):
        cs = ctypes.c_uint32()
        check(rt().mi355x_unpack(self.h, count, base, pos, src, nbytes, ctypes.byref(cs) if checksum else None,
                                 stream), "mi355x_unpack")
        return cs.value if checksum else None

    def pack_host(self, count, base, pos, dst, nbytes):
        """the same window on host memory (no GPU)"""
        check(rt().mi355x_pack_host(self.h, count, base, pos, dst, nbytes), "mi355x_pack_host")

    def unpack_host(self, count, base, pos, src, nbytes):
        check(rt().mi355x_unpack_host(self.h, count, base, pos, src, nbytes), "mi355x_unpack_host")

    def raw(self, count, iov_num=5):
        """opal_convertor_raw's walk: a list of calls, each a list of (offset, length) pieces of at
        most iov_num entries; the last call returns 1 (no GPU)"""
        pos = ctypes.c_size_t(0)
        calls = []
        while True:
            disp = (ctypes.c_int64 * iov_num)()
            lens = (ctypes.c_size_t * iov_num)()
            cnt, got = ctypes.c_uint32(iov_num), ctypes.c_size_t(0)
            rc = rt().mi355x_ddt_raw(self.h, count, ctypes.byref(pos), disp, lens, ctypes.byref(cnt), ctypes.byref(got))
            if rc < 0:
                check(rc, "mi355x_ddt_raw")
            calls.append([(disp[k], lens[k]) for k in range(cnt.value)])
            assert sum(ln for _, ln in calls[-1]) == got.value
            if rc == 1:
                return calls

    def destroy(self):
        if self.h:
            rt().mi355x_ddt_destroy(self.h)
            self.h = None


def ddt_tune(unroll_pack: int = 0, unroll_unpack: int = 0, threads: int = 0, nontemporal: int = -2) -> None:
    """launch shape of the single-run pack/unpack kernel (see mi355x_ddt_tune)"""
    check(rt().mi355x_ddt_tune(unroll_pack, unroll_unpack, threads, nontemporal), "mi355x_ddt_tune")


def ddt_tune_rows(mode: int) -> None:
    """pack/unpack kernel choice (mi355x_ddt_tune_rows): 2 default, 3 unit kernel with W-byte units
    only, 1 16-B row kernel only, 0 the general kernel only"""
    check(rt().mi355x_ddt_tune_rows(mode), "mi355x_ddt_tune_rows")


def sched_program(kind: int, n: int, alg: int, block: int) -> list[int]:
    buf = (ctypes.c_int * 4096)()
    k = rt().mi355x_sched_program(kind, n, alg, block, buf, 4096)
    check(0 if k >= 0 else k, "mi355x_sched_program")
    return list(buf[:k])


def env_flag(name: str, default: str = "") -> str:
    return os.environ.get(name, default)
