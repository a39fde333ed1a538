"""The drop-in boundary, checked on CPU (no GPU needed):

* libmi355x_rt.so exports every entry point include/mi355x_rt.h declares;
* mca_op_hip.so / mca_coll_mi355x.so export the MCA component symbols (mca_<type>_<name>_component,
  opal/mca/base/mca_base_component_find.c:619-631) and the reference-signature entry points;
* the component structs carry the framework names/versions the MCA loader checks;
* the ABI mirror (include/ompi_abi.h) has the offsets derived from the reference definitions;
* op/hip goes through the restated ompi_op_base_op_select: every GPU slot is installed, the NULL
  pattern of the base table is kept, host buffers are routed to the base (reference) loops, and
  the module reference counts balance despite op_base_op_select.c:162-168;
* coll/mi355x's comm_query installs exactly the five collectives and declines where coll/tuned
  does (inter-communicators, size 1) and for multi-node jobs.
"""
from __future__ import annotations

import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import opdata
from conftest import REPO
from mini import mini


def _declared(header):
    txt = (REPO / "include" / header).read_text()
    return sorted(set(re.findall(r"^\s*(?:int|void|size_t|const char \*)\s*\*?(mi355x_\w+)\s*\(", txt, re.M)))


def _exports(so):
    out = subprocess.check_output(["nm", "-D", "--defined-only", str(so)], text=True)
    return {ln.split()[-1] for ln in out.splitlines() if ln.strip()}


def test_rt_exports_every_declared_symbol(pkg):
    names = _declared("mi355x_rt.h")
    assert len(names) >= 40, names
    ex = _exports(pkg.lib_path())
    missing = [n for n in names if n not in ex]
    assert not missing, missing


def test_component_symbols(pkg):
    op = _exports(pkg.lib_path("mca_op_hip.so"))
    for s in ("mca_op_hip_component", "mca_op_hip_2buff", "mca_op_hip_3buff"):
        assert s in op
    coll = _exports(pkg.lib_path("mca_coll_mi355x.so"))
    for s in ("mca_coll_mi355x_component", "mca_coll_mi355x_allreduce", "mca_coll_mi355x_reduce_scatter_block",
              "mca_coll_mi355x_reduce_scatter", "mca_coll_mi355x_allgather", "mca_coll_mi355x_bcast",
              "mca_coll_mi355x_reduce", "mca_coll_mi355x_iallreduce", "mca_coll_mi355x_ireduce",
              "mca_coll_mi355x_ireduce_scatter_block", "mca_coll_mi355x_iallgather", "mca_coll_mi355x_ibcast",
              "mca_coll_mi355x_gather", "mca_coll_mi355x_gatherv", "mca_coll_mi355x_scatter",
              "mca_coll_mi355x_scatterv", "mca_coll_mi355x_allgatherv", "mca_coll_mi355x_alltoall",
              "mca_coll_mi355x_alltoallv", "mca_coll_mi355x_scan", "mca_coll_mi355x_exscan"):
        assert s in coll


class _Comp(ctypes.Structure):
    _fields_ = [("maj", ctypes.c_int), ("min", ctypes.c_int), ("rel", ctypes.c_int),
                ("type_name", ctypes.c_char * 32), ("tmaj", ctypes.c_int), ("tmin", ctypes.c_int),
                ("trel", ctypes.c_int), ("name", ctypes.c_char * 64)]


def test_component_headers():
    m = mini()
    op = _Comp.from_address(m.component_ptr(m.op_hip, "mca_op_hip_component"))
    assert (op.maj, op.min, op.rel) == (2, 0, 0)
    assert op.type_name == b"op" and (op.tmaj, op.tmin, op.trel) == (1, 0, 0) and op.name == b"hip"
    co = _Comp.from_address(m.component_ptr(m.coll, "mca_coll_mi355x_component"))
    assert co.type_name == b"coll" and (co.tmaj, co.tmin, co.trel) == (2, 0, 0) and co.name == b"mi355x"


def test_abi_offsets():
    """offsets derived by hand from the reference struct definitions (x86-64, non-debug)"""
    L = mini().lib
    want = {
        0: 16 + 64 + 4 + 4,          # ompi_op_t.o_f_to_c_index (op.h:138-188)
        1: 96,                       # ompi_op_t.o_func
        2: 96 + 39 * 8 * 2,          # ompi_op_t.o_3buff_intrinsic (union = intrinsic fns+modules)
        3: 32,                       # ompi_op_base_module_t.opm_fns (op.h:357-373)
        4: 32 + 39 * 8,              # ompi_op_base_module_t.opm_3buff_fns
        5: 368,                      # ompi_datatype_t.id = sizeof(opal_datatype_t)
        6: 24,                       # opal_datatype_t.size
        12: 3 * 4 + 32 + 3 * 4 + 64 + 3 * 4 + 4 + 4 * 8 + 32,  # mca_base_component_2_0_0_t
        13: 368,
        14: 368 + 4 + 4 + 8 + 8 + 8 + 64,
        10: 16 + 8 + 2 * 8,          # coll module: allreduce is the 3rd fn after enable
        11: 16 + 8 + 44 * 8,         # ft_event after 17 + 17 + 10 fns
        16: 44 * 16,                 # mca_coll_base_comm_coll_t: 44 (fn, module) pairs
        17: 16 + 8 + 19 * 8,         # coll module: iallreduce = 3rd nonblocking fn (coll.h:418-420)
        # ompi_request_t (request.h:98-110): free-list item 56 B (list item 40 = object 16 +
        # next/prev 16 + item_free 4 + pad), req_type 4 + pad, status 24, flags, 4 fn pointers, union
        18: 144,
        19: 64,                      # req_status
        20: 104,                     # req_free
        21: 19 * 16,                 # comm coll table: iallreduce pair after 17 blocking + 2
        22: 8 * 32,                  # ompi_predefined_request_t padded to 32 pointers
        23: 16 + 8 + 14 * 8,         # coll module: scan = 15th blocking fn (coll.h:390-409)
        24: 16 * 16,                 # comm coll table: scatterv pair = 17th (coll.h:469-504)
        25: 9 * 16,                  # comm coll table: gather pair = 10th
        # mca_pml_base_module_t (pml.h:497-531): 21 function pointers, then two 4-byte limits
        26: 7 * 8,                   # pml_irecv: 8th (add/del procs, enable, progress, add/del comm, irecv_init)
        27: 10 * 8,                  # pml_isend: 11th
        28: 13 * 8,                  # pml_probe: 14th
        29: 21 * 8 + 4,              # pml_max_tag after pml_max_contextid
        30: 21 * 8 + 8,
        31: 4 * 4 + 8,               # ompi_status_public_t (mpi.h.in:344-356)
    }
    for k, v in want.items():
        assert L.mini_offsetof(k) == v, (k, L.mini_offsetof(k), v)
    # communicator: c_contextid right after the 64-B name that follows the 64-B opal_mutex_t
    assert L.mini_offsetof(15) == 16 + 64 + 64
    assert L.mini_offsetof(7) == L.mini_offsetof(15) + 4


@pytest.mark.parametrize("opname", ["MAX", "MIN", "SUM", "PROD", "LAND", "BAND", "LOR", "BOR", "LXOR", "BXOR",
                                    "MAXLOC", "MINLOC"])
def test_op_select_installs_and_routes_host(pkg, oracle, opname):
    m = mini()
    m.install_oracle_base(oracle)
    code = pkg.OP[opname]
    op = m.select_op(code)
    f2 = m.addr(m.op_hip, "mca_op_hip_2buff")
    hip_mod = None
    installed = 0
    for slot in range(39):
        base = oracle.oracle_has_op(code, slot)
        fn = m.lib.mini_op_fn2(op, slot)
        assert bool(fn) == bool(base), slot          # NULL pattern kept (op_base_op_select.c:185-201)
        if base and pkg.op_supported(code, slot):
            assert fn == f2, (opname, slot)
            installed += 1
            hip_mod = m.lib.mini_op_module2(op, slot)
            assert m.lib.mini_op_module3(op, slot) == hip_mod
    assert installed == sum(pkg.op_supported(code, t) for t in range(39))
    # references held by the op's tables == the module's count, despite :162-168
    nslots = sum(1 for t in range(39) if m.lib.mini_op_module2(op, t) == hip_mod) + \
        sum(1 for t in range(39) if m.lib.mini_op_module3(op, t) == hip_mod)
    assert m.lib.mini_obj_refcount(hip_mod) == nslots
    # host buffers are reduced by the base (reference) loop: MPI_Reduce_local semantics
    for slot in range(39):
        if not oracle.oracle_has_op(code, slot):
            continue
        dt = m.dtype_for_slot(slot)
        if dt is None:
            continue
        tname = pkg.TYPES[slot]
        a = opdata.make(tname, 97, 1)
        b = opdata.make(tname, 97, 2)
        want = b.copy()
        oracle.oracle_op_2buff(code, slot, a.ctypes.data, want.ctypes.data, 97)
        got = b.copy()
        m.lib.mini_op_reduce(op, a.ctypes.data, got.ctypes.data, 97, dt)
        opdata.assert_same(tname, opname, got, want, "host route")
    m.lib.mini_op_destroy(op)   # must not double free


def _coll_env(monkeypatch, world=4, local=4):
    monkeypatch.setenv("OMPI_COMM_WORLD_SIZE", str(world))
    monkeypatch.setenv("OMPI_COMM_WORLD_LOCAL_SIZE", str(local))


class _CollComp(ctypes.Structure):
    _fields_ = [("version", ctypes.c_char * (200)), ("data", ctypes.c_char * 36),
                ("init_query", ctypes.c_void_p), ("comm_query", ctypes.c_void_p)]


def _comm_query(m, comm):
    comp = _CollComp.from_address(m.component_ptr(m.coll, "mca_coll_mi355x_component"))
    fn = ctypes.CFUNCTYPE(ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int))(comp.comm_query)
    prio = ctypes.c_int(-1)
    mod = fn(comm, ctypes.byref(prio))
    return mod, prio.value


def test_coll_comm_query(monkeypatch):
    m = mini()
    assert ctypes.sizeof(_CollComp) >= 200
    _coll_env(monkeypatch)
    comm = m.lib.mini_comm_create(0, 4, 7)
    mod, prio = _comm_query(m, comm)
    assert mod and prio == 90
    # the module provides exactly allreduce, reduce_scatter(_block), allgather, bcast, reduce
    m.lib.mini_comm_install(comm, mod)
    names = ["mca_coll_mi355x_allreduce", "mca_coll_mi355x_reduce_scatter_block", "mca_coll_mi355x_reduce_scatter",
             "mca_coll_mi355x_allgather", "mca_coll_mi355x_bcast", "mca_coll_mi355x_reduce",
             "mca_coll_mi355x_iallreduce", "mca_coll_mi355x_ireduce", "mca_coll_mi355x_ireduce_scatter_block",
             "mca_coll_mi355x_iallgather", "mca_coll_mi355x_ibcast"]
    for which, n in enumerate(names):
        assert m.lib.mini_comm_fn(comm, which) == m.addr(m.coll, n)
    m.lib.mini_comm_destroy(comm)
    # declines: size 1, multi-node job
    one = m.lib.mini_comm_create(0, 1, 8)
    assert _comm_query(m, one)[0] is None
    _coll_env(monkeypatch, world=16, local=8)
    c2 = m.lib.mini_comm_create(0, 4, 9)
    assert _comm_query(m, c2)[0] is None


def _chan_rank(rank, size, name, q):
    try:
        m = mini()
        L = m.lib
        comm = L.mini_comm_create(rank, size, 11)
        assert L.mini_comm_set_channel(comm, name.encode()) == 0
        L.mini_comm_install(comm, L.mini_stub_module())
        byte = ctypes.addressof(ctypes.c_char.in_dll(L, "ompi_mpi_byte"))
        for k in range(50):
            root = k % size
            buf = (ctypes.c_char * 64)()
            if rank == root:
                buf.value = f"key-{k}-{root}".encode()
            assert L.mini_bcast(comm, ctypes.addressof(buf), 64, byte, root) == 0
            assert buf.value == f"key-{k}-{root}".encode(), (k, buf.value)
        L.mini_comm_destroy(comm)
        q.put((rank, "ok"))
    except BaseException as e:  # noqa: BLE001
        q.put((rank, repr(e)))


def test_harness_host_bcast_channel():
    """the harness's stand-in for the lower-priority modules' host transport (what coll/mi355x's
    module_enable uses to agree on its rendezvous key): 3 processes, 50 bcasts with rotating roots"""
    import multiprocessing as mp
    import uuid
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    name = "t" + uuid.uuid4().hex[:10]
    ps = [ctx.Process(target=_chan_rank, args=(r, 3, name, q)) for r in range(3)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(30)
    assert res == {0: "ok", 1: "ok", 2: "ok"}, res


def test_pml_hook_install_and_close():
    """coll/mi355x's init_query hooks the PML slot only when a device is there (and
    OMPI_MCA_coll_mi355x_pml_hook is not 0); component close puts the saved entries back"""
    m = mini()
    L = m.lib
    comp = m.component_ptr(m.coll, "mca_coll_mi355x_component")
    saved = [L.mini_pml_fn(w) for w in range(6)]
    names = ["isend", "send", "irecv", "recv", "iprobe", "probe"]
    rc = L.mini_coll_init(comp)
    now = [L.mini_pml_fn(w) for w in range(6)]
    if rc != 0:  # no GPU here: the component declines and the PML is untouched
        assert now == saved
    else:
        assert now == [m.addr(m.coll, f"mca_coll_mi355x_pml_{n}") for n in names]
    assert L.mini_coll_close(comp) == 0
    assert [L.mini_pml_fn(w) for w in range(6)] == saved


def test_mca_variables_registered(monkeypatch):
    """coll_mi355x_priority / _allreduce_algorithm / _pml_hook / _mixed_buffers and op_hip_priority go through
    mca_base_component_var_register when the process provides it (here: the harness's variable
    system standing in for libopen-pal, which reads OMPI_MCA_<name>); the stored value is what
    comm_query / op_query then use"""
    m = mini()
    L = m.lib
    coll = m.component_ptr(m.coll, "mca_coll_mi355x_component")
    oph = m.component_ptr(m.op_hip, "mca_op_hip_component")
    prio = ctypes.c_int.in_dll(m.coll, "mca_coll_mi355x_priority")
    oprio = ctypes.c_int.in_dll(m.op_hip, "mca_op_hip_priority")
    saved = prio.value, oprio.value
    try:
        monkeypatch.setenv("OMPI_MCA_coll_mi355x_priority", "77")
        monkeypatch.setenv("OMPI_MCA_op_hip_priority", "33")
        monkeypatch.setenv("OMPI_MCA_coll_mi355x_rcache_size_limit", str(3 << 30))
        assert L.mini_component_register(coll) == 0 and L.mini_component_register(oph) == 0
        names = {L.mini_var_name(i).decode(): L.mini_var_int(i) for i in range(L.mini_var_count())}
        assert names["coll_mi355x_priority"] == 77 and prio.value == 77
        assert names["op_hip_priority"] == 33 and oprio.value == 33
        assert "coll_mi355x_allreduce_algorithm" in names and names["coll_mi355x_pml_hook"] == 1
        assert names["coll_mi355x_mixed_buffers"] == 1  # mixed host / device buffers: on by default
        # the peer-mapping cache bounds (mpool_rgpusm_rcache_size_limit: bytes, unsigned long long)
        assert names["coll_mi355x_rcache_max_maps"] == 0
        assert ctypes.c_ulonglong.in_dll(m.coll, "mca_coll_mi355x_rcache_size_limit").value == 3 << 30
        # the engine's crossovers (coll_tuned_component.c:115-170 style), with the engine's defaults
        engine_vars = {"pipe_min_ranks": 4, "pipe_chunk_kib": 0, "pipe_wg_per_cu": 2, "pipe_wt": 1,
                       "one_phase_max": 1 << 20, "svc_max": 32 << 10, "svc_pull_max": 128 << 10,
                       "svc_copy_max": 1 << 20, "svc_idle_us": 1000, "svc_shrink_us": 100, "selftest": 1,
                       "timeout_s": 0}
        for name, dflt in engine_vars.items():
            assert names.get("coll_mi355x_" + name) == dflt, (name, names.get("coll_mi355x_" + name))
        _coll_env(monkeypatch)
        comm = L.mini_comm_create(0, 4, 17)
        mod, p = _comm_query(m, comm)
        assert mod and p == 77
    finally:
        prio.value, oprio.value = saved
        ctypes.c_ulonglong.in_dll(m.coll, "mca_coll_mi355x_rcache_size_limit").value = 0


# ---- the MPI-2 pair types as libmpi builds them (DECLARE_MPI2_COMPOSED_{STRUCT,BLOCK}_DDT,
#      ompi_datatype_module.c:391-437, instantiated :471-509) and the engine's datatype gate
OMPI_PREDEFINED, OMPI_DATA_INT, OMPI_DATA_C = 0x0200, 0x1000, 0x4000   # ompi_datatype.h:51-59
OPAL_PREDEFINED = 0x0002                                               # opal_datatype.h:66
PAIRS = {  # name: (ompi id, struct members as (opal basic, displacement) | block of 2, extra flags)
    "2INT": (0x1A, "block", "INT4", OMPI_DATA_C | OMPI_DATA_INT),
    "FLOAT_INT": (0x20, [("FLOAT4", 0), ("INT4", 4)], None, OMPI_DATA_C),
    "DOUBLE_INT": (0x21, [("FLOAT8", 0), ("INT4", 8)], None, OMPI_DATA_C),
    "LONG_DOUBLE_INT": (0x22, [("FLOAT16", 0), ("INT4", 16)], None, OMPI_DATA_C),
    "LONG_INT": (0x23, [("INT8", 0), ("INT4", 8)], None, OMPI_DATA_C | OMPI_DATA_INT),
    "SHORT_INT": (0x24, [("INT2", 0), ("INT4", 4)], None, OMPI_DATA_C | OMPI_DATA_INT),
}


def _restated_pair(name):
    """the pair type through the restated opal_datatype_add (oracle/opal_types.py), then the
    OPAL -> OMPI predefined flag swap of ompi_datatype_module.c:415-416 / :431-432"""
    import opal_types as ot
    _, members, block, extra = PAIRS[name]
    if members == "block":
        t = ot.contiguous(2, ot.OpalType.basic(block))
    else:
        t = ot.struct_([1, 1], [d for _, d in members], [ot.OpalType.basic(b) for b, _ in members])
    t.commit()
    flags = (t.flags | extra) & ~OPAL_PREDEFINED | OMPI_PREDEFINED
    return t, flags


@pytest.mark.parametrize("name", list(PAIRS))
def test_pair_types_as_libmpi_builds_them(name):
    """the harness's pair types carry what a real Open MPI 1.8.5 passes: OPAL predefined flag
    cleared, MPI predefined set, the struct's size / bounds / contiguity (DOUBLE_INT and LONG_INT
    12 bytes in a 16-byte extent, SHORT_INT 6 with a hole in 8, LONG_DOUBLE_INT 20 in 32) and its
    committed description records"""
    import sys
    sys.path.insert(0, str(REPO / "oracle"))
    m = mini()
    L = m.lib
    L.mini_datatype_fields.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64)]
    L.mini_datatype_desc.restype = ctypes.c_void_p
    L.mini_datatype_desc.argtypes = [ctypes.c_void_p]
    t, flags = _restated_pair(name)
    dt = L.mini_datatype(PAIRS[name][0])
    f = (ctypes.c_int64 * 7)()
    L.mini_datatype_fields(dt, f)
    assert list(f[:6]) == [flags, t.size, t.lb, t.ub, t.true_lb, t.true_ub], (name, list(f), flags, t.size, t.ub)
    assert not (f[0] & OPAL_PREDEFINED) and f[0] & OMPI_PREDEFINED
    desc = t.desc_bytes()
    assert f[6] * 32 + 32 == len(desc)           # `used` excludes commit's END_LOOP (optimize.c:257)
    assert ctypes.string_at(L.mini_datatype_desc(dt), len(desc)) == desc
    # the engine's gate: the pair's op slot, by MPI-predefined flag + ompi_op_ddt_map + extent
    L2 = m.coll
    L2.mca_coll_mi355x_reducible_type.argtypes = [ctypes.c_void_p]
    assert L2.mca_coll_mi355x_reducible_type(dt) == m.pkg.T[name]
    assert m.pkg.type_size(m.pkg.T[name]) == t.ub - t.lb


def test_reducible_type_gate(pkg):
    """every predefined reducible type maps to its slot; a derived type, a resized predefined-id
    type and a type offset from its lower bound do not"""
    m = mini()
    fn = m.coll.mca_coll_mi355x_reducible_type
    fn.argtypes = [ctypes.c_void_p]
    for slot in range(39):
        dt = m.dtype_for_slot(slot)
        if dt is not None:
            assert fn(dt) == slot, pkg.TYPES[slot]
    import ddtcases
    desc, used, tsize, lb, ub = ddtcases.opal_vector(4, 4, 8)
    d = m.derived(desc, used, tsize, lb, ub)
    assert fn(d) == -1
    m.lib.mini_datatype_destroy(d)
