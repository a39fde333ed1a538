"""op/hip and coll/mi355x driven exactly as Open MPI drives them (restated selection + dispatch
in the mini-OMPI harness), on device buffers, vs the oracle.

* op/hip: every slot through ompi_op_reduce / ompi_3buff_op_reduce dispatch with device
  operands; mixed host/device operands; x87 long double slots staged to the base loop.
* coll/mi355x: two processes each select the component over a stub lower-priority module, then
  MPI_Allreduce / MPI_Reduce_scatter_block / MPI_Allgather / MPI_Bcast on device buffers go
  through the engine (checked vs the oracle), and host buffers go to the stub.
"""
from __future__ import annotations

import ctypes
import os
import pathlib
import subprocess
import sys
import uuid

import numpy as np
import pytest

import opdata
from mini import mini

pytestmark = pytest.mark.gpu
HERE = pathlib.Path(__file__).parent


def _dev(torch, a):
    return torch.from_numpy(a.view(np.uint8).copy()).cuda()


def test_op_hip_device_dispatch(gpu, pkg, oracle):
    torch = gpu
    m = mini()
    m.install_oracle_base(oracle)
    n = 10_007
    bad = []
    for code in range(1, 13):
        op = m.select_op(code)
        for slot in range(39):
            if not oracle.oracle_has_op(code, slot):
                continue
            dt = m.dtype_for_slot(slot)
            if dt is None:
                continue
            tname, opname = pkg.TYPES[slot], pkg.OPS[code]
            a = opdata.make(tname, n, 1)
            b = opdata.make(tname, n, 2)
            da, db = _dev(torch, a), _dev(torch, b)
            torch.cuda.synchronize()
            m.lib.mini_op_reduce(op, da.data_ptr(), db.data_ptr(), n, dt)        # device / device
            want = b.copy()
            oracle.oracle_op_2buff(code, slot, a.ctypes.data, want.ctypes.data, n)
            got = db.cpu().numpy().view(a.dtype)
            try:
                opdata.assert_same(tname, opname, got, want, "2buff dev")
            except AssertionError as e:
                bad.append(str(e))
            hb = b.copy()                                                          # device in, host inout
            m.lib.mini_op_reduce(op, da.data_ptr(), hb.ctypes.data, n, dt)
            try:
                opdata.assert_same(tname, opname, hb, want, "2buff mixed")
            except AssertionError as e:
                bad.append(str(e))
            do = torch.empty_like(da)
            m.lib.mini_op_reduce_3buff(op, da.data_ptr(), _dev(torch, b).data_ptr(), do.data_ptr(), n, dt)
            want3 = np.zeros_like(a)
            oracle.oracle_op_3buff(code, slot, a.ctypes.data, b.ctypes.data, want3.ctypes.data, n)
            try:
                opdata.assert_same(tname, opname, do.cpu().numpy().view(a.dtype), want3, "3buff dev")
            except AssertionError as e:
                bad.append(str(e))
        m.lib.mini_op_destroy(op)
    assert not bad, "\n".join(bad[:10])


def test_op_hip_concurrent_callers(gpu, pkg, oracle):
    """MPI_THREAD_MULTIPLE: several threads reduce through the same MPI_Op's table at once, all-
    device operands (the lock-free path) mixed with staged host operands (the locked path); every
    result must match the oracle"""
    import threading
    torch = gpu
    m = mini()
    m.install_oracle_base(oracle)
    code, slot = pkg.OP["SUM"], pkg.T["INT32"]
    op = m.select_op(code)
    dt = m.dtype_for_slot(slot)
    n, iters, nthreads = 300_001, 25, 6
    errors = []

    def worker(k):
        try:
            a = np.arange(n, dtype=np.int32) * (k + 1)
            da = torch.from_numpy(a).cuda()
            for it in range(iters):
                b = np.full(n, it - k, dtype=np.int32)
                want = b + a
                if k % 3 == 2:  # host inout: staged through the module's scratch under its lock
                    m.lib.mini_op_reduce(op, da.data_ptr(), b.ctypes.data, n, dt)
                    got = b
                else:
                    db = torch.from_numpy(b).cuda()
                    torch.cuda.synchronize()
                    m.lib.mini_op_reduce(op, da.data_ptr(), db.data_ptr(), n, dt)
                    got = db.cpu().numpy()
                if not np.array_equal(got, want):
                    errors.append((k, it))
        except Exception as e:  # noqa: BLE001
            errors.append((k, repr(e)))

    ts = [threading.Thread(target=worker, args=(k,)) for k in range(nthreads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(120)
    m.lib.mini_op_destroy(op)
    assert not errors, errors[:5]


@pytest.mark.parametrize("size", [2, 3, 4])  # 4: the pipelined allreduce is the default from 4 ranks
def test_coll_component_processes(gpu, size):
    key = uuid.uuid4().hex[:10]
    env = dict(os.environ, MI355X_TIMEOUT_S="60", OMPI_COMM_WORLD_SIZE=str(size),
               OMPI_COMM_WORLD_LOCAL_SIZE=str(size), OMPI_MCA_ess_base_jobid=key)
    procs = []
    for r in range(size):
        e = dict(env, OMPI_COMM_WORLD_LOCAL_RANK=str(r), OMPI_COMM_WORLD_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, str(HERE / "coll_worker.py"), str(r), str(size), key], env=e,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=300)
        except subprocess.TimeoutExpired:
            p.kill()
            out, _ = p.communicate()
        outs.append(out)
    for r, p in enumerate(procs):
        assert p.returncode == 0, f"rank {r}:\n{outs[r][-3000:]}"


def test_split_communicators_same_cid(gpu):
    """two disjoint 2-rank communicators of one job with the same context id (the MPI_Comm_split
    case, comm.c:610) selecting coll/mi355x and running collectives concurrently: the rendezvous
    key is agreed per communicator (rank 0 picks it, the lower-priority bcast spreads it), so the
    groups never meet in one control segment"""
    key = uuid.uuid4().hex[:10]
    env = dict(os.environ, MI355X_TIMEOUT_S="60", OMPI_COMM_WORLD_SIZE="4", OMPI_COMM_WORLD_LOCAL_SIZE="4",
               OMPI_MCA_ess_base_jobid=key)
    procs = [subprocess.Popen([sys.executable, str(HERE / "coll_worker.py"), str(w), "4", key, "split"],
                              env=dict(env, OMPI_COMM_WORLD_LOCAL_RANK=str(w), OMPI_COMM_WORLD_RANK=str(w)),
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True) for w in range(4)]
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=300)
        except subprocess.TimeoutExpired:
            p.kill()
            out, _ = p.communicate()
        outs.append(out)
    for w, p in enumerate(procs):
        assert p.returncode == 0 and f"rank {w} split OK" in outs[w], f"rank {w}:\n{outs[w][-3000:]}"


def _run_workers(size, mode, extra_env=None, timeout=300):
    """coll_worker.py <rank> <size> <key> <mode> as `size` processes; every rank must print
    'rank <r> <mode> OK'"""
    key = uuid.uuid4().hex[:10]
    env = dict(os.environ, MI355X_TIMEOUT_S="60", OMPI_COMM_WORLD_SIZE=str(size),
               OMPI_COMM_WORLD_LOCAL_SIZE=str(size), OMPI_MCA_ess_base_jobid=key, **(extra_env or {}))
    for k in [k for k in env if k.startswith("OMPI_MCA_coll_tuned_")]:
        del env[k]   # coll/tuned's variables come from the variable system in these tests
    procs = [subprocess.Popen([sys.executable, str(HERE / "coll_worker.py"), str(r), str(size), key, mode],
                              env=dict(env, OMPI_COMM_WORLD_LOCAL_RANK=str(r), OMPI_COMM_WORLD_RANK=str(r)),
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True) for r in range(size)]
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            p.kill()
            out, _ = p.communicate()
        outs.append(out)
    for r, p in enumerate(procs):
        assert p.returncode == 0 and f"rank {r} {mode} OK" in outs[r], f"rank {r}:\n{outs[r][-3000:]}"


@pytest.mark.parametrize("size", [2, 3])
def test_pml_slot_device_p2p(gpu, size):
    """MPI point-to-point through the PML slot (`mca_pml`): coll/mi355x's init_query hooks the
    selected PML the way pml/v does (pml_v_component.c:110-131); on the engine communicator every
    call -- MPI_Send/Ssend/Bsend/Recv/Isend/Irecv/Iprobe/Probe, persistent Send_init/Recv_init/Start,
    Mprobe/Mrecv/Improbe/Imrecv, Cancel -- goes to the engine's one matching queue whatever the
    buffer kinds (dev->host, host->dev, dev->dev, host->host; ANY_SOURCE and same-tag order across
    kinds; derived types either side), nothing reaches the saved PML, close restores the table"""
    _run_workers(size, "pml")


def test_tuned_variables_through_mca_var_system(gpu):
    """coll/tuned's use_dynamic_rules / allreduce_algorithm / dynamic_rules_filename as the MCA
    variable system holds them (registered the way tuned_register does, values from a parameter
    file, nothing in the environment) reach the engine: the forced algorithm's operand order,
    then the rules file's (coll_tuned_component.c:151-167, coll_tuned_allreduce.c:949-1005)"""
    _run_workers(2, "tuned_vars")


def test_pml_hook_opt_out(gpu, monkeypatch):
    """coll_mi355x_pml_hook=0 (MCA variable, here through OMPI_MCA_*) leaves the PML table alone;
    by default init_query hooks it and close restores it"""
    m = mini()
    L = m.lib
    comp = m.component_ptr(m.coll, "mca_coll_mi355x_component")
    saved = [L.mini_pml_fn(w) for w in range(6)]
    hook = ctypes.c_int.in_dll(m.coll, "mca_coll_mi355x_pml_hook")
    try:
        monkeypatch.setenv("OMPI_MCA_coll_mi355x_pml_hook", "0")
        assert L.mini_component_register(comp) == 0 and hook.value == 0
        assert L.mini_coll_init(comp) == 0
        assert [L.mini_pml_fn(w) for w in range(6)] == saved, "opted out, yet the PML was hooked"
        assert L.mini_coll_close(comp) == 0
        monkeypatch.setenv("OMPI_MCA_coll_mi355x_pml_hook", "1")
        assert L.mini_component_register(comp) == 0 and hook.value == 1
        assert L.mini_coll_init(comp) == 0
        assert L.mini_pml_fn(1) == m.addr(m.coll, "mca_coll_mi355x_pml_send")
    finally:
        assert L.mini_coll_close(comp) == 0
        hook.value = 1
    assert [L.mini_pml_fn(w) for w in range(6)] == saved


@pytest.mark.parametrize("size", [2, 3])
def test_declined_reductions_staged_through_host(gpu, size):
    """coll/cuda's host staging (coll_cuda_allreduce.c:43-75, coll_cuda_reduce.c,
    coll_cuda_reduce_scatter_block.c:45-83, coll_cuda_scan.c, coll_cuda_exscan.c) for every reduction
    the engine declines, over a lower-priority module that reduces on the CPU and fails on device
    memory: a user MPI_Op on device buffers, blocking and
    nonblocking, exact; MAXLOC/MINLOC over all six pair types (flags as libmpi sets them; the 32-byte
    MPI_LONG_DOUBLE_INT through the gather-then-fold form) and MAX/MIN over MPI_LONG_DOUBLE served by
    the engine, exact vs the oracle"""
    _run_workers(size, "staging")


def test_engine_crossovers_are_mca_variables(gpu):
    """coll_mi355x_pipe_min_ranks / svc_max (and the other crossovers) registered as MCA variables
    (coll_tuned_component.c:115-170 style) decide the engine's flows: pipe_min_ranks = 2 puts a
    2-rank communicator's large allreduce on the pipelined flow, svc_max = 0 keeps small calls off the
    resident service; the defaults do neither at 2 ranks; results exact (coll_worker.py::mca_vars_main)"""
    _run_workers(2, "mca_vars")
