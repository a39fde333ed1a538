"""One rank of test_components_gpu.test_coll_component_processes: a mini-OMPI communicator whose
lower-priority module is a stub; coll/mi355x selected on top; collectives on device buffers must
match the oracle, host buffers must reach the stub."""
from __future__ import annotations

import ctypes
import pathlib
import sys

import numpy as np

sys.path.insert(0, str(pathlib.Path(__file__).parent))
from conftest import load_oracle  # noqa: E402
from mini import mini  # noqa: E402
import opdata  # noqa: E402


def main():
    rank, size = int(sys.argv[1]), int(sys.argv[2])
    import torch
    ndev = torch.cuda.device_count()
    torch.cuda.set_device(rank % ndev)
    m = mini()
    oracle = load_oracle()
    m.install_oracle_base(oracle)
    comm = m.lib.mini_comm_create(rank, size, 42)
    m.lib.mini_comm_install(comm, m.lib.mini_stub_module())
    prio = m.lib.mini_coll_select(comm, m.component_ptr(m.coll, "mca_coll_mi355x_component"))
    assert prio == 90, prio
    ptrs = lambda arrs: (ctypes.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])
    pkg = m.pkg
    for opname, tname in [("SUM", "FLOAT"), ("MAXLOC", "DOUBLE_INT"), ("PROD", "C_DOUBLE_COMPLEX"), ("BXOR", "INT32")]:
        code, slot = pkg.OP[opname], pkg.T[tname]
        dt = m.dtype_for_slot(slot)
        op = m.select_op(code)
        for count in (3, 4001, 200_003):
            xs = [opdata.make(tname, count, 500 + r) for r in range(size)]
            outs = [np.zeros_like(xs[0]) for _ in range(size)]
            oracle.oracle_allreduce(0, size, count, slot, code, 0, ptrs(xs), ptrs(outs))
            dx = torch.from_numpy(xs[rank].view(np.uint8).copy()).cuda()
            dr = torch.zeros_like(dx)
            torch.cuda.synchronize()
            assert m.lib.mini_allreduce(comm, dx.data_ptr(), dr.data_ptr(), count, dt, op) == 0
            opdata.assert_same(tname, opname, dr.cpu().numpy().view(xs[0].dtype), outs[rank], "component allreduce")
        # reduce_scatter_block
        rcount = 1001
        xs = [opdata.make(tname, rcount * size, 600 + r) for r in range(size)]
        outs = [np.zeros(rcount, dtype=xs[0].dtype) for _ in range(size)]
        oracle.oracle_reduce_scatter_block(size, rcount, slot, code, ptrs(xs), ptrs(outs))
        dx = torch.from_numpy(xs[rank].view(np.uint8).copy()).cuda()
        dr = torch.zeros(rcount * xs[0].dtype.itemsize, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        assert m.lib.mini_reduce_scatter_block(comm, dx.data_ptr(), dr.data_ptr(), rcount, dt, op) == 0
        opdata.assert_same(tname, opname, dr.cpu().numpy().view(xs[0].dtype), outs[rank], "component rsb")
        m.lib.mini_op_destroy(op)
    # allgather + bcast (MPI_FLOAT)
    fdt = m.dtype_for_slot(pkg.T["FLOAT"])
    n = 12345
    src = torch.full((n,), float(rank + 1), device="cuda")
    dst = torch.zeros(n * size, device="cuda")
    torch.cuda.synchronize()
    assert m.lib.mini_allgather(comm, src.data_ptr(), n, fdt, dst.data_ptr(), n, fdt) == 0
    for r in range(size):
        assert bool((dst[r * n:(r + 1) * n] == r + 1).all())
    buf = torch.full((n,), float(rank), device="cuda")
    torch.cuda.synchronize()
    assert m.lib.mini_bcast(comm, buf.data_ptr(), n, fdt, size - 1) == 0
    assert bool((buf == size - 1).all())
    # host buffers -> the lower-priority (stub) module
    h = np.zeros(16, dtype=np.float32)
    op = m.select_op(pkg.OP["SUM"])
    assert m.lib.mini_allreduce(comm, h.ctypes.data, h.ctypes.data, 16, fdt, op) == m.lib.mini_stub_marker()
    assert m.lib.mini_stub_calls(0) == 1
    m.lib.mini_comm_destroy(comm)
    print(f"rank {rank} OK", flush=True)


if __name__ == "__main__":
    main()
