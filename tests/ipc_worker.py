"""One rank of the multi-process coll/mi355x test (test_coll_ipc_gpu.py).

argv: key rank size device.  Every rank builds every rank's input deterministically, runs the
collectives through the IPC path (mi355x_comm_create + hipIpc* handles), and checks its own
result against the oracle's simulation of the reference schedule.  Exit 0 on success.
"""
from __future__ import annotations

import ctypes
import os
import pathlib
import sys

import numpy as np

sys.path.insert(0, str(pathlib.Path(__file__).parent))
from conftest import load_oracle, load_pkg  # noqa: E402
import opdata  # noqa: E402


def realloc_same_address(pkg, comm, rank, size):
    """free + hipMalloc usually returns the same address: the registration caches must notice the
    new allocation (buffer id) instead of reusing the stale IPC mapping"""
    lib = pkg.rt()
    n = 1 << 18
    nbytes = n * 4
    addrs = []
    for gen in range(3):
        p = ctypes.c_void_p()
        assert lib.mi355x_malloc(ctypes.byref(p), nbytes) == 0
        addrs.append(p.value)
        host = np.full(n, float(rank + 1 + 10 * gen), dtype=np.float32)
        assert lib.mi355x_memcpy(p, host.ctypes.data, nbytes) == 0
        comm.allreduce(None, p.value, n, pkg.T["FLOAT"], pkg.OP["SUM"])  # MPI_IN_PLACE
        out = np.empty(n, dtype=np.float32)
        assert lib.mi355x_memcpy(out.ctypes.data, p, nbytes) == 0
        want = sum(r + 1 + 10 * gen for r in range(size))
        assert np.all(out == want), (gen, out[:4], want)
        comm.barrier()  # every rank is done with the peers' allocations before they are freed
        assert lib.mi355x_free(p) == 0
    print(f"rank {rank} realloc addresses {'same' if len(set(addrs)) == 1 else 'differ'}", flush=True)
    # small allocations of changing sizes share blocks: a freed allocation's stale mapping must
    # not make the next import fail (direct path: LL off)
    comm.set("LL_MAX_BYTES", 0)
    for gen, kib in enumerate((64, 200, 48, 800, 96, 1500, 32)):
        n = kib * 256
        p = ctypes.c_void_p()
        assert lib.mi355x_malloc(ctypes.byref(p), n * 4) == 0
        host = np.full(n, float(rank + 1 + gen), dtype=np.float32)
        assert lib.mi355x_memcpy(p, host.ctypes.data, n * 4) == 0
        comm.allreduce(None, p.value, n, pkg.T["FLOAT"], pkg.OP["SUM"])
        out = np.empty(n, dtype=np.float32)
        assert lib.mi355x_memcpy(out.ctypes.data, p, n * 4) == 0
        assert np.all(out == sum(r + 1 + gen for r in range(size))), ("growing realloc", kib)
        comm.barrier()
        assert lib.mi355x_free(p) == 0
    comm.set("LL_MAX_BYTES", 0)


def ll_checks(pkg, comm, rank, size, oracle, torch, knob="LL_MAX_BYTES"):
    """the one-shot low-latency protocol -- per-call LL kernels (coll_ll.hip, knob LL_MAX_BYTES) or
    the resident service (coll_svc.hip, knob SVC_MAX_BYTES): every forced allreduce algorithm
    against the oracle's schedule simulation, in place and not, allgather / bcast, and many
    back-to-back calls (parity reuse of the LL slots)"""
    ptrs = lambda arrs: (ctypes.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])
    path = "LL" if knob == "LL_MAX_BYTES" else "SVC"
    if knob == "LL_MAX_BYTES":
        assert comm.get("LL_MAX_BYTES") == 0, "the LL path is off by default"
    saved_svc = comm.get("SVC_MAX_BYTES")
    comm.set("SVC_MAX_BYTES", 0)
    comm.set(knob, 256 << 10)
    assert comm.get(knob) > 0, f"the creation-time self-test disabled the {path} path"
    for alg in (0, 1, 2, 3, 4, 5):
        comm.set("ALLREDUCE_ALG", alg)
        for opname, tname in [("SUM", "FLOAT"), ("MAX", "DOUBLE"), ("MINLOC", "FLOAT_INT"), ("PROD", "C_DOUBLE_COMPLEX")]:
            op, ty = pkg.OP[opname], pkg.T[tname]
            esz = pkg.type_size(ty)
            for count in (1, 3, 2500 // esz + 3, 9001, (256 << 10) // esz):
                xs = [opdata.make(tname, count, 700 + 10 * alg + r) for r in range(size)]
                outs = [np.zeros_like(xs[0]) for _ in range(size)]
                ran = oracle.oracle_allreduce(alg, size, count, ty, op, 0, ptrs(xs), ptrs(outs))
                for inplace in (False, True):
                    dx = torch.from_numpy(xs[rank].view(np.uint8).copy()).cuda()
                    dr = dx.clone() if inplace else torch.zeros_like(dx)
                    torch.cuda.synchronize()
                    comm.allreduce(None if inplace else dx.data_ptr(), dr.data_ptr(), count, ty, op)
                    got = dr.cpu().numpy().view(xs[0].dtype)
                    opdata.assert_same(tname, opname, got, outs[rank],
                                       f"{path} allreduce alg={alg} count={count} inplace={inplace} rank={rank}")
                    assert comm.last_algorithm() == ran, (comm.last_algorithm(), ran)
    comm.set("ALLREDUCE_ALG", 0)
    # MPI_Reduce: LL (every rank pushes to the root) and, above the LL size, owner-computes
    oracle.oracle_reduce.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_size_t, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_uint32, ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p]
    for alg in (0, 1, 2, 3, 4, 5):
        comm.set("REDUCE_ALG", alg)
        for opname, tname in [("SUM", "FLOAT"), ("MAXLOC", "DOUBLE_INT")]:
            op, ty = pkg.OP[opname], pkg.T[tname]
            for count in (3, 5001, 100_003):
                xs = [opdata.make(tname, count, 750 + 10 * alg + r) for r in range(size)]
                for root in (0, size - 1):
                    want = np.zeros_like(xs[0])
                    oracle.oracle_reduce(alg, size, root, count, ty, op, 0, ptrs(xs), want.ctypes.data)
                    dx = torch.from_numpy(xs[rank].view(np.uint8).copy()).cuda()
                    dr = torch.zeros_like(dx)
                    torch.cuda.synchronize()
                    comm.reduce(dx.data_ptr(), dr.data_ptr() if rank == root else None, count, ty, op, root)
                    if rank == root:
                        opdata.assert_same(tname, opname, dr.cpu().numpy().view(xs[0].dtype), want,
                                           f"reduce alg={alg} count={count} root={root}")
    comm.set("REDUCE_ALG", 0)
    # back to back: 64 calls, each checked (slot parity reuse)
    x = torch.empty(1000, device="cuda")
    y = torch.empty_like(x)
    for k in range(64):
        x.fill_(float(rank + k))
        comm.allreduce(x.data_ptr(), y.data_ptr(), 1000, pkg.T["FLOAT"], pkg.OP["SUM"])
        want = sum(r + k for r in range(size))
        assert bool(torch.all(y == want)), ("back-to-back", k)
    for nb in (1, 4097, 200_003):
        for inplace in (False, True):
            src = torch.full((nb,), rank + 1, dtype=torch.uint8, device="cuda")
            dst = torch.zeros(nb * size, dtype=torch.uint8, device="cuda")
            if inplace:
                dst[rank * nb:(rank + 1) * nb] = rank + 1
            torch.cuda.synchronize()
            comm.allgather(None if inplace else src.data_ptr(), dst.data_ptr(), nb)
            # LL (3) unless the ranks sharing this GPU could not all be resident at once
            # (one 4 KiB block per CU for the ranks together, coll_comm.cpp::ll_usable)
            cus = torch.cuda.get_device_properties(0).multi_processor_count
            if ((nb + 4095) // 4096) * size <= cus:
                assert comm.last_algorithm() == 3
            for r in range(size):
                assert int(dst[r * nb:(r + 1) * nb].min()) == r + 1 == int(dst[r * nb:(r + 1) * nb].max()), ("LL ag", nb, r)
        for root in range(size):
            b = torch.full((nb,), rank, dtype=torch.uint8, device="cuda")
            torch.cuda.synchronize()
            comm.bcast(b.data_ptr(), nb, root)
            assert int(b.min()) == root == int(b.max()), ("LL bcast", nb, root)
    # nonblocking through the progress thread: an LL-sized and a large allreduce posted together
    xs = torch.full((1000,), float(rank + 1), device="cuda")
    xl = torch.full((3_000_000,), float(rank + 1), device="cuda")
    ys, yl = torch.empty_like(xs), torch.empty_like(xl)
    reqs = [comm.iallreduce(xs.data_ptr(), ys.data_ptr(), xs.numel(), pkg.T["FLOAT"], pkg.OP["SUM"]),
            comm.iallreduce(xl.data_ptr(), yl.data_ptr(), xl.numel(), pkg.T["FLOAT"], pkg.OP["SUM"])]
    for q in reqs:
        q.wait()
    want = size * (size + 1) / 2
    assert bool(torch.all(ys == want)) and bool(torch.all(yl == want)), "nonblocking allreduce"
    comm.set(knob, 0)
    comm.set("SVC_MAX_BYTES", saved_svc)
    print(f"rank {rank} {path} OK", flush=True)


def svc_pull_checks(pkg, comm, rank, size, oracle, torch):
    """the one-phase ring-ordered allreduce served by the resident service from the peers' mapped
    inputs (LL_PULL, coll_svc.hip): sizes between the service's LL limit and the pull limit, odd
    counts (a tail shorter than a 16-B vector), every ring algorithm against the oracle's schedule
    simulation; in place and 1-byte types (BXOR INT8) take the host-synchronised flows"""
    ptrs = lambda arrs: (ctypes.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])
    saved = comm.get("SVC_PULL_MAX_BYTES")
    comm.set("SVC_PULL_MAX_BYTES", 1 << 20)
    assert comm.get("SVC_PULL_MAX_BYTES") == 1 << 20
    svc_max = comm.get("SVC_MAX_BYTES")
    calls0 = comm.get("SVC_CALLS")
    for alg in (0, 4, 5):
        comm.set("ALLREDUCE_ALG", alg)
        for opname, tname in [("SUM", "FLOAT"), ("MAX", "DOUBLE"), ("MINLOC", "FLOAT_INT"), ("PROD", "C_DOUBLE_COMPLEX"),
                              ("BXOR", "INT8")]:
            op, ty = pkg.OP[opname], pkg.T[tname]
            esz = pkg.type_size(ty)
            for count in (svc_max // esz + 1, 100_003 // esz, (1 << 20) // esz - 3, (1 << 20) // esz):
                xs = [opdata.make(tname, count, 800 + 10 * alg + r) for r in range(size)]
                outs = [np.zeros_like(xs[0]) for _ in range(size)]
                ran = oracle.oracle_allreduce(alg, size, count, ty, op, 0, ptrs(xs), ptrs(outs))
                for inplace in (False, True):
                    dx = torch.from_numpy(xs[rank].view(np.uint8).copy()).cuda()
                    dr = dx.clone() if inplace else torch.full_like(dx, 0x5a)
                    torch.cuda.synchronize()
                    comm.allreduce(None if inplace else dx.data_ptr(), dr.data_ptr(), count, ty, op)
                    got = dr.cpu().numpy().view(xs[0].dtype)
                    opdata.assert_same(tname, opname, got, outs[rank],
                                       f"pull allreduce alg={alg} count={count} inplace={inplace} rank={rank}")
                    assert comm.last_algorithm() == ran, (comm.last_algorithm(), ran)
                    # the caller reuses its input at once: the peers must be done reading it
                    dx.fill_(0x7f)
    served = comm.get("SVC_CALLS") - calls0
    assert served >= 3 * 4 * 4, f"the service served {served} pull calls"
    comm.set("ALLREDUCE_ALG", 0)
    # allgather / bcast copied by the service (LL_PULL_AG / LL_PULL_BC): 16-B multiples, odd sizes
    # (word and byte copies), odd offsets, in place
    assert comm.get("SVC_PULL_COPY_MAX_BYTES") == 1 << 20
    comm.set("SVC_PULL_COPY_MAX_BYTES", 1 << 19)
    assert comm.get("SVC_PULL_COPY_MAX_BYTES") == 1 << 19
    comm.set("SVC_PULL_COPY_MAX_BYTES", 1 << 20)
    calls1 = comm.get("SVC_CALLS")
    # the last size is above the copy limit: host-synchronised flows, not counted
    for nb in (svc_max + 16, svc_max + 1, 100_003, (1 << 20) - 4, (1 << 20) + 16):
        for inplace in (False, True):
            for shift in (0, 3):
                src = torch.full((nb + shift,), (rank * 3 + nb) % 251, dtype=torch.uint8, device="cuda")
                dst = torch.zeros(nb * size + shift, dtype=torch.uint8, device="cuda")
                if inplace:
                    dst[shift + rank * nb: shift + (rank + 1) * nb] = (rank * 3 + nb) % 251
                torch.cuda.synchronize()
                comm.allgather(None if inplace else src.data_ptr() + shift, dst.data_ptr() + shift, nb)
                assert comm.last_algorithm() == 1
                for r in range(size):
                    blk = dst[shift + r * nb: shift + (r + 1) * nb]
                    assert bool(torch.all(blk == (r * 3 + nb) % 251).item()), ("pull allgather", nb, inplace, shift, r)
                src.fill_(0)  # reused at once: every peer is done reading it
        for root in range(size):
            b = torch.full((nb + 5,), (rank * 7 + nb) % 251, dtype=torch.uint8, device="cuda")
            torch.cuda.synchronize()
            comm.bcast(b.data_ptr() + 5, nb, root)
            assert bool(torch.all(b[5:] == (root * 7 + nb) % 251).item()), ("pull bcast", nb, root)
    copies = comm.get("SVC_CALLS") - calls1
    assert copies == 4 * 2 * 2 + 4 * size, f"the service served {copies} allgather / bcast calls"
    comm.set("SVC_PULL_MAX_BYTES", saved)
    # the reduce_scatter form (on by default; MI355X_SVC_RS=0 turns it off on every rank)
    rs = svc_rs_checks(pkg, comm, rank, size, oracle, torch) if os.environ.get("MI355X_SVC_RS", "1") != "0" else 0
    print(f"rank {rank} pull OK ({served} allreduce, {copies} allgather / bcast, {rs} reduce_scatter service calls)",
          flush=True)


def svc_rs_checks(pkg, comm, rank, size, oracle, torch):
    """reduce_scatter(_block) evaluated by the resident service from the peers' mapped inputs
    (LL_PULL_RS, coll_svc.hip): every reduce_scatter algorithm (decision, non-overlapping's reduce
    tree, recursive halving's trees, ring folds) over 1- to 16-byte types, single-element, ragged,
    empty and 128 KiB blocks, against the oracle's schedule simulation; a block above the pull
    limit and the in-place forms take the host-synchronised flows"""
    ptrs = lambda arrs: (ctypes.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])
    limit = comm.get("SVC_PULL_MAX_BYTES")
    calls0 = comm.get("SVC_CALLS")
    expect = 0
    for rsalg in (0, 1, 2, 3):
        comm.set("REDUCE_SCATTER_ALG", rsalg)
        for opname, tname in [("SUM", "FLOAT"), ("MAX", "DOUBLE"), ("MINLOC", "FLOAT_INT"), ("PROD", "C_DOUBLE_COMPLEX"),
                              ("BXOR", "INT8"), ("SUM", "INT16")]:
            op, ty = pkg.OP[opname], pkg.T[tname]
            esz = pkg.type_size(ty)
            for rcounts in ([1] * size, [7 * r + 3 for r in range(size)], [0 if r == 1 else 5000 + r for r in range(size)],
                            [limit // esz - r for r in range(size)], [limit // esz + 1] + [3] * (size - 1)):
                total = sum(rcounts)
                xs = [opdata.make(tname, total, 900 + 10 * rsalg + r) for r in range(size)]
                outs = [np.zeros(max(k, 1), dtype=xs[0].dtype) for k in rcounts]
                rc = (ctypes.c_int * size)(*rcounts)
                assert oracle.oracle_reduce_scatter_alg(rsalg, size, rc, ty, op, ptrs(xs), ptrs(outs)) >= 0
                dx = torch.from_numpy(xs[rank].view(np.uint8).copy()).cuda()
                dr = torch.full((max(rcounts[rank], 1) * esz,), 0x5a, dtype=torch.uint8, device="cuda")
                torch.cuda.synchronize()
                comm.reduce_scatter(dx.data_ptr(), dr.data_ptr(), rcounts, ty, op)
                mine = rcounts[rank]
                if mine:
                    got = dr.cpu().numpy().view(xs[0].dtype)[:mine]
                    opdata.assert_same(tname, opname, got, outs[rank][:mine],
                                       f"service rs alg={rsalg} rcounts={rcounts[:3]} rank={rank}")
                dx.fill_(0x7f)  # reused at once: every peer is done reading it
                expect += max(rcounts) * esz <= limit
    comm.set("REDUCE_SCATTER_ALG", 0)
    # reduce_scatter_block (the reduce decision's program per block), not in place and in place
    for opname, tname in [("SUM", "FLOAT"), ("MAXLOC", "DOUBLE_INT"), ("BAND", "UINT8")]:
        op, ty = pkg.OP[opname], pkg.T[tname]
        esz = pkg.type_size(ty)
        for rcount in (1, 1001, limit // esz):
            xs = [opdata.make(tname, rcount * size, 950 + r) for r in range(size)]
            outs = [np.zeros(rcount, dtype=xs[0].dtype) for _ in range(size)]
            assert oracle.oracle_reduce_scatter_block(size, rcount, ty, op, ptrs(xs), ptrs(outs)) >= 0
            for inplace in (False, True):
                dx = torch.from_numpy(xs[rank].view(np.uint8).copy()).cuda()
                dr = dx.clone() if inplace else torch.full((rcount * esz,), 0x5a, dtype=torch.uint8, device="cuda")
                torch.cuda.synchronize()
                comm.reduce_scatter_block(None if inplace else dx.data_ptr(), dr.data_ptr(), rcount, ty, op)
                got = dr[:rcount * esz].cpu().numpy().view(xs[0].dtype)
                opdata.assert_same(tname, opname, got, outs[rank], f"service rsb rcount={rcount} inplace={inplace} rank={rank}")
                dx.fill_(0x7f)
                expect += not inplace
    served = comm.get("SVC_CALLS") - calls0
    assert served == expect, f"the service served {served} reduce_scatter calls, expected {expect}"
    return served


def svc_all_slots(pkg, comm, rank, size, oracle, torch):
    """every (op, type) slot through the resident service -- the LL form's tree program (recursive
    doubling, < 10000 B), its ring order, and the reduce-scatter form -- against the oracle's
    schedule simulation.  The service's evaluation keeps the ranks' values of an element in one
    vector register tuple for the integer and floating types and in an array for the others
    (complex, value-index pairs), so every element type is run, not a sample"""
    ptrs = lambda arrs: (ctypes.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])
    saved = comm.get("SVC_MAX_BYTES")
    comm.set("SVC_MAX_BYTES", 32 << 10)
    calls0 = comm.get("SVC_CALLS")
    bad = []
    k = ncalls = 0
    for code in range(1, 13):
        for ty in range(len(pkg.TYPES)):
            if not (oracle.oracle_has_op(code, ty) and pkg.comm_op_supported(code, ty) and pkg.type_size(ty) <= 16):
                continue
            tname, opname = pkg.TYPES[ty], pkg.OPS[code]
            esz = pkg.type_size(ty)
            for count in (3 + k % 5, (12 << 10) // esz + k % 7):
                xs = [opdata.make(tname, count, 9000 + 11 * k + r) for r in range(size)]
                outs = [np.zeros_like(xs[0]) for _ in range(size)]
                ran = oracle.oracle_allreduce(0, size, count, ty, code, 0, ptrs(xs), ptrs(outs))
                dx = torch.from_numpy(xs[rank].view(np.uint8).copy()).cuda()
                dr = torch.full_like(dx, 0x5a)
                torch.cuda.synchronize()
                comm.allreduce(dx.data_ptr(), dr.data_ptr(), count, ty, code)
                ncalls += 1
                try:
                    opdata.assert_same(tname, opname, dr.cpu().numpy().view(xs[0].dtype), outs[rank],
                                       f"service slot {opname}/{tname} count={count}")
                    assert comm.last_algorithm() == ran, (opname, tname, count, comm.last_algorithm(), ran)
                except AssertionError as e:
                    bad.append(str(e)[:300])
            rcount = 5 + k % 9
            xs = [opdata.make(tname, rcount * size, 9500 + 11 * k + r) for r in range(size)]
            outs = [np.zeros(rcount, dtype=xs[0].dtype) for _ in range(size)]
            assert oracle.oracle_reduce_scatter_block(size, rcount, ty, code, ptrs(xs), ptrs(outs)) >= 0
            dx = torch.from_numpy(xs[rank].view(np.uint8).copy()).cuda()
            dr = torch.full((rcount * esz,), 0x5a, dtype=torch.uint8, device="cuda")
            torch.cuda.synchronize()
            comm.reduce_scatter_block(dx.data_ptr(), dr.data_ptr(), rcount, ty, code)
            ncalls += 1
            try:
                opdata.assert_same(tname, opname, dr.cpu().numpy().view(xs[0].dtype), outs[rank],
                                   f"service rsb slot {opname}/{tname} rcount={rcount}")
            except AssertionError as e:
                bad.append(str(e)[:300])
            k += 1
    served = comm.get("SVC_CALLS") - calls0
    comm.set("SVC_MAX_BYTES", saved)
    assert not bad, "\n".join(bad[:8])
    assert k >= 100, k  # every GPU slot ran
    assert served == ncalls, f"the service served {served} of {ncalls} calls"
    print(f"rank {rank} service slots OK ({k} slots, {served} service calls)", flush=True)


def staged(pkg, comm, rank, size, torch, key):
    """allocations too large for hipIpc* (forced here: every allocation; for real: >= 2 GiB, which
    hipIpcOpenMemHandle cannot map on this platform) through real IPC, twice: on a communicator
    with the dmabuf path disabled (staged flow, 1 MiB staging) and on the main one (dmabuf fds
    passed with SCM_RIGHTS over the communicator's Unix datagram sockets)"""
    import os
    os.environ["MI355X_DMABUF"] = "0"
    c2 = pkg.Comm.create(key + "_st", rank, size, torch.cuda.current_device())
    try:
        large_calls(pkg, c2, rank, size, torch)
    finally:
        c2.destroy()
        del os.environ["MI355X_DMABUF"]
    large_calls(pkg, comm, rank, size, torch)
    print(f"rank {rank} staged OK", flush=True)


def large_calls(pkg, comm, rank, size, torch):
    comm.set("IPC_MAX_BYTES", 0)
    comm.set("STAGE_BYTES", 1 << 20)
    n = 700_001
    x = torch.full((n,), float(rank + 1), device="cuda")
    y = torch.empty_like(x)
    want = size * (size + 1) / 2
    torch.cuda.synchronize()
    comm.allreduce(x.data_ptr(), y.data_ptr(), n, pkg.T["FLOAT"], pkg.OP["SUM"])
    assert bool(torch.all(y == want)), "staged allreduce"
    r = torch.empty((n // size,), device="cuda")
    comm.reduce_scatter_block(x.data_ptr(), r.data_ptr(), n // size, pkg.T["FLOAT"], pkg.OP["SUM"])
    assert bool(torch.all(r == want)), "staged rsb"
    g = torch.empty((n // size * size,), device="cuda")
    comm.allgather(r.data_ptr(), g.data_ptr(), r.numel() * 4)
    assert bool(torch.all(g == want)), "staged allgather"
    b = torch.full((3_000_001,), rank, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    comm.bcast(b.data_ptr(), b.numel(), 0)
    assert int(b.max()) == 0, "staged bcast"
    comm.set("IPC_MAX_BYTES", 1 << 31)
    comm.set("STAGE_BYTES", 256 << 20)
    del x, y, r, g, b
    if size == 2:
        big = torch.full(((1 << 28) + (1 << 20),), float(rank + 1), dtype=torch.float64, device="cuda")  # 2 GiB + 8 MiB
        torch.cuda.synchronize()
        comm.allreduce(None, big.data_ptr(), big.numel(), pkg.T["DOUBLE"], pkg.OP["SUM"])
        assert bool(torch.all(big == want)), "allreduce on a >= 2 GiB allocation"
        out = torch.empty((big.numel() // 2,), dtype=torch.float64, device="cuda")
        comm.reduce_scatter_block(big.data_ptr(), out.data_ptr(), out.numel(), pkg.T["DOUBLE"], pkg.OP["SUM"])
        assert bool(torch.all(out == size * want)), "rsb on a >= 2 GiB allocation"
        del big, out
        torch.cuda.empty_cache()


def max_count(pkg, comm, rank, size, torch):
    """the largest count an MPI_Allreduce can pass (INT_MAX elements, `int count` at coll.h:189-191)
    of fp32: 8 GiB per buffer, dmabuf-exported allocations, byte offsets past 2^32 -- two-phase and
    pipelined flows, in place and not; x_r = r + 1 -> every element n(n+1)/2 exactly"""
    n = 2**31 - 1
    want = size * (size + 1) / 2
    x = torch.full((n,), float(rank + 1), device="cuda")
    y = torch.full((n,), -1.0, device="cuda")
    torch.cuda.synchronize()
    try:
        for pipe in (0, 1):
            comm.set("PIPE", pipe)
            comm.allreduce(x.data_ptr(), y.data_ptr(), n, pkg.T["FLOAT"], pkg.OP["SUM"])
            assert bool(torch.all(y == want)), ("INT_MAX-count allreduce", pipe)
            y.fill_(float(rank + 1))
            torch.cuda.synchronize()
            comm.allreduce(None, y.data_ptr(), n, pkg.T["FLOAT"], pkg.OP["SUM"])
            assert bool(torch.all(y == want)), ("INT_MAX-count allreduce in place", pipe)
    finally:
        comm.set("PIPE", 1 if size >= 4 else 0)
    del x, y
    torch.cuda.empty_cache()
    print(f"rank {rank} maxcount OK", flush=True)


def pipe_checks(pkg, comm, rank, size, oracle, torch):
    """the pipelined allreduce (coll_pipe.hip: fold + pulls in one launch, device-side chunk
    flags) against the oracle's schedule simulation and against the two-phase flow: ring and
    segmented-ring regions, order-sensitive data, in place, every rank's buffers at a different
    misalignment (scalar fold, per-peer pull paths), many back-to-back calls (flags and the work
    queue reused)"""
    ptrs = lambda arrs: (ctypes.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])
    assert comm.get("PIPE") == (1 if size >= 4 else 0)  # default: on from 4 ranks up
    assert comm.get("PIPE_WT") == 1
    comm.set("PIPE", 1)
    comm.set("LL_MAX_BYTES", 0)
    cases = [("SUM", "FLOAT", 300_007), ("SUM", "FLOAT", size * (1 << 18) * 2 + 12_345),
             ("PROD", "C_DOUBLE_COMPLEX", 100_003), ("MAXLOC", "DOUBLE_INT", 70_001), ("BAND", "INT64", 4099)]
    for opname, tname, count, wt in [c + (w,) for c in cases for w in (0, 1)]:
        comm.set("PIPE_WT", wt)  # fenced publishing, then write-through publishing
        op, ty = pkg.OP[opname], pkg.T[tname]
        esz = pkg.type_size(ty)
        xs = [opdata.make(tname, count, 3000 + r) for r in range(size)]
        outs = [np.zeros_like(xs[0]) for _ in range(size)]
        ran = oracle.oracle_allreduce(0, size, count, ty, op, 0, ptrs(xs), ptrs(outs))
        for skew in (False, True):
            for inplace in (False, True):
                # skew: this rank's buffers start (4 * rank) bytes into their allocations
                off = (4 * rank) % 16 if skew else 0
                raw = torch.zeros(count * esz + 64, dtype=torch.uint8, device="cuda")
                dx = raw[off:off + count * esz]
                dx.copy_(torch.from_numpy(xs[rank].view(np.uint8).copy()).cuda())
                rraw = torch.zeros(count * esz + 64, dtype=torch.uint8, device="cuda")
                roff = (16 - off) % 16 if skew else 0
                dr = dx if inplace else rraw[roff:roff + count * esz]
                torch.cuda.synchronize()
                comm.allreduce(None if inplace else dx.data_ptr(), dr.data_ptr(), count, ty, op)
                got = dr.cpu().numpy().view(xs[0].dtype)
                opdata.assert_same(tname, opname, got, outs[rank],
                                   f"pipe allreduce {opname}/{tname} count={count} skew={skew} inplace={inplace} wt={wt}")
                assert comm.last_algorithm() == ran
    # back to back, values change every call; then the same with the two-phase flow
    x = torch.empty(1 << 20, device="cuda")
    y = torch.empty_like(x)
    for pipe, wt in ((1, 0), (0, 0), (1, 1), (1, 0), (1, 1)):
        comm.set("PIPE", pipe)
        comm.set("PIPE_WT", wt)
        for k in range(16):
            x.fill_(float(rank + k))
            comm.allreduce(x.data_ptr(), y.data_ptr(), x.numel(), pkg.T["FLOAT"], pkg.OP["SUM"])
            assert bool(torch.all(y == sum(r + k for r in range(size)))), ("pipe back-to-back", pipe, wt, k)
    comm.set("PIPE", 1 if size >= 4 else 0)
    comm.set("PIPE_WT", 1)
    comm.set("LL_MAX_BYTES", 0)
    print(f"rank {rank} pipe OK", flush=True)


def pipe_all_slots(pkg, comm, rank, size, oracle, torch):
    """every (op, type) slot of the pipelined kernel (one instantiation each) on the ring path,
    fenced and write-through publishing, against the oracle's schedule simulation"""
    ptrs = lambda arrs: (ctypes.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])
    comm.set("PIPE", 1)
    comm.set("LL_MAX_BYTES", 0)
    bad = []
    k = 0
    for code in range(1, 13):
        for ty in range(len(pkg.TYPES)):
            if not (oracle.oracle_has_op(code, ty) and pkg.comm_op_supported(code, ty) and pkg.type_size(ty) <= 16):
                continue
            tname, opname = pkg.TYPES[ty], pkg.OPS[code]
            esz = pkg.type_size(ty)
            count = (64 << 10) // esz + 2 * k + 1  # above the ring threshold, odd, a different tail per slot
            xs = [opdata.make(tname, count, 5000 + 7 * k + r) for r in range(size)]
            outs = [np.zeros_like(xs[0]) for _ in range(size)]
            ran = oracle.oracle_allreduce(0, size, count, ty, code, 0, ptrs(xs), ptrs(outs))
            if ran not in (4, 5):
                continue
            comm.set("PIPE_WT", k & 1)
            dx = torch.from_numpy(xs[rank].view(np.uint8).copy()).cuda()
            dr = torch.zeros_like(dx)
            torch.cuda.synchronize()
            comm.allreduce(dx.data_ptr(), dr.data_ptr(), count, ty, code)
            try:
                opdata.assert_same(tname, opname, dr.cpu().numpy().view(xs[0].dtype), outs[rank],
                                   f"pipe slot {opname}/{tname} count={count}")
            except AssertionError as e:
                bad.append(str(e)[:300])
            k += 1
    comm.set("PIPE", 1 if size >= 4 else 0)
    comm.set("PIPE_WT", 1)
    assert not bad, "\n".join(bad[:8])
    assert k >= 100, k  # every GPU slot ran
    print(f"rank {rank} pipe slots OK ({k})", flush=True)


def _pattern_chunk(torch, lo, hi):
    """int32 words lo..hi-1 of the big-bcast pattern (an LCG of the word index, wraps in int32)"""
    return torch.arange(lo, hi, dtype=torch.int32, device="cuda") * 1103515245 + 12345


def big_bcast(pkg, comm, rank, size, torch):
    """BASELINE configs[4]: a 4 GiB MPI_Bcast (MPI_FLOAT x 2^30) on a >= 2 GiB allocation (the
    dmabuf path: hipIpcOpenMemHandle cannot map it), root size-1, every word checked exactly"""
    nbytes = 4 << 30
    words = nbytes // 4
    chunk = 1 << 26
    buf = torch.zeros(nbytes, dtype=torch.uint8, device="cuda")
    b32 = buf.view(torch.int32)
    root = size - 1
    if rank == root:
        for lo in range(0, words, chunk):
            b32[lo:lo + chunk] = _pattern_chunk(torch, lo, lo + chunk)
    torch.cuda.synchronize()
    comm.bcast(buf.data_ptr(), nbytes, root)
    assert comm.last_algorithm() == 2, comm.last_algorithm()  # scatter + allgather shape
    for lo in range(0, words, chunk):
        assert torch.equal(b32[lo:lo + chunk], _pattern_chunk(torch, lo, lo + chunk)), ("4 GiB bcast", lo)
    comm.barrier()
    del buf, b32
    torch.cuda.empty_cache()
    print(f"rank {rank} bcast4g OK", flush=True)


def p2p_checks(pkg, comm, rank, size, oracle, torch):
    """device point-to-point across processes (IPC-mapped sender buffers pulled by the receiver)"""
    def pattern(src, n, salt):
        return np.random.default_rng(1000 * src + salt).integers(0, 256, n, dtype=np.uint8)

    nxt, prv = (rank + 1) % size, (rank - 1) % size
    for salt, n in enumerate([0, 1, 4096, 1 << 20, (64 << 20) + 3]):
        s = torch.from_numpy(pattern(rank, n, salt)).cuda() if n else None
        d = torch.zeros(max(n, 1), dtype=torch.uint8, device="cuda")
        st = comm.sendrecv(s.data_ptr() if n else None, n, nxt, salt, d.data_ptr(), n, prv, salt)
        assert st == (prv, salt, 0, n), st
        assert np.array_equal(d[:n].cpu().numpy(), pattern(prv, n, salt)), f"sendrecv {n} bytes"
    # every rank to every other, received with MPI_ANY_SOURCE
    srcs = {q: torch.from_numpy(pattern(rank, 1000 + rank, 50 + q)).cuda() for q in range(size) if q != rank}
    outs = [torch.zeros(4096, dtype=torch.uint8, device="cuda") for _ in range(size - 1)]
    rreqs = [comm.irecv(o.data_ptr(), 4096, pkg.ANY_SOURCE, 77) for o in outs]
    sreqs = [comm.isend(srcs[q].data_ptr(), srcs[q].numel(), q, 77) for q in srcs]
    sts = [r.wait() for r in rreqs]
    for r in sreqs:
        r.wait()
    assert sorted(s[0] for s in sts) == [q for q in range(size) if q != rank], sts
    for s, o in zip(sts, outs):
        assert np.array_equal(o[:s[3]].cpu().numpy(), pattern(s[0], 1000 + s[0], 50 + rank)), "any-source bytes"
    # more messages in flight than envelopes: queued sends, order kept
    k = 80
    src = torch.from_numpy(pattern(rank, 64 * k, 99)).cuda()
    dst = torch.zeros(64 * k, dtype=torch.uint8, device="cuda")
    rreqs = [comm.irecv(dst[i * 64:(i + 1) * 64].data_ptr(), 64, prv, pkg.ANY_TAG) for i in range(k)]
    sreqs = [comm.isend(src[i * 64:(i + 1) * 64].data_ptr(), 64, nxt, i) for i in range(k)]
    for i, r in enumerate(rreqs):
        assert r.wait()[1] == i
    for r in sreqs:
        r.wait()
    assert np.array_equal(dst.cpu().numpy(), pattern(prv, 64 * k, 99)), "queued messages"
    # more small DEVICE sends in flight than the 32 envelopes of a pair, none received yet: every
    # send (standard small = eager, and MPI_Bsend) must complete locally -- a send that finds the
    # ring full takes the host copy at once instead of waiting for a receiver's claim -- and the
    # receiver gets them all, in order, only after every send has completed
    k2 = 48
    src2 = [torch.from_numpy(pattern(rank, 1024, 600 + i)).cuda() for i in range(k2)]
    torch.cuda.synchronize()
    sreqs = [comm.isend(src2[i].data_ptr(), 1024, nxt, 700 + i, mode="BUFFERED" if i % 5 == 4 else None)
             for i in range(k2)]
    for r in sreqs:
        r.wait()      # before any receive is posted anywhere (the barrier below)
    for i in range(k2):
        src2[i].fill_(0)   # the caller may reuse an eager send's buffer
    comm.barrier()
    dst2 = torch.zeros(k2 * 1024, dtype=torch.uint8, device="cuda")
    for i in range(k2):
        st = comm.recv(dst2[i * 1024:(i + 1) * 1024].data_ptr(), 1024, prv, pkg.ANY_TAG)
        assert st[1] == 700 + i, ("order of eager device sends", i, st)
    for i in range(k2):
        assert np.array_equal(dst2[i * 1024:(i + 1) * 1024].cpu().numpy(), pattern(prv, 1024, 600 + i)), ("eager", i)
    # MPI_Type_vector(stride 2, block 64) floats: packed by the sender, received contiguous
    nvec = 1000
    od = oracle.oracle_ddt_vector(nvec, 64, 128, 4)
    dv = pkg.Ddt.vector(nvec, 64, 128, 4)
    vsrc = pattern(rank, nvec * 128 * 4, 7)
    d = torch.zeros(nvec * 64 * 4, dtype=torch.uint8, device="cuda")
    s = comm.isend(torch.from_numpy(vsrc).cuda().data_ptr(), 1, nxt, 5, ddt=dv)
    comm.recv(d.data_ptr(), nvec * 64 * 4, prv, 5)
    s.wait()
    want = np.zeros(nvec * 64 * 4, dtype=np.uint8)
    pv = pattern(prv, nvec * 128 * 4, 7)
    oracle.oracle_ddt_pack(od, 1, pv.ctypes.data, 0, want.ctypes.data, want.size)
    assert np.array_equal(d.cpu().numpy(), want), "vector send"
    oracle.oracle_ddt_free(od)
    dv.destroy()
    # host buffers across processes, in the same queue: host -> host through the sender's shared-
    # memory arena (sizes that outgrow it: new segment generations the receiver maps by name),
    # host -> device, device -> host (pulled into device staging, then copied out)
    for salt, n in enumerate([5, 4097, 3 << 20, (40 << 20) + 1]):
        hs = pattern(rank, n, 200 + salt)
        want = pattern(prv, n, 200 + salt)
        hd = np.zeros(n, dtype=np.uint8)
        st = comm.sendrecv(hs.ctypes.data, n, nxt, 300 + salt, hd.ctypes.data, n, prv, 300 + salt)
        assert st == (prv, 300 + salt, 0, n) and np.array_equal(hd, want), f"host->host {n}"
        dd = torch.zeros(n, dtype=torch.uint8, device="cuda")
        comm.sendrecv(hs.ctypes.data, n, nxt, 400 + salt, dd.data_ptr(), n, prv, 400 + salt)
        assert np.array_equal(dd.cpu().numpy(), want), f"host->device {n}"
        ds = torch.from_numpy(hs).cuda()
        torch.cuda.synchronize()
        hd[:] = 0
        comm.sendrecv(ds.data_ptr(), n, nxt, 500 + salt, hd.ctypes.data, n, prv, 500 + salt)
        assert np.array_equal(hd, want), f"device->host {n}"
    if size == 2:   # a send buffer inside an allocation of >= 2 GiB: dmabuf export
        big = torch.full(((1 << 31) + (8 << 20),), rank + 1, dtype=torch.uint8, device="cuda")
        tail = 16 << 20
        torch.cuda.synchronize()
        if rank == 0:
            comm.send(big[-tail:].data_ptr(), tail, 1, 123)
        else:
            d = torch.zeros(tail, dtype=torch.uint8, device="cuda")
            assert comm.recv(d.data_ptr(), tail, 0, 123) == (0, 123, 0, tail)
            assert int(d.min()) == 1 and int(d.max()) == 1, "send from a >= 2 GiB allocation"
        comm.barrier()
        del big
        torch.cuda.empty_cache()
    comm.barrier()
    print(f"rank {rank} p2p OK", flush=True)


def _fd_report(rank):
    import os
    import resource
    try:
        n = len(os.listdir("/proc/self/fd"))
    except OSError:
        n = -1
    print(f"rank {rank} open fds {n}, RLIMIT_NOFILE {resource.getrlimit(resource.RLIMIT_NOFILE)}", flush=True)


def concurrent_comms(key, rank, size, dev):
    """4 communicators over the same ranks, each driven by its own thread and stream, running 1 GiB
    fp32 allreduces at the same time with the pipelined flow on: the per-GPU admission token lets
    one communicator's persistent grids onto a GPU at a time and sends the others down the
    two-phase flow, so nothing waits on a grid that cannot be resident.  Every result exact, no
    timeout (concurrent communicators)."""
    import threading
    import torch
    torch.cuda.set_device(dev)
    pkg = load_pkg()
    ncomm, n, iters = 4, (1 << 30) // 4, 3
    comms = [pkg.Comm.create(f"{key}_c{i}", rank, size, dev) for i in range(ncomm)]
    for c in comms:
        c.set("PIPE", 1)
        c.set("TIMEOUT_S", 60)
    xs = [torch.empty(n, device="cuda") for _ in range(ncomm)]
    ys = [torch.empty(n, device="cuda") for _ in range(ncomm)]
    errs, bad = [], []
    start = threading.Barrier(ncomm)

    def run(i):
        try:
            torch.cuda.set_device(dev)
            st = torch.cuda.Stream()
            with torch.cuda.stream(st):
                for it in range(iters):
                    xs[i].fill_(float(rank + 1 + 10 * i + 100 * it))
                    ys[i].fill_(float("nan"))
                    if it == 0:
                        st.synchronize()
                        start.wait()   # every thread's first call at the same moment
                    comms[i].allreduce(xs[i].data_ptr(), ys[i].data_ptr(), n, pkg.T["FLOAT"], pkg.OP["SUM"],
                                       stream=st.cuda_stream)
                    want = size * (size + 1) / 2 + size * (10 * i + 100 * it)
                    if not bool(torch.all(ys[i] == want).item()):
                        bad.append((i, it))
        except Exception as e:  # noqa: BLE001
            errs.append(repr(e))

    ts = [threading.Thread(target=run, args=(i,)) for i in range(ncomm)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(240)
    assert not any(t.is_alive() for t in ts), "a communicator's allreduce never returned"
    assert not errs, errs
    assert not bad, f"wrong results {bad}"
    refused = sum(c.get("PIPE_REFUSED") for c in comms)
    print(f"rank {rank} concurrent: {ncomm} communicators x {iters} calls exact; {refused} calls fell back "
          "to two phases", flush=True)
    for c in comms:
        c.barrier()
        c.destroy()
    print(f"rank {rank} concurrent OK", flush=True)


def svc_mode(key, rank, size, dev):
    """the resident LL service (coll_svc.hip on a private HSA queue, svc_queue.cpp) beside the rest of
    the process: while it stays resident (MI355X_SVC_IDLE_MS=3000 here) hipDeviceSynchronize and work
    on fresh streams do not wait for it; back-to-back calls reuse one launch; it leaves when idle and
    comes back on the next call.  One service per process, owned by the communicator that issues the
    small calls: claimed at a communicator's first small call, kept while it is busy
    (MI355X_SVC_HANDOVER_MS=200 here), handed over to the other communicator once it has been idle;
    the communicator without it computes exactly on the per-call paths"""
    import os
    import time
    import torch
    torch.cuda.set_device(dev)
    pkg = load_pkg()
    f32, SUM = pkg.T["FLOAT"], pkg.OP["SUM"]
    a = pkg.Comm.create(key + "_a", rank, size, dev)
    b = pkg.Comm.create(key + "_b", rank, size, dev)
    a.set("SVC_MAX_BYTES", 64 << 10)
    b.set("SVC_MAX_BYTES", 64 << 10)
    assert a.get("SVC_OWNER") == 0 and b.get("SVC_OWNER") == 0, "nothing is claimed before a small call"
    x = torch.full((1000,), float(rank + 1), device="cuda")
    y = torch.empty_like(x)
    want = size * (size + 1) / 2

    def ar(c, k=0):
        x.fill_(float(rank + 1 + k))
        y.fill_(-1)
        torch.cuda.synchronize()
        c.allreduce(x.data_ptr(), y.data_ptr(), 1000, f32, SUM)
        assert bool(torch.all(y == want + size * k).item()), "allreduce next to the service"

    for c in (a, b, a, b):  # b asks while a is busy: a keeps it
        ar(c)
    assert a.get("SVC_OWNER") == 1 and b.get("SVC_OWNER") == 0
    assert b.get("SVC_CALLS") == 0 and a.get("SVC_CALLS") >= 2
    # resident now (idle limit 3 s): the device synchronizes without it, a fresh stream runs
    assert a.get("SVC_LAUNCHES") >= 1
    t0 = time.perf_counter()
    torch.cuda.synchronize()
    dt_sync = time.perf_counter() - t0
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        z = x * 2
    t0 = time.perf_counter()
    st.synchronize()
    dt_stream = time.perf_counter() - t0
    assert dt_sync < 0.5 and dt_stream < 0.5, (dt_sync, dt_stream)
    assert bool(torch.all(z == 2 * (rank + 1)).item())
    launches = a.get("SVC_LAUNCHES")
    for k in range(200):
        ar(a, k)
    relaunched = a.get("SVC_LAUNCHES") - launches
    assert relaunched <= 2, f"{relaunched} relaunches over 200 back-to-back calls"
    # a idle longer than the handover time: b's next claim takes the service over, on every rank
    time.sleep(0.3)
    for k in range(40):
        ar(b, k)
    assert b.get("SVC_OWNER") == 1 and a.get("SVC_OWNER") == 0, (b.get("SVC_OWNER"), a.get("SVC_OWNER"))
    assert b.get("SVC_CALLS") > 0
    handed = b.get("SVC_CALLS")
    # idle longer than SVC_SHRINK_US (100 us) but not the idle limit: every workgroup but the first
    # leaves; a small call is served by it alone (no launch), a 16-slice call relaunches the full grid
    assert b.get("SVC_SHRINK_US") == 100
    l0, g0 = b.get("SVC_LAUNCHES"), b.get("SVC_REGROWS")
    for k in range(3):
        time.sleep(0.002)
        ar(b, k)
    assert b.get("SVC_LAUNCHES") == l0 and b.get("SVC_REGROWS") == g0, "the shrunk service serves small calls"
    xb = torch.full((16384,), float(rank + 1), device="cuda")  # 64 KiB: 16 slices
    yb = torch.empty_like(xb)
    torch.cuda.synchronize()
    b.allreduce(xb.data_ptr(), yb.data_ptr(), xb.numel(), f32, SUM)
    assert bool(torch.all(yb == want).item()), "allreduce after the grid regrew"
    assert b.get("SVC_REGROWS") == g0 + 1 and b.get("SVC_LAUNCHES") == l0 + 1, (b.get("SVC_REGROWS"), b.get("SVC_LAUNCHES"))
    for k in range(5):  # a without the service: the per-call paths, exact
        ar(a, k)
    # idle exit and relaunch (a short idle limit on a fresh owner)
    a.barrier()
    a.destroy()
    b.barrier()
    b.destroy()
    os.environ["MI355X_SVC_IDLE_MS"] = "2"
    c = pkg.Comm.create(key + "_c", rank, size, dev)
    c.set("SVC_MAX_BYTES", 64 << 10)
    for k in range(20):
        ar(c, k)
        time.sleep(0.01)  # longer than the idle limit: the service has left; the next call relaunches
    assert c.get("SVC_OWNER") == 1, "a communicator created after the owners left gets the service"
    assert c.get("SVC_LAUNCHES") >= 10, c.get("SVC_LAUNCHES")
    print(f"rank {rank} svc: sync {dt_sync * 1e3:.2f} ms, fresh stream {dt_stream * 1e3:.2f} ms while resident; "
          f"{relaunched} relaunches over 200 calls; handed over after idle ({handed} calls served on the second "
          f"communicator); {c.get('SVC_LAUNCHES')} launches over 20 spaced calls", flush=True)
    c.barrier()
    c.destroy()
    print(f"rank {rank} svc OK", flush=True)


def svc_dup(key, rank, size, dev):
    """MPI_COMM_WORLD created first, then a dup that issues the small allreduces (the usual gradient-
    communicator pattern): the dup is served by the resident service; world's own small calls later
    take it back once the dup has been idle, and the dup again after world; every result exact and
    every rank reports the same owner at every step"""
    import time
    import torch
    torch.cuda.set_device(dev)
    pkg = load_pkg()
    f32, SUM = pkg.T["FLOAT"], pkg.OP["SUM"]
    world = pkg.Comm.create(key + "_w", rank, size, dev)
    dup = pkg.Comm.create(key + "_d", rank, size, dev)
    x = torch.empty(2048, device="cuda")
    y = torch.empty_like(x)
    owners = []

    def burst(c, tag, calls=100):
        for k in range(calls):
            x.fill_(float(rank + 1 + k))
            y.fill_(-1)
            torch.cuda.synchronize()
            c.allreduce(x.data_ptr(), y.data_ptr(), 2048, f32, SUM)
            assert bool(torch.all(y == size * (size + 1) / 2 + size * k).item()), (tag, k)
        owners.append(f"{tag}:world={world.get('SVC_OWNER')},dup={dup.get('SVC_OWNER')}")

    l0 = dup.get("SVC_LAUNCHES")
    burst(dup, "dup")
    assert dup.get("SVC_OWNER") == 1 and dup.get("SVC_LAUNCHES") > l0, "the dup is served"
    assert world.get("SVC_OWNER") == 0
    time.sleep(0.05)                  # dup idle: world's small calls take the service over
    burst(world, "world")
    assert world.get("SVC_OWNER") == 1 and dup.get("SVC_OWNER") == 0
    time.sleep(0.05)
    burst(dup, "dup2")
    assert dup.get("SVC_OWNER") == 1 and world.get("SVC_OWNER") == 0
    print(f"rank {rank} owners {' '.join(owners)} claims world={world.get('SVC_CLAIMS')} dup={dup.get('SVC_CLAIMS')}",
          flush=True)
    for c in (dup, world):
        c.barrier()
        c.destroy()
    print(f"rank {rank} svc_dup OK", flush=True)


def selftest(key, rank, size, dev):
    """the creation-time / first-claim flow self-tests: with MI355X_SELFTEST_FAIL=<flow> on one rank
    (fault injection), that flow is off on EVERY rank (FLOWS / FLOWS_FAILED agree) and calls of every
    kind stay exact vs the oracle; with no injection every flow is on.  Creation time is printed."""
    import torch
    torch.cuda.set_device(dev)
    pkg = load_pkg()
    oracle = load_oracle()
    ptrs = lambda arrs: (ctypes.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])
    # SVC_OPEN: the service cannot open on one rank -> no rank claims it, nothing is self-tested
    open_fail = os.environ.get("SELFTEST_EXPECT", "") == "SVC_OPEN"
    expect = pkg.FLOW.get(os.environ.get("SELFTEST_EXPECT", ""), 0)
    comm = pkg.Comm.create(key, rank, size, dev)
    create_us, st_us = comm.get("CREATE_US"), comm.get("SELFTEST_US")
    f32, i32, SUM = pkg.T["FLOAT"], pkg.T["INT32"], pkg.OP["SUM"]
    x = torch.full((1000,), float(rank + 1), device="cuda")
    y = torch.empty_like(x)
    torch.cuda.synchronize()
    comm.allreduce(x.data_ptr(), y.data_ptr(), 1000, f32, SUM)  # the first small call claims the service
    assert bool(torch.all(y == size * (size + 1) / 2).item())
    flows, failed = comm.get("FLOWS"), comm.get("FLOWS_FAILED")
    assert failed == expect, f"flows failed {failed:#x}, expected {expect:#x}"
    assert flows == 0x1f & ~expect, f"flows {flows:#x}"
    assert comm.get("SVC_OWNER") == (0 if expect == pkg.FLOW["SVC_LL"] or open_fail else 1)
    if expect == pkg.FLOW["PIPE"]:
        comm.set("PIPE", 1)
        assert comm.get("PIPE") == 0, "a flow that failed its self-test cannot be forced on"
    else:
        comm.set("PIPE", 1)
    calls0 = comm.get("SVC_CALLS")
    # every kind of call, each size class, exact vs the oracle's schedule simulation
    for count in (3, 2048, 12288, 100_003, size * 300_000):
        xs = [opdata.make("FLOAT", count, 60 + r) for r in range(size)]
        outs = [np.zeros_like(xs[0]) for _ in range(size)]
        oracle.oracle_allreduce(0, size, count, f32, SUM, 0, ptrs(xs), ptrs(outs))
        dx = torch.from_numpy(xs[rank].view(np.uint8).copy()).cuda()
        dr = torch.full_like(dx, 0x5a)
        torch.cuda.synchronize()
        comm.allreduce(dx.data_ptr(), dr.data_ptr(), count, f32, SUM)
        opdata.assert_same("FLOAT", "SUM", dr.cpu().numpy().view(np.float32), outs[rank], f"selftest allreduce {count}")
    for nb in (100, 48 << 10, 1 << 20):
        src = torch.full((nb,), rank + 3, dtype=torch.uint8, device="cuda")
        dst = torch.zeros(nb * size, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        comm.allgather(src.data_ptr(), dst.data_ptr(), nb)
        for r in range(size):
            assert int(dst[r * nb:(r + 1) * nb].min()) == r + 3 == int(dst[r * nb:(r + 1) * nb].max()), ("ag", nb, r)
        b = torch.full((nb,), rank, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        comm.bcast(b.data_ptr(), nb, size - 1)
        assert int(b.min()) == size - 1 == int(b.max()), ("bcast", nb)
    for rcount in (5, 4096, 70_000):
        xs = [opdata.make("INT32", rcount * size, 90 + r) for r in range(size)]
        outs = [np.zeros(rcount, dtype=xs[0].dtype) for _ in range(size)]
        oracle.oracle_reduce_scatter_block(size, rcount, i32, SUM, ptrs(xs), ptrs(outs))
        dx = torch.from_numpy(xs[rank].view(np.uint8).copy()).cuda()
        dr = torch.full((rcount * 4,), 0x5a, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        comm.reduce_scatter_block(dx.data_ptr(), dr.data_ptr(), rcount, i32, SUM)
        opdata.assert_same("INT32", "SUM", dr.cpu().numpy().view(xs[0].dtype), outs[rank], f"selftest rsb {rcount}")
    served = comm.get("SVC_CALLS") - calls0
    if open_fail:
        assert served == 0 and comm.get("SVC_LAUNCHES") == 0, "a service that could not open on one rank serves no rank"
    print(f"rank {rank} flows {flows:#x} failed {failed:#x} create_us {create_us} selftest_us {st_us} "
          f"claim_selftest_us {comm.get('SELFTEST_US') - st_us} served {served}", flush=True)
    # a dup of the same processes takes the verdicts over (no tests): a flow that failed anywhere is
    # off for the dup too, on every rank, and its calls stay exact
    import time
    dup = pkg.Comm.create(key + "dup", rank, size, dev)
    comm.barrier()
    t0 = time.perf_counter()
    dup.allreduce(x.data_ptr(), y.data_ptr(), 1000, f32, SUM)
    dup_ms = (time.perf_counter() - t0) * 1e3
    assert bool(torch.all(y == size * (size + 1) / 2).item())
    assert dup.get("SELFTEST_REUSED") == (1 if open_fail else 2), dup.get("SELFTEST_REUSED")
    assert dup.get("SELFTEST_US") == 0
    assert dup.get("FLOWS") == comm.get("FLOWS") and dup.get("FLOWS_FAILED") == comm.get("FLOWS_FAILED"), \
        (dup.get("FLOWS"), dup.get("FLOWS_FAILED"))
    if expect == pkg.FLOW["PIPE"]:
        dup.set("PIPE", 1)
        assert dup.get("PIPE") == 0, "a flow that failed its self-test cannot be forced on in a dup"
    for count in (3, 12288, size * 300_000):
        xs = [opdata.make("FLOAT", count, 160 + r) for r in range(size)]
        outs = [np.zeros_like(xs[0]) for _ in range(size)]
        oracle.oracle_allreduce(0, size, count, f32, SUM, 0, ptrs(xs), ptrs(outs))
        dx = torch.from_numpy(xs[rank].view(np.uint8).copy()).cuda()
        dr = torch.full_like(dx, 0x5a)
        torch.cuda.synchronize()
        dup.allreduce(dx.data_ptr(), dr.data_ptr(), count, f32, SUM)
        opdata.assert_same("FLOAT", "SUM", dr.cpu().numpy().view(np.float32), outs[rank], f"dup allreduce {count}")
    print(f"rank {rank} dup: first device call {dup_ms:.2f} ms, setup_us {dup.get('SETUP_US')}", flush=True)
    dup.barrier()
    dup.destroy()
    comm.barrier()
    comm.destroy()
    print(f"rank {rank} selftest OK", flush=True)


def svc_stress(key, rank, size, dev):
    """a long random mix of calls every rank makes in the same order (shared seed): small allreduces
    and reduces through the resident service's LL form, 32-128 KiB ones through its pull form, in
    place (host flows), 1 MiB ones (host flows: the service steps aside), allgather and bcast up to
    128 KiB (LL and pull-copy forms), and pauses shorter and longer than the idle limit (the service leaves and comes back, and
    a pause can end just as it leaves) -- every result checked exactly"""
    import time
    import torch
    torch.cuda.set_device(dev)
    pkg = load_pkg()
    comm = pkg.Comm.create(key + "_stress", rank, size, dev)
    assert comm.get("SVC_MAX_BYTES") > 0, "the stress communicator owns the service"
    rng = np.random.default_rng(20261017)
    f32, f64, i32 = pkg.T["FLOAT"], pkg.T["DOUBLE"], pkg.T["INT32"]
    SUM, MAX = pkg.OP["SUM"], pkg.OP["MAX"]
    iters = int(os.environ.get("SVC_STRESS_ITERS", "6000"))
    kinds = ["ar_small", "ar_pull", "ar_inplace", "ar_host", "reduce", "allgather", "bcast", "pause", "rs"]
    probs = [0.3, 0.14, 0.08, 0.05, 0.1, 0.09, 0.07, 0.09, 0.08]
    counts = {k: 0 for k in kinds}
    calls0, launches0 = comm.get("SVC_CALLS"), comm.get("SVC_LAUNCHES")
    for it in range(iters):
        kind = kinds[rng.choice(len(kinds), p=probs)]
        counts[kind] += 1
        base = float(1 + it % 5)
        if kind == "pause":
            time.sleep(float(rng.choice([0.0002, 0.0009, 0.0011, 0.003])))
            continue
        if kind in ("ar_small", "ar_pull", "ar_inplace", "ar_host"):
            nbytes = {"ar_small": int(rng.integers(1, 32 << 10)), "ar_pull": int(rng.integers((32 << 10) + 16, 128 << 10)),
                      "ar_inplace": int(rng.integers(1, 128 << 10)), "ar_host": 1 << 20}[kind]
            ty, tdt = [(f32, torch.float32), (f64, torch.float64), (i32, torch.int32)][it % 3]
            esz = 8 if ty == f64 else 4
            n = max(1, nbytes // esz)
            op = MAX if ty == i32 else SUM
            x = torch.full((n,), base + rank, dtype=tdt, device="cuda")
            want = (base + size - 1) if op == MAX else sum(base + r for r in range(size))
            if kind == "ar_inplace":
                torch.cuda.synchronize()
                comm.allreduce(None, x.data_ptr(), n, ty, op)
                y = x
            else:
                y = torch.full_like(x, -7)
                torch.cuda.synchronize()
                comm.allreduce(x.data_ptr(), y.data_ptr(), n, ty, op)
            assert bool(torch.all(y == want).item()), (it, kind, n, ty, op)
        elif kind == "reduce":
            n = int(rng.integers(1, 8 << 10))
            root = int(rng.integers(0, size))
            x = torch.full((n,), base + rank, dtype=torch.float32, device="cuda")
            y = torch.full_like(x, -7)
            torch.cuda.synchronize()
            comm.reduce(x.data_ptr(), y.data_ptr() if rank == root else None, n, f32, SUM, root)
            if rank == root:
                assert bool(torch.all(y == sum(base + r for r in range(size))).item()), (it, kind, n, root)
        elif kind == "allgather":
            nb = int(rng.integers(1, 128 << 10))
            src = torch.full((nb,), (rank + it) % 251, dtype=torch.uint8, device="cuda")
            dst = torch.zeros(nb * size, dtype=torch.uint8, device="cuda")
            torch.cuda.synchronize()
            comm.allgather(src.data_ptr(), dst.data_ptr(), nb)
            for r in range(size):
                assert bool(torch.all(dst[r * nb:(r + 1) * nb] == (r + it) % 251).item()), (it, kind, nb, r)
        elif kind == "rs":  # reduce_scatter_block: service pull form, or the host flow in place
            n = int(rng.integers(1, 40 << 10))
            inplace = it % 4 == 0
            x = torch.full((n * size,), base + rank, dtype=torch.float32, device="cuda")
            y = x if inplace else torch.full((n,), -7.0, dtype=torch.float32, device="cuda")
            torch.cuda.synchronize()
            comm.reduce_scatter_block(None if inplace else x.data_ptr(), y.data_ptr(), n, f32, SUM)
            assert bool(torch.all(y[:n] == sum(base + r for r in range(size))).item()), (it, kind, n, inplace)
        else:  # bcast
            nb = int(rng.integers(1, 128 << 10))
            root = int(rng.integers(0, size))
            b = torch.full((nb,), (rank * 7 + it) % 251, dtype=torch.uint8, device="cuda")
            torch.cuda.synchronize()
            comm.bcast(b.data_ptr(), nb, root)
            assert bool(torch.all(b == (root * 7 + it) % 251).item()), (it, kind, nb, root)
    served, launches = comm.get("SVC_CALLS") - calls0, comm.get("SVC_LAUNCHES") - launches0
    assert served > iters // 3, served
    print(f"rank {rank} svc stress: {iters} calls {counts}, {served} served by the service, {launches} launches",
          flush=True)
    comm.barrier()
    comm.destroy()
    print(f"rank {rank} svc_stress OK", flush=True)


def lazy_setup(key, rank, size, dev):
    """smcuda's lazy rule (btl/smcuda/README:36-40): creating a communicator does no device work.
    Five communicators are created after a barrier of an existing one (an MPI_Comm_dup of an
    already-synchronised group): each is host-only until its first device-buffer collective
    (DEV_SETUP 0; no device memory taken on the GPU, which every rank shares here), creation is
    timed; then one allreduce on device buffers runs the device setup and is exact."""
    import json
    import time
    import torch
    torch.cuda.set_device(dev)
    torch.zeros(1, device="cuda")  # this process's HIP context and allocator first
    torch.cuda.synchronize()
    pkg = load_pkg()
    base = pkg.Comm.create(key + "b", rank, size, dev)
    base.barrier()
    free0 = torch.cuda.mem_get_info()[0]
    base.barrier()
    comms, wall = [], []
    for rep in range(5):
        base.barrier()
        t0 = time.perf_counter()
        c = pkg.Comm.create(f"{key}d{rep}", rank, size, dev)
        wall.append((time.perf_counter() - t0) * 1e6)
        comms.append(c)
        assert c.get("DEV_SETUP") == 0, "device setup ran at creation"
        c.barrier()  # host-only use
        assert c.vote(0) == 0
    base.barrier()
    free1 = torch.cuda.mem_get_info()[0]
    base.barrier()
    assert free1 == free0, f"host-only communicators took {free0 - free1} bytes of device memory"
    assert all(c.get("DEV_SETUP") == 0 for c in comms)
    create_us = [c.get("CREATE_US") for c in comms]
    # the first device-buffer collective runs the setup, collectively
    c = comms[-1]
    x = torch.full((4096,), float(rank + 1), device="cuda")
    y = torch.empty_like(x)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    c.allreduce(x.data_ptr(), y.data_ptr(), 4096, pkg.T["FLOAT"], pkg.OP["SUM"])
    first_ms = (time.perf_counter() - t0) * 1e3
    assert bool(torch.all(y == size * (size + 1) / 2).item())
    assert c.get("DEV_SETUP") == 1 and all(k.get("DEV_SETUP") == 0 for k in comms[:-1])
    assert c.get("SELFTEST_REUSED") == 0 or c.get("SELFTEST_US") == 0
    setup_us = c.get("SETUP_US")
    # the next communicator of the same processes (a dup): the flow verdicts are taken over
    c2 = comms[-2]
    base.barrier()
    t0 = time.perf_counter()
    c2.allreduce(x.data_ptr(), y.data_ptr(), 4096, pkg.T["FLOAT"], pkg.OP["SUM"])
    dup_ms = (time.perf_counter() - t0) * 1e3
    assert bool(torch.all(y == size * (size + 1) / 2).item())
    assert c2.get("SELFTEST_REUSED") >= 1 and c2.get("SELFTEST_US") == 0, (c2.get("SELFTEST_REUSED"), c2.get("SELFTEST_US"))
    dup_setup_us = c2.get("SETUP_US")
    for k in comms:
        k.barrier()
        k.destroy()
    base.barrier()
    base.destroy()
    wall.sort()
    print(json.dumps({"rank": rank, "n": size, "create_wall_us": [round(w, 1) for w in wall],
                      "create_us_knob": create_us, "device_bytes_taken": free0 - free1,
                      "first_device_call_ms": round(first_ms, 2), "device_setup_us": setup_us,
                      "dup_first_device_call_ms": round(dup_ms, 2), "dup_device_setup_us": dup_setup_us}), flush=True)
    print(f"rank {rank} lazy OK", flush=True)


def done_words(key, rank, size, dev):
    """MI355X_DONE_WORDS=1 (finish points by command-processor-written completion words, off by
    default: slower back to back on this platform, profiles/r03_small_latency.jsonl): every flow that
    ends in a finish point stays exact -- one-phase and two-phase allreduce, reduce_scatter_block,
    allgather, bcast"""
    import os
    import torch
    os.environ["MI355X_DONE_WORDS"] = "1"
    torch.cuda.set_device(dev)
    pkg = load_pkg()
    comm = pkg.Comm.create(key + "_dw", rank, size, dev)
    comm.set("PIPE", 0)
    f32, SUM = pkg.T["FLOAT"], pkg.OP["SUM"]
    for it, n in enumerate((2, 16384, 262144, 4_000_000)):
        x = torch.full((n * size,), float(rank + 1 + it), device="cuda")
        y = torch.empty_like(x)
        torch.cuda.synchronize()
        comm.allreduce(x.data_ptr(), y.data_ptr(), n * size, f32, SUM)
        want = sum(r + 1 + it for r in range(size))
        assert bool(torch.all(y == want).item()), ("done-words allreduce", n)
        r = torch.empty(n, device="cuda")
        comm.reduce_scatter_block(x.data_ptr(), r.data_ptr(), n, f32, SUM)
        assert bool(torch.all(r == want).item()), ("done-words rsb", n)
        g = torch.empty(n * size, device="cuda")
        comm.allgather(r.data_ptr(), g.data_ptr(), n * 4)
        assert bool(torch.all(g == want).item()), ("done-words allgather", n)
        b = torch.full((n,), float(rank), device="cuda")
        torch.cuda.synchronize()
        comm.bcast(b.data_ptr(), n * 4, size - 1)
        assert bool(torch.all(b == size - 1).item()), ("done-words bcast", n)
    comm.barrier()
    comm.destroy()
    print(f"rank {rank} done_words OK", flush=True)


def host_bw(key, rank, size, dev):
    """host -> host point-to-point rate between two processes, one JSON line per (pattern, size) from
    rank 0: `oneway` (rank 0 sends, rank 1 is already waiting in MPI_Recv; a 1-byte reply closes
    each round) and `sendrecv` (both directions at once); MI355X_P2P_STREAM_MIN selects the copy-in
    protocol"""
    import json
    import os
    import time
    import torch
    torch.cuda.set_device(dev)
    pkg = load_pkg()
    comm = pkg.Comm.create(key, rank, size, dev)
    peer = 1 - rank
    ack = np.zeros(1, dtype=np.uint8)
    for pattern in ("oneway", "sendrecv"):
        for n in (1 << 20, 8 << 20, 64 << 20):
            src = np.random.default_rng(rank + n).integers(0, 256, n, dtype=np.uint8)
            dst = np.zeros(n, dtype=np.uint8)
            reps = max(4, min(40, (512 << 20) // n))

            def once():
                if pattern == "sendrecv":
                    comm.sendrecv(src.ctypes.data, n, peer, 9, dst.ctypes.data, n, peer, 9)
                elif rank == 0:
                    comm.send(src.ctypes.data, n, 1, 9)
                    comm.recv(ack.ctypes.data, 1, 1, 10)
                else:
                    comm.recv(dst.ctypes.data, n, 0, 9)
                    comm.send(ack.ctypes.data, 1, 0, 10)

            for _ in range(2):
                once()
            comm.barrier()
            t0 = time.perf_counter()
            for _ in range(reps):
                once()
            comm.barrier()
            dt = (time.perf_counter() - t0) / reps
            if pattern == "sendrecv" or rank == 1:
                assert np.array_equal(dst, np.random.default_rng(peer + n).integers(0, 256, n, dtype=np.uint8))
            if rank == 0:
                print(json.dumps({"leg": "host_p2p_" + pattern, "bytes": n, "us": round(dt * 1e6, 1),
                                  "GBs_per_direction": round(n / dt / 1e9, 2),
                                  "stream_min": os.environ.get("MI355X_P2P_STREAM_MIN", "default"),
                                  "frag": os.environ.get("MI355X_P2P_STREAM_FRAG", "default")}), flush=True)
    comm.barrier()
    comm.destroy()
    print(f"rank {rank} host_bw OK", flush=True)


def rcache_p2p(key, rank, size, dev):
    """the bounded peer-mapping cache in a point-to-point-only phase: 2 ranks, bound 4;
    rank 0 sends 24 distinct device buffers to rank 1 (the receiver pulls each from the sender's
    allocation), then sends the first 8 again -- mappings evicted meanwhile are opened again (a
    dmabuf fd asked for again from the sender, which serves the request while it waits in its send);
    the receiver's open mappings stay within the bound, every payload exact"""
    import torch
    torch.cuda.set_device(dev)
    pkg = load_pkg()
    comm = pkg.Comm.create(key, rank, size, dev)
    comm.set("RCACHE_MAX_MAPS", 4)
    keep = []
    peak = 0
    for k in list(range(24)) + list(range(8)):
        n = (1 << 18) + k * (1 << 17)
        if rank == 0:
            if k >= len(keep):
                keep.append(torch.full((n,), float(k + 1), device="cuda"))
                torch.cuda.synchronize()
            comm.send(keep[k].data_ptr(), n * 4, 1, k)
        else:
            y = torch.zeros(n, device="cuda")
            torch.cuda.synchronize()
            comm.recv(y.data_ptr(), n * 4, 0, k)
            torch.cuda.synchronize()
            assert bool(torch.all(y == float(k + 1)).item()), ("rcache_p2p payload", k)
            peak = max(peak, comm.get("PEER_MAPS"))
    ev = comm.get("RCACHE_EVICTIONS")
    if rank == 1:
        assert peak <= 4, f"{peak} peer mappings open under a bound of 4"
        assert ev > 0, "no evictions"
        print(f"rank {rank} rcache_p2p: peak {peak} mappings, {ev} evictions", flush=True)
    comm.barrier()
    comm.destroy()
    print(f"rank {rank} rcache_p2p OK", flush=True)


def rcache(key, rank, size, dev):
    """the bounded peer-mapping cache (RCACHE_MAX_MAPS, mpool/rgpusm's LRU): 64 distinct allocations
    per rank, each one a 1 MiB allreduce's input and output, then freed and 64 more -- the open
    mappings of peers' allocations never exceed the bound, evictions happen, every result exact"""
    import torch
    torch.cuda.set_device(dev)
    pkg = load_pkg()
    comm = pkg.Comm.create(key, rank, size, dev)
    bound = int(os.environ.get("RCACHE_BOUND", "16"))  # (experiments: 0 = unbounded)
    comm.set("RCACHE_MAX_MAPS", bound)
    assert comm.get("RCACHE_MAX_MAPS") == bound
    n = (1 << 20) // 4
    peak = 0
    for rnd in range(int(os.environ.get("RCACHE_ROUNDS", "2"))):
        keep = []
        for k in range(64):
            # distinct allocations: each larger than the last, all alive until the round ends
            # rank r contributes m * 256**r (m = 1 + k + 64 rnd < 256): a wrong sum names, digit by
            # digit, whose buffer of which call every rank's contribution came from
            m = 1 + k + 64 * rnd
            x = torch.full((n + k * (1 << 19),), float(m * 256 ** rank), device="cuda")
            y = torch.full_like(x, float("nan"))
            torch.cuda.synchronize()
            comm.allreduce(x.data_ptr(), y.data_ptr(), n, pkg.T["FLOAT"], pkg.OP["SUM"])
            want = sum(m * 256 ** r for r in range(size))
            bad = (y[:n] != want).nonzero()
            if bad.numel():
                got = int(y[int(bad[0])].item())
                print("rcache: wrong sum", rnd, k, "per-rank m:", [(got >> (8 * r)) & 255 for r in range(size)],
                      "want", m, "bad", bad.numel(), "alg", comm.last_algorithm(), "maps", comm.get("PEER_MAPS"),
                      hex(x.data_ptr()), hex(y.data_ptr()), flush=True)
            assert bad.numel() == 0, ("rcache allreduce", rnd, k)
            peak = max(peak, comm.get("PEER_MAPS"))
            keep += [x, y]
        comm.barrier()  # no peer still reads them
        del keep, x, y
        torch.cuda.empty_cache()
    ev = comm.get("RCACHE_EVICTIONS")
    print(f"rank {rank} rcache export mismatches: {comm.get('EXPORT_MISMATCHES')}", flush=True)
    assert peak <= 16, f"{peak} peer mappings open under a bound of 16"
    assert ev > 0, "no evictions"
    print(f"rank {rank} rcache: peak {peak} mappings, {ev} evictions", flush=True)
    comm.barrier()
    comm.destroy()
    print(f"rank {rank} rcache OK", flush=True)


def p2p_fault(key, rank, size, dev):
    """a small device send offered two ways (device buffer + host copy) whose host copy FAILS on the
    sender (MI355X_P2P_INJECT=1) while the receiver cannot map the device buffer at first
    (P2P_EXPECT=ok: the first mapping fails, INJECT=2) or ever (P2P_EXPECT=fail, INJECT=4): the sender
    publishes claim 3, the receiver maps again and pulls (exact) or fails its receive with an error,
    and the sender's send completes either way -- neither side waits for the other forever"""
    expect = os.environ.get("P2P_EXPECT", "ok")
    # (read by the engine at its first point-to-point pass)
    os.environ["MI355X_P2P_INJECT"] = "1" if rank == 0 else ("2" if expect == "ok" else "4")
    os.environ["MI355X_P2P_DUAL_DELAY_US"] = "0"
    import torch
    torch.cuda.set_device(dev)
    pkg = load_pkg()
    comm = pkg.Comm.create(key, rank, size, dev)
    n = 1000  # > the inline limit, <= the 4 KiB eager limit: a dual offer
    data = (np.arange(n) * 7 % 251).astype(np.uint8)
    # a first host message sets up (and registers) the sender's host arena: only then are small
    # device sends offered two ways
    warm = np.arange(2000, dtype=np.uint8)
    if rank == 0:
        comm.send(warm.ctypes.data, warm.nbytes, 1, 4)
    else:
        got = np.zeros_like(warm)
        comm.recv(got.ctypes.data, got.nbytes, 0, 4)
        assert np.array_equal(got, warm)
    if rank == 0:
        s = torch.from_numpy(data).cuda()
        torch.cuda.synchronize()
        comm.send(s.data_ptr(), n, 1, 5)
    else:
        d = torch.zeros(n, dtype=torch.uint8, device="cuda")
        req = comm.irecv(d.data_ptr(), n, 0, 5)
        try:
            req.wait()
            assert expect == "ok", "the receive succeeded although the buffer was never readable"
            assert np.array_equal(d.cpu().numpy(), data), "p2p fault: wrong bytes"
        except pkg.MI355XError as e:
            assert expect == "fail", f"the receive failed: {e}"
            assert "readable" in str(e), e
    comm.barrier()
    comm.destroy()
    print(f"rank {rank} p2p_fault: {expect}", flush=True)
    print(f"rank {rank} p2p_fault OK", flush=True)


def p2p_in_coll(key, rank, size, dev):
    """MPI's progress rule across a collective: rank 0 posts a receive of a device payload (pulled
    from the sender's allocation: a peer mapping to open) and enters an allreduce; rank 1 completes
    a blocking send of it first (its FIN comes only once rank 0 has read the payload), then enters
    the allreduce.  Rank 0's progress inside the collective's barrier must serve the receive (ob1
    progresses a posted receive inside any blocking call).  Twice: the receive on the collective's
    own communicator, then on a second one"""
    import torch
    torch.cuda.set_device(dev)
    pkg = load_pkg()
    comm = pkg.Comm.create(key, rank, size, dev)
    other = pkg.Comm.create(key + "_p", rank, size, dev)
    n = 4 << 20  # 16 MiB of fp32: neither inline nor a dual offer
    x = torch.full((256,), float(rank + 1), device="cuda")
    y = torch.zeros_like(x)
    for it, pc in enumerate((comm, other)):
        if rank == 0:
            d = torch.zeros(n, device="cuda")
            torch.cuda.synchronize()
            req = pc.irecv(d.data_ptr(), n * 4, 1, 7 + it)
            comm.allreduce(x.data_ptr(), y.data_ptr(), 256, pkg.T["FLOAT"], pkg.OP["SUM"])
            req.wait()
            torch.cuda.synchronize()
            assert bool(torch.all(d == float(11 + it)).item()), ("p2p_in_coll payload", it)
        else:
            s = torch.full((n,), float(11 + it), device="cuda")
            torch.cuda.synchronize()
            pc.send(s.data_ptr(), n * 4, 0, 7 + it)
            comm.allreduce(x.data_ptr(), y.data_ptr(), 256, pkg.T["FLOAT"], pkg.OP["SUM"])
        torch.cuda.synchronize()
        assert bool(torch.all(y == float(size * (size + 1) // 2)).item()), ("p2p_in_coll allreduce", it)
    comm.barrier()
    other.destroy()
    comm.destroy()
    print(f"rank {rank} p2p_in_coll OK", flush=True)


def carved(key, rank, size, dev):
    """the bounded cache's dmabuf export check is on identity, not contents: the runtime carves small
    hipMallocs out of one buffer object and exports the whole object from its start, so a carved
    allocation's fd names another range.  Every rank takes a carved 64 KiB allocation (found here by
    its fd's size) whose bytes at the old content check's three sample offsets are zero -- as are the
    object's first bytes (every allocation of the object zero-filled) -- makes it its allreduce input,
    and the engine must send it the hipIpc way (EXPORT_MISMATCHES + 1) with an exact result"""
    import torch
    torch.cuda.set_device(dev)
    hip = ctypes.CDLL("libamdhip64.so")
    vp, sz_t = ctypes.c_void_p, ctypes.c_size_t
    hip.hipMalloc.argtypes = [ctypes.POINTER(vp), sz_t]
    hip.hipMemset.argtypes = [vp, ctypes.c_int, sz_t]
    hip.hipMemcpy.argtypes = [vp, vp, sz_t, ctypes.c_int]
    hip.hipFree.argtypes = [vp]
    hip.hipMemGetHandleForAddressRange.argtypes = [ctypes.POINTER(ctypes.c_int), vp, sz_t, ctypes.c_int,
                                                   ctypes.c_ulonglong]
    pkg = load_pkg()
    comm = pkg.Comm.create(key, rank, size, dev)
    comm.set("RCACHE_MAX_MAPS", 16)   # a bounded cache: allocations go as dmabuf fds
    nb = 64 << 10
    allocs, found = [], None
    for _ in range(32):
        p = vp()
        assert hip.hipMalloc(ctypes.byref(p), nb) == 0
        assert hip.hipMemset(p, 0, nb) == 0
        allocs.append(p.value)
    for p in allocs:
        fd = ctypes.c_int(-1)
        if hip.hipMemGetHandleForAddressRange(ctypes.byref(fd), vp(p), nb, 1, 0) != 0:
            continue
        end = os.lseek(fd.value, 0, os.SEEK_END)
        os.close(fd.value)
        if end > nb:
            found = p
            break
    assert found is not None, "no carved allocation among 32 small hipMallocs"
    count = nb // 4
    x = np.arange(count, dtype=np.float32) * (rank + 1) + 7 * rank + 1
    for o in (0, (nb // 2) & ~15, nb - 16):   # the old check's sample offsets: zero, like the object's start
        x[o // 4:o // 4 + 4] = 0
    assert hip.hipMemcpy(vp(found), vp(x.ctypes.data), nb, 1) == 0   # hipMemcpyHostToDevice
    y = torch.full((count,), float("nan"), device="cuda")
    torch.cuda.synchronize()
    before = comm.get("EXPORT_MISMATCHES")
    comm.allreduce(found, y.data_ptr(), count, pkg.T["FLOAT"], pkg.OP["SUM"])
    want = sum(np.arange(count, dtype=np.float32) * (r + 1) + 7 * r + 1 for r in range(size))
    for o in (0, (nb // 2) & ~15, nb - 16):
        want[o // 4:o // 4 + 4] = 0
    got = y.cpu().numpy()
    assert np.array_equal(got, want), ("carved allreduce", np.nonzero(got != want)[0][:8])
    mism = comm.get("EXPORT_MISMATCHES") - before
    assert mism >= 1, "the carved allocation was exported as a dmabuf fd"
    comm.barrier()
    for p in allocs:
        hip.hipFree(vp(p))
    comm.destroy()
    print(f"rank {rank} carved: mismatches +{mism}", flush=True)
    print(f"rank {rank} carved OK", flush=True)


def vote_dead(key, rank, size, dev):
    """a peer process that dies without a word (os._exit right after creation): the surviving
    host-buffer rank waiting in the buffer-kind vote (an unbounded wait) returns an error within
    seconds instead of spinning forever"""
    import time
    import torch
    torch.cuda.set_device(dev)
    pkg = load_pkg()
    comm = pkg.Comm.create(key, rank, size, dev)
    comm.barrier()
    if rank == 1:
        os._exit(0)
    t0 = time.time()
    try:
        comm.vote(False)
        raise AssertionError("the vote returned although its peer is gone")
    except pkg.MI355XError as e:
        assert "gone" in str(e), e
    dt = time.time() - t0
    assert dt < 30, dt
    print(f"rank {rank} vote: dead peer noticed after {dt:.2f} s", flush=True)
    print(f"rank {rank} vote_dead OK", flush=True)


def dead_peer(key, rank, size, dev):
    """a peer process that dies without a word after one device allreduce: the surviving rank's next
    small device allreduce -- through the resident service, a per-call LL launch or the host flow
    (DEAD_FLOW, set up by the caller's environment) -- returns an error naming the gone peer within
    seconds, although every wait's bound is far away (MI355X_TIMEOUT_S=100): the host finds the peer
    gone by its pid and sends the waiting kernel away through the error word"""
    import time
    import torch
    torch.cuda.set_device(dev)
    pkg = load_pkg()
    comm = pkg.Comm.create(key, rank, size, dev)
    x = torch.full((256,), float(rank + 1), device="cuda")
    y = torch.zeros_like(x)
    comm.allreduce(x.data_ptr(), y.data_ptr(), 256, pkg.T["FLOAT"], pkg.OP["SUM"])
    torch.cuda.synchronize()
    assert bool(torch.all(y == 3.0).item())
    comm.barrier()
    if rank == 1:
        os._exit(0)
    time.sleep(0.5)
    t0 = time.time()
    try:
        comm.allreduce(x.data_ptr(), y.data_ptr(), 256, pkg.T["FLOAT"], pkg.OP["SUM"])
        torch.cuda.synchronize()
        raise AssertionError("the allreduce returned although its peer is gone")
    except pkg.MI355XError as e:
        assert "gone" in str(e) or "aborted" in str(e), e
    dt = time.time() - t0
    assert dt < 30, dt
    print(f"rank {rank} dead peer ({os.environ.get('DEAD_FLOW')}): noticed after {dt:.2f} s", flush=True)
    print(f"rank {rank} dead_peer OK", flush=True)


def token_hold(key, dev):
    """a one-rank communicator takes its GPU's pipelined-grid admission token (as a rank inside a
    pipelined allreduce holds it) and sleeps until the test SIGKILLs it"""
    import time
    import torch
    torch.cuda.set_device(dev)
    pkg = load_pkg()
    comm = pkg.Comm.create(key, 0, 1, dev)
    assert comm.debug_pipe_token(True), "the admission token of a free GPU"
    print("holding", flush=True)
    time.sleep(300)


def token_check(key, rank, size, dev):
    """pipelined 64 MiB allreduces (MI355X_PIPE=1): exact, and PIPE_REFUSED reported for the test to
    compare with whether another process holds this GPU's admission token"""
    import torch
    torch.cuda.set_device(dev)
    pkg = load_pkg()
    comm = pkg.Comm.create(key, rank, size, dev)
    comm.set("PIPE", 1)
    n = (64 << 20) // 4
    for it in range(3):
        x = torch.full((n,), float(rank + 1 + it), device="cuda")
        y = torch.full_like(x, float("nan"))
        torch.cuda.synchronize()
        comm.allreduce(x.data_ptr(), y.data_ptr(), n, pkg.T["FLOAT"], pkg.OP["SUM"])
        assert bool(torch.all(y == sum(r + 1 + it for r in range(size))).item()), ("token check", it)
    print(f"rank {rank} refused {comm.get('PIPE_REFUSED')}", flush=True)
    comm.barrier()
    comm.destroy()
    print(f"rank {rank} token_check OK", flush=True)


def main():
    try:
        _main()
    except BaseException:
        _fd_report(int(sys.argv[2]))
        raise


def _main():
    key, rank, size, dev = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    if len(sys.argv) > 5 and sys.argv[5] == "concurrent":
        return concurrent_comms(key, rank, size, dev)
    if len(sys.argv) > 5 and sys.argv[5] == "svc_dup":
        return svc_dup(key, rank, size, dev)
    if len(sys.argv) > 5 and sys.argv[5] == "selftest":
        return selftest(key, rank, size, dev)
    if len(sys.argv) > 5 and sys.argv[5] == "vote_dead":
        return vote_dead(key, rank, size, dev)
    if len(sys.argv) > 5 and sys.argv[5] == "dead_peer":
        return dead_peer(key, rank, size, dev)
    if len(sys.argv) > 5 and sys.argv[5] == "rcache":
        return rcache(key, rank, size, dev)
    if len(sys.argv) > 5 and sys.argv[5] == "rcache_p2p":
        return rcache_p2p(key, rank, size, dev)
    if len(sys.argv) > 5 and sys.argv[5] == "carved":
        return carved(key, rank, size, dev)
    if len(sys.argv) > 5 and sys.argv[5] == "p2p_fault":
        return p2p_fault(key, rank, size, dev)
    if len(sys.argv) > 5 and sys.argv[5] == "p2p_in_coll":
        return p2p_in_coll(key, rank, size, dev)
    if len(sys.argv) > 5 and sys.argv[5] == "token_hold":
        return token_hold(key, dev)
    if len(sys.argv) > 5 and sys.argv[5] == "token_check":
        return token_check(key, rank, size, dev)
    if len(sys.argv) > 5 and sys.argv[5] == "done_words":
        return done_words(key, rank, size, dev)
    if len(sys.argv) > 5 and sys.argv[5] == "lazy":
        return lazy_setup(key, rank, size, dev)
    if len(sys.argv) > 5 and sys.argv[5] == "host_bw":
        return host_bw(key, rank, size, dev)
    if len(sys.argv) > 5 and sys.argv[5] == "svc":
        return svc_mode(key, rank, size, dev)
    if len(sys.argv) > 5 and sys.argv[5] == "svc_stress":
        return svc_stress(key, rank, size, dev)
    import faulthandler
    faulthandler.dump_traceback_later(150, exit=True)  # a rank stuck in a HIP call names its line
    import torch
    torch.cuda.set_device(dev)
    pkg = load_pkg()
    oracle = load_oracle()
    comm = pkg.Comm.create(key, rank, size, dev)
    ptrs = lambda arrs: (ctypes.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])
    for opname, tname in [("SUM", "FLOAT"), ("MAXLOC", "DOUBLE_INT"), ("PROD", "C_FLOAT_COMPLEX")]:
        op, ty = pkg.OP[opname], pkg.T[tname]
        for count in (5, 3001, 300_007):
            xs = [opdata.make(tname, count, 400 + r) for r in range(size)]
            outs = [np.zeros_like(xs[0]) for _ in range(size)]
            oracle.oracle_allreduce(0, size, count, ty, op, 0, ptrs(xs), ptrs(outs))
            dx = torch.from_numpy(xs[rank].view(np.uint8).copy()).cuda()
            dr = torch.zeros_like(dx)
            torch.cuda.synchronize()
            for rep in range(2):  # second call hits the registration caches
                comm.allreduce(dx.data_ptr(), dr.data_ptr(), count, ty, op)
                got = dr.cpu().numpy().view(xs[0].dtype)
                opdata.assert_same(tname, opname, got, outs[rank], f"ipc allreduce rank={rank} rep={rep}")
    # bcast + allgather through IPC
    nb = 1_000_003
    buf = torch.full((nb,), rank, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    comm.bcast(buf.data_ptr(), nb, size - 1)
    assert int(buf.min()) == size - 1 and int(buf.max()) == size - 1
    src = torch.full((nb,), rank + 1, dtype=torch.uint8, device="cuda")
    dst = torch.zeros(nb * size, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    comm.allgather(src.data_ptr(), dst.data_ptr(), nb)
    for r in range(size):
        assert int(dst[r * nb:(r + 1) * nb].min()) == r + 1
    realloc_same_address(pkg, comm, rank, size)
    pipe_checks(pkg, comm, rank, size, oracle, torch)
    if size == 3:
        pipe_all_slots(pkg, comm, rank, size, oracle, torch)
    ll_checks(pkg, comm, rank, size, oracle, torch)
    calls0 = comm.get("SVC_CALLS")
    ll_checks(pkg, comm, rank, size, oracle, torch, knob="SVC_MAX_BYTES")
    served, launches = comm.get("SVC_CALLS") - calls0, comm.get("SVC_LAUNCHES")
    assert served > 100, f"the resident service served {served} calls"
    print(f"rank {rank} resident service: {served} calls, {launches} launches", flush=True)
    if size in (2, 3):
        svc_all_slots(pkg, comm, rank, size, oracle, torch)
    svc_pull_checks(pkg, comm, rank, size, oracle, torch)
    p2p_checks(pkg, comm, rank, size, oracle, torch)
    _fd_report(rank)
    staged(pkg, comm, rank, size, torch, key)
    if size in (2, 3):
        big_bcast(pkg, comm, rank, size, torch)
    if size == 2:
        max_count(pkg, comm, rank, size, torch)
    comm.barrier()
    comm.destroy()
    print(f"rank {rank} OK", flush=True)


if __name__ == "__main__":
    main()
