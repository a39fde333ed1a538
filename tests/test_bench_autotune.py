"""bench_coll.autotune on CPU (gloo, 2 processes, a fake engine): a flow that fails on one rank
only is dropped by both (they agree before acting), the communicator is rebuilt under a new key,
a candidate whose result is stale on one rank is dropped by both, the remaining one is timed and
chosen, and every rank ends with the same choice."""
from __future__ import annotations

import ctypes
import multiprocessing as mp
import os
import pathlib
import sys

import pytest

REPO = pathlib.Path(__file__).resolve().parents[1]


class FakeError(RuntimeError):
    pass


class FakeComm:
    created = []

    def __init__(self, key, rank):
        self.key, self.rank, self.knobs, self.destroyed = key, rank, {}, False
        FakeComm.created.append(key)

    def set(self, k, v):
        self.knobs[k] = v

    def get(self, k):
        return self.knobs.get(k, 0)

    def destroy(self):
        self.destroyed = True

    def allreduce(self, sbuf, rbuf, n, ty, op):
        if self.knobs.get("PIPE") == 1 and self.rank == 0:  # the pipelined flow fails on rank 0 only
            raise FakeError("pipelined allreduce timed out waiting for a peer")
        # 2 ranks, x_r = r + 1 + 3k (bench_coll.check_calls) -> sum = 3 + 6k; the two-phase flow
        # with a 1024-block grid returns the previous call's sum on rank 1 (a stale hand-off)
        v = ctypes.c_float.from_address(sbuf if sbuf else rbuf).value  # sbuf None: MPI_IN_PLACE
        k = round((v - self.rank - 1) / 3)
        stale = self.knobs.get("BLOCKS_PER_CU") == 1024 and self.rank == 1
        want = (ctypes.c_float * n)(*([3.0 + 6 * (k - (1 if stale else 0))] * n))
        ctypes.memmove(rbuf, want, 4 * n)


class FakePkg:
    MI355XError = FakeError

    class Comm:
        @staticmethod
        def create(key, rank, size, dev):
            return FakeComm(key, rank)


def _rank(rank, port, q):
    try:
        sys.path.insert(0, str(REPO))
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        import torch
        import torch.distributed as dist
        import bench_coll
        dist.init_process_group("gloo", rank=rank, world_size=2)
        n = 64
        x = torch.full((n,), float(rank + 1))
        y = torch.zeros(n)
        cands = [{"pipe": 1, "pipe_wg_per_cu": 2, "pipe_chunk_kib": 0, "pipe_wt": 1},
                 {"pipe": 1, "pipe_wg_per_cu": 4, "pipe_chunk_kib": 0, "pipe_wt": 1},
                 {"pipe": 0, "blocks_per_cu": 1024, "copy_block_kib": 4},
                 {"pipe": 0, "blocks_per_cu": 8, "copy_block_kib": 4}]
        comm0 = FakeComm("k", rank)
        comm, key, tried, ok, best = bench_coll.autotune(
            comm0, "k", cands, pkg=FakePkg, dist=dist, rank=rank, world=2, local=0, x=x, y=y, n=n, ty=0, op=3,
            want=3.0, sync=lambda: None)
        dist.destroy_process_group()
        q.put((rank, dict(key=key, best=best, ok=ok, tried=tried, old_destroyed=comm0.destroyed,
                          new_pipe=comm.knobs.get("PIPE"))))
    except BaseException as e:  # noqa: BLE001
        q.put((rank, repr(e)))


def test_autotune_drops_a_flow_failing_on_one_rank():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29700 + os.getpid() % 200
    ps = [ctx.Process(target=_rank, args=(r, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=180) for _ in ps)
    for p in ps:
        p.join(30)
    for r in (0, 1):
        out = res[r]
        assert isinstance(out, dict), out
        assert out["key"] == "k_r" and out["old_destroyed"], out      # rebuilt once, on both ranks
        assert out["best"]["pipe"] == 0 and out["new_pipe"] == 0, out  # the surviving flow, applied
        assert out["best"]["blocks_per_cu"] == 8, out                  # not the stale candidate
        assert out["ok"], out
        pipe_rows = [t for t in out["tried"] if t["pipe"] == 1]
        assert len(pipe_rows) == 1 and pipe_rows[0]["ms"] is None, out  # the flow dropped after its first failure
        assert "error" in pipe_rows[0]
        stale = [t for t in out["tried"] if t.get("blocks_per_cu") == 1024]
        assert len(stale) == 1 and stale[0]["ms"] is None and "wrong result" in stale[0]["error"], out
    assert res[0]["best"] == res[1]["best"]
