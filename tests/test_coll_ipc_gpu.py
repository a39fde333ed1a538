"""coll/mi355x through the real multi-process path: 2 processes, hipIpcGetMemHandle /
hipIpcOpenMemHandle, node-local shm control segment.  On a one-GPU box both ranks share device 0
(IPC within one device); on an 8-GPU node the same code maps peer devices over xGMI."""
from __future__ import annotations

import os
import pathlib
import subprocess
import sys
import uuid

import pytest

pytestmark = pytest.mark.gpu

HERE = pathlib.Path(__file__).parent


@pytest.mark.parametrize("size", [2, 3, 8])
def test_ipc_ranks(gpu, size):
    key = "t" + uuid.uuid4().hex[:12]
    ndev = gpu.cuda.device_count()
    env = dict(os.environ, MI355X_TIMEOUT_S="60")
    procs = [subprocess.Popen([sys.executable, str(HERE / "ipc_worker.py"), key, str(r), str(size), str(r % ndev)],
                              env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
             for r in range(size)]
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=300)
        except subprocess.TimeoutExpired:
            p.kill()
            out, _ = p.communicate()
        outs.append(out)
    failed = [r for r, p in enumerate(procs) if p.returncode != 0]
    assert not failed, "\n".join(f"rank {r} failed (rc {procs[r].returncode}):\n{outs[r][-2500:]}" for r in failed)
    for r, p in enumerate(procs):
        stages = ("pipe OK", "LL OK", "SVC OK", "pull OK", "p2p OK", "staged OK", "OK") + (("bcast4g OK",) if size in (2, 3) else ()) \
            + (("maxcount OK",) if size == 2 else ()) \
            + (("pipe slots OK",) if size == 3 else ())
        for stage in stages:
            assert f"rank {r} {stage}" in outs[r], f"rank {r} did not report '{stage}':\n{outs[r][-3000:]}"


def _run_mode(gpu, mode, size=2, timeout=280, extra_env=None):
    key = "t" + uuid.uuid4().hex[:12]
    ndev = gpu.cuda.device_count()
    env = dict(os.environ, MI355X_TIMEOUT_S="60", **(extra_env or {}))
    procs = [subprocess.Popen([sys.executable, str(HERE / "ipc_worker.py"), key, str(r), str(size), str(r % ndev), mode],
                              env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True) for r in range(size)]
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
    return outs


@pytest.mark.parametrize("size", [2, 3])
def test_resident_service(gpu, size):
    """the resident LL service beside the rest of the process (ipc_worker.py::svc_mode)"""
    outs = _run_mode(gpu, "svc", size, extra_env={"MI355X_SVC_IDLE_MS": "3000"})
    print(next(line for line in outs[0].splitlines() if "svc:" in line))


@pytest.mark.parametrize("size", [2, 3])
def test_resident_service_stress(gpu, size):
    """6000 random calls in the same order on every rank -- the service's LL and pull forms, host
    flows it steps aside for, pauses around its idle limit -- every result exact
    (ipc_worker.py::svc_stress)"""
    outs = _run_mode(gpu, "svc_stress", size, timeout=250)
    print(next(line for line in outs[0].splitlines() if "svc stress:" in line))


@pytest.mark.parametrize("size", [2, 3])
def test_done_words(gpu, size):
    """finish points by device-written completion words (MI355X_DONE_WORDS=1) stay exact"""
    _run_mode(gpu, "done_words", size)


@pytest.mark.parametrize("stream_min", ["default", "off"] + [f"frag{k}" for k in
                                                           os.environ.get("MI355X_P2P_FRAG_SWEEP", "").split(",") if k])
def test_host_p2p_between_processes(gpu, stream_min):
    """host -> host sendrecv between two processes through the shared-memory arenas, 1-64 MiB,
    with the fragment pipeline (default) and with whole-message copy-in (off); exact both ways,
    the rates printed (tools/gpu_r03_p2p.sh keeps them)"""
    extra = {} if stream_min == "default" else {"MI355X_P2P_STREAM_MIN": str(1 << 62)}
    if stream_min.startswith("frag"):
        extra = {"MI355X_P2P_STREAM_FRAG": stream_min[4:]}
    outs = _run_mode(gpu, "host_bw", 2, extra_env=extra)
    for line in outs[0].splitlines():
        if line.startswith("{"):
            print("\n" + line)


def test_concurrent_communicators(gpu):
    """4 communicators over the same 2 ranks, 4 threads each, concurrent 1 GiB pipelined-flow
    allreduces: exact, no timeout (per-GPU admission of the persistent grid, coll_comm.cpp)"""
    key = "t" + uuid.uuid4().hex[:12]
    ndev = gpu.cuda.device_count()
    env = dict(os.environ, MI355X_TIMEOUT_S="60")
    procs = [subprocess.Popen([sys.executable, str(HERE / "ipc_worker.py"), key, str(r), "2", str(r % ndev), "concurrent"],
                              env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True) for r in range(2)]
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=280)
        except subprocess.TimeoutExpired:
            p.kill()
            out, _ = p.communicate()
        outs.append(out)
    for r, p in enumerate(procs):
        assert p.returncode == 0 and f"rank {r} concurrent OK" in outs[r], f"rank {r}:\n{outs[r][-3000:]}"
    print(outs[0].strip().splitlines()[-2])
