"""The C ABI from plain C (tests/c/coll_ranks.c): N forked processes, one rank each, every engine
collective and device point-to-point checked exactly -- the engine as an MPI library's C code
would call it, no Python in the data path."""
from __future__ import annotations

import os
import pathlib
import subprocess

import pytest

pytestmark = pytest.mark.gpu
EXE = pathlib.Path(__file__).resolve().parent / "c" / "build" / "coll_ranks"


@pytest.mark.parametrize("n", [2, 4])
def test_c_abi_ranks(gpu, n):
    if not EXE.exists():
        pytest.fail(f"{EXE} missing: run __graft_entry__.build()")
    p = subprocess.run([str(EXE), str(n)], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, MI355X_TIMEOUT_S="60"))
    assert p.returncode == 0, p.stdout + p.stderr
    for r in range(n):
        assert f"rank {r} C-ABI OK" in p.stdout, p.stdout + p.stderr
