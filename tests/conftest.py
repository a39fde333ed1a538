"""Shared pytest fixtures: package/oracle loaders, GPU gating.

`-m "not gpu"` runs here (no GPU); `-m gpu` runs on an MI355X box.  GPU tests call the HIP path
through the C ABI (libmi355x_rt.so / the MCA component DSOs) and compare with the CPU oracle
(oracle/build/liboracle.so), which is test infrastructure only.
"""
from __future__ import annotations

import ctypes
import importlib.util
import pathlib
import subprocess
import sys

import pytest

REPO = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")


def load_pkg():
    name = "ompi_release_amd"
    if name in sys.modules:
        return sys.modules[name]
    spec = importlib.util.spec_from_file_location(name, REPO / "ompi-release_amd" / "__init__.py")
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


_oracle = None


def load_oracle() -> ctypes.CDLL:
    global _oracle
    if _oracle is None:
        so = REPO / "oracle" / "build" / "liboracle.so"
        if not so.exists():
            subprocess.check_call(["make", "-s", "-C", str(REPO / "oracle")])
        lib = ctypes.CDLL(str(so))
        c = ctypes
        vp, sz, i = c.c_void_p, c.c_size_t, c.c_int
        lib.oracle_type_size.restype = sz
        lib.oracle_type_size.argtypes = [i]
        lib.oracle_has_op.argtypes = [i, i]
        lib.oracle_op_2buff.argtypes = [i, i, vp, vp, sz]
        lib.oracle_op_3buff.argtypes = [i, i, vp, vp, vp, sz]
        lib.oracle_op_3buff_mt.argtypes = [i, i, vp, vp, vp, sz, i]
        lib.oracle_allreduce.argtypes = [i, i, sz, i, i, c.c_uint32, c.POINTER(vp), c.POINTER(vp)]
        lib.oracle_cpu_allreduce.argtypes = [i, sz, i, i, c.c_uint32, c.POINTER(vp), c.POINTER(vp), i, i,
                                             c.POINTER(c.c_double)]
        lib.oracle_allreduce_decision.argtypes = [i, sz, i, c.POINTER(c.c_uint32)]
        lib.oracle_reduce.argtypes = [i, i, i, sz, i, i, c.c_uint32, c.POINTER(vp), vp]
        lib.oracle_reduce_decision.argtypes = [i, sz, i, c.POINTER(c.c_uint32)]
        lib.oracle_reduce_fo.argtypes = [i, i, i, i, sz, i, i, c.POINTER(vp), vp]
        lib.oracle_reduce_scatter_alg.argtypes = [i, i, c.POINTER(i), i, i, c.POINTER(vp), c.POINTER(vp)]
        lib.oracle_reduce_scatter_block.argtypes = [i, sz, i, i, c.POINTER(vp), c.POINTER(vp)]
        lib.oracle_scan.argtypes = [i, i, sz, i, i, c.POINTER(vp), c.POINTER(vp)]
        lib.oracle_ring_fold_order.argtypes = [i, sz, sz, c.POINTER(c.c_int)]
        i64 = c.c_int64
        lib.oracle_ddt_contiguous.restype = vp
        lib.oracle_ddt_contiguous.argtypes = [i64, i64]
        lib.oracle_ddt_vector.restype = vp
        lib.oracle_ddt_vector.argtypes = [i64, i64, i64, i64]
        lib.oracle_ddt_indexed.restype = vp
        lib.oracle_ddt_indexed.argtypes = [i, c.POINTER(i), c.POINTER(i), i64]
        lib.oracle_ddt_struct.restype = vp
        lib.oracle_ddt_struct.argtypes = [i, c.POINTER(i64), c.POINTER(i64), c.POINTER(i64), i64]
        lib.oracle_ddt_free.argtypes = [vp]
        lib.oracle_ddt_size.restype = i64
        lib.oracle_ddt_size.argtypes = [vp]
        lib.oracle_ddt_extent.restype = i64
        lib.oracle_ddt_extent.argtypes = [vp]
        lib.oracle_ddt_round_position.restype = i64
        lib.oracle_ddt_round_position.argtypes = [vp, i64, i64]
        lib.oracle_ddt_pack.argtypes = [vp, i64, vp, i64, vp, i64]
        lib.oracle_ddt_unpack.argtypes = [vp, i64, vp, i64, vp, i64]
        lib.oracle_uicsum_partial.restype = c.c_ulong
        lib.oracle_uicsum_partial.argtypes = [vp, sz, c.POINTER(c.c_uint), c.POINTER(sz)]
        lib.oracle_ddt_pack_checksum.restype = c.c_uint32
        lib.oracle_ddt_pack_checksum.argtypes = [vp, i64, vp, vp]
        lib.oracle_ddt_pack_runs.argtypes = [vp, i64, vp, vp]
        lib.oracle_ompi_fn2.restype = vp
        lib.oracle_ompi_fn2.argtypes = [i, i]
        lib.oracle_ompi_fn3.restype = vp
        lib.oracle_ompi_fn3.argtypes = [i, i]
        _oracle = lib
    return _oracle


@pytest.fixture(scope="session")
def pkg():
    return load_pkg()


@pytest.fixture(scope="session")
def oracle():
    return load_oracle()


@pytest.fixture(scope="session")
def gpu():
    """torch with a visible MI355X; the HIP library loaded."""
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu-marked test run without a visible GPU")
    p = load_pkg()
    p.rt()
    return torch

# a failed rank must not leave its peers in a 10-minute barrier
import os as _os  # noqa: E402
_os.environ.setdefault("MI355X_TIMEOUT_S", "60")
