"""The x87 extended-precision add / subtract / multiply the GPU's long double SUM / PROD slots run
(ompi-release_amd/csrc/rt/f80_arith.hpp) against this host's x87 unit, which is what the reference's
`long double` loops execute on x86-64 (op_base_functions.c:110-170, `*(out) += *(in)` / `*=`).

CPU only: tools/f80_check.cpp compiles the header for the host and compares it bit for bit with
native `long double` arithmetic on every ordered pair of adversarial encodings (zeros, denormals,
pseudo-denormals, unnormals, pseudo-NaN / -infinity, signalling and quiet NaNs, infinities, the
exponent extremes) and on random pairs over the whole exponent range (overflow, gradual underflow,
near-cancellation).  Both the normal-operand fast paths and the general path are covered."""
import json
import os
import platform
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(platform.machine() != "x86_64" or shutil.which("g++") is None,
                    reason="needs an x87 unit and g++")
def test_f80_arith_matches_host_x87(tmp_path):
    exe = tmp_path / "f80_check"
    subprocess.run(["g++", "-O2", "-o", str(exe), os.path.join(REPO, "tools", "f80_check.cpp")], check=True)
    r = subprocess.run([str(exe), "2000000"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["mismatches"] == 0
    assert res["checked"] == 3 * (res["adversarial_pairs"] + res["random_pairs"])
