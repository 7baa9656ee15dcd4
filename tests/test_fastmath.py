"""The exact-division identities the compact kernel uses instead of general divisions
(kube-scheduler-simulator_amd/csrc/kss_fastmath.cuh), checked on the host against the plain
divisions: integer floor quotients from a perturbed float reciprocal, int64 quotients from
a double reciprocal, and the correctly rounded float64 quotient RN(a/b) from two FMA
residual steps on RN(1/b) (Markstein).  tests/csrc/fastmath_check.c replays the device's
operation sequence; the samples cover the operand ranges the device path admits."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
def test_fastmath_identities(tmp_path):
    exe = tmp_path / "fmc"
    subprocess.check_call(["gcc", "-O2", "-ffp-contract=off", "-o", str(exe),
                           os.path.join(HERE, "csrc", "fastmath_check.c"), "-lm"])
    out = subprocess.check_output([str(exe), "4000000"], text=True).split()
    assert out == ["0", "0", "0"], f"mismatches small_div / quot_small_i64 / div_rn: {out}"
