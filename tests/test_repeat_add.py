"""The PE T / P drift's closed form (csrc/ws_repeat_add.h: n rounded additions of a constant
taken a binade at a time) against the plain loop of rounded additions it replaces, on the host:
tests/native/repeat_add_check.cpp, 800 000 random cases in fp32 and fp64 -- the drift's own
range, binade tops, ties (c = (k + 1/2) ulp), negative, tiny, zero, subnormal, inf / nan --
must agree bit for bit. (On the device the same function runs in affine2_kernel; the PE parity
suites compare its output with the reference fixtures and step-by-step runs.)"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_repeat_add_matches_the_loop(tmp_path):
    exe = tmp_path / "rac"
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-std=c++17",
                    "-I", os.path.join(ROOT, "nvidia-jetson-workload_amd", "csrc"),
                    os.path.join(ROOT, "tests", "native", "repeat_add_check.cpp"), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout
    assert out.stdout.strip().endswith("mismatches 0 cases 800000"), out.stdout
