"""CPU check of the FP32-enclosed slab test (myraytracer_amd/csrc/slab32.h) against the
reference's FP64 slab (hitAABB, RTContext.swift:557-565).  Builds and runs
tests/cpp/slab32_test.cpp; no GPU needed."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_slab32_encloses_fp64(tmp_path):
    exe = str(tmp_path / "slab32_test")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-o", exe,
                    os.path.join(HERE, "cpp", "slab32_test.cpp")], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failures" in r.stdout
