"""The C++ host mirror (include/rt_engine.hpp) drives the C ABI from compiled code, as the Swift
RayTracerEngine would ("tests drive the shim from C++").  tests/cpp/engine_test is
built by myraytracer_amd/build.py (build_cpp_tests) and run as a child process."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "cpp", "engine_test")


def _run(mode, timeout):
    assert os.path.exists(EXE), f"{EXE} missing: run `python -c 'import __graft_entry__ as g; g.build()'`"
    p = subprocess.run([EXE, mode], capture_output=True, text=True, timeout=timeout)
    print(p.stdout)
    print(p.stderr)
    assert p.returncode == 0, p.stdout + p.stderr
    assert f"{mode}: ok" in p.stdout
    return p.stdout


def test_cpp_host_without_gpu_reports_device_error():
    if os.path.exists("/dev/kfd") and os.access("/dev/kfd", os.R_OK | os.W_OK):
        pytest.skip("a GPU is present (the gpu variant covers this host)")
    _run("cpu", 60)


@pytest.mark.gpu
def test_cpp_host_renders_match_oracle():
    out = _run("gpu", 120)
    assert "c1: L-inf" in out and "grid cam1" in out
