"""Build recipes (hipcc / g++ invoked directly; no CMake needed).

  libmyrt.so        product: HIP kernels (gfx950) + host scene build + PLY + C ABI
  oracle/liboracle.so   test-only CPU restatement of the reference (g++)
  oracle/_ref/libcply_ref.so  the reference's own CPly, compiled from /root/reference
                              when present (PLY golden vectors; oracle/build_ref.sh)
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "myraytracer_amd")
CSRC = os.path.join(PKG, "csrc")
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"

PRODUCT_SOURCES = ["render.hip", "scene.cpp", "ply.cpp", "sceneio.cpp"]
# -ffp-contract=off on host AND device: the reference does no FMA contraction
COMMON_FLAGS = ["-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared"]


def _run(cmd, cwd=ROOT):
    print("+", " ".join(cmd), flush=True)
    subprocess.run(cmd, cwd=cwd, check=True)


def _stale(target, sources):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in sources)


def build_product(force: bool = False) -> str:
    out = os.path.join(PKG, "libmyrt.so")
    srcs = [os.path.join(CSRC, s) for s in PRODUCT_SOURCES]
    deps = srcs + [os.path.join(CSRC, h) for h in ("layout.h", "scene.h", "device.h", "wide.h", "render_full.h")] + [os.path.join(ROOT, "include", "rtcore.h")]
    if force or _stale(out, deps):
        _run([HIPCC, "--offload-arch=gfx950", *COMMON_FLAGS, "-o", out, *srcs])
    return out


def build_oracle(force: bool = False) -> str:
    src = os.path.join(ROOT, "oracle", "rt_oracle.cpp")
    out = os.path.join(ROOT, "oracle", "liboracle.so")
    if force or _stale(out, [src, os.path.join(ROOT, "include", "rtcore.h")]):
        _run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared", "-o", out, src, "-lpthread"])
    return out


def build_ref(force: bool = False) -> str:
    """Compile the reference's CPly (if /root/reference is present) into oracle/_ref/."""
    script = os.path.join(ROOT, "oracle", "build_ref.sh")
    out = os.path.join(ROOT, "oracle", "_ref", "libcply_ref.so")
    if not os.path.isdir("/root/reference/Sources/CPly"):
        return out if os.path.exists(out) else ""
    if force or not os.path.exists(out):
        _run(["bash", script])
    return out


def build_cpp_tests(force: bool = False) -> str:
    """tests/cpp/engine_test: the C++ host (include/rt_engine.hpp) driving libmyrt.so, checked
    against the oracle (test infrastructure; run by tests/test_cpp_host.py)."""
    src = os.path.join(ROOT, "tests", "cpp", "engine_test.cpp")
    out = os.path.join(ROOT, "tests", "cpp", "engine_test")
    deps = [src, os.path.join(ROOT, "include", "rt_engine.hpp"), os.path.join(ROOT, "include", "rtcore.h"),
            os.path.join(PKG, "libmyrt.so"), os.path.join(ROOT, "oracle", "liboracle.so")]
    if force or _stale(out, deps):
        _run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-I", os.path.join(ROOT, "include"), "-o", out, src,
              "-L", PKG, "-lmyrt", "-L", os.path.join(ROOT, "oracle"), "-loracle", "-L/opt/rocm/lib",
              "-Wl,-rpath,$ORIGIN/../../myraytracer_amd", "-Wl,-rpath,$ORIGIN/../../oracle",
              "-Wl,-rpath,/opt/rocm/lib", "-lpthread"])
    return out


def build_all(force: bool = False):
    build_product(force)
    build_oracle(force)
    build_ref(force)
    build_cpp_tests(force)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
