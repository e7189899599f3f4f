"""The C-ABI library loads and exports every symbol include/rtcore.h declares; the ctypes
mirror matches the header's struct layout; error codes without a GPU (no compute)."""
import ctypes as C
import os
import re
import subprocess

import pytest

import myraytracer_amd as M
from myraytracer_amd import _abi as A

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "rtcore.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(rt_[a-z0-9_]+)\s*\(", src)) - {"rt_progress_fn"})


def test_library_exports_every_declared_symbol():
    lib = M.load_library()
    declared = header_functions()
    assert len(declared) >= 14
    missing = [f for f in declared if not hasattr(lib, f)]
    assert not missing, missing
    assert set(A.EXPORTED_SYMBOLS) <= set(declared)
    out = subprocess.run(["nm", "-D", "--defined-only", M.engine.LIB_PATH], capture_output=True, text=True).stdout
    for f in declared:
        assert re.search(rf"\bT {f}\b", out), f


STRUCTS = ["rt_vec3", "rt_material", "rt_point_light", "rt_area_light", "rt_camera", "rt_object", "rt_scene_desc",
           "rt_stats", "rt_scene_info", "rt_work_counters", "rt_ply_mesh"]


def test_ctypes_layout_matches_header(tmp_path):
    prog = tmp_path / "sizes.c"
    body = "\n".join(f'printf("{s} %zu\\n", sizeof({s}));' for s in STRUCTS)
    offs = [("rt_object", f) for f, _ in A.rt_object._fields_] + [("rt_scene_desc", f) for f, _ in A.rt_scene_desc._fields_] + \
           [("rt_camera", f) for f, _ in A.rt_camera._fields_]
    body += "\n" + "\n".join(f'printf("{s}.{f} %zu\\n", offsetof({s}, {f}));' for s, f in offs)
    prog.write_text(f'#include <stdio.h>\n#include <stddef.h>\n#include "{HEADER}"\nint main(void){{\n{body}\nreturn 0;}}\n')
    exe = tmp_path / "sizes"
    subprocess.run(["gcc", "-std=c99", "-o", str(exe), str(prog)], check=True)
    got = dict(line.split() for line in subprocess.run([str(exe)], capture_output=True, text=True).stdout.splitlines())
    for s in STRUCTS:
        assert int(got[s]) == C.sizeof(getattr(A, s)), s
    for s, f in offs:
        assert int(got[f"{s}.{f}"]) == getattr(getattr(A, s), f).offset, (s, f)


def test_rows_for_chunks_agrees():
    lib = M.load_library()
    for H in [1, 7, 8, 9, 100, 600, 1080, 2160]:
        for first, step in [(0, 1), (1, 2), (3, 8), (0, 5), (20, 3)]:
            assert lib.rt_rows_for_chunks(H, first, step) == M.rows_for_chunks(H, first, step)
    assert lib.rt_rows_for_chunks(1080, 0, 1) == 1080
    assert sum(lib.rt_rows_for_chunks(1080, r, 8) for r in range(8)) == 1080


def test_error_codes_without_compute():
    lib = M.load_library()
    h = C.c_void_p()
    assert lib.rt_scene_create(None, None, 0, C.byref(h)) == A.RT_ERR_NO_SCENE
    assert lib.rt_render(None, 0, 0, 1, None, None, None, A.RT_PROGRESS_FN(0), None) == A.RT_ERR_NO_SCENE
    assert b"scene" in lib.rt_last_error().lower()
    assert lib.rt_render_device(None, 0, 0, 0, 1, None, None, None) == A.RT_ERR_NO_SCENE
    st = A.rt_scene_info()
    assert lib.rt_scene_info_get(None, C.byref(st)) == A.RT_ERR_NO_SCENE
    m = A.rt_ply_mesh()
    assert lib.rt_ply_load(b"/nonexistent.ply", C.byref(m)) == A.RT_ERR_PLY
    assert lib.rt_version().startswith(b"myraytracer_amd")
    assert f"(abi {A.RT_ABI_VERSION},".encode() in lib.rt_version()   # RT_ABI_VERSION (rtcore.h)
    v = C.c_int64()
    assert lib.rt_scene_set_option(None, b"wide", 0) == A.RT_ERR_NO_SCENE
    assert lib.rt_scene_get_option(None, b"wide", C.byref(v)) == A.RT_ERR_NO_SCENE
    assert lib.rt_scene_set_unsafe_option(None, b"wide_delta_scale", 0) == A.RT_ERR_NO_SCENE


def test_header_declares_the_abi_version_and_struct_sizes():
    """rtcore.h's RT_ABI_VERSION and the ctypes mirror agree; the structs that grew in version 3
    (rt_stats.rewalked, rt_scene_info.scratch_bytes) have the header's layout."""
    import os
    import re
    hdr = open(os.path.join(os.path.dirname(__file__), "..", "include", "rtcore.h")).read()
    assert int(re.search(r"#define RT_ABI_VERSION (\d+)", hdr).group(1)) == A.RT_ABI_VERSION
    assert C.sizeof(A.rt_stats) == 11 * 8 and A.rt_stats.rewalked.offset == 10 * 8
    assert C.sizeof(A.rt_scene_info) == 12 * 8 and A.rt_scene_info.scratch_bytes.offset == 11 * 8


def test_product_fails_loudly_without_gpu():
    torch = pytest.importorskip("torch")
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from myraytracer_amd import scenes
    with pytest.raises(M.RenderError) as e:
        M.RayTracerEngine(scenes.scene_c1(8, 8))
    assert e.value.code == A.RT_ERR_DEVICE
