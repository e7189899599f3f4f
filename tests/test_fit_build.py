"""Host build of the flattened instance tree (scene.cpp build_fit; the walk is wide.h fit_walk),
CPU only: every leaf run of every instance is one pair of the tree, the tree fits the device stack,
and the build does not depend on the thread count.  Scenes the exactness argument does not cover
(transforms with a condition number above 2^12) and identity scenes get no tree."""
import ctypes as C
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import myraytracer_amd as M
from myraytracer_amd import scenes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _fit(sc):
    lib = M.load_library()
    if not hasattr(lib, "rt_debug_fit_build"):
        pytest.skip("library without rt_debug_fit_build")
    pk = sc.to_desc()
    out = (C.c_int64 * 5)()
    rc = lib.rt_debug_fit_build(pk.ptr, out)
    assert rc == 0, lib.rt_last_error()
    return [int(v) for v in out]


def _rot(a, b):
    ca, sa, cb, sb = np.cos(a), np.sin(a), np.cos(b), np.sin(b)
    return np.array([[ca, -sa, 0.0], [sa, ca, 0.0], [0.0, 0.0, 1.0]]) @ np.array([[cb, 0.0, sb], [0.0, 1.0, 0.0],
                                                                                  [-sb, 0.0, cb]])


def _instanced(scales=(0.5, 0.9, 1.3, 1.7)):
    sc = scenes.scaled(scenes.scene_c2(inline=True), 8, 8)
    base = sc.objects[0]
    objs = [base]
    for k, s in enumerate(scales):
        M4 = np.eye(4)
        M4[:3, :3] = _rot(0.3 * k, 0.7 * k) @ np.diag(np.atleast_1d(s) * np.ones(3))
        M4[:3, 3] = (1.5 * k, -0.5 * k, 0.25 * k)
        objs.append(M.MeshInstance(id=40 + k, base_mesh_id=base.id, material="1", transform=tuple(M4.T.reshape(-1))))
    sc.objects = objs
    return sc


def test_every_leaf_run_of_every_instance_is_one_pair():
    pairs, nodes, depth, runs, h = _fit(_instanced())
    assert pairs > 0 and pairs == runs
    assert nodes >= (pairs + 3) // 4
    assert 3 * depth + 2 <= 128


def test_c3i_tree():
    pairs, nodes, depth, runs, h = _fit(scenes.scene_c3_instanced(inline=True))
    assert pairs == runs > 500_000
    assert 3 * depth + 2 <= 128


def test_ill_conditioned_transforms_and_identity_scenes_get_no_tree():
    sc = _instanced(scales=(0.5, np.array([1.0, 1.0, 1e-4])))        # condition number 1e4 > 2^12
    pairs, _, _, runs, _ = _fit(sc)
    assert pairs == 0 and runs > 0
    pairs, _, _, _, _ = _fit(scenes.scaled(scenes.scene_c2(inline=True), 8, 8))   # identity scene
    assert pairs == 0


def test_the_tree_does_not_depend_on_the_thread_count():
    code = ("import ctypes as C, json, sys; sys.path.insert(0, %r); sys.path.insert(0, %r); "
            "import myraytracer_amd as M; from test_fit_build import _fit, _instanced; "
            "from myraytracer_amd import scenes; "
            "print(json.dumps([_fit(_instanced()), _fit(scenes.scene_c3_instanced(inline=True))]))"
            % (ROOT, os.path.join(ROOT, "tests")))
    res = []
    for t in ("1", "8"):
        env = dict(os.environ, MYRT_BUILD_THREADS=t)
        p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=600)
        assert p.returncode == 0, p.stderr[-2000:]
        res.append(json.loads(p.stdout.strip().splitlines()[-1]))
    assert res[0] == res[1]
