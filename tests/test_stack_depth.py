"""Traversal-stack capacity (ADVICE r1 "high").

The reference gives the TLAS walk and each BLAS walk their own 64-entry stacks
(RTContext.swift:550, 623) and overflowing one is undefined behaviour, so a BVH deeper than
that is refused (RT_ERR_STACK).  The device walks keep TLAS and BLAS entries on ONE per-lane
stack of kStackCap = 128 entries (16 in LDS, the rest private), which holds both walks at
their limits; the host computes what a scene needs and refuses anything beyond the cap.

Scenes: triangles perpendicular to x at x = 16^k.  With 12 SAH bins every split peels off
the largest one, so a mesh of n such triangles has a BLAS n-2 levels deep, and n such meshes
a TLAS as deep.  A ray along +x hits both children of every node on the spine, so it pushes
one entry per level: a deep TLAS over a deep BLAS drives the stack to ~126 entries.
"""
import ctypes as C

import numpy as np
import pytest

import myraytracer_amd as M
from myraytracer_amd import _abi as A
from myraytracer_amd import scenes
import oracle


def _wall_mesh(xs, mid):
    V, F = [], []
    for k, x in enumerate(xs):
        V += [[x, -0.1, -0.1], [x, 0.2, -0.1], [x, -0.1, 0.2]]
        F.append([3 * k, 3 * k + 1, 3 * k + 2])
    return M.Mesh(id=mid, material="1", positions=np.array(V, float), indices=np.array(F, np.int32),
                  indices_one_based=False, shading_mode="flat")


def deep_scene(n_tlas, n_blas, width=32, height=24):
    objs = [_wall_mesh([16.0 ** k for k in range(n_blas)], 1)]
    objs += [_wall_mesh([1.5 * 16.0 ** k], 100 + k) for k in range(n_tlas)]
    sc = scenes.scene_c1(width, height)
    sc.objects = objs
    c = sc.cameras[0]
    c.position, c.gaze_point, c.up, c.fovy = (-1.0, 0.04, 0.04), (10.0, 0.04, 0.04), (0.0, 1.0, 0.0), 8.0
    return sc


def host_build(sc):
    lib = M.load_library()
    pk = sc.to_desc()
    hs = (C.c_uint64 * 512)()
    n = C.c_int32()
    info = A.rt_scene_info()
    rc = lib.rt_debug_host_build(pk.ptr, hs, 512, C.byref(n), C.byref(info))
    return rc, info


@pytest.mark.parametrize("n,ok", [(40, True), (64, True), (65, False), (80, False)])
def test_blas_deeper_than_the_reference_stack_is_refused(n, ok):
    rc, info = host_build(deep_scene(0, n))
    if ok:
        assert rc == A.RT_OK and info.max_depth == (n - 2) + 2   # one mesh: TLAS depth 0
    else:
        assert rc == A.RT_ERR_STACK


def test_deep_tlas_over_deep_blas_fits_the_device_stack():
    rc, info = host_build(deep_scene(64, 64))
    assert rc == A.RT_OK
    assert 120 <= info.max_depth <= 128            # far past the round-1 80-entry stack
    rc, _ = host_build(deep_scene(66, 60))         # TLAS deeper than the reference's stack
    assert rc == A.RT_ERR_STACK


def _axis_rays():
    xs = [16.0 ** k for k in range(64)]
    o = [[-1.0, 0.01, 0.02], [-1.0, 0.05, -0.05]]
    o += [[x + 0.25, 0.02, 0.01] for x in xs[::3]]                    # start between walls
    d = [[1.0, 0.0, 0.0]] * len(o)
    o += [[2.0 * xs[-1], 0.01, 0.01], [3.0, 0.03, 0.0]]                # walking back down
    d += [[-1.0, 0.0, 0.0], [-1.0, 0.0, 0.0]]
    rng = np.random.RandomState(3)
    dd = np.array([[1.0, 0.0, 0.0]] * 16) + rng.normal(scale=1e-3, size=(16, 3))
    o += [[-1.0, 0.02, 0.02]] * 16
    d += list(dd / np.linalg.norm(dd, axis=1, keepdims=True))
    return np.array(o, float), np.array(d, float)


@pytest.mark.gpu
@pytest.mark.parametrize("n_tlas,n_blas", [(0, 64), (40, 40), (64, 64)])
def test_deep_walks_match_the_oracle(n_tlas, n_blas):
    sc = deep_scene(n_tlas, n_blas)
    O, D = _axis_rays()
    eng = M.RayTracerEngine(sc)
    tg, pg, ng, mg = eng.trace_rays(O, D)
    to, po, no, mo = oracle.OracleScene(sc).trace_rays(O, D)
    hit = np.isfinite(to)
    assert hit.sum() >= len(O) // 2
    assert np.array_equal(tg, to) and np.array_equal(mg, mo)
    assert np.array_equal(pg[hit], po[hit]) and np.array_equal(ng[hit], no[hit])
    og = eng.occluded_rays(O, D, np.full(len(O), 1e300))
    oo = oracle.OracleScene(sc).occluded_rays(O, D, np.full(len(O), 1e300))
    assert np.array_equal(og, oo)
    res = eng.render(0)                              # the megakernel's walk on the same scene
    ref, ref8, _ = oracle.OracleScene(sc).render(0, threads=0, rgba=True)
    assert float(np.abs(res.rgb - ref).max()) <= 1e-5 and np.array_equal(res.rgba8, ref8)
    eng.close()
