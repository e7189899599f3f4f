"""Host scene build (product, libmyrt.so) vs the oracle's restatement of BVHBuilder and
RTContext.init: identical BVH topology, node bounds and leaf primitive order (the
canonical preorder hash), for every instance and the TLAS.  CPU only (no device)."""
import ctypes as C

import numpy as np
import pytest

import myraytracer_amd as M
from myraytracer_amd import _abi as A
from myraytracer_amd import scenes
import oracle


def product_hashes(sc):
    lib = M.load_library()
    pk = sc.to_desc()
    hs = (C.c_uint64 * 256)()
    n = C.c_int32()
    info = A.rt_scene_info()
    rc = lib.rt_debug_host_build(pk.ptr, hs, 256, C.byref(n), C.byref(info))
    assert rc == 0, lib.rt_last_error()
    return [hs[i] for i in range(n.value + 1)], info


def oracle_hashes(sc):
    o = oracle.OracleScene(sc)
    return [o.bvh_hash(i) for i in range(o.num_instances())] + [o.bvh_hash(-1)]


def _mesh(V, F, mid=1, mat="1", smooth="smooth", **kw):
    return M.Mesh(id=mid, material=mat, positions=np.asarray(V, float), indices=np.asarray(F, np.int32),
                  indices_one_based=False, shading_mode=smooth, **kw)


def _scene(objs):
    sc = scenes.scene_c1(8, 8)
    sc.objects = objs
    return sc


def test_c1_c2_bvh_identical():
    for sc in [scenes.scene_c1(), scenes.scaled(scenes.scene_c2(inline=True), 16, 16)]:
        p, info = product_hashes(sc)
        assert p == oracle_hashes(sc)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_random_soup_bvh_identical(seed):
    rng = np.random.RandomState(seed)
    n = 3000
    base = rng.uniform(-10, 10, size=(n, 1, 3))
    V = (base + rng.normal(scale=0.3, size=(n, 3, 3))).reshape(-1, 3).astype(np.float32).astype(np.float64)
    F = np.arange(3 * n).reshape(-1, 3)
    sc = _scene([_mesh(V, F, smooth="flat")])
    assert product_hashes(sc)[0] == oracle_hashes(sc)


def test_degenerate_centroids_and_tiny_meshes():
    # identical centroids cannot be split: a leaf holding > maxLeaf prims (BVH.swift:161-162)
    tri = np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0]], float)
    V = np.concatenate([tri, tri * 2 - 0.5, tri * 0.5 + 0.25 / 3])      # same centroid (1/3,1/3,0)
    F = np.arange(9).reshape(-1, 3)
    for objs in [[_mesh(V, F)], [_mesh(tri, [[0, 1, 2]])], [_mesh(V[:6], F[:2])]]:
        sc = _scene(objs)
        assert product_hashes(sc)[0] == oracle_hashes(sc)


def test_multi_object_instances_tlas_identical():
    pos, faces = scenes.geometry_c2(segments=32, rings=16)
    m1 = _mesh(pos, faces, mid=1, mat="1")
    m2 = _mesh(pos * 0.5 + 2.0, faces, mid=2, mat="1", smooth="flat")
    objs = [m1, M.Triangle(vertices=((0, 0, 0), (1, 0, 0), (0, 1, 0)), material="1"), m2,
            M.MeshInstance(id=5, base_mesh_id=1, material="1", transform=M.translation(3, 0, 0)),
            M.MeshInstance(id=6, base_mesh_id=5, transform=M.translation(0, 2, 0)),
            M.MeshInstance(id=7, base_mesh_id=99)]   # unknown base -> skipped (RTContext.swift:387)
    sc = _scene(objs)
    p, info = product_hashes(sc)
    o = oracle_hashes(sc)
    assert len(p) == len(o) == 6      # tri, inst5, inst6, mesh1, mesh2 + TLAS
    assert p == o


def test_c3_scene_bvh_identical_and_stack_bound():
    sc = scenes.scene_c3(inline=True)
    p, info = product_hashes(sc)
    assert p == oracle_hashes(sc)
    assert info.triangles == 1015808
    assert 0 < info.max_depth < 64          # RTContext.swift:550 64-entry stack
