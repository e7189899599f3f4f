"""Traversal parity on explicit rays (rt_debug_trace_rays / rt_debug_occluded_rays vs the
oracle's intersectTLAS / occludedTLAS, RTContext.swift:619-781).

Camera rays almost never have a zero direction component, so the frame tests exercise the
`FAST` slab only.  These rays are built to hit the exact-semantics paths and the tie rules:
axis-aligned and signed-zero directions (1/d = +-inf, NaN slab products), rays
through shared vertices and edges of a grid (equal-t triangles: first visited wins, H2),
grazing rays along box faces, and rays mixed in one wave with ordinary ones.  Hits must be
bit-identical: t, world point, world normal and material.

Identity scenes run on three walks (render options, rt_scene_set_option): the conservative
four-wide FP32 walk (wide.h, the default), the binary unified walk (wide = 0) and the nested
walk of intersectTLAS (unified = 0)."""
import dataclasses

import numpy as np
import pytest

import myraytracer_amd as M
from myraytracer_amd import scenes
import oracle

pytestmark = pytest.mark.gpu

# walk name -> render options (identity scenes: wide / unified / general; instanced scenes:
# transformed / general)
WALKS = {"wide": {}, "unified": {"wide": 0}, "general": {"unified": 0},
         "transformed": {}, "transformed_tw": {"fit": 0}, "transformed_binary": {"wide": 0},
         "nested": {"unified_transformed": 0}}


def _engine(sc, walk):
    eng = M.RayTracerEngine(sc)
    for k, v in WALKS[walk].items():
        eng.set_option(k, v)
    return eng


def _axis_dirs():
    d = []
    for a in range(3):
        for s in (1.0, -1.0):
            v = [0.0, 0.0, 0.0]; v[a] = s; d.append(v)
    for a in range(3):                                   # one zero component, incl. -0.0
        for z in (0.0, -0.0):
            v = [0.6, -0.8, 0.3]; v[a] = z
            d.append(list(np.asarray(v) / np.linalg.norm(v)))
    return np.array(d)


def _ray_set(center, radius, n_random, seed):
    rng = np.random.RandomState(seed)
    o = center + rng.uniform(-radius, radius, size=(n_random, 3))
    d = rng.normal(size=(n_random, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    ax = _axis_dirs()
    oa = np.repeat(center[None, :] + rng.uniform(-0.3 * radius, 0.3 * radius, size=(len(ax), 3)), 1, axis=0)
    # interleave so axis-aligned rays share waves with ordinary ones
    O = np.concatenate([o[: n_random // 2], oa, o[n_random // 2:], oa + 0.25 * radius])
    D = np.concatenate([d[: n_random // 2], ax, d[n_random // 2:], -ax])
    return O, D


def _check_closest(sc, O, D, tmin=None, time=None, walk="wide"):
    eng = _engine(sc, walk)
    tg, pg, ng, mg = eng.trace_rays(O, D, tmin, time)
    to, po, no, mo = oracle.OracleScene(sc).trace_rays(O, D, tmin, time)
    eng.close()
    hit = np.isfinite(to)
    assert np.array_equal(tg, to), f"t differs on {int((tg != to).sum())} of {len(to)} rays"
    assert np.array_equal(mg, mo)
    assert np.array_equal(pg[hit], po[hit]) and np.array_equal(ng[hit], no[hit])
    return hit


def _check_occluded(sc, O, D, tmax, time=None, walk="wide"):
    eng = _engine(sc, walk)
    g = eng.occluded_rays(O, D, tmax, time)
    o = oracle.OracleScene(sc).occluded_rays(O, D, tmax, time)
    eng.close()
    assert np.array_equal(g, o), f"occlusion differs on {int((g != o).sum())} rays"
    return o


@pytest.mark.parametrize("walk", ["wide", "unified", "general"])
def test_c2_random_and_axis_rays(walk):
    sc = scenes.scaled(scenes.scene_c2(inline=True), 8, 8)
    O, D = _ray_set(np.array([0.0, 0.0, 0.0]), 2.5, 4000, 7)
    hit = _check_closest(sc, O, D, walk=walk)
    assert 0.2 < hit.mean() < 0.95
    tmax = np.random.RandomState(3).uniform(0.05, 4.0, size=len(O))
    occ = _check_occluded(sc, O, D, tmax, walk=walk)
    assert 0.05 < occ.mean() < 0.95


@pytest.mark.parametrize("walk", ["wide", "unified"])
def test_grid_vertices_edges_and_faces(walk):
    """Vertical rays through heightfield grid vertices, edge midpoints and cell centres:
    1/d has +-inf components and several triangles share the exact hit.  Then the same points
    from tilted directions (every 1/d finite: the four-wide walk takes them) - rays through
    shared vertices and edges whose triangles may meet at the same t."""
    hp, hf = scenes.heightfield(64, 20.0, 2.0, 5)
    hp32 = hp.astype(np.float32).astype(np.float64)
    mesh = M.Mesh(id=1, material="1", positions=hp32, indices=hf.astype(np.int32), indices_one_based=False,
                  shading_mode="flat")
    sc = scenes.scaled(scenes.scene_c1(8, 8), 8, 8)
    sc.objects = [mesh]
    rng = np.random.RandomState(11)
    verts = hp32[rng.choice(len(hp32), 300, replace=False)]
    tri = hf[rng.choice(len(hf), 300, replace=False)]
    a, b, c = hp32[tri[:, 0]], hp32[tri[:, 1]], hp32[tri[:, 2]]
    pts = np.concatenate([verts, 0.5 * (a + b), 0.5 * (b + c), (a + b + c) / 3.0])
    O = pts + np.array([0.0, 10.0, 0.0])
    D = np.tile([0.0, -1.0, 0.0], (len(O), 1))
    hit = _check_closest(sc, O, D, walk=walk)
    # MT is not watertight: exactly on shared vertices/edges both triangles can reject the
    # ray (u, v rounding), in the reference as here; the centroids always hit
    assert hit[-300:].all() and hit.mean() > 0.25
    Dt = np.array([0.3, -1.0, 0.2]) / np.linalg.norm([0.3, -1.0, 0.2])
    Ot = pts - 10.0 * Dt
    _check_closest(sc, Ot, np.tile(Dt, (len(Ot), 1)), walk=walk)
    _check_occluded(sc, Ot, np.tile(Dt, (len(Ot), 1)), np.full(len(Ot), 9.999), walk=walk)
    # grazing: rays in the plane of the grid's bounding faces, along +x and -z
    lo, hi = hp32.min(0), hp32.max(0)
    ys = np.linspace(lo[1], hi[1], 40)
    Og = np.concatenate([np.stack([np.full(40, lo[0] - 1), ys, np.full(40, lo[2])], 1),
                         np.stack([np.full(40, hi[0]), ys, np.full(40, hi[2] + 1)], 1)])
    Dg = np.concatenate([np.tile([1.0, 0.0, 0.0], (40, 1)), np.tile([0.0, 0.0, -1.0], (40, 1))])
    _check_closest(sc, Og, Dg, walk=walk)
    _check_occluded(sc, O, D, np.full(len(O), 9.999), walk=walk)


@pytest.mark.parametrize("walk", ["transformed", "nested"])
def test_instances_transforms_and_primitives(walk):
    """Transformed mesh instances, spheres, planes and a triangle: the unified transformed walk
    (one stack, per-instance ray switches at marker entries, device.h ut_walk) and the nested
    general walk both give the oracle's intersectTLAS / occludedTLAS bit for bit."""
    sc = scenes.scaled(scenes.scene_c2(inline=True), 8, 8)
    base = sc.objects[0]
    sc.objects = [base,
                  M.MeshInstance(id=11, base_mesh_id=base.id, material="1",
                                 transform=(2, 0, 0, 0, 0, 2, 0, 0, 0, 0, 2, 0, 3.0, 0.5, -2.0, 1)),
                  M.Sphere(center=(-2.5, 0.3, 0.5), radius=0.7, material="1"),
                  M.Plane(center=(0.0, -1.5, 0.0), normal=(0.0, 1.0, 0.0), material="1"),
                  M.Triangle(vertices=((-3, -1, -3), (3, -1, -3), (0, 2, -3.5)), material="1")]
    O, D = _ray_set(np.array([0.5, 0.0, 0.0]), 4.0, 3000, 21)
    _check_closest(sc, O, D, walk=walk)
    _check_occluded(sc, O, D, np.random.RandomState(5).uniform(0.1, 6.0, size=len(O)), walk=walk)


@pytest.mark.parametrize("walk", ["transformed", "nested"])
def test_motion_blur_times_and_tmin(walk):
    sc = scenes.scaled(scenes.scene_c2(inline=True), 8, 8)
    base = sc.objects[0]
    base.motion_blur = (0.0, 0.2, 0.0)
    sc.objects = [base, M.MeshInstance(id=21, base_mesh_id=base.id, material="1",
                                       transform=M.translation(0.5, 0.0, 0.5), motion_blur=(0.3, 0.0, 0.0))]
    O, D = _ray_set(np.array([0.0, 0.0, 0.0]), 2.5, 2000, 9)
    rng = np.random.RandomState(2)
    _check_closest(sc, O, D, tmin=rng.uniform(0.0, 0.5, size=len(O)), time=rng.uniform(0, 1, size=len(O)), walk=walk)


def _rotation(rng):
    q = rng.normal(size=4)
    q /= np.linalg.norm(q)
    w, x, y, z = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


@pytest.mark.parametrize("walk", ["wide", "unified", "general"])
def test_near_degenerate_grazing_hits_and_the_pruning_margin(walk):
    """Large, nearly coplanar triangles and rays grazing them through a corner (|det| just
    above eps): Moeller-Trumbore's t then carries an error of up to ~1e-4 relative and can
    undercut the entry distance of the triangle's own box - far beyond the round-1 margin
    (1e-7 rel + 1e-9 diag), measured on CPU.  The margin now bounds that error
    (scene.cpp, "pruning margin"), so pruning still never drops a node whose triangle the
    reference would accept: hits stay bit-identical to the unpruned oracle."""
    rng = np.random.default_rng(17)
    R0 = _rotation(rng)
    V, F, corners = [], [], []
    for k in range(48):
        L = 10 ** rng.uniform(1.7, 2.7)
        Rk = R0 @ _rotation(np.random.default_rng(1000 + k))[:, :] if k % 4 == 0 else R0
        tilt = np.eye(3) + rng.normal(scale=1e-9, size=(3, 3))
        v0 = rng.normal(scale=1e-6, size=3) + np.array([0.0, 0.0, 0.05 * (k % 3)])
        e1 = Rk @ tilt @ np.array([L, 0.0, 0.0])
        e2 = Rk @ tilt @ np.array([0.3 * L, L, 0.0])
        V += [v0, v0 + e1, v0 + e2]
        F.append([3 * k, 3 * k + 1, 3 * k + 2])
        corners.append((v0, e1, e2, Rk @ np.array([0.0, 0.0, 1.0])))
    mesh = M.Mesh(id=1, material="1", positions=np.array(V), indices=np.array(F, np.int32),
                  indices_one_based=False, shading_mode="flat")
    sc = scenes.scaled(scenes.scene_c1(8, 8), 8, 8)
    sc.objects = [mesh]
    O, D = [], []
    for i in range(6000):
        v0, e1, e2, nrm = corners[rng.integers(len(corners))]
        tgt = v0 + rng.uniform(0, 1e-9) * e1 + rng.uniform(0, 1e-9) * e2
        inplane = (e1 + e2) / np.linalg.norm(e1 + e2) + rng.uniform(-0.1, 0.1) * e1 / np.linalg.norm(e1)
        inplane /= np.linalg.norm(inplane)
        d = inplane + 10 ** rng.uniform(-13, -7) * rng.choice([-1.0, 1.0]) * nrm
        d /= np.linalg.norm(d)
        O.append(tgt - d * 10 ** rng.uniform(0, 3))
        D.append(d)
    O, D = np.array(O), np.array(D)
    hit = _check_closest(sc, O, D, walk=walk)
    assert hit.mean() > 0.3
    t, *_ = oracle.OracleScene(sc).trace_rays(O, D)
    tmax = np.where(np.isfinite(t), t * (1 + rng.choice([-1e-12, 1e-12], size=len(t))), 1e3)
    _check_occluded(sc, O, D, tmax, walk=walk)


def _twin_meshes():
    """Two meshes holding the SAME triangles (same vertices, same order) with different
    materials: every hit is an exact tie between two instances, and the reference keeps the
    first it visits (strict t < hit.t, RTContext.swift:494)."""
    hp, hf = scenes.heightfield(24, 8.0, 1.0, 3)
    hp32 = hp.astype(np.float32).astype(np.float64)
    a = M.Mesh(id=1, material="1", positions=hp32, indices=hf.astype(np.int32), indices_one_based=False,
               shading_mode="flat")
    b = M.Mesh(id=2, material="2", positions=hp32.copy(), indices=hf.astype(np.int32)[:, [0, 1, 2]],
               indices_one_based=False, shading_mode="smooth")
    sc = scenes.scaled(scenes.scene_c1(8, 8), 48, 40)
    sc.materials = [sc.materials[0], dataclasses.replace(sc.materials[0], diffuse=(0.1, 0.9, 0.2))]
    sc.objects = [a, b]
    sc.cameras[0].position = (0.5, 7.0, 7.5)
    sc.cameras[0].gaze_point = (0.0, 0.0, 0.0)
    sc.point_lights[0].position = (1.0, 9.0, 2.0)
    return sc, hp32


@pytest.mark.parametrize("walk", ["wide", "unified"])
def test_equal_t_ties_between_instances(walk):
    """Every hit of the twin-mesh scene is an exact tie: the four-wide walk must hand each such
    ray to the reference-order walk (rewalked > 0) and return the reference's instance -
    material, point and normal (flat vs smooth) tell the two apart."""
    sc, hp = _twin_meshes()
    rng = np.random.RandomState(4)
    D = rng.normal(size=(3000, 3)) * np.array([0.4, 1.0, 0.4]) - np.array([0.0, 2.0, 0.0])
    D /= np.linalg.norm(D, axis=1, keepdims=True)
    lo, hi = hp.min(0), hp.max(0)
    tgt = rng.uniform(lo, hi, size=(3000, 3))
    O = tgt - 12.0 * D
    hit = _check_closest(sc, O, D, walk=walk)
    assert hit.mean() > 0.5
    eng = _engine(sc, walk)
    rgb, rgba, st = eng.render_rows(0, 0, 1, True)
    ref, ref8, _ = oracle.OracleScene(sc).render(0, 0, 1, threads=0, rgba=True)
    eng.close()
    assert float(np.abs(rgb - ref).max()) <= 1e-5 and np.array_equal(rgba, ref8)
    if walk == "wide":
        assert st.rewalked > 0, "no tie was handed to the reference-order walk"
    else:
        assert st.rewalked == 0


@pytest.mark.parametrize("variant", ["area_light", "glass"])
def test_equal_t_ties_in_the_full_trace_passes(variant):
    """The twin-mesh ties through the full trace() kernels (k_level / k_events walk, k_shade,
    render_full): an area light (jitterIndex events) or glass on the second twin (dielectric
    paths).  Frames equal the oracle's and the re-walks are counted (rt_stats.rewalked > 0)."""
    sc, hp = _twin_meshes()
    if variant == "area_light":
        sc.area_lights = [M.AreaLight(position=(0.0, 9.0, 1.0), normal=(0.0, -1.0, 0.1), radiance=(400.0, 380.0, 350.0),
                                      size=2.0)]
    else:
        sc.materials[1] = M.Material(ambient=(0.0, 0.0, 0.0), diffuse=(0.05, 0.05, 0.05), specular=(0.5, 0.5, 0.5),
                                     phong=60.0, ior=1.5, absorption=(0.02, 0.04, 0.08), type="dielectric")
        sc.objects[0], sc.objects[1] = sc.objects[1], sc.objects[0]     # the glass twin is visited first
    eng = _engine(sc, "wide")
    rgb, rgba, st = eng.render_rows(0, 0, 1, True)
    ref, ref8, _ = oracle.OracleScene(sc).render(0, 0, 1, threads=0, rgba=True)
    eng.close()
    assert float(np.abs(rgb - ref).max()) <= 1e-5 and np.array_equal(rgba, ref8)
    assert st.rewalked > 0, "ties in the full trace() passes are not counted"


def _transformed_instances():
    """Instances of one mesh under scales, rotations and translations - triangles only, nothing
    moving."""
    sc = scenes.scaled(scenes.scene_c2(inline=True), 8, 8)
    base = sc.objects[0]
    rng = np.random.RandomState(31)
    objs = [base]
    for k in range(5):
        Rm = _rotation(rng) * (0.4 + 0.5 * k)
        t = rng.uniform(-3.0, 3.0, size=3)
        M4 = np.eye(4)
        M4[:3, :3] = Rm
        M4[:3, 3] = t
        objs.append(M.MeshInstance(id=40 + k, base_mesh_id=base.id, material="1",
                                   transform=tuple(M4.T.reshape(-1))))
    sc.objects = objs
    return sc


@pytest.mark.parametrize("walk", ["transformed", "transformed_tw", "transformed_binary", "nested"])
def test_transformed_mesh_instances(walk):
    """Rotated / scaled / translated mesh instances: the flattened instance tree (wide.h
    fit_walk, the default), the four-wide transformed walk (tw_walk, option fit = 0), the unified
    transformed walk (device.h ut_walk, option wide = 0) and the nested walk give the oracle's
    intersectTLAS / occludedTLAS bit for bit - including axis-aligned and signed-zero directions
    in local space."""
    sc = _transformed_instances()
    O, D = _ray_set(np.array([0.0, 0.0, 0.0]), 4.0, 3000, 23)
    _check_closest(sc, O, D, walk=walk)
    _check_occluded(sc, O, D, np.random.RandomState(6).uniform(0.1, 8.0, size=len(O)), walk=walk)


@pytest.mark.parametrize("walk", ["transformed", "transformed_tw", "transformed_binary", "nested"])
def test_equal_t_ties_between_transformed_instances(walk):
    """Two instances of one mesh under the same rotation and scale, with different materials:
    every hit is a tie between them, and the walks must return the reference's instance (the
    first intersectTLAS visits; strict t < hit.t, RTContext.swift:494)."""
    hp, hf = scenes.heightfield(24, 8.0, 1.0, 3)
    hp32 = hp.astype(np.float32).astype(np.float64)
    a = M.Mesh(id=1, material="1", positions=hp32, indices=hf.astype(np.int32), indices_one_based=False,
               shading_mode="flat")
    c, sn = np.cos(0.5), np.sin(0.5)                    # about y, so the camera still sees the grid
    Mt = np.eye(4)
    Mt[:3, :3] = np.array([[c, 0.0, sn], [0.0, 1.0, 0.0], [-sn, 0.0, c]]) * 0.75
    Mt[:3, 3] = (0.25, -0.5, 0.125)
    T = tuple(Mt.T.reshape(-1))
    sc = scenes.scaled(scenes.scene_c1(8, 8), 48, 40)
    sc.materials = [sc.materials[0], dataclasses.replace(sc.materials[0], diffuse=(0.1, 0.9, 0.2))]
    sc.objects = [a, M.MeshInstance(id=5, base_mesh_id=1, material="1", transform=T),
                  M.MeshInstance(id=6, base_mesh_id=1, material="2", transform=T)]
    sc.cameras[0].position = (0.5, 7.0, 7.5)
    sc.cameras[0].gaze_point = (0.0, 0.0, 0.0)
    sc.point_lights[0].position = (1.0, 9.0, 2.0)
    rng = np.random.RandomState(4)
    D = rng.normal(size=(3000, 3)) * np.array([0.4, 1.0, 0.4]) - np.array([0.0, 2.0, 0.0])
    D /= np.linalg.norm(D, axis=1, keepdims=True)
    loc = hp32[rng.randint(len(hp32), size=3000)] + rng.uniform(-0.05, 0.05, size=(3000, 3)) * np.array([1, 0, 1])
    tgt = loc @ Mt[:3, :3].T + Mt[:3, 3]
    O = tgt - 12.0 * D
    hit = _check_closest(sc, O, D, walk=walk)
    assert hit.mean() > 0.3
    eng = _engine(sc, walk)
    rgb, rgba, st = eng.render_rows(0, 0, 1, True)
    ref, ref8, _ = oracle.OracleScene(sc).render(0, 0, 1, threads=0, rgba=True)
    eng.close()
    assert float(np.abs(rgb - ref).max()) <= 1e-5 and np.array_equal(rgba, ref8)
    if walk in ("transformed", "transformed_tw"):    # four-wide (fit_walk / tw_walk): ties re-walked
        assert st.rewalked > 0
    else:                                            # the binary walks keep the reference order
        assert st.rewalked == 0


def test_fast_reciprocal_is_ieee_division():
    """device.h rcp_rn (1/det of the triangle tests when RenderParams::fast_rcp holds) equals
    IEEE 1.0/x bit for bit over its range 2^-700 <= |x| <= 2^1000: random mantissas at every
    exponent, both signs, powers of two, all-ones mantissas and the range ends."""
    import ctypes as C
    lib = M.load_library()
    rng = np.random.RandomState(7)
    exps = np.arange(-700, 1001)
    xs = [np.ldexp(1.0 + rng.random_sample(exps.size), exps),           # random mantissas
          np.ldexp(np.ones(exps.size), exps),                            # powers of two
          np.ldexp(np.full(exps.size, 2.0 - 2.0 ** -52), exps),          # all-ones mantissas
          np.ldexp(1.0 + 2.0 ** -52 * np.arange(1, exps.size + 1), exps),
          rng.uniform(1e-9, 1e9, 200000),                                 # determinants seen in scenes
          np.array([2.0 ** -700, 2.0 ** 1000, 3.0, 1.0 / 3.0, 0.1, 1e-7, 7e-300, 6e299])]
    x = np.concatenate(xs)
    x = np.concatenate([x, -x]).astype(np.float64)
    fast = np.empty_like(x)
    div = np.empty_like(x)
    p = lambda a: a.ctypes.data_as(C.POINTER(C.c_double))
    assert lib.rt_debug_rcp(int(x.size), p(x), p(fast), p(div)) == 0
    assert np.array_equal(div.view(np.uint64), (1.0 / x).view(np.uint64))   # the GPU division is IEEE
    bad = np.flatnonzero(fast.view(np.uint64) != div.view(np.uint64))
    assert bad.size == 0, (x[bad[:5]], fast[bad[:5]], div[bad[:5]])
