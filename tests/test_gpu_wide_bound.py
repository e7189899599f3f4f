"""The four-wide walk's widening bound, pushed to its edge (VERDICT r4 "next" #1).

The default walk of identity scenes (wide.h) tests inner boxes in FP32 against boxes widened per
render by wdelta = R * 2^-21 (render.hip set_wide; R bounds every box and ray-origin coordinate).
Its exactness proof (wide.h header) says the FP32 test then passes whenever the reference's FP64
hitAABB of a leaf below passes (RTContext.swift:557-565, 600-606).  These tests stress that:

* scenes translated and scaled to coordinates of 1e3, 1e5 and 1e6 with the camera far off the
  origin (FP32 rounding of the slab offsets grows with the coordinates, not with the geometry);
* explicit rays aimed a hair from triangle vertices (the hit point sits on or next to the corner or
  edge of its leaf box), through the vertices and along the edges;
* rays that touch a leaf box EXACTLY: FP64 tmax == max(tmin, eps), entering one face at the very
  t it leaves another (flat right triangles at dyadic coordinates, so the FP64 slab values are
  exact while their FP32 offsets are not), and hit the triangle there (u = 0 exactly);
* |1/d| at the wide walk's limits 2^-100 and 2^100 and just past them (binary walk);
* the full frame of C3 translated to 1e6.
Every set must equal the oracle bit for bit at the production widening.  Then the test-only render
option `wide_delta_scale` (per mille of the bound) shows the sets have teeth: with no widening (0)
the same sets produce mismatches, so they really reach the bound.
"""
import copy

import numpy as np
import pytest

import myraytracer_amd as M
from myraytracer_amd import _abi as A
from myraytracer_amd import scenes
import oracle

pytestmark = pytest.mark.gpu
TOL = 1e-5

# (scale, offset): geometry scaled, then translated; coordinates of ~1e3, ~1e5, ~1e6
PLACEMENTS = {"1e3": (10.0, (1.0e3, -7.0e2, 5.0e2)),
              "1e5": (1.0e3, (1.0e5, 3.0e4, -8.0e4)),
              "1e6": (1.0e4, (1.0e6, -6.0e5, 9.0e5))}


def _far(sc, scale, offset):
    """The same scene scaled by `scale` and moved by `offset`, as an identity scene (the geometry
    itself moves, float32-exact like PLY positions; no instance transform).  Camera, near plane,
    lights (intensity x scale^2: same image) and the shadow-ray epsilon follow."""
    s = copy.deepcopy(sc)
    off = np.asarray(offset, np.float64)
    for obj in s.objects:
        obj.positions = (np.asarray(obj.positions) * scale + off).astype(np.float32).astype(np.float64)
    for c in s.cameras:
        c.position = tuple(np.asarray(c.position) * scale + off)
        c.gaze_point = tuple(np.asarray(c.gaze_point) * scale + off)
        c.near_distance = c.near_distance * scale
    for L in s.point_lights:
        L.position = tuple(np.asarray(L.position) * scale + off)
        L.intensity = tuple(np.asarray(L.intensity) * scale * scale)
    s.shadow_ray_epsilon = s.shadow_ray_epsilon * scale
    return s


def _engine(sc, permille=None, fit=None):
    eng = M.RayTracerEngine(sc)
    if permille is not None:
        eng.set_unsafe_option("wide_delta_scale", permille)
    if fit is not None:
        eng.set_option("fit", fit)
    assert eng.get_option("wide") == 1
    return eng


def _closest_mismatch(sc, O, D, permille=None, orc=None, fit=None):
    """Rays whose closest hit (t, point, normal, material) differs from the oracle's."""
    eng = _engine(sc, permille, fit)
    tg, pg, ng, mg = eng.trace_rays(O, D)
    eng.close()
    to, po, no, mo = (orc or oracle.OracleScene(sc)).trace_rays(O, D)
    bad = (tg.view(np.uint64) != to.view(np.uint64)) | (mg != mo)
    hit = np.isfinite(to) & np.isfinite(tg)
    bad |= hit & ((pg != po).any(1) | (ng != no).any(1))
    return bad, np.isfinite(to)


def _occluded_mismatch(sc, O, D, tmax, permille=None, orc=None, fit=None):
    eng = _engine(sc, permille, fit)
    g = eng.occluded_rays(O, D, tmax)
    eng.close()
    o = (orc or oracle.OracleScene(sc)).occluded_rays(O, D, tmax)
    return g != o, o


def _near_vertex_rays(P, F, n, rng, reach):
    """Rays aimed at points a hair from a triangle vertex (relative offsets 1e-9 .. 1e-3 along both
    edges), exactly at the vertex, and on an edge: the hit points lie on or next to a corner or an
    edge of the triangle's leaf box, where FP32 slab values round across the FP64 ones."""
    tri = F[rng.randint(len(F), size=n)]
    k = rng.randint(3, size=n)
    a = P[tri[np.arange(n), k]]
    b = P[tri[np.arange(n), (k + 1) % 3]]
    c = P[tri[np.arange(n), (k + 2) % 3]]
    al = 10.0 ** rng.uniform(-9, -3, size=n)
    be = 10.0 ** rng.uniform(-9, -3, size=n)
    kind = rng.randint(8, size=n)
    al[kind == 0] = 0.0
    be[kind <= 1] = 0.0                                   # exactly at the vertex / on edge a-b
    tgt = a + al[:, None] * (b - a) + be[:, None] * (c - a)
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    O = tgt - d * (reach * rng.uniform(0.2, 2.0, size=n))[:, None]
    return O, d


def _far_c2(place):
    scale, off = PLACEMENTS[place]
    return _far(scenes.scaled(scenes.scene_c2(inline=True), 160, 120), scale, off), scale, np.asarray(off)


@pytest.mark.parametrize("place", list(PLACEMENTS))
def test_far_scene_rays_and_frame(place):
    """C2 at 1e3 / 1e5 / 1e6: random rays, near-vertex rays (closest + any hit) and the frame
    (L-inf <= 1e-5, exact RGBA8) equal the oracle's at the production widening."""
    sc, scale, off = _far_c2(place)
    mesh = sc.objects[0]
    P, F = np.asarray(mesh.positions), np.asarray(mesh.indices)
    rng = np.random.RandomState(61)
    orc = oracle.OracleScene(sc)
    Or = off + rng.uniform(-3.0, 3.0, size=(4000, 3)) * scale
    Dr = rng.normal(size=(4000, 3))
    Dr /= np.linalg.norm(Dr, axis=1, keepdims=True)
    Ov, Dv = _near_vertex_rays(P, F, 12000, rng, 3.0 * scale)
    O, D = np.concatenate([Or, Ov]), np.concatenate([Dr, Dv])
    bad, hit = _closest_mismatch(sc, O, D, orc=orc)
    assert not bad.any(), f"{int(bad.sum())} of {len(O)} closest hits differ"
    assert hit.mean() > 0.3
    t, *_ = orc.trace_rays(O, D)
    # shadow limits just past / just short of the closest hit, and far beyond
    tmax = np.where(np.isfinite(t), t * (1 + rng.choice([-1e-9, 1e-9], size=len(t))), 1e3 * scale)
    bado, occ = _occluded_mismatch(sc, O, D, tmax, orc=orc)
    assert not bado.any(), f"{int(bado.sum())} occlusion results differ"
    assert 0.05 < occ.mean() < 0.95
    eng = _engine(sc)
    rgb, rgba, st = eng.render_rows(0, 0, 1, True)
    eng.close()
    ref, ref8, _ = orc.render(0, 0, 1, threads=0, rgba=True)
    assert float(np.abs(rgb - ref).max()) <= TOL and np.array_equal(rgba, ref8)
    assert float(ref8[..., :3].std()) > 5.0                    # a real image, not a blank frame


def _touching_grid(offset, S=4.0, n=12):
    """Flat right triangles v0 = (X, Y, Z), v0 + (S, 0, 0), v0 + (0, S, 0) on a grid at a large
    dyadic offset: each triangle's own box is [X, X+S] x [Y, Y+S] x [Z, Z], and its edges x = X and
    y = Y lie on box faces."""
    X0, Y0, Z0 = offset
    V, Fc, corners = [], [], []
    for a in range(n):
        for b in range(n):
            x, y, z = X0 + 3 * S * a, Y0 + 3 * S * b, Z0    # one plane: every box is flat in z
            base = len(V)
            V += [(x, y, z), (x + S, y, z), (x, y + S, z)]
            Fc.append((base, base + 1, base + 2))
            corners.append((x, y, z))
    return np.array(V, np.float64), np.array(Fc, np.int32), np.array(corners)


def _touching_rays(corners, S, rng, n):
    """Rays that enter a triangle's box through the face x = X (or y = Y) at exactly the t at which
    they cross the flat z-slab, and hit the triangle there on its edge (u = 0 or v = 0 exactly):
    FP64 hitAABB gives tmax == tmin.  Directions and the path from the origin are dyadic, so the
    FP64 slab values are exact; the origins' large coordinates are not floats, so the FP32 plane
    offsets round."""
    idx = rng.randint(len(corners), size=n)
    x, y, z = corners[idx].T
    along = rng.randint(1, 16, size=n) / 16.0 * S
    on_x = rng.rand(n) < 0.5
    tgt = np.stack([np.where(on_x, x, x + along), np.where(on_x, y + along, y), z], 1)
    p2 = lambda lo, hi, m: 2.0 ** rng.randint(lo, hi, size=m)
    dz = -p2(-3, 2, n) * np.where(rng.rand(n) < 0.5, 1.0, -1.0)
    dx = np.where(on_x, p2(-3, 2, n), (rng.randint(-8, 9, size=n)) / 16.0)
    dy = np.where(on_x, (rng.randint(-8, 9, size=n)) / 16.0, p2(-3, 2, n))
    D = np.stack([dx, dy, dz], 1)
    t0 = p2(2, 8, n) + rng.randint(0, 64, size=n) / 64.0          # dyadic path length
    O = tgt - t0[:, None] * D
    return O, D, t0


def test_exactly_touching_leaf_boxes():
    """tmax == max(tmin, eps) exactly in the reference's FP64 hitAABB, on wide-eligible rays (every
    |1/d| in [2^-100, 2^100]): hits and occlusion equal the oracle's; and the rays do hit (u = 0)."""
    V, Fc, corners = _touching_grid((1048576.0, -524288.0, 786432.0))
    mesh = M.Mesh(id=1, material="1", positions=V, indices=Fc, indices_one_based=False, shading_mode="flat")
    sc = scenes.scaled(scenes.scene_c1(8, 8), 8, 8)
    sc.objects = [mesh]
    sc.cameras[0].position = tuple(corners.mean(0) + np.array([0.0, 0.0, 300.0]))
    sc.cameras[0].gaze_point = tuple(corners.mean(0))
    rng = np.random.RandomState(5)
    O, D, t0 = _touching_rays(corners, 4.0, rng, 6000)
    orc = oracle.OracleScene(sc)
    t, *_ = orc.trace_rays(O, D)
    assert (t == t0).mean() > 0.5, "the constructed rays should hit their triangle at t0"
    bad, _ = _closest_mismatch(sc, O, D, orc=orc)
    assert not bad.any(), f"{int(bad.sum())} of {len(O)} closest hits differ"
    tmax = t0 * (1 + 2.0 ** -40)
    bado, occ = _occluded_mismatch(sc, O, D, tmax, orc=orc)
    assert not bado.any() and occ.mean() > 0.5


def test_reciprocal_direction_at_the_wide_limits():
    """|1/d| = 2^-100 and 2^100 (the four-wide walk's limits, wide.h wide_ok) and just past them
    (2^-101, 2^101: those rays take the binary walk), mixed in the same waves, at 1e6."""
    sc, scale, off = _far_c2("1e6")
    rng = np.random.RandomState(8)
    n = 4096
    O = off + rng.uniform(-3.0, 3.0, size=(n, 3)) * scale
    D = rng.normal(size=(n, 3))
    D /= np.linalg.norm(D, axis=1, keepdims=True)
    ax = rng.randint(3, size=n)
    e = rng.choice([100, -100, 101, -101], size=n)
    # a component of magnitude 2^-e: |1/d| = 2^e along that axis
    D[np.arange(n), ax] = np.sign(rng.normal(size=n)) * 2.0 ** (-e.astype(np.float64))
    # |1/d| = 2^-100 on every axis: all components 2^100 (t shrinks, the FP32 products stay finite)
    big = rng.rand(n) < 0.1
    D[big] = np.sign(D[big]) * 2.0 ** 100
    bad, hit = _closest_mismatch(sc, O, D)
    assert not bad.any(), f"{int(bad.sum())} of {n} closest hits differ"
    assert hit.mean() > 0.1
    bado, _ = _occluded_mismatch(sc, O, D, np.full(n, np.inf))
    assert not bado.any()


def test_translated_c3_full_frame():
    """C3 (1.02M triangles) translated to 1e6 with the camera far off the origin: the full
    1920x1080 frame through the bench's call (RGBA8 into page-locked memory) equals the oracle."""
    sc = _far(scenes.scene_c3(inline=True), 1.0e4, (1.0e6, -6.0e5, 9.0e5))
    ref, ref8, ost = oracle.OracleScene(sc).render(0, threads=0, rgba=True)
    eng = _engine(sc)
    H, W = ref.shape[:2]
    rgba = M.pinned_array((H, W, 4), np.uint8)
    rgba.fill(0)
    st = eng.render_into(0, 0, 1, rgb=None, rgba=rgba, frame_layout=True)
    rgb, _, _ = eng.render_rows(0, 0, 1, False)
    eng.close()
    assert np.array_equal(rgba, ref8), f"RGBA8 differs on {int((rgba != ref8).any(-1).sum())} px"
    assert float(np.abs(rgb - ref).max()) <= TOL
    assert st.primary_rays == ost.primary_rays and st.shadow_rays_traced == ost.shadow_rays_used


def test_test_hooks_are_refused_by_the_production_entry_point():
    """wide_delta_scale (voids the exactness proof below 1000) and debug_fail_replica (injects
    failures) are test hooks: rt_scene_set_option refuses them with RT_ERR_INVALID_ARG and leaves
    the option at its production value; only rt_scene_set_unsafe_option (ABI 4, not for
    production) sets them.  Every ordinary option still goes through rt_scene_set_option."""
    eng = M.RayTracerEngine(scenes.scene_c1(16, 16))
    for name, val, default in (("wide_delta_scale", 0, 1000), ("wide_delta_scale", 1000, 1000),
                               ("debug_fail_replica", 0, -1)):
        with pytest.raises(M.RenderError) as e:
            eng.set_option(name, val)
        assert e.value.code == A.RT_ERR_INVALID_ARG and "test hook" in str(e.value)
        assert eng.get_option(name) == default
    eng.set_unsafe_option("wide_delta_scale", 500)
    assert eng.get_option("wide_delta_scale") == 500
    eng.set_unsafe_option("wide_delta_scale", 1000)
    eng.set_option("queue", 0)                               # an ordinary option
    assert eng.get_option("queue") == 0
    eng.close()


def test_the_sets_reach_the_bound():
    """Teeth: with the widening switched off (wide_delta_scale = 0) the near-vertex rays at 1e6 and
    the exactly touching rays DO produce mismatches against the oracle - so at the production
    widening (the tests above) they exercise the bound, not a slack case."""
    sc, scale, off = _far_c2("1e6")
    mesh = sc.objects[0]
    rng = np.random.RandomState(61)
    Ov, Dv = _near_vertex_rays(np.asarray(mesh.positions), np.asarray(mesh.indices), 12000, rng, 3.0 * scale)
    bad0, _ = _closest_mismatch(sc, Ov, Dv, permille=0)
    bad1, _ = _closest_mismatch(sc, Ov, Dv, permille=1000)
    assert not bad1.any()
    V, Fc, corners = _touching_grid((1048576.0, -524288.0, 786432.0))
    tsc = scenes.scaled(scenes.scene_c1(8, 8), 8, 8)
    tsc.objects = [M.Mesh(id=1, material="1", positions=V, indices=Fc, indices_one_based=False, shading_mode="flat")]
    O, D, t0 = _touching_rays(corners, 4.0, np.random.RandomState(5), 6000)
    badt0, _ = _closest_mismatch(tsc, O, D, permille=0)
    occ0, _ = _occluded_mismatch(tsc, O, D, t0 * (1 + 2.0 ** -40), permille=0)
    print(f"no widening: near-vertex {int(bad0.sum())} / {len(Ov)}, touching {int(badt0.sum())} / {len(O)} "
          f"closest, {int(occ0.sum())} occlusion mismatches")
    # measured on the GPU box (round 5): 512 / 12000 near-vertex, 85 / 6000 touching closest hits
    # and 226 / 6000 touching occlusion results differ without the widening
    assert bad0.any(), "near-vertex rays: no mismatch without widening, the set does not reach the bound"
    assert badt0.any() and occ0.any(), "touching rays: no mismatch without widening"


def _rot(rng):
    q = rng.normal(size=4)
    q /= np.linalg.norm(q)
    w, x, y, z = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def _far_instances():
    """C2's mesh far from the origin in its own space (1e6) under three rotated / scaled /
    translated instances placed far from the world origin (the four-wide transformed walk,
    wide.h tw_walk: world-space TLAS, local-space BLAS widened per ray)."""
    sc, scale, off = _far_c2("1e6")
    base = sc.objects[0]
    rng = np.random.RandomState(77)
    mats = []
    for k in range(3):
        M4 = np.eye(4)
        M4[:3, :3] = _rot(rng) * (0.5 + 0.4 * k)
        M4[:3, 3] = np.array([-3.0e5, 7.0e5, 2.0e5]) + rng.uniform(-1, 1, size=3) * 8.0e4 - M4[:3, :3] @ off
        mats.append(M4)
    base.transform = tuple(mats[0].T.reshape(-1))
    sc.objects = [base] + [M.MeshInstance(id=50 + k, base_mesh_id=base.id, material="1",
                                          transform=tuple(mats[k].T.reshape(-1))) for k in (1, 2)]
    centre = np.array([-3.0e5, 7.0e5, 2.0e5])
    sc.cameras[0].position = tuple(centre + np.array([0.0, 2.0e4, 9.0e4]))
    sc.cameras[0].gaze_point = tuple(centre)
    sc.point_lights[0].position = tuple(centre + np.array([4.0e4, 9.0e4, 6.0e4]))
    return sc, mats, centre


@pytest.mark.parametrize("fit", [1, 0])
def test_transformed_instances_far_away_and_teeth(fit):
    """Near-vertex rays at instances of a far mesh (world and local coordinates ~1e6): bit-exact
    closest hits and occlusion through the flattened instance tree (fit = 1, wide.h fit_walk) and
    the four-wide transformed walk (fit = 0, tw_walk), and the frame; without the widening
    (wide_delta_scale = 0, world and local) the same rays differ from the oracle."""
    sc, mats, centre = _far_instances()
    mesh = sc.objects[0]
    P, F = np.asarray(mesh.positions), np.asarray(mesh.indices)
    rng = np.random.RandomState(91)
    Os, Ds = [], []
    for M4 in mats:
        Pw = P @ M4[:3, :3].T + M4[:3, 3]
        O, D = _near_vertex_rays(Pw, F, 5000, rng, 4.0e4)
        Os.append(O); Ds.append(D)
    O, D = np.concatenate(Os), np.concatenate(Ds)
    orc = oracle.OracleScene(sc)
    bad, hit = _closest_mismatch(sc, O, D, orc=orc, fit=fit)
    assert not bad.any(), f"{int(bad.sum())} of {len(O)} closest hits differ"
    assert hit.mean() > 0.3
    t, *_ = orc.trace_rays(O, D)
    tmax = np.where(np.isfinite(t), t * (1 + rng.choice([-1e-9, 1e-9], size=len(t))), 1e7)
    bado, occ = _occluded_mismatch(sc, O, D, tmax, orc=orc, fit=fit)
    assert not bado.any()
    eng = _engine(sc, fit=fit)
    rgb, rgba, st = eng.render_rows(0, 0, 1, True)
    eng.close()
    ref, ref8, _ = orc.render(0, 0, 1, threads=0, rgba=True)
    assert float(np.abs(rgb - ref).max()) <= TOL and np.array_equal(rgba, ref8)
    bad0, _ = _closest_mismatch(sc, O, D, permille=0, orc=orc, fit=fit)
    print(f"transformed (fit = {fit}), no widening: {int(bad0.sum())} / {len(O)} closest hits differ")
    # tw_walk's local FP32 boxes are tight: the set reaches their bound.  The flattened tree's world
    # boxes of ROTATED instances are loose (AABB.transformed of a rotated leaf box), so the set
    # cannot: its teeth are test_fit_tree_reaches_the_bound (translated instances, tight boxes).
    if not fit:
        assert bad0.any(), "no mismatch without widening: the set does not reach the bound"


def test_fit_tree_reaches_the_bound():
    """The flattened instance tree at its edge: C2's mesh at 1e6 as a TRANSLATED instance (local
    coordinates = the far geometry minus the offset, exactly; the pair boxes equal the identity
    scene's leaf boxes), near-vertex rays bit-exact (closest + any hit) at the production widening,
    and mismatches without it - so wide.h fit_walk's widening is what keeps them exact."""
    sc, scale, off = _far_c2("1e6")
    mesh = sc.objects[0]
    Pw = np.asarray(mesh.positions)
    F = np.asarray(mesh.indices)
    mesh.positions = Pw - off                             # exact: multiples of 2^-4 below 2^15
    assert np.array_equal(mesh.positions + off, Pw)
    M4 = np.eye(4)
    M4[:3, 3] = off
    mesh.transform = tuple(M4.T.reshape(-1))
    rng = np.random.RandomState(61)
    O, D = _near_vertex_rays(Pw, F, 12000, rng, 3.0 * scale)
    orc = oracle.OracleScene(sc)
    bad, hit = _closest_mismatch(sc, O, D, orc=orc)
    assert not bad.any(), f"{int(bad.sum())} of {len(O)} closest hits differ"
    assert hit.mean() > 0.3
    t, *_ = orc.trace_rays(O, D)
    tmax = np.where(np.isfinite(t), t * (1 + rng.choice([-1e-9, 1e-9], size=len(t))), 1e3 * scale)
    bado, _ = _occluded_mismatch(sc, O, D, tmax, orc=orc)
    assert not bado.any()
    bad0, _ = _closest_mismatch(sc, O, D, permille=0, orc=orc)
    bad0t, _ = _closest_mismatch(sc, O, D, permille=0, orc=orc, fit=0)
    print(f"translated instance, no widening: fit {int(bad0.sum())} / {len(O)}, tw {int(bad0t.sum())} closest hits differ")
    assert bad0.any(), "no mismatch without widening: the set does not reach the fit tree's bound"
