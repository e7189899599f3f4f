"""Pin the CPU oracle (oracle/rt_oracle.cpp) with known answers derived from the
reference's formulas.  The Swift reference cannot run anywhere here, so
these KATs are the oracle's only anchor for the render path:

  * PCG32 streams (Object+Extension.swift:556-589) from an independent pure-Python PCG32;
  * the whole C1 frame from an independent vectorised numpy restatement of
    Renderer.render + trace for a single flat triangle (camera basis, per-pixel jitter,
    image-plane tMin, Moeller-Trumbore, Blinn-Phong, 1/d^2, shadow ray);
  * a closed-form centre-pixel check;
  * slab-test NaN/inf semantics and Moeller-Trumbore edge cases.
"""
import math

import numpy as np
import pytest

import oracle
from myraytracer_amd import scenes

M64 = (1 << 64) - 1


class PyPCG32:
    def __init__(self, seed):
        self.state, self.inc = 0, ((seed << 1) | 1) & M64
        self.next()
        self.state = (self.state + 0x9E3779B97F4A7C15) & M64
        self.next()

    def next(self):
        old = self.state
        self.state = (old * 6364136223846793005 + self.inc) & M64
        xs = (((old >> 18) ^ old) >> 27) & 0xFFFFFFFF
        rot = old >> 59
        return ((xs >> rot) | (xs << ((-rot) & 31))) & 0xFFFFFFFF

    def next_float(self):
        return float(self.next()) * 2.3283064365386963e-10


def test_pcg32_known_stream():
    # SURVEY.md §8c KAT (1): jitter-table seed
    assert oracle.pcg32_stream(0x123456789ABCDEF, 4) == [4216580722, 2511589146, 1215133729, 2029482206]


def test_pcg32_pixel_seed_floats():
    # pixel (0,0): seed ((0<<32)^0) &+ 0x9E3779B97F4A7C15 (Object+Extension.swift:294)
    r = PyPCG32(0x9E3779B97F4A7C15)
    got = [r.next_float() for _ in range(3)]
    assert got == [0.7661335312295705, 0.6387690156698227, 0.09951749863103032]
    u = oracle.pcg32_stream(0x9E3779B97F4A7C15, 3)
    assert [x * 2.3283064365386963e-10 for x in u] == got


@pytest.mark.parametrize("seed", [0, 1, 0xDEADBEEF, (7 << 32) ^ 5, M64])
def test_pcg32_matches_python(seed):
    r = PyPCG32(seed)
    assert oracle.pcg32_stream(seed, 16) == [r.next() for _ in range(16)]


# ------------------------------------------------------- numpy restatement of C1
def _np_pcg_init(seed):
    with np.errstate(over="ignore"):
        inc = (seed << np.uint64(1)) | np.uint64(1)
        state = np.zeros_like(seed)
        state, _ = _np_pcg_next(state, inc)
        state = state + np.uint64(0x9E3779B97F4A7C15)
        state, _ = _np_pcg_next(state, inc)
    return state, inc


def _np_pcg_next(state, inc):
    with np.errstate(over="ignore"):
        old = state
        state = old * np.uint64(6364136223846793005) + inc
        xs = (((old >> np.uint64(18)) ^ old) >> np.uint64(27)) & np.uint64(0xFFFFFFFF)
        rot = old >> np.uint64(59)
        out = ((xs >> rot) | (xs << ((np.uint64(32) - rot) & np.uint64(31)))) & np.uint64(0xFFFFFFFF)
    return state, out


def _dot(a, b):
    return (a[..., 0] * b[..., 0] + a[..., 1] * b[..., 1]) + a[..., 2] * b[..., 2]


def _cross(a, b):
    return np.stack([a[..., 1] * b[..., 2] - a[..., 2] * b[..., 1],
                     a[..., 2] * b[..., 0] - a[..., 0] * b[..., 2],
                     a[..., 0] * b[..., 1] - a[..., 1] * b[..., 0]], axis=-1)


def _normalize(v):
    return v * (1.0 / np.sqrt(_dot(v, v)))[..., None]


def _slab(lo, hi, o, inv, eps):
    t1 = (lo - o) * inv
    t2 = (hi - o) * inv
    mn, mx = np.fmin(t1, t2), np.fmax(t1, t2)
    smax = lambda x, y: np.where(y >= x, y, x)
    smin = lambda x, y: np.where(y < x, y, x)
    tmin = smax(smax(mn[..., 0], mn[..., 1]), mn[..., 2])
    tmax = smin(mx[..., 0], smin(mx[..., 1], mx[..., 2]))
    return np.where(tmax >= smax(tmin, eps), tmin, np.inf)


def numpy_render_c1(sc):
    """Vectorised restatement of Renderer.render/trace for a single flat triangle, spp=1."""
    cam = sc.cameras[0]
    W, H = cam.image_resolution
    eye = np.array(cam.position, float)
    gaze = np.array(cam.gaze_point, float) - eye
    w = -_normalize(gaze)
    up = _normalize(np.array(cam.up, float))
    u = _normalize(_cross(up, w))
    v = _normalize(_cross(w, u))
    nd = cam.near_distance
    t = nd * math.tan((cam.fovy * math.pi) / (2.0 * 180.0))
    r = t * (W / H)
    l, b = -r, -t
    du, dv = (r - l) / W, (t - b) / H
    m = eye - w * nd
    q00 = (m + u * l) + v * t
    jj, ii = np.meshgrid(np.arange(H, dtype=np.uint64), np.arange(W, dtype=np.uint64), indexing="ij")
    with np.errstate(over="ignore"):
        seed = ((jj << np.uint64(32)) ^ ii) + np.uint64(0x9E3779B97F4A7C15)
    st, inc = _np_pcg_init(seed)
    st, a = _np_pcg_next(st, inc)
    st, bb = _np_pcg_next(st, inc)
    st, c = _np_pcg_next(st, inc)
    xi1, xi2 = a.astype(np.float64) * 2.3283064365386963e-10, bb.astype(np.float64) * 2.3283064365386963e-10
    cI = ii.astype(np.float64) + (0.0 + xi1) / 1.0
    cJ = jj.astype(np.float64) + (0.0 + xi2) / 1.0
    s = (q00 - v * (cJ * dv)[..., None]) + u * (cI * du)[..., None]
    d = _normalize(s - eye)
    denom = _dot(d, np.broadcast_to(w, d.shape))
    timg = _dot(np.broadcast_to((eye - w * nd) - eye, d.shape), np.broadcast_to(w, d.shape)) / denom
    tlo = np.where(0.0 >= timg, 0.0, timg)
    inv = 1.0 / d
    V = np.array(sc.objects[0].positions, float)
    v0, v1, v2 = V
    e1, e2 = v1 - v0, v2 - v0
    eps = sc.intersection_test_epsilon
    lo, hi = np.minimum(v0, np.minimum(v1, v2)), np.maximum(v0, np.maximum(v1, v2))
    # TLAS root box = instance world bounds = AABB.transformed(identity) = c -/+ e
    c0, ex = 0.5 * (lo + hi), 0.5 * (hi - lo)
    wlo, whi = c0 - ex, c0 + ex
    o = np.broadcast_to(eye, d.shape)
    box_ok = (_slab(wlo, whi, o, inv, eps) != np.inf) & (_slab(lo, hi, o, inv, eps) != np.inf)
    p = _cross(d, np.broadcast_to(e2, d.shape))
    det = _dot(np.broadcast_to(e1, d.shape), p)
    with np.errstate(divide="ignore", invalid="ignore"):
        invdet = 1.0 / det
        tv = o - v0
        uu = _dot(tv, p) * invdet
        q = _cross(tv, np.broadcast_to(e1, d.shape))
        vv = _dot(d, q) * invdet
        tt = _dot(np.broadcast_to(e2, d.shape), q) * invdet
    hit = box_ok & ~(np.abs(det) < eps) & ~((uu < 0) | (uu > 1)) & ~((vv < 0) | (uu + vv > 1)) & \
        ~(tt <= np.where(tlo >= eps, tlo, eps))
    pl = (v0 + uu[..., None] * e1) + vv[..., None] * e2
    nl = _normalize(_cross(e1, e2))
    # instance: identity localToWorld / normalMatrix, literally multiplied
    P = ((1.0 * pl[..., 0:1] * np.array([1, 0, 0]) + pl[..., 1:2] * np.array([0, 1, 0])) +
         pl[..., 2:3] * np.array([0, 0, 1])) + 1.0 * np.array([0.0, 0.0, 0.0])
    n3 = (nl[0] * np.array([1.0, 0, 0]) + nl[1] * np.array([0, 1.0, 0])) + nl[2] * np.array([0, 0, 1.0])
    Ng = np.broadcast_to(_normalize(n3), d.shape)
    front = _dot(d, Ng) < 0
    N = np.where(front[..., None], Ng, -Ng)
    mat = sc.materials[0]
    Lo = np.broadcast_to(np.array(sc.ambient_light) * np.array(mat.ambient), d.shape).copy()
    L = sc.point_lights[0]
    wi = np.array(L.position) - P
    dist = np.sqrt(_dot(wi, wi))
    wi = _normalize(wi)
    # shadow ray vs the only triangle (cannot be occluded by itself here: it starts on the lit side)
    NdotL = _dot(N, wi)
    NdotL = np.where(NdotL >= 0.0, NdotL, 0.0)
    view = _normalize(-d)
    h = _normalize(wi + view)
    NdotH = _dot(N, h)
    NdotH = np.where(NdotH >= 0.0, NdotH, 0.0)
    shin = mat.phong if mat.phong >= 1.0 else 1.0
    Ld = np.array(mat.diffuse) * NdotL[..., None]
    Ls = np.array(mat.specular) * np.power(NdotH, shin)[..., None]
    att = np.array(L.intensity) / np.where(dist * dist >= 1e-12, dist * dist, 1e-12)[..., None]
    Lo = Lo + np.where((NdotL > 0)[..., None], (Ld + Ls) * att, 0.0)
    img = np.where(hit[..., None], Lo, np.array(sc.background_color, float))
    return img


def test_c1_frame_matches_numpy_restatement():
    sc = scenes.scene_c1()
    ref = numpy_render_c1(sc)
    got, st = oracle.OracleScene(sc).render(0, threads=4)
    assert got.shape == ref.shape == (256, 256, 3)
    assert float(np.abs(got - ref).max()) <= 1e-12
    assert np.mean(got == ref) > 0.99           # bit-identical almost everywhere
    hit = ~(got == np.array(sc.background_color)).all(-1)
    assert st.primary_rays == 256 * 256 and st.shadow_rays == int(hit.sum())


def test_c1_centre_pixel_closed_form():
    sc = scenes.scene_c1()
    got, _ = oracle.OracleScene(sc).render(0, threads=1)
    # pixel (128,128): the ray passes within half a pixel of the optical axis and hits z=-3
    cam_t = math.tan(math.radians(30.0))
    r = PyPCG32(((128 << 32) ^ 128) + 0x9E3779B97F4A7C15 & M64)
    xi1, xi2 = r.next_float(), r.next_float()
    x = (-cam_t + (128 + xi1) * (2 * cam_t / 256))
    y = (cam_t - (128 + xi2) * (2 * cam_t / 256))
    d = np.array([x, y, -1.0]) / math.sqrt(x * x + y * y + 1.0)
    p = d * (3.0 / -d[2])
    L = np.array([2.0, 2.0, 0.0]) - p
    dist = np.linalg.norm(L)
    wi = L / dist
    n = np.array([0.0, 0.0, 1.0])
    hv = wi - d
    hv /= np.linalg.norm(hv)
    col = 25.0 + (np.array([0.8, 0.5, 0.3]) * (wi @ n) + 0.5 * max(hv @ n, 0.0) ** 32) * 3e3 / dist ** 2
    assert np.allclose(got[128, 128], col, rtol=0, atol=1e-9)


# --------------------------------------------------------------- edge cases
def test_slab_nan_semantics():
    lo, hi = np.zeros(3), np.ones(3)
    # origin on the x=0 face, direction parallel to it: (0-0)*inf = NaN, suppressed by
    # simd.min/max (fmin/fmax); Swift.max/min then give tmin = inf > tmax -> miss
    assert oracle.hit_aabb(lo, hi, [0.0, 0.5, 0.5], [0.0, 1.0, 0.0], 1e-6) == math.inf
    # inside the box: the (negative) entry distance is returned (tmax >= max(tmin, eps));
    # y/z slabs are (-inf, +inf) and Swift.max keeps the x entry -0.5
    assert oracle.hit_aabb(lo, hi, [0.5, 0.5, 0.5], [1.0, 0.0, 0.0], 1e-6) == -0.5
    assert oracle.hit_aabb(lo, hi, [-1.0, 0.5, 0.5], [1.0, 0.25, 0.0], 1e-6) == 1.0
    # box entirely behind the origin
    assert oracle.hit_aabb(lo, hi, [2.0, 0.5, 0.5], [1.0, 0.0, 0.0], 1e-6) == math.inf
    # exit exactly at eps counts (tmax >= max(tmin, eps))
    assert oracle.hit_aabb(lo, hi, [-0.5, 0.5, 0.5], [1.0, 0.0, 0.0], 1.5) == 0.5
    assert oracle.hit_aabb(lo, hi, [-0.5, 0.5, 0.5], [1.0, 0.0, 0.0], 1.5000001) == math.inf


def test_moller_trumbore_edges():
    v0, v1, v2 = [0.0, 0.0, 0.0], [1.0, 0.0, 0.0], [0.0, 1.0, 0.0]
    t, p, n = oracle.intersect_triangle(v0, v1, v2, [0.25, 0.25, 1.0], [0.0, 0.0, -1.0])
    assert t == 1.0 and list(p) == [0.25, 0.25, 0.0] and list(n) == [0.0, 0.0, 1.0]
    # exactly on the hypotenuse u+v == 1 is accepted
    t, _, _ = oracle.intersect_triangle(v0, v1, v2, [0.5, 0.5, 1.0], [0.0, 0.0, -1.0])
    assert t == 1.0
    # parallel ray: |det| < eps -> miss
    t, _, _ = oracle.intersect_triangle(v0, v1, v2, [0.2, 0.2, 1.0], [1.0, 0.0, 0.0])
    assert t == math.inf
    # behind tMin
    t, _, _ = oracle.intersect_triangle(v0, v1, v2, [0.25, 0.25, 1.0], [0.0, 0.0, -1.0], tmin=1.0)
    assert t == math.inf
    # no backface culling
    t, _, _ = oracle.intersect_triangle(v0, v1, v2, [0.25, 0.25, -2.0], [0.0, 0.0, 1.0])
    assert t == 2.0
