"""Seeded synthetic scenes for the BASELINE.json configs.

There is no Stanford bunny or any other asset in the container, so every config is
generated here, deterministically, and written as binary-little-endian float32 PLY
(float32 positions, no ASCII rounding quirks).  No degenerate triangles
are produced (H15): heightfields are regular grids, spheres use pole fans.

  C1  single triangle, 256x256                     (config[0])
  C2  ~69k-tri displaced UV sphere + ground, 800x600, smooth        (config[1])
  C3  ~1.02M-tri heightfield + 24 icospheres, 1920x1080, shadows    (config[2], the bench workload)
  C4  = C3 tile-partitioned over GPUs                                 (config[3])
  C5  ~10M tris: 2048^2 heightfield + mirror icospheres, 3840x2160, depth 4 (config[4])
"""
from __future__ import annotations

import math
import os
from typing import Dict, Tuple

import numpy as np

from .scene import AreaLight, Camera, Material, Mesh, MeshInstance, PointLight, Scene


# ----------------------------------------------------------------------------- PLY
def write_ply(path: str, positions: np.ndarray, faces: np.ndarray, normals: np.ndarray = None,
              fmt: str = "binary_little_endian") -> None:
    """Write a PLY with float32 x,y,z[,nx,ny,nz] and a `list uchar int vertex_indices` face list."""
    pos = np.ascontiguousarray(positions, dtype=np.float32)
    f = np.ascontiguousarray(faces, dtype=np.int32)
    nv, nf = pos.shape[0], f.shape[0]
    props = "property float x\nproperty float y\nproperty float z\n"
    if normals is not None:
        props += "property float nx\nproperty float ny\nproperty float nz\n"
    header = (f"ply\nformat {fmt} 1.0\ncomment myraytracer_amd synthetic scene\n"
              f"element vertex {nv}\n{props}element face {nf}\nproperty list uchar int vertex_indices\nend_header\n")
    verts = pos if normals is None else np.concatenate([pos, np.asarray(normals, np.float32)], axis=1)
    with open(path, "wb") as fh:
        fh.write(header.encode("ascii"))
        if fmt == "ascii":
            for row in verts:
                fh.write((" ".join(repr(float(x)) for x in row) + "\n").encode())
            for tri in f:
                fh.write(("3 " + " ".join(str(int(x)) for x in tri) + "\n").encode())
            return
        endian = "<" if fmt == "binary_little_endian" else ">"
        fh.write(np.ascontiguousarray(verts.astype(endian + "f4")).tobytes())
        rec = np.zeros(nf, dtype=[("n", "u1"), ("i", endian + "i4", (3,))])
        rec["n"] = 3
        rec["i"] = f
        fh.write(rec.tobytes())


# ------------------------------------------------------------------------ geometry
def value_noise_2d(x: np.ndarray, y: np.ndarray, seed: int, octaves: int = 5) -> np.ndarray:
    """Smooth lattice value noise, sum of octaves, in [-1, 1]-ish."""
    rng = np.random.RandomState(seed)
    out = np.zeros_like(x, dtype=np.float64)
    amp, freq, norm = 1.0, 1.0, 0.0
    for _ in range(octaves):
        lat = rng.uniform(-1.0, 1.0, size=(257, 257))
        fx, fy = x * freq, y * freq
        ix, iy = np.floor(fx).astype(np.int64), np.floor(fy).astype(np.int64)
        tx, ty = fx - ix, fy - iy
        sx, sy = tx * tx * (3 - 2 * tx), ty * ty * (3 - 2 * ty)
        ix0, iy0 = ix % 256, iy % 256
        a, b = lat[ix0, iy0], lat[ix0 + 1, iy0]
        c, d = lat[ix0, iy0 + 1], lat[ix0 + 1, iy0 + 1]
        out += amp * ((a * (1 - sx) + b * sx) * (1 - sy) + (c * (1 - sx) + d * sx) * sy)
        norm += amp
        amp *= 0.5
        freq *= 2.0
    return out / norm


def heightfield(n: int, size: float, height: float, seed: int) -> Tuple[np.ndarray, np.ndarray]:
    """(n+1)^2 vertices, 2*n^2 triangles over [-size/2, size/2]^2 in xz, y = noise."""
    g = np.linspace(-size / 2, size / 2, n + 1)
    X, Z = np.meshgrid(g, g, indexing="ij")
    Y = height * value_noise_2d((X / size + 0.5) * 8.0, (Z / size + 0.5) * 8.0, seed)
    pos = np.stack([X, Y, Z], axis=-1).reshape(-1, 3)
    i, j = np.meshgrid(np.arange(n), np.arange(n), indexing="ij")
    v00 = (i * (n + 1) + j).reshape(-1)
    v10, v01, v11 = v00 + (n + 1), v00 + 1, v00 + (n + 1) + 1
    # counter-clockwise seen from +y
    t1 = np.stack([v00, v01, v10], axis=1)
    t2 = np.stack([v10, v01, v11], axis=1)
    faces = np.empty((2 * n * n, 3), dtype=np.int64)
    faces[0::2], faces[1::2] = t1, t2
    return pos, faces


def icosphere(level: int) -> Tuple[np.ndarray, np.ndarray]:
    """Unit icosphere with 20*4^level faces (outward CCW)."""
    t = (1.0 + 5 ** 0.5) / 2.0
    v = np.array([[-1, t, 0], [1, t, 0], [-1, -t, 0], [1, -t, 0], [0, -1, t], [0, 1, t], [0, -1, -t], [0, 1, -t],
                  [t, 0, -1], [t, 0, 1], [-t, 0, -1], [-t, 0, 1]], dtype=np.float64)
    v /= np.linalg.norm(v, axis=1, keepdims=True)
    f = np.array([[0, 11, 5], [0, 5, 1], [0, 1, 7], [0, 7, 10], [0, 10, 11], [1, 5, 9], [5, 11, 4], [11, 10, 2],
                  [10, 7, 6], [7, 1, 8], [3, 9, 4], [3, 4, 2], [3, 2, 6], [3, 6, 8], [3, 8, 9], [4, 9, 5],
                  [2, 4, 11], [6, 2, 10], [8, 6, 7], [9, 8, 1]], dtype=np.int64)
    verts = [tuple(x) for x in v]
    for _ in range(level):
        cache: Dict[Tuple[int, int], int] = {}
        vl = verts

        def mid(a, b):
            key = (a, b) if a < b else (b, a)
            if key in cache:
                return cache[key]
            p = (np.asarray(vl[a]) + np.asarray(vl[b])) * 0.5
            p /= np.linalg.norm(p)
            vl.append(tuple(p))
            cache[key] = len(vl) - 1
            return cache[key]

        nf = []
        for a, b, c in f:
            ab, bc, ca = mid(a, b), mid(b, c), mid(c, a)
            nf += [[a, ab, ca], [b, bc, ab], [c, ca, bc], [ab, bc, ca]]
        f = np.array(nf, dtype=np.int64)
        verts = vl
    return np.asarray(verts, dtype=np.float64), f


def uv_sphere(segments: int, rings: int) -> Tuple[np.ndarray, np.ndarray]:
    """UV sphere with pole triangle fans: 2*segments*(rings-1) faces."""
    verts = [(0.0, 1.0, 0.0)]
    for r in range(1, rings):
        th = math.pi * r / rings
        for s in range(segments):
            ph = 2 * math.pi * s / segments
            verts.append((math.sin(th) * math.cos(ph), math.cos(th), math.sin(th) * math.sin(ph)))
    verts.append((0.0, -1.0, 0.0))
    V = np.asarray(verts)
    bottom = len(verts) - 1
    faces = []
    ring = lambda r, s: 1 + (r - 1) * segments + (s % segments)
    for s in range(segments):
        faces.append([0, ring(1, s + 1), ring(1, s)])
    for r in range(1, rings - 1):
        for s in range(segments):
            a, b = ring(r, s), ring(r, s + 1)
            c, d = ring(r + 1, s), ring(r + 1, s + 1)
            faces.append([a, b, d])
            faces.append([a, d, c])
    for s in range(segments):
        faces.append([bottom, ring(rings - 1, s), ring(rings - 1, s + 1)])
    return V, np.asarray(faces, dtype=np.int64)


def _displace(V: np.ndarray, amp: float, seed: int) -> np.ndarray:
    """Radial smooth displacement of unit-sphere vertices."""
    rng = np.random.RandomState(seed)
    k = rng.normal(size=(6, 3))
    ph = rng.uniform(0, 2 * np.pi, size=6)
    d = np.zeros(len(V))
    for q in range(6):
        d += np.sin(3.0 * (V @ k[q]) + ph[q])
    return V * (1.0 + amp * d / 6.0)[:, None]


def _merge(parts):
    pos, faces, off = [], [], 0
    for p, f in parts:
        pos.append(p)
        faces.append(f + off)
        off += len(p)
    return np.concatenate(pos), np.concatenate(faces)


# --------------------------------------------------------------------------- configs
def _std_material(diffuse=(0.8, 0.6, 0.4), mtype="") -> Material:
    return Material(ambient=(0.1, 0.1, 0.1), diffuse=diffuse, specular=(0.4, 0.4, 0.4), phong=24.0,
                    mirror=(0.6, 0.6, 0.6) if mtype == "mirror" else (0.0, 0.0, 0.0), type=mtype)


def scene_c1(width: int = 256, height: int = 256) -> Scene:
    """Single triangle."""
    tri = np.array([[-1.0, -1.0, -3.0], [1.0, -1.0, -3.0], [0.0, 1.0, -3.0]])
    mesh = Mesh(id=1, material="1", positions=tri, indices=np.array([[1, 2, 3]], np.int32), shading_mode="flat")
    mat = Material(ambient=(1, 1, 1), diffuse=(0.8, 0.5, 0.3), specular=(0.5, 0.5, 0.5), phong=32.0)
    cam = Camera(position=(0.0, 0.0, 0.0), gaze_point=(0.0, 0.0, -1.0), up=(0.0, 1.0, 0.0), fovy=60.0,
                 near_distance=1.0, image_resolution=(width, height), type="lookAt", image_name="c1.png")
    return Scene(cameras=[cam], materials=[mat], objects=[mesh],
                 point_lights=[PointLight((2.0, 2.0, 0.0), (3e3, 3e3, 3e3))], ambient_light=(25.0, 25.0, 25.0),
                 background_color=(10.0, 20.0, 30.0), shadow_ray_epsilon=1e-3, intersection_test_epsilon=1e-6,
                 max_recursion_depth=6)


def geometry_c2(segments: int = 256, rings: int = 136, seed: int = 1):
    V, F = uv_sphere(segments, rings)
    V = _displace(V, 0.08, seed) * 1.0
    ground = (np.array([[-4.0, -1.2, -4.0], [4.0, -1.2, -4.0], [4.0, -1.2, 4.0], [-4.0, -1.2, 4.0]]),
              np.array([[0, 2, 1], [0, 3, 2]]))
    return _merge([(V, F), ground])


def geometry_c3(grid: int = 512, spheres: int = 24, level: int = 5, seed: int = 42):
    hp, hf = heightfield(grid, 100.0, 6.0, seed)
    rng = np.random.RandomState(seed + 1)
    Vs, Fs = icosphere(level)
    parts = [(hp, hf)]
    for q in range(spheres):
        r = rng.uniform(1.0, 3.0)
        cx, cz = rng.uniform(-22, 22), rng.uniform(-22, 22)
        V = _displace(Vs, 0.05, seed + 10 + q) * r + np.array([cx, 5.0 + r, cz])
        parts.append((V, Fs))
    return _merge(parts)


def geometry_c5(grid: int = 2048, spheres: int = 80, level: int = 5, seed: int = 5):
    hp, hf = heightfield(grid, 120.0, 6.0, seed)
    rng = np.random.RandomState(seed + 1)
    Vs, Fs = icosphere(level)
    parts = []
    for q in range(spheres):
        r = rng.uniform(0.8, 2.5)
        cx, cz = rng.uniform(-50, 50), rng.uniform(-50, 50)
        parts.append((_displace(Vs, 0.03, seed + 10 + q) * r + np.array([cx, 6.0 + r, cz]), Fs))
    return (hp, hf), _merge(parts)


def _ply_or_inline(path_dir, name, pos, faces, smooth, mid, mat, inline):
    if inline or path_dir is None:
        return Mesh(id=mid, material=mat, positions=pos.astype(np.float32).astype(np.float64),
                    indices=faces.astype(np.int32), indices_one_based=False, shading_mode=smooth)
    os.makedirs(path_dir, exist_ok=True)
    path = os.path.join(path_dir, name)
    if not os.path.exists(path):
        # several ranks may generate the same scene at once: write privately, publish atomically
        tmp = f"{path}.{os.getpid()}.tmp"
        write_ply(tmp, pos, faces)
        os.replace(tmp, path)
    return Mesh(id=mid, material=mat, ply_path=path, shading_mode=smooth)


def scene_c2(path_dir: str = None, width: int = 800, height: int = 600, inline: bool = False) -> Scene:
    pos, faces = geometry_c2()
    mesh = _ply_or_inline(path_dir, "c2_bunny_standin.ply", pos, faces, "smooth", 1, "1", inline)
    cam = Camera(position=(0.0, 0.6, 4.2), gaze_point=(0.0, -0.1, 0.0), up=(0.0, 1.0, 0.0), fovy=45.0,
                 near_distance=1.0, image_resolution=(width, height), image_name="c2.png")
    return Scene(cameras=[cam], materials=[_std_material((0.7, 0.7, 0.6))], objects=[mesh],
                 point_lights=[PointLight((3.0, 5.0, 4.0), (2.0e3, 2.0e3, 2.0e3))], ambient_light=(20.0, 20.0, 20.0),
                 background_color=(15.0, 25.0, 40.0), shadow_ray_epsilon=1e-3, intersection_test_epsilon=1e-6,
                 max_recursion_depth=4)


def scene_c3(path_dir: str = None, width: int = 1920, height: int = 1080, inline: bool = False) -> Scene:
    pos, faces = geometry_c3()
    mesh = _ply_or_inline(path_dir, "c3_terrain_spheres_1m.ply", pos, faces, "smooth", 1, "1", inline)
    # oblique view, ~18% sky (miss) pixels
    cam = Camera(position=(0.0, 18.0, 42.0), gaze_point=(0.0, 0.0, 8.0), up=(0.0, 1.0, 0.0), fovy=50.0,
                 near_distance=1.0, image_resolution=(width, height), image_name="c3.png")
    return Scene(cameras=[cam], materials=[_std_material((0.6, 0.7, 0.5))], objects=[mesh],
                 point_lights=[PointLight((30.0, 40.0, 40.0), (3.0e5, 3.0e5, 3.0e5))], ambient_light=(15.0, 15.0, 15.0),
                 background_color=(40.0, 60.0, 90.0), shadow_ray_epsilon=1e-3, intersection_test_epsilon=1e-6,
                 max_recursion_depth=4)


def scene_c5(path_dir: str = None, width: int = 3840, height: int = 2160, inline: bool = False) -> Scene:
    (hp, hf), (sp, sf) = geometry_c5()
    terrain = _ply_or_inline(path_dir, "c5_terrain_8m.ply", hp, hf, "smooth", 1, "1", inline)
    mirrors = _ply_or_inline(path_dir, "c5_mirror_spheres_1p6m.ply", sp, sf, "smooth", 2, "2", inline)
    cam = Camera(position=(0.0, 25.0, 90.0), gaze_point=(0.0, 2.0, 0.0), up=(0.0, 1.0, 0.0), fovy=50.0,
                 near_distance=1.0, image_resolution=(width, height), image_name="c5.png")
    return Scene(cameras=[cam], materials=[_std_material((0.6, 0.7, 0.5)), _std_material((0.2, 0.2, 0.2), "mirror")],
                 objects=[terrain, mirrors], point_lights=[PointLight((40.0, 80.0, 60.0), (4.0e5, 4.0e5, 4.0e5))],
                 ambient_light=(15.0, 15.0, 15.0), background_color=(40.0, 60.0, 90.0), shadow_ray_epsilon=1e-3,
                 intersection_test_epsilon=1e-6, max_recursion_depth=4)


def _placement(s: float, tx: float, ty: float, tz: float):
    """Column-major localToWorld of a uniform scale s followed by a translation."""
    return (s, 0.0, 0.0, 0.0, 0.0, s, 0.0, 0.0, 0.0, 0.0, s, 0.0, tx, ty, tz, 1.0)


def scene_c3_instanced(path_dir: str = None, width: int = 1920, height: int = 1080, inline: bool = False) -> Scene:
    """C3's geometry as mesh instances with non-identity transforms (the literal intersectTLAS
    walk, RTContext.swift:619-720, every object an instance, :122-241, 384-401): the 512^2
    terrain translated, one displaced level-5 icosphere base mesh placed by scale + translation,
    and 23 MeshInstances of it placed the way C3 places its 24 spheres.  1,015,808 triangles
    traced (524,288 + 24 x 20,480), 2 BLASes, a TLAS of 25 instances; same camera and light."""
    seed = 42
    hp, hf = heightfield(512, 100.0, 6.0, seed)
    rng = np.random.RandomState(seed + 1)
    Vs, Fs = icosphere(5)
    Vb = _displace(Vs, 0.05, seed + 10)
    places = []
    for q in range(24):
        r = rng.uniform(1.0, 3.0)
        cx, cz = rng.uniform(-22, 22), rng.uniform(-22, 22)
        places.append(_placement(r, cx, 5.0 + r, cz))
    terrain = _ply_or_inline(path_dir, "c3i_terrain.ply", hp, hf, "smooth", 1, "1", inline)
    terrain.transform = _placement(1.0, 0.0, -0.25, 0.0)
    base = _ply_or_inline(path_dir, "c3i_icosphere.ply", Vb, Fs, "smooth", 2, "1", inline)
    base.transform = places[0]
    objs = [terrain, base] + [MeshInstance(id=3 + q, base_mesh_id=2, transform=places[q]) for q in range(1, 24)]
    cam = Camera(position=(0.0, 18.0, 42.0), gaze_point=(0.0, 0.0, 8.0), up=(0.0, 1.0, 0.0), fovy=50.0,
                 near_distance=1.0, image_resolution=(width, height), image_name="c3i.png")
    return Scene(cameras=[cam], materials=[_std_material((0.6, 0.7, 0.5))], objects=objs,
                 point_lights=[PointLight((30.0, 40.0, 40.0), (3.0e5, 3.0e5, 3.0e5))], ambient_light=(15.0, 15.0, 15.0),
                 background_color=(40.0, 60.0, 90.0), shadow_ray_epsilon=1e-3, intersection_test_epsilon=1e-6,
                 max_recursion_depth=4)


def scene_c3_glass(path_dir: str = None, width: int = 1920, height: int = 1080, inline: bool = False,
                   area_lights: bool = True, rough: bool = False) -> Scene:
    """C3's geometry with the 24 spheres made of glass (dielectric with Beer absorption, two
    child rays per bounce, Object+Extension.swift:207-251) and two area lights next to the
    point light (:145-186, the chunk-sequential jitterIndex): the full trace() kernels
    (render_full, k_events + k_jscan).  Terrain and spheres are two meshes, maxRecursionDepth 4.
    area_lights=False: the point light alone (C3d: dielectric paths without the events passes).
    rough=True (C3r): the glass is rough (roughness 0.05, Object+Extension.swift:191-198, 209-216):
    PCG32 draws inside trace() fix the walk order, so the area-light frame takes the depth-first
    k_events pass instead of the level passes."""
    seed = 42
    hp, hf = heightfield(512, 100.0, 6.0, seed)
    rng = np.random.RandomState(seed + 1)
    Vs, Fs = icosphere(5)
    parts = []
    for q in range(24):
        r = rng.uniform(1.0, 3.0)
        cx, cz = rng.uniform(-22, 22), rng.uniform(-22, 22)
        parts.append((_displace(Vs, 0.05, seed + 10 + q) * r + np.array([cx, 5.0 + r, cz]), Fs))
    sp, sf = _merge(parts)
    terrain = _ply_or_inline(path_dir, "c3g_terrain.ply", hp, hf, "smooth", 1, "1", inline)
    glass = _ply_or_inline(path_dir, "c3g_spheres.ply", sp, sf, "smooth", 2, "2", inline)
    cam = Camera(position=(0.0, 18.0, 42.0), gaze_point=(0.0, 0.0, 8.0), up=(0.0, 1.0, 0.0), fovy=50.0,
                 near_distance=1.0, image_resolution=(width, height), image_name="c3g.png")
    mats = [_std_material((0.6, 0.7, 0.5)),
            Material(ambient=(0.0, 0.0, 0.0), diffuse=(0.05, 0.05, 0.05), specular=(0.5, 0.5, 0.5), phong=60.0,
                     ior=1.5, absorption=(0.02, 0.04, 0.08), roughness=0.05 if rough else 0.0, type="dielectric")]
    return Scene(cameras=[cam], materials=mats, objects=[terrain, glass],
                 point_lights=[PointLight((30.0, 40.0, 40.0), (3.0e5, 3.0e5, 3.0e5))],
                 area_lights=[AreaLight(position=(-20.0, 30.0, 10.0), normal=(0.5, -1.0, -0.2), radiance=(900.0, 850.0, 800.0),
                                        size=4.0),
                              AreaLight(position=(25.0, 20.0, -10.0), normal=(-1.0, -0.6, 0.3),
                                        radiance=(300.0, 400.0, 600.0), size=3.0)] if area_lights else [],
                 ambient_light=(15.0, 15.0, 15.0), background_color=(40.0, 60.0, 90.0), shadow_ray_epsilon=1e-3,
                 intersection_test_epsilon=1e-6, max_recursion_depth=4)


def scaled(scene: Scene, width: int, height: int) -> Scene:
    """Same scene, different image resolution (parity tests at oracle-friendly sizes)."""
    import copy
    s = copy.deepcopy(scene)
    for c in s.cameras:
        c.image_resolution = (width, height)
    return s
