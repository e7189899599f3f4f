"""Scene description types — the stand-in for the reference's ParsingKit `Scene`.

The reference reads scenes through ParsingKit (`SceneLoader.load`, RayTracer.swift:30-49),
which is not available.  These dataclasses carry exactly the fields the
hot path reads (RTContext.swift:94-418, Object+Extension.swift:52-433) under the
ParsingKit names, and `to_desc()` packs them into the C structs of include/rtcore.h.
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple, Union

import numpy as np

from . import _abi as A

Vec3 = Tuple[float, float, float]
IDENTITY = tuple(float(x) for x in np.eye(4).reshape(-1))


def _v(x) -> A.rt_vec3:
    return A.rt_vec3(float(x[0]), float(x[1]), float(x[2]))


def material_index(mid: Optional[Union[str, int]]) -> int:
    """RTContext.materialIndex(for:) (RTContext.swift:423-426): Int(id) or -1."""
    if mid is None:
        return -1
    if isinstance(mid, int):
        return mid
    try:
        return int(str(mid), 10)
    except ValueError:
        return -1


@dataclass
class Material:
    ambient: Vec3 = (0.0, 0.0, 0.0)
    diffuse: Vec3 = (0.0, 0.0, 0.0)
    specular: Vec3 = (0.0, 0.0, 0.0)
    mirror: Vec3 = (0.0, 0.0, 0.0)
    phong: float = 1.0
    ior: float = 0.0
    absorption_index: float = 0.0
    roughness: float = 0.0
    absorption: Vec3 = (0.0, 0.0, 0.0)
    type: str = ""          # "", "mirror", "dielectric", "conductor"


@dataclass
class PointLight:
    position: Vec3
    intensity: Vec3


@dataclass
class AreaLight:
    position: Vec3
    normal: Vec3
    radiance: Vec3
    size: float


@dataclass
class Camera:
    position: Vec3
    up: Vec3
    image_resolution: Tuple[int, int]
    type: str = "lookAt"                 # "lookAt" or anything else (nearPlane camera)
    gaze_point: Vec3 = (0.0, 0.0, -1.0)
    gaze: Vec3 = (0.0, 0.0, -1.0)
    fovy: Optional[float] = None
    near_distance: float = 1.0
    near_plane: Tuple[float, float, float, float] = (-1.0, 1.0, -1.0, 1.0)
    num_samples: int = 1
    aperture_size: float = 0.0
    focus_distance: float = 0.0
    image_name: Optional[str] = None
    id: Optional[str] = None


@dataclass
class Mesh:
    """A mesh object.  Either `ply_path` (0-based indices, RTContext.swift:251-261) or
    inline `positions` + `indices` (faces.data, 1-based unless `indices_one_based=False`)."""
    id: int
    material: Optional[Union[str, int]] = "1"
    ply_path: Optional[str] = None
    positions: Optional[np.ndarray] = None     # (V,3) float64
    indices: Optional[np.ndarray] = None       # (T,3) int32
    normals: Optional[np.ndarray] = None       # (V,3) float64, PLY-branch normals
    indices_one_based: bool = True
    shading_mode: str = "flat"
    transform: Sequence[float] = IDENTITY      # column-major 4x4 localToWorld
    motion_blur: Vec3 = (0.0, 0.0, 0.0)


@dataclass
class Triangle:
    vertices: Tuple[Vec3, Vec3, Vec3]
    material: Optional[Union[str, int]] = "1"
    transform: Sequence[float] = IDENTITY
    motion_blur: Vec3 = (0.0, 0.0, 0.0)
    id: int = -1


@dataclass
class Sphere:
    center: Vec3
    radius: float
    material: Optional[Union[str, int]] = "1"
    transform: Sequence[float] = IDENTITY
    id: int = -1


@dataclass
class Plane:
    center: Vec3
    normal: Vec3
    material: Optional[Union[str, int]] = "1"
    transform: Sequence[float] = IDENTITY
    id: int = -1


@dataclass
class MeshInstance:
    id: int
    base_mesh_id: int
    material: Optional[Union[str, int]] = None     # None -> the base mesh's material
    transform: Sequence[float] = IDENTITY
    motion_blur: Vec3 = (0.0, 0.0, 0.0)


SceneObject = Union[Mesh, Triangle, Sphere, Plane, MeshInstance]


@dataclass
class Scene:
    cameras: List[Camera]
    materials: List[Material]
    objects: List[SceneObject]
    point_lights: List[PointLight] = field(default_factory=list)
    area_lights: List[AreaLight] = field(default_factory=list)
    ambient_light: Vec3 = (0.0, 0.0, 0.0)
    background_color: Vec3 = (0.0, 0.0, 0.0)
    shadow_ray_epsilon: float = 1e-3
    intersection_test_epsilon: float = 1e-6
    max_recursion_depth: int = 6
    path: Optional[str] = None           # directory of the scene file (Scene.path, RayTracer.swift:34)

    # ------------------------------------------------------------------ packing
    def to_desc(self) -> "PackedScene":
        return PackedScene(self)


class PackedScene:
    """Owns the ctypes arrays behind an `rt_scene_desc` (keep it alive while used)."""

    def __init__(self, scene: Scene):
        s = scene
        self._keep = []
        mats = (A.rt_material * max(1, len(s.materials)))()
        for i, m in enumerate(s.materials):
            mats[i] = A.rt_material(_v(m.ambient), _v(m.diffuse), _v(m.specular), _v(m.mirror), _v(m.absorption),
                                    float(m.phong), float(m.ior), float(m.absorption_index), float(m.roughness),
                                    A.RT_MAT.get(m.type, 0), 0)
        pls = (A.rt_point_light * max(1, len(s.point_lights)))()
        for i, l in enumerate(s.point_lights):
            pls[i] = A.rt_point_light(_v(l.position), _v(l.intensity))
        als = (A.rt_area_light * max(1, len(s.area_lights)))()
        for i, l in enumerate(s.area_lights):
            als[i] = A.rt_area_light(_v(l.position), _v(l.normal), _v(l.radiance), float(l.size))
        cams = (A.rt_camera * max(1, len(s.cameras)))()
        for i, c in enumerate(s.cameras):
            cc = A.rt_camera()
            cc.type = A.RT_CAM_LOOKAT if (c.type or "").lower() == "lookat" else A.RT_CAM_NEARPLANE
            cc.width, cc.height = int(c.image_resolution[0]), int(c.image_resolution[1])
            cc.num_samples = int(c.num_samples)
            cc.position, cc.gaze_point, cc.gaze, cc.up = _v(c.position), _v(c.gaze_point), _v(c.gaze), _v(c.up)
            cc.fovy = float("nan") if c.fovy is None else float(c.fovy)
            cc.near_distance = float(c.near_distance)
            for k in range(4):
                cc.near_plane[k] = float(c.near_plane[k])
            cc.aperture_size, cc.focus_distance = float(c.aperture_size), float(c.focus_distance)
            cams[i] = cc
        objs = (A.rt_object * max(1, len(s.objects)))()
        base_material = {o.id: o.material for o in s.objects if isinstance(o, Mesh)}
        for i, o in enumerate(s.objects):
            r = A.rt_object()
            r.transform[:] = [float(x) for x in np.asarray(o.transform, dtype=np.float64).reshape(-1)]
            r.id = int(getattr(o, "id", -1))
            r.indices_one_based = 1
            if isinstance(o, Mesh):
                r.kind = A.RT_OBJ_MESH
                r.material_id = material_index(o.material)
                r.smooth = 1 if o.shading_mode == "smooth" else 0
                r.motion_blur = _v(o.motion_blur)
                if o.ply_path is not None:
                    b = o.ply_path.encode()
                    self._keep.append(b)
                    r.ply_path = b
                else:
                    pos = np.ascontiguousarray(o.positions, dtype=np.float64).reshape(-1)
                    idx = np.ascontiguousarray(o.indices, dtype=np.int32).reshape(-1)
                    self._keep += [pos, idx]
                    r.positions = pos.ctypes.data_as(A.c_double_p)
                    r.num_positions = pos.size // 3
                    r.indices = idx.ctypes.data_as(A.c_int32_p)
                    r.num_indices = idx.size
                    r.indices_one_based = 1 if o.indices_one_based else 0
                    if o.normals is not None:
                        nrm = np.ascontiguousarray(o.normals, dtype=np.float64).reshape(-1)
                        if nrm.size != pos.size:
                            raise ValueError(f"mesh normals: {nrm.size // 3} xyz triples for "
                                             f"{pos.size // 3} positions (one normal per vertex expected)")
                        self._keep.append(nrm)
                        r.normals = nrm.ctypes.data_as(A.c_double_p)
                        r.num_normals = nrm.size // 3
            elif isinstance(o, Triangle):
                r.kind = A.RT_OBJ_TRIANGLE
                r.material_id = material_index(o.material)
                for k in range(3):
                    r.v[k] = _v(o.vertices[k])
                r.motion_blur = _v(o.motion_blur)
            elif isinstance(o, Sphere):
                r.kind = A.RT_OBJ_SPHERE
                r.material_id = material_index(o.material)
                r.center, r.radius = _v(o.center), float(o.radius)
            elif isinstance(o, Plane):
                r.kind = A.RT_OBJ_PLANE
                r.material_id = material_index(o.material)
                r.center, r.normal = _v(o.center), _v(o.normal)
            elif isinstance(o, MeshInstance):
                r.kind = A.RT_OBJ_MESH_INSTANCE
                mat = o.material if o.material not in (None, "") else base_material.get(o.base_mesh_id)
                r.material_id = material_index(mat)
                r.base_mesh_id = int(o.base_mesh_id)
                r.motion_blur = _v(o.motion_blur)
            else:
                raise TypeError(f"unknown scene object {type(o)!r}")
            objs[i] = r
        self._keep += [mats, pls, als, cams, objs]
        d = A.rt_scene_desc()
        d.background_color, d.ambient_light = _v(s.background_color), _v(s.ambient_light)
        d.shadow_ray_epsilon, d.intersection_test_epsilon = float(s.shadow_ray_epsilon), float(s.intersection_test_epsilon)
        d.max_recursion_depth = int(s.max_recursion_depth)
        d.num_materials, d.materials = len(s.materials), mats
        d.num_point_lights, d.point_lights = len(s.point_lights), pls
        d.num_area_lights, d.area_lights = len(s.area_lights), als
        d.num_objects, d.objects = len(s.objects), objs
        d.num_cameras, d.cameras = len(s.cameras), cams
        self.desc = d

    @property
    def ptr(self):
        return C.byref(self.desc)


def translation(tx: float, ty: float, tz: float) -> Tuple[float, ...]:
    m = np.eye(4)
    m[0:3, 3] = (tx, ty, tz)
    return tuple(m.T.reshape(-1))       # column-major


def fovy_deg(value: float) -> float:
    return float(value) if value is not None else math.nan
