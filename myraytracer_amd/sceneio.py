"""Scene files -> `Scene` (the reference's `SceneLoader.load`, RayTracer.swift:30-49).

The reference decodes its scene through ParsingKit's `SceneLoader.load(.url / .data(format: .auto))`
(`SceneFormat` = auto/json/xml, Models/SceneFormat.swift:8-10).  ParsingKit's scene model is not in
the container: only its v1.0.0 decoding helpers survive in the SwiftPM mirror pack
(`.build/repositories/ParsingKit-f301aefd`), and this module follows their conventions:

* `ParsingKit.decode(_:from:rootKey:)` (RootDecoding.swift:12-26): the document's "Scene" object is
  the root;
* `Flexible<T>` / `pkDouble` / `pkInt` (PropertyWrapper.swift:13-30, FlexibleDecoding.swift:31-44):
  a scalar is a JSON number or a numeric string (surrounding whitespace trimmed);
* `FlexibleVec3` (PropertyWrapper.swift:58-88) and `pkVectorStrings` (FlexibleDecoding.swift:47-61):
  a vector is a whitespace-separated string or a JSON array;
* `OneOrMany<T>` (PropertyWrapper.swift:36-44): a single object or an array of them.

XML input is turned into the same dictionary shape first (ParsingKit's XML2JSON.swift, whose source
is missing): attributes become "_name" keys, the text of an element with attributes becomes
"_data", repeated child elements become arrays.  Key names are those of the scene format the
reference's fields come from (RTContext.swift:94-418, Object+Extension.swift:52-433): `Cameras/Camera`,
`Lights/{AmbientLight,PointLight,AreaLight}`, `Materials/Material`, `Transformations`, `VertexData`,
`Objects/{Mesh,Triangle,Sphere,Plane,MeshInstance}`.

Parity here is **unpinned** (the key set, the object order and `Scene.composeTransform` live in the
missing dependency).  The fixed decisions, each in one place below:

* object order: Mesh, Triangle, Sphere, Plane, MeshInstance, each in file order (`_OBJECT_ORDER`);
  it only matters for TLAS instance order (H11);
* `composeTransform(tokens:reset:base:)` (called at RTContext.swift:127,162,195,374,388): tokens
  `t<id> s<id> r<id> c<id>` are applied in the order listed, M = T_n ... T_1; a MeshInstance
  composes on top of its base mesh's transform unless `_resetTransform` is true (`compose`);
* rotation `"angle ax ay az"` is in degrees about the normalised axis (Rodrigues); a Composite's 16
  numbers are row-major;
* `materialIndex(for:)` keeps the reference's Int(id) (RTContext.swift:423-426): material ids index
  the file-ordered material list 1-based (Object+Extension.swift:105-106), as in the reference;
* a mesh's `_plyFile` is resolved against the scene file's directory, else the current directory
  (RTContext.swift:251-254).
"""
from __future__ import annotations

import json
import math
import os
import xml.etree.ElementTree as ET
from typing import Any, Dict, List, Optional, Sequence, Tuple, Union

import numpy as np

from .scene import (AreaLight, Camera, Material, Mesh, MeshInstance, Plane, PointLight, Scene, Sphere,
                    Triangle)

SceneSource = Union[str, bytes, os.PathLike]

_OBJECT_ORDER = ("Mesh", "Triangle", "Sphere", "Plane", "MeshInstance")


class SceneLoadError(ValueError):
    """ParsingKit `SceneLoadError` / `PKDecodingError` (FlexibleDecoding.swift:10-22)."""


# ----------------------------------------------------------------------------- XML -> dict
def _xml_to_obj(el: ET.Element) -> Any:
    """One element -> str (text only) or dict (attributes "_k", children, text as "_data")."""
    kids = list(el)
    text = (el.text or "").strip()
    if not el.attrib and not kids:
        return text
    out: Dict[str, Any] = {f"_{k}": v for k, v in el.attrib.items()}
    for ch in kids:
        v = _xml_to_obj(ch)
        if ch.tag in out:
            prev = out[ch.tag]
            if isinstance(prev, list):
                prev.append(v)
            else:
                out[ch.tag] = [prev, v]
        else:
            out[ch.tag] = v
    if text:
        out["_data"] = text
    return out


def xml_to_dict(data: Union[str, bytes]) -> Dict[str, Any]:
    root = ET.fromstring(data)
    return {root.tag: _xml_to_obj(root)}


# ----------------------------------------------------------------------------- flexible scalars
def _text(v: Any) -> Any:
    """An element given with attributes keeps its text under "_data"."""
    if isinstance(v, dict) and "_data" in v:
        return v["_data"]
    return v


def _one_or_many(v: Any) -> List[Any]:
    """OneOrMany<T> (PropertyWrapper.swift:36-44)."""
    if v is None:
        return []
    return list(v) if isinstance(v, list) else [v]


def _double(v: Any, key: str) -> float:
    """pkDouble / Flexible<Double> (FlexibleDecoding.swift:39-44, PropertyWrapper.swift:13-30)."""
    v = _text(v)
    if isinstance(v, bool):
        raise SceneLoadError(f"Expected double-like value for {key}")
    if isinstance(v, (int, float)):
        return float(v)
    if isinstance(v, str):
        try:
            return float(v.strip())
        except ValueError:
            pass
    raise SceneLoadError(f"Expected double-like value for {key}")


def _int(v: Any, key: str) -> int:
    """pkInt (FlexibleDecoding.swift:32-37): int, numeric string, or a double truncated."""
    v = _text(v)
    if isinstance(v, bool):
        raise SceneLoadError(f"Expected int-like value for {key}")
    if isinstance(v, int):
        return v
    if isinstance(v, str):
        try:
            return int(v.strip(), 10)
        except ValueError:
            pass
    if isinstance(v, float):
        return int(v)
    raise SceneLoadError(f"Expected int-like value for {key}")


def _strings(v: Any, key: str) -> List[str]:
    """pkVectorStrings (FlexibleDecoding.swift:47-61)."""
    v = _text(v)
    if isinstance(v, str):
        return v.split()
    if isinstance(v, list):
        return [str(x) for x in v if isinstance(x, (int, float, str)) and not isinstance(x, bool)]
    if isinstance(v, (int, float)) and not isinstance(v, bool):
        return [str(v)]
    raise SceneLoadError(f"Expected vector-like value for {key}")


def _doubles(v: Any, key: str, n: Optional[int] = None) -> List[float]:
    parts = _strings(v, key)
    try:
        vals = [float(p) for p in parts]
    except ValueError:
        raise SceneLoadError(f"Invalid vector element for {key}") from None
    if n is not None and len(vals) < n:
        raise SceneLoadError(f"{key} requires {n} components")
    return vals


def _vec3(v: Any, key: str) -> Tuple[float, float, float]:
    """FlexibleVec3 (PropertyWrapper.swift:58-88): the first three components."""
    x = _doubles(v, key, 3)
    return (x[0], x[1], x[2])


def _opt(d: Dict[str, Any], key: str, conv, default=None):
    return conv(d[key], key) if key in d and d[key] is not None and _text(d[key]) != "" else default


def _id(d: Dict[str, Any]) -> Optional[str]:
    v = d.get("_id", d.get("id"))
    return None if v is None else str(v)


def _bool(v: Any) -> bool:
    v = _text(v)
    if isinstance(v, bool):
        return v
    return str(v).strip().lower() in ("true", "1", "yes")


# ----------------------------------------------------------------------------- transforms
def _translation(t) -> np.ndarray:
    m = np.eye(4)
    m[0:3, 3] = t
    return m


def _scaling(s) -> np.ndarray:
    return np.diag([s[0], s[1], s[2], 1.0])


def _rotation(angle_deg: float, axis) -> np.ndarray:
    a = np.asarray(axis, dtype=np.float64)
    n = math.sqrt(float(a @ a))
    if n == 0.0:
        raise SceneLoadError("rotation axis is zero")
    x, y, z = a / n
    th = math.radians(angle_deg)
    c, s, C = math.cos(th), math.sin(th), 1.0 - math.cos(th)
    m = np.eye(4)
    m[0:3, 0:3] = [[c + x * x * C, x * y * C - z * s, x * z * C + y * s],
                   [y * x * C + z * s, c + y * y * C, y * z * C - x * s],
                   [z * x * C - y * s, z * y * C + x * s, c + z * z * C]]
    return m


class _Transforms:
    """Scene.transformations: id -> 4x4 (row-major numpy) per kind."""

    def __init__(self, d: Optional[Dict[str, Any]]):
        self.table: Dict[str, np.ndarray] = {}
        d = d or {}
        for kind, letter in (("Translation", "t"), ("Scaling", "s"), ("Rotation", "r"), ("Composite", "c")):
            for e in _one_or_many(d.get(kind)):
                if not isinstance(e, dict):
                    raise SceneLoadError(f"{kind} needs an _id")
                tid = _id(e)
                vals = _doubles(e.get("_data"), kind)
                if kind == "Translation":
                    m = _translation(vals[:3])
                elif kind == "Scaling":
                    m = _scaling(vals[:3])
                elif kind == "Rotation":
                    if len(vals) < 4:
                        raise SceneLoadError("Rotation needs angle and axis")
                    m = _rotation(vals[0], vals[1:4])
                else:
                    if len(vals) < 16:
                        raise SceneLoadError("Composite needs 16 numbers")
                    m = np.asarray(vals[:16], dtype=np.float64).reshape(4, 4)
                self.table[f"{letter}{tid}"] = m

    def compose(self, tokens: Optional[str], base: Optional[np.ndarray] = None, reset: bool = False) -> np.ndarray:
        """Scene.composeTransform(tokens:reset:base:): tokens applied in order (M = T_n...T_1),
        on top of `base` unless `reset`."""
        m = np.eye(4) if (base is None or reset) else base.copy()
        for tok in (tokens or "").split():
            key = tok[0].lower() + tok[1:]
            if key not in self.table:
                raise SceneLoadError(f"unknown transformation {tok!r}")
            m = self.table[key] @ m
        return m


def _colmajor(m: np.ndarray) -> Tuple[float, ...]:
    return tuple(float(x) for x in np.asarray(m, dtype=np.float64).T.reshape(-1))


# ----------------------------------------------------------------------------- decoding
def _camera(c: Dict[str, Any]) -> Camera:
    res = _strings(c.get("ImageResolution", "0 0"), "ImageResolution")
    if len(res) < 2:
        raise SceneLoadError("ImageResolution requires 2 components")
    ctype = str(_text(c.get("_type", ""))) or "simple"
    fovy = _opt(c, "FovY", _double)
    return Camera(
        position=_vec3(c.get("Position", "0 0 0"), "Position"),
        up=_vec3(c.get("Up", "0 1 0"), "Up"),
        image_resolution=(int(float(res[0])), int(float(res[1]))),
        type=ctype,
        gaze_point=_opt(c, "GazePoint", _vec3, (0.0, 0.0, -1.0)),
        gaze=_opt(c, "Gaze", _vec3, (0.0, 0.0, -1.0)),
        fovy=fovy,
        near_distance=_opt(c, "NearDistance", _double, 1.0),
        near_plane=tuple(_opt(c, "NearPlane", lambda v, k: _doubles(v, k, 4)[:4], [-1.0, 1.0, -1.0, 1.0])),
        num_samples=_opt(c, "NumSamples", _int, 1),
        aperture_size=_opt(c, "ApertureSize", _double, 0.0),
        focus_distance=_opt(c, "FocusDistance", _double, 0.0),
        image_name=_opt(c, "ImageName", lambda v, k: str(_text(v)).strip()),
        id=_id(c),
    )


def _material(m: Dict[str, Any]) -> Material:
    z = (0.0, 0.0, 0.0)
    return Material(
        ambient=_opt(m, "AmbientReflectance", _vec3, z),
        diffuse=_opt(m, "DiffuseReflectance", _vec3, z),
        specular=_opt(m, "SpecularReflectance", _vec3, z),
        mirror=_opt(m, "MirrorReflectance", _vec3, z),
        phong=_opt(m, "PhongExponent", _double, 1.0),
        ior=_opt(m, "RefractionIndex", _double, 0.0),
        absorption_index=_opt(m, "AbsorptionIndex", _double, 0.0),
        roughness=_opt(m, "Roughness", _double, 0.0),
        absorption=_opt(m, "AbsorptionCoefficient", _vec3, z),
        type=str(_text(m.get("_type", ""))).strip(),
    )


def _vertex_data(v: Any) -> np.ndarray:
    if v is None:
        return np.zeros((0, 3))
    vals = _doubles(v, "VertexData")
    if len(vals) % 3:
        raise SceneLoadError("VertexData length is not a multiple of 3")
    return np.asarray(vals, dtype=np.float64).reshape(-1, 3)


def _vertex(vd: np.ndarray, idx: int, what: str) -> Tuple[float, float, float]:
    """scene.vertexData.data[i - 1] (RTContext.swift:124,167,199-201)."""
    if not (1 <= idx <= vd.shape[0]):
        raise SceneLoadError(f"{what}: vertex index {idx} out of range 1..{vd.shape[0]}")
    return tuple(float(x) for x in vd[idx - 1])


def _material_ref(o: Dict[str, Any]) -> Optional[str]:
    v = o.get("Material")
    if v is None:
        return None
    return str(_text(v)).strip()


def decode(doc: Dict[str, Any], base_dir: Optional[str] = None) -> Scene:
    """ParsingKit.decode(Scene.self, from:, rootKey: "Scene") (RootDecoding.swift:13-25)."""
    if not isinstance(doc, dict) or not isinstance(doc.get("Scene"), dict):
        raise SceneLoadError("Root key not found: Scene")
    doc = doc["Scene"]
    tf = _Transforms(doc.get("Transformations"))
    vd = _vertex_data(doc.get("VertexData"))

    cams = [_camera(c) for c in _one_or_many((doc.get("Cameras") or {}).get("Camera"))]
    mats = [_material(m) for m in _one_or_many((doc.get("Materials") or {}).get("Material"))]
    lights = doc.get("Lights") or {}
    ambient = _opt(lights, "AmbientLight", _vec3, (0.0, 0.0, 0.0))
    points = [PointLight(_vec3(p.get("Position"), "Position"), _vec3(p.get("Intensity"), "Intensity"))
              for p in _one_or_many(lights.get("PointLight"))]
    areas = [AreaLight(_vec3(a.get("Position"), "Position"), _vec3(a.get("Normal"), "Normal"),
                       _vec3(a.get("Radiance"), "Radiance"), _double(a.get("Size"), "Size"))
             for a in _one_or_many(lights.get("AreaLight"))]

    objs_in = doc.get("Objects") or {}
    objects = []
    mesh_transform: Dict[str, np.ndarray] = {}      # id -> composed transform (meshes and instances)
    for kind in _OBJECT_ORDER:
        for o in _one_or_many(objs_in.get(kind)):
            if not isinstance(o, dict):
                raise SceneLoadError(f"{kind} must be an object")
            oid = _id(o)
            mat = _material_ref(o)
            reset = _bool(o.get("_resetTransform", "false"))
            tokens = _text(o.get("Transformations"))
            if kind == "Mesh":
                M = tf.compose(tokens, reset=reset)
                faces = o.get("Faces")
                ply = faces.get("_plyFile") if isinstance(faces, dict) else None
                mesh = Mesh(id=_numeric_id(oid), material=mat, shading_mode=str(_text(o.get("_shadingMode", "flat"))),
                            transform=_colmajor(M),
                            motion_blur=_opt(o, "MotionBlur", _vec3, (0.0, 0.0, 0.0)))
                if ply:
                    mesh.ply_path = os.path.join(base_dir or os.getcwd(), str(ply))
                else:
                    idx = np.asarray([int(float(x)) for x in _strings(_text(faces) if faces is not None else "",
                                                                        "Faces")], dtype=np.int64)
                    if idx.size % 3:
                        raise SceneLoadError(f"Mesh {oid}: face index count is not a multiple of 3")
                    off = _opt(faces, "_vertexOffset", _int, 0) if isinstance(faces, dict) else 0
                    idx = idx + off
                    if idx.size and (idx.min() < 1 or idx.max() > vd.shape[0]):
                        raise SceneLoadError(f"Mesh {oid}: face index out of range 1..{vd.shape[0]}")
                    mesh.positions = vd
                    mesh.indices = idx.astype(np.int32).reshape(-1, 3)
                    mesh.indices_one_based = True
                mesh_transform[oid] = M
                objects.append(mesh)
            elif kind == "Triangle":
                ii = [int(float(x)) for x in _strings(o.get("Indices"), "Indices")]
                if len(ii) < 3:
                    raise SceneLoadError("Triangle needs 3 indices")
                verts = tuple(_vertex(vd, k, "Triangle") for k in ii[:3])
                objects.append(Triangle(vertices=verts, material=mat, transform=_colmajor(tf.compose(tokens, reset=reset)),
                                        id=_numeric_id(oid)))
            elif kind == "Sphere":
                ci = _int(o.get("Center"), "Center")
                objects.append(Sphere(center=_vertex(vd, ci, "Sphere"), radius=_double(o.get("Radius"), "Radius"),
                                      material=mat, transform=_colmajor(tf.compose(tokens, reset=reset)),
                                      id=_numeric_id(oid)))
            elif kind == "Plane":
                ci = _int(o.get("Point", o.get("Center")), "Point")
                objects.append(Plane(center=_vertex(vd, ci, "Plane"), normal=_vec3(o.get("Normal"), "Normal"),
                                     material=mat, transform=_colmajor(tf.compose(tokens, reset=reset)),
                                     id=_numeric_id(oid)))
            else:
                base = str(_text(o.get("_baseMeshId", "")))
                if base not in mesh_transform:
                    # RTContext.swift:386: `guard let baseData = instanceByID[baseMeshID] else { continue }`
                    continue
                M = tf.compose(tokens, base=mesh_transform[base], reset=reset)
                mesh_transform[oid] = M
                objects.append(MeshInstance(id=_numeric_id(oid), base_mesh_id=_numeric_id(base), material=mat,
                                            transform=_colmajor(M),
                                            motion_blur=_opt(o, "MotionBlur", _vec3, (0.0, 0.0, 0.0))))

    sc = Scene(cameras=cams, materials=mats, objects=objects, point_lights=points, area_lights=areas,
               ambient_light=ambient,
               background_color=_opt(doc, "BackgroundColor", _vec3, (0.0, 0.0, 0.0)),
               shadow_ray_epsilon=_opt(doc, "ShadowRayEpsilon", _double, 1e-3),
               intersection_test_epsilon=_opt(doc, "IntersectionTestEpsilon", _double, 1e-6),
               max_recursion_depth=_opt(doc, "MaxRecursionDepth", _int, 6),
               path=base_dir)
    return sc


def _numeric_id(oid: Optional[str]) -> int:
    """rt_object.id is an int; scene-file ids are strings (Int(id) like materialIndex, else a hash)."""
    if oid is None:
        return -1
    try:
        return int(oid, 10)
    except ValueError:
        import zlib
        return (zlib.crc32(oid.encode()) & 0x3FFFFFFF) | 0x40000000


def detect_format(data: Union[str, bytes]) -> str:
    """SceneFormat.auto: '<' -> xml, '{' / '[' -> json."""
    s = data.lstrip()[:1]
    if s in ("<", b"<"):
        return "xml"
    if s in ("{", "[", b"{", b"["):
        return "json"
    raise SceneLoadError("cannot detect scene format (expected JSON or XML)")


def loads(data: Union[str, bytes], format: str = "auto", base_dir: Optional[str] = None) -> Scene:
    """SceneLoader.load(.data(data, format:)) (RayTracer.swift:35-36)."""
    fmt = detect_format(data) if format == "auto" else format
    try:
        if fmt == "json":
            doc = json.loads(data)
        elif fmt == "xml":
            doc = xml_to_dict(data)
        else:
            raise SceneLoadError(f"unknown scene format {format!r}")
    except (json.JSONDecodeError, ET.ParseError) as e:
        raise SceneLoadError(f"scene decode failed: {e}") from e
    return decode(doc, base_dir)


def load(path: Union[str, os.PathLike], format: str = "auto") -> Scene:
    """SceneLoader.load(.url(url)); scene.path = url (RayTracer.swift:33-34)."""
    path = os.fspath(path)
    with open(path, "rb") as f:
        data = f.read()
    if format == "auto":
        ext = os.path.splitext(path)[1].lower()
        format = {".json": "json", ".xml": "xml"}.get(ext, "auto")
    return loads(data, format, base_dir=os.path.dirname(os.path.abspath(path)))


# ----------------------------------------------------------------------------- PNG
def save_png(rgba8: np.ndarray, path: str) -> None:
    """ImageHelper.savePNG(makeCGImage(rgba)) (Helpers/Image.swift:14-42): 8-bit RGB, alpha skipped
    (`CGImageAlphaInfo.noneSkipLast`), row 0 = top."""
    import struct
    import zlib

    a = np.ascontiguousarray(rgba8)
    if a.ndim != 3 or a.shape[2] not in (3, 4) or a.dtype != np.uint8:
        raise ValueError("expected (H, W, 4) or (H, W, 3) uint8")
    h, w = a.shape[:2]
    rows = np.concatenate([np.zeros((h, 1), np.uint8), a[:, :, :3].reshape(h, w * 3)], axis=1)

    def chunk(tag: bytes, payload: bytes) -> bytes:
        return struct.pack(">I", len(payload)) + tag + payload + struct.pack(">I", zlib.crc32(tag + payload) & 0xFFFFFFFF)

    png = b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 2, 0, 0, 0)) \
        + chunk(b"IDAT", zlib.compress(rows.tobytes(), 6)) + chunk(b"IEND", b"")
    tmp = path + ".tmp"
    with open(tmp, "wb") as f:
        f.write(png)
    os.replace(tmp, path)
