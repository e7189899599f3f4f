"""Scene-file loader: RayTracerEngine.init(from:data:) -> SceneLoader.load
(RayTracer.swift:30-49), ParsingKit's flexible decoding conventions (FlexibleDecoding.swift,
PropertyWrapper.swift, RootDecoding.swift of the v1.0.0 mirror pack), and the PNG epilogue
(Helpers/Image.swift:14-42).  CPU only: decoded scenes are compared with hand-built ones, and the
CPU oracle renders both bit-identically.  Parity of the key set itself is unpinned (ParsingKit's
scene model is missing)."""
import json
import math
import os
import shutil
import struct
import zlib

import numpy as np
import pytest

import myraytracer_amd as M
from myraytracer_amd import scenes, sceneio

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "scenes")


def _canon(x):
    """Comparable form of a Scene (numpy arrays -> nested lists)."""
    if isinstance(x, np.ndarray):
        return ("nd", x.dtype.kind, x.tolist())
    if hasattr(x, "__dataclass_fields__"):
        return (type(x).__name__, tuple((k, _canon(getattr(x, k))) for k in x.__dataclass_fields__))
    if isinstance(x, (list, tuple)):
        return tuple(_canon(v) for v in x)
    return x


@pytest.fixture(scope="module")
def mixed_dir(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("mixed"))
    for f in ("mixed.json", "mixed.xml"):
        shutil.copy(os.path.join(GOLDEN, f), d)
    V, F = scenes.icosphere(1)
    scenes.write_ply(os.path.join(d, "ico.ply"), V * 0.7, F)
    return d


def test_json_and_xml_decode_to_the_same_scene(mixed_dir):
    a = sceneio.load(os.path.join(mixed_dir, "mixed.json"))
    b = sceneio.load(os.path.join(mixed_dir, "mixed.xml"))
    assert _canon(a) == _canon(b)
    # auto-detection from bytes gives the same result as the extension
    with open(os.path.join(mixed_dir, "mixed.xml"), "rb") as f:
        c = sceneio.loads(f.read(), base_dir=mixed_dir)
    assert _canon(c) == _canon(b)


def _translation(x, y, z):
    m = np.eye(4); m[0:3, 3] = (x, y, z); return m


def _rot_y(deg):
    t = math.radians(deg)
    m = np.eye(4)
    m[0, 0] = math.cos(t); m[0, 2] = math.sin(t); m[2, 0] = -math.sin(t); m[2, 2] = math.cos(t)
    return m


def _cm(m):
    return tuple(float(v) for v in m.T.reshape(-1))


def test_decoded_fields_and_transform_composition(mixed_dir):
    s = sceneio.load(os.path.join(mixed_dir, "mixed.json"))
    assert s.max_recursion_depth == 4 and s.background_color == (12.0, 18.0, 30.0)
    assert s.shadow_ray_epsilon == 1e-3 and s.intersection_test_epsilon == 1e-6
    assert s.ambient_light == (20.0, 20.0, 20.0)
    assert [l.position for l in s.point_lights] == [(4.0, 6.0, 5.0), (-5.0, 3.0, 2.0)]
    c0, c1 = s.cameras
    assert c0.type == "lookAt" and c0.fovy == 45.0 and c0.image_resolution == (96, 72)
    assert c0.gaze_point == (0.0, 0.4, 0.0) and c0.image_name == "mixed_lookat.png" and c0.id == "1"
    assert c1.type != "lookAt" and c1.fovy is None and c1.near_plane == (-0.6, 0.6, -0.45, 0.45)
    assert c1.image_resolution == (80, 60)
    assert [m.type for m in s.materials] == ["", "mirror", ""] and s.materials[1].phong == 64.0
    kinds = [type(o).__name__ for o in s.objects]
    assert kinds == ["Mesh", "Mesh", "Triangle", "Sphere", "Sphere", "Plane", "MeshInstance", "MeshInstance"]
    mesh1, mesh2, tri, sph6, sph7, pln, inst3, inst4 = s.objects
    # r1 then t2: M = T(2.2,0,0) * Ry(30)
    np.testing.assert_allclose(np.array(mesh1.transform), _cm(_translation(2.2, 0, 0) @ _rot_y(30)), atol=1e-15)
    assert mesh1.indices.tolist()[0] == [1, 2, 3] and mesh1.indices_one_based and mesh1.positions.shape == (10, 3)
    assert mesh2.ply_path == os.path.join(mixed_dir, "ico.ply") and mesh2.shading_mode == "smooth"
    # Composite is row-major: translation column (-2, 0.3, 0.5)
    assert tuple(mesh2.transform[12:15]) == (-2.0, 0.3, 0.5)
    assert tri.vertices == ((-3.0, -1.0, -3.0), (3.0, -1.0, -3.0), (0.0, 2.5, -3.2))
    assert sph6.center == (-1.6, 0.0, 0.0) and sph6.radius == 1.0 and sph6.material == "2"
    np.testing.assert_array_equal(np.array(sph7.transform), _cm(_translation(0.4, 0, -1.5) @ np.diag([2, 2, 2, 1.0])))
    assert pln.center == (0.0, -1.0, 0.0) and pln.normal == (0.0, 1.0, 0.0)
    # MeshInstance 3 composes t1 on top of its base mesh; 4 resets (its base is instance 3)
    np.testing.assert_allclose(np.array(inst3.transform),
                               _cm(_translation(0.4, 0, -1.5) @ _translation(2.2, 0, 0) @ _rot_y(30)), atol=1e-15)
    assert inst3.base_mesh_id == 1 and inst3.material == "2"
    np.testing.assert_array_equal(np.array(inst4.transform), np.array(sph7.transform))
    assert inst4.base_mesh_id == 3 and inst4.material is None


def test_flexible_scalars_vectors_and_one_or_many():
    doc = {"Scene": {
        "MaxRecursionDepth": 3.0, "BackgroundColor": [1, "2", 3.5], "ShadowRayEpsilon": " 0.01 ",
        "Cameras": {"Camera": {"Position": [0, 0, 0], "Gaze": "0 0 -1", "Up": "0 1 0",
                               "ImageResolution": "8 8", "NumSamples": " 4"}},
        "Materials": {"Material": {"_id": 1, "DiffuseReflectance": {"_data": "1 1 1"}}},
        "VertexData": "0 0 0 1 0 0 0 1 0",
        "Objects": {"Mesh": {"_id": 1, "Material": 1, "Faces": "1 2 3"}}}}
    s = sceneio.decode(doc)
    assert s.max_recursion_depth == 3 and s.background_color == (1.0, 2.0, 3.5) and s.shadow_ray_epsilon == 0.01
    assert len(s.cameras) == 1 and s.cameras[0].num_samples == 4
    assert s.materials[0].diffuse == (1.0, 1.0, 1.0)
    assert s.objects[0].indices.tolist() == [[1, 2, 3]] and s.objects[0].material == "1"


@pytest.mark.parametrize("doc,msg", [
    ({"NotScene": 1}, "Root key"),
    ({"Scene": {"BackgroundColor": "1 2"}}, "requires 3"),
    ({"Scene": {"MaxRecursionDepth": "x"}}, "int-like"),
    ({"Scene": {"VertexData": "0 0 0 1", "Objects": {}}}, "multiple of 3"),
    ({"Scene": {"VertexData": "0 0 0", "Objects": {"Sphere": {"Center": "2", "Radius": "1"}}}}, "out of range"),
    ({"Scene": {"VertexData": "0 0 0", "Objects": {"Mesh": {"_id": "1", "Faces": "1 1 2"}}}}, "out of range"),
    ({"Scene": {"Objects": {"Sphere": {"Center": "1", "Radius": "1", "Transformations": "t9"}},
                "VertexData": "0 0 0"}}, "unknown transformation"),
])
def test_decode_errors(doc, msg):
    with pytest.raises(sceneio.SceneLoadError, match=msg):
        sceneio.decode(doc)


def test_format_detection_and_bad_documents():
    assert sceneio.detect_format(b"  <Scene/>") == "xml" and sceneio.detect_format(' {"Scene": {}}') == "json"
    with pytest.raises(sceneio.SceneLoadError):
        sceneio.loads("Scene: yaml")
    with pytest.raises(sceneio.SceneLoadError):
        sceneio.loads("{not json", format="json")
    with pytest.raises(sceneio.SceneLoadError):
        sceneio.loads("<Scene><Cameras></Scene>", format="xml")


def test_instance_of_missing_base_is_dropped():
    """RTContext.swift:386: `guard let baseData = instanceByID[baseMeshID] else { continue }`."""
    doc = {"Scene": {"VertexData": "0 0 0 1 0 0 0 1 0",
                     "Objects": {"MeshInstance": {"_id": "2", "_baseMeshId": "9"},
                                 "Mesh": {"_id": "1", "Faces": "1 2 3"}}}}
    s = sceneio.decode(doc)
    assert [type(o).__name__ for o in s.objects] == ["Mesh"]


def test_loaded_c1_equals_built_c1_on_the_oracle():
    """The C1 scene written as a scene file renders bit-identically to scenes.scene_c1 on the oracle."""
    import oracle
    doc = {"Scene": {
        "MaxRecursionDepth": "6", "BackgroundColor": "10 20 30", "ShadowRayEpsilon": "1e-3",
        "IntersectionTestEpsilon": "1e-6",
        "Cameras": {"Camera": {"_id": "1", "_type": "lookAt", "Position": "0 0 0", "GazePoint": "0 0 -1",
                               "Up": "0 1 0", "FovY": "60", "NearDistance": "1", "ImageResolution": "64 48",
                               "ImageName": "c1.png"}},
        "Lights": {"AmbientLight": "25 25 25", "PointLight": {"_id": "1", "Position": "2 2 0",
                                                             "Intensity": "3e3 3e3 3e3"}},
        "Materials": {"Material": {"_id": "1", "AmbientReflectance": "1 1 1", "DiffuseReflectance": "0.8 0.5 0.3",
                                   "SpecularReflectance": "0.5 0.5 0.5", "PhongExponent": "32"}},
        "VertexData": "-1 -1 -3 1 -1 -3 0 1 -3",
        "Objects": {"Mesh": {"_id": "1", "_shadingMode": "flat", "Material": "1", "Faces": "1 2 3"}}}}
    loaded = sceneio.loads(json.dumps(doc))
    built = scenes.scene_c1(64, 48)
    a, _ = oracle.OracleScene(loaded).render(0, threads=0)
    b, _ = oracle.OracleScene(built).render(0, threads=0)
    assert np.array_equal(a, b)


def inline_plys(scene):
    """Copy of `scene` whose PLY meshes carry the file's float32-widened arrays inline (0-based),
    the form the CPU oracle takes (PLYReader.swift:85-102)."""
    import copy
    import oracle
    s = copy.deepcopy(scene)
    for o in s.objects:
        if isinstance(o, M.Mesh) and o.ply_path:
            d = oracle.RefCPly().load(o.ply_path) if os.path.exists(oracle.REF_CPLY) else M.ply_load(o.ply_path)
            o.positions = np.asarray(d["positions"], np.float64).reshape(-1, 3)
            o.indices = np.asarray(d["indices"], np.int32).reshape(-1, 3)
            o.normals = d["normals"]
            o.indices_one_based = False
            o.ply_path = None
    return s


def test_mixed_scene_renders_on_the_oracle(mixed_dir):
    """Every object kind of the loader reaches the (test-only) CPU restatement and is hit."""
    import oracle
    s = inline_plys(sceneio.load(os.path.join(mixed_dir, "mixed.json")))
    for cam in range(2):
        img, st = oracle.OracleScene(s).render(cam, threads=0)
        assert np.isfinite(img).all() and st.primary_rays == np.prod(s.cameras[cam].image_resolution)
        bg = np.array(s.background_color)
        assert (np.abs(img - bg).max(axis=-1) > 0).mean() > 0.3      # most pixels hit geometry


def _png_decode(path):
    data = open(path, "rb").read()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat, hdr = 8, b"", None
    while pos < len(data):
        n, = struct.unpack(">I", data[pos:pos + 4]); tag = data[pos + 4:pos + 8]; body = data[pos + 8:pos + 8 + n]
        crc, = struct.unpack(">I", data[pos + 8 + n:pos + 12 + n])
        assert crc == zlib.crc32(tag + body) & 0xFFFFFFFF
        if tag == b"IHDR":
            hdr = struct.unpack(">IIBBBBB", body)
        elif tag == b"IDAT":
            idat += body
        pos += 12 + n
    w, h, depth, ctype = hdr[:4]
    assert depth == 8 and ctype == 2
    raw = np.frombuffer(zlib.decompress(idat), np.uint8).reshape(h, 1 + 3 * w)
    assert (raw[:, 0] == 0).all()
    return raw[:, 1:].reshape(h, w, 3)


def test_png_epilogue_roundtrip(tmp_path):
    rng = np.random.default_rng(3)
    rgba = rng.integers(0, 256, size=(17, 23, 4), dtype=np.uint8)
    p = str(tmp_path / "x.png")
    sceneio.save_png(rgba, p)
    assert np.array_equal(_png_decode(p), rgba[:, :, :3])
