"""The C-ABI scene-file decoder (rt_scene_file_*, myraytracer_amd/csrc/sceneio.cpp) for compiled
hosts: RayTracerEngine.init(from:data:) -> SceneLoader.load (RayTracer.swift:30-49).

It must decode every document exactly like the Python mirror (myraytracer_amd/sceneio.py, whose
conventions tests/test_sceneio.py pins to ParsingKit's surviving helpers): the descriptor it
hands to rt_scene_create is compared field by field with the one PackedScene builds from the
Python decode.  Transforms are compared to 1e-15 (numpy's matmul may round differently from the
plain dot products of the C++ composition); everything else must be identical.  CPU only.
"""
import ctypes as C
import json
import math
import os
import shutil

import numpy as np
import pytest

import myraytracer_amd as M
from myraytracer_amd import _abi as A
from myraytracer_amd import scenes, sceneio

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "scenes")


def _v(v):
    return (v.x, v.y, v.z)


def _canon(d):
    """rt_scene_desc -> comparable tuples (arrays copied out of the C memory)."""
    out = {"background": _v(d.background_color), "ambient": _v(d.ambient_light),
           "eps": (d.shadow_ray_epsilon, d.intersection_test_epsilon), "depth": d.max_recursion_depth}
    out["materials"] = [(_v(m.ambient), _v(m.diffuse), _v(m.specular), _v(m.mirror), _v(m.absorption), m.phong,
                         m.ior, m.absorption_index, m.roughness, m.type) for m in d.materials[:d.num_materials]]
    out["points"] = [(_v(l.position), _v(l.intensity)) for l in d.point_lights[:d.num_point_lights]]
    out["areas"] = [(_v(l.position), _v(l.normal), _v(l.radiance), l.size) for l in d.area_lights[:d.num_area_lights]]
    cams = []
    for c in d.cameras[:d.num_cameras]:
        cams.append((c.type, c.width, c.height, c.num_samples, _v(c.position), _v(c.gaze_point), _v(c.gaze),
                     _v(c.up), "nan" if math.isnan(c.fovy) else c.fovy, c.near_distance, tuple(c.near_plane),
                     c.aperture_size, c.focus_distance))
    out["cameras"] = cams
    objs, xf = [], []
    for o in d.objects[:d.num_objects]:
        pos = tuple(o.positions[:3 * o.num_positions]) if o.positions else ()
        idx = tuple(o.indices[:o.num_indices]) if o.indices else ()
        nrm = tuple(o.normals[:3 * o.num_normals]) if o.normals else ()
        objs.append((o.kind, o.material_id, o.smooth, o.id, o.base_mesh_id, o.indices_one_based, _v(o.motion_blur),
                     o.ply_path.decode() if o.ply_path else None, pos, idx, nrm,
                     tuple(_v(x) for x in o.v), _v(o.center), _v(o.normal), o.radius))
        xf.append(list(o.transform))
    out["objects"] = objs
    return out, np.array(xf).reshape(-1, 16) if xf else np.zeros((0, 16))


class NativeFile:
    def __init__(self, path=None, data=None, fmt=A.RT_SCENE_FORMAT_AUTO, base_dir=None):
        self.lib = M.load_library()
        self.h = C.c_void_p()
        if path is not None:
            rc = self.lib.rt_scene_file_load(path.encode(), fmt, C.byref(self.h))
        else:
            b = data.encode() if isinstance(data, str) else data
            rc = self.lib.rt_scene_file_parse(b, len(b), fmt, base_dir.encode() if base_dir else None, C.byref(self.h))
        self.rc = rc
        self.err = self.lib.rt_scene_file_last_error().decode() if rc else ""

    def desc(self):
        return self.lib.rt_scene_file_desc(self.h).contents

    def close(self):
        if self.h:
            self.lib.rt_scene_file_destroy(self.h)
            self.h = C.c_void_p()


def _assert_same(native_desc, scene):
    a, xa = _canon(native_desc)
    b, xb = _canon(scene.to_desc().desc)
    assert a == b
    np.testing.assert_allclose(xa, xb, rtol=0, atol=1e-15)


@pytest.fixture(scope="module")
def mixed_dir(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("mixed_native"))
    for f in ("mixed.json", "mixed.xml"):
        shutil.copy(os.path.join(GOLDEN, f), d)
    V, F = scenes.icosphere(1)
    scenes.write_ply(os.path.join(d, "ico.ply"), V * 0.7, F)
    return d


@pytest.mark.parametrize("name", ["mixed.json", "mixed.xml"])
def test_golden_scene_files_decode_like_the_python_mirror(mixed_dir, name):
    path = os.path.join(mixed_dir, name)
    nf = NativeFile(path=path)
    assert nf.rc == 0, nf.err
    py = sceneio.load(path)
    _assert_same(nf.desc(), py)
    names = [nf.lib.rt_scene_file_image_name(nf.h, k) for k in range(2)]
    assert [n.decode() for n in names] == [c.image_name for c in py.cameras]
    assert nf.lib.rt_scene_file_image_name(nf.h, 5) is None
    nf.close()


def test_in_memory_data_auto_detection_and_base_dir(mixed_dir):
    with open(os.path.join(mixed_dir, "mixed.xml"), "rb") as f:
        data = f.read()
    nf = NativeFile(data=b"\xef\xbb\xbf  " + data, base_dir=mixed_dir)   # BOM + whitespace, auto format
    assert nf.rc == 0, nf.err
    _assert_same(nf.desc(), sceneio.loads(data, base_dir=mixed_dir))
    nf.close()


def test_flexible_scalars_vectors_and_one_or_many():
    doc = {"Scene": {
        "MaxRecursionDepth": 3.0, "BackgroundColor": [1, "2", 3.5], "ShadowRayEpsilon": " 0.01 ",
        "Cameras": {"Camera": [{"Position": [0, 0, 0], "Gaze": "0 0 -1", "Up": "0 1 0",
                                "ImageResolution": "8 8", "NumSamples": " 4", "_type": "LookAt", "FovY": 50,
                                "GazePoint": "0 0 -1"},
                               {"ImageResolution": [16, 9.0], "NearPlane": "-1 1 -0.5 0.5 9"}]},
        "Lights": {"PointLight": [{"Position": "1 2 3", "Intensity": [4, 5, 6]}],
                   "AreaLight": {"Position": "0 4 0", "Normal": "0 -1 0", "Radiance": "9 9 9", "Size": "0.5"}},
        "Materials": {"Material": [{"_id": 1, "DiffuseReflectance": {"_data": "1 1 1"}},
                                   {"_id": "2", "_type": "dielectric", "RefractionIndex": 1.5,
                                    "AbsorptionCoefficient": "0.1 0.2 0.3"}]},
        "VertexData": "0 0 0 1 0 0 0 1 0 \n 1 1 0",
        "Transformations": {"Rotation": {"_id": 2, "_data": "90 1 1 0"},
                            "Composite": {"_id": "1", "_data": [1, 0, 0, 1, 0, 1, 0, 2, 0, 0, 1, 3, 0, 0, 0, 1]}},
        "Objects": {"Mesh": [{"_id": 1, "Material": 1, "Faces": "1 2 3", "_shadingMode": "smooth",
                              "Transformations": "r2 c1", "MotionBlur": "0 0.1 0"},
                             {"_id": "sky", "Material": "x", "Faces": {"_vertexOffset": "1", "_data": "0 1 2"}}],
                    "MeshInstance": [{"_id": 5, "_baseMeshId": 1, "Transformations": "c1"},
                                     {"_id": 6, "_baseMeshId": "sky", "Material": "2",
                                      "_resetTransform": "true", "Transformations": "r2"}],
                    "Triangle": {"Indices": "1 2 4", "Material": 2},
                    "Sphere": {"Center": 4, "Radius": "0.25"},
                    "Plane": {"Point": "1", "Normal": "0 1 0"}}}}
    text = json.dumps(doc)
    nf = NativeFile(data=text, base_dir="/tmp")
    assert nf.rc == 0, nf.err
    _assert_same(nf.desc(), sceneio.loads(text, base_dir="/tmp"))
    nf.close()


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
def test_decode_errors_match(doc, msg):
    with pytest.raises(sceneio.SceneLoadError, match=msg):
        sceneio.decode(doc)
    nf = NativeFile(data=json.dumps(doc))
    assert nf.rc == A.RT_ERR_SCENE_FILE and msg in nf.err, nf.err


@pytest.mark.parametrize("data,fmt", [("Scene: yaml", A.RT_SCENE_FORMAT_AUTO), ("{not json", A.RT_SCENE_FORMAT_JSON),
                                      ("<Scene><Cameras></Scene>", A.RT_SCENE_FORMAT_XML),
                                      ('{"Scene": {}} x', A.RT_SCENE_FORMAT_JSON)])
def test_bad_documents(data, fmt):
    nf = NativeFile(data=data, fmt=fmt)
    assert nf.rc == A.RT_ERR_SCENE_FILE and nf.err


@pytest.mark.parametrize("data,fmt", [("[" * 300000 + "]" * 300000, A.RT_SCENE_FORMAT_JSON),
                                      ('{"a":' * 200000 + "1" + "}" * 200000, A.RT_SCENE_FORMAT_JSON),
                                      ("<a>" * 200000 + "</a>" * 200000, A.RT_SCENE_FORMAT_XML)])
def test_deep_nesting_fails_instead_of_overflowing_the_stack(data, fmt):
    """The recursive decoders stop at 512 levels with RT_ERR_SCENE_FILE (a few hundred
    thousand levels used to overflow the host stack and crash the process)."""
    nf = NativeFile(data=data, fmt=fmt)
    assert nf.rc == A.RT_ERR_SCENE_FILE and "nesting too deep" in nf.err, nf.err
    ok = NativeFile(data='{"Scene": {"x": ' + "[" * 500 + "]" * 500 + "}}", fmt=A.RT_SCENE_FORMAT_JSON)
    assert ok.rc == 0, ok.err
    ok.close()


def test_missing_file():
    nf = NativeFile(path="/nonexistent/scene.json")
    assert nf.rc == A.RT_ERR_SCENE_FILE and "cannot open" in nf.err


def test_instance_of_missing_base_is_dropped():
    doc = {"Scene": {"VertexData": "0 0 0 1 0 0 0 1 0",
                     "Objects": {"MeshInstance": {"_id": "2", "_baseMeshId": "9"},
                                 "Mesh": {"_id": "1", "Faces": "1 2 3"}}}}
    nf = NativeFile(data=json.dumps(doc))
    assert nf.rc == 0 and nf.desc().num_objects == 1
    nf.close()


def test_xml_entities_comments_cdata_and_attributes():
    xml = """<?xml version="1.0"?>
<!-- a comment -->
<Scene>
  <BackgroundColor><![CDATA[1 2 3]]></BackgroundColor>
  <MaxRecursionDepth> 2 </MaxRecursionDepth>
  <Cameras><Camera id='c&amp;1' type="lookAt"><ImageResolution>4 &#50;</ImageResolution>
    <GazePoint>0 0 -1</GazePoint><!-- inner --></Camera></Cameras>
  <VertexData>0 0 0 1 0 0 0 1 0</VertexData>
  <Objects><Mesh id="1"><Faces>1 2 3</Faces><Material>1</Material></Mesh></Objects>
</Scene>"""
    nf = NativeFile(data=xml)
    assert nf.rc == 0, nf.err
    _assert_same(nf.desc(), sceneio.loads(xml))
    assert nf.desc().cameras[0].height == 2
    nf.close()


def test_loaded_c1_hashes_equal_the_built_scene():
    """The C1 scene as a file, decoded natively, builds the same BVH (host build, no device)."""
    doc = {"Scene": {
        "MaxRecursionDepth": "6", "BackgroundColor": "10 20 30",
        "Cameras": {"Camera": {"_id": "1", "_type": "lookAt", "Position": "0 0 0", "GazePoint": "0 0 -1",
                               "Up": "0 1 0", "FovY": "60", "NearDistance": "1", "ImageResolution": "64 48"}},
        "Lights": {"AmbientLight": "25 25 25", "PointLight": {"Position": "2 2 0", "Intensity": "3e3 3e3 3e3"}},
        "Materials": {"Material": {"_id": "1", "AmbientReflectance": "1 1 1", "DiffuseReflectance": "0.8 0.5 0.3",
                                   "SpecularReflectance": "0.5 0.5 0.5", "PhongExponent": "32"}},
        "VertexData": "-1 -1 -3 1 -1 -3 0 1 -3",
        "Objects": {"Mesh": {"_id": "1", "_shadingMode": "flat", "Material": "1", "Faces": "1 2 3"}}}}
    nf = NativeFile(data=json.dumps(doc))
    assert nf.rc == 0
    lib = M.load_library()
    hs = (C.c_uint64 * 8)()
    n = C.c_int32()
    info = A.rt_scene_info()
    assert lib.rt_debug_host_build(C.byref(nf.desc()), hs, 8, C.byref(n), C.byref(info)) == 0
    hs2 = (C.c_uint64 * 8)()
    pk = scenes.scene_c1(64, 48).to_desc()
    assert lib.rt_debug_host_build(pk.ptr, hs2, 8, C.byref(n), C.byref(info)) == 0
    assert list(hs)[:2] == list(hs2)[:2]
    nf.close()
