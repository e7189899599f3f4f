"""oracle — TEST INFRASTRUCTURE ONLY.

ctypes wrapper around liboracle.so, the C++ CPU restatement of the reference's
per-pixel trace path (oracle/rt_oracle.cpp), and around oracle/_ref/libcply_ref.so,
the reference's own CPly compiled here (oracle/build_ref.sh).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
package; the product (myraytracer_amd) never does.

Render parity with the Swift reference binary is UNPINNED (the Swift path cannot be
built or run: SURVEY.md §0, §8c); the restatement is pinned by known-answer tests
(tests/test_oracle_kat.py).  PLY parsing is pinned by the reference's own CPly.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")
REF_CPLY = os.path.join(HERE, "_ref", "libcply_ref.so")


class oracle_stats(C.Structure):
    _fields_ = [("primary_rays", C.c_int64), ("shadow_rays", C.c_int64), ("secondary_rays", C.c_int64),
                ("node_visits", C.c_int64), ("node_fetches", C.c_int64), ("tri_tests", C.c_int64),
                ("smooth_hits", C.c_int64), ("pixels", C.c_int64), ("milliseconds", C.c_double),
                ("threads", C.c_int32), ("shadow_rays_used", C.c_int64)]


_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            raise RuntimeError(f"{LIB} missing; build with __graft_entry__.build()")
        L = C.CDLL(LIB)
        L.oracle_scene_create.argtypes = [C.c_void_p, C.POINTER(C.c_void_p)]
        L.oracle_scene_create.restype = C.c_int32
        L.oracle_scene_destroy.argtypes = [C.c_void_p]
        L.oracle_scene_destroy.restype = None
        L.oracle_render.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                                    C.POINTER(C.c_double), C.POINTER(C.c_uint8), C.POINTER(oracle_stats)]
        L.oracle_render.restype = C.c_int32
        L.oracle_last_error.restype = C.c_char_p
        L.oracle_bvh_hash.argtypes = [C.c_void_p, C.c_int32]
        L.oracle_bvh_hash.restype = C.c_uint64
        L.oracle_num_instances.argtypes = [C.c_void_p]
        L.oracle_num_instances.restype = C.c_int32
        L.oracle_pcg32_stream.argtypes = [C.c_uint64, C.c_int32, C.POINTER(C.c_uint32)]
        L.oracle_pcg32_stream.restype = None
        d3 = C.POINTER(C.c_double)
        L.oracle_hit_aabb.argtypes = [d3, d3, d3, d3, C.c_double]
        L.oracle_hit_aabb.restype = C.c_double
        L.oracle_intersect_triangle.argtypes = [d3, d3, d3, d3, d3, C.c_double, C.c_double, d3, d3]
        L.oracle_intersect_triangle.restype = C.c_double
        i32 = C.POINTER(C.c_int32)
        L.oracle_trace_rays.argtypes = [C.c_void_p, C.c_int32, d3, d3, d3, d3, d3, d3, d3, i32]
        L.oracle_trace_rays.restype = C.c_int32
        L.oracle_occluded_rays.argtypes = [C.c_void_p, C.c_int32, d3, d3, d3, d3, C.POINTER(C.c_uint8)]
        L.oracle_occluded_rays.restype = C.c_int32
        _lib = L
    return _lib


def _dp(a):
    return np.ascontiguousarray(a, dtype=np.float64).ctypes.data_as(C.POINTER(C.c_double))


class OracleScene:
    """CPU restatement of RTContext + Renderer for one scene (scene.to_desc() input)."""

    def __init__(self, scene):
        self._packed = scene.to_desc()
        h = C.c_void_p()
        rc = lib().oracle_scene_create(C.cast(self._packed.ptr, C.c_void_p), C.byref(h))
        if rc != 0:
            raise RuntimeError(f"oracle_scene_create: {rc} {lib().oracle_last_error().decode()}")
        self._h = h
        self.scene = scene

    def close(self):
        if getattr(self, "_h", None):
            lib().oracle_scene_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def render(self, camera_index=0, chunk_first=0, chunk_step=1, threads=0, rgba=False):
        cam = self.scene.cameras[camera_index]
        W, H = max(1, cam.image_resolution[0]), max(1, cam.image_resolution[1])
        nchunks = (H + 7) // 8
        rows = sum(min(8, H - 8 * c) for c in range(chunk_first, nchunks, chunk_step))
        out = np.empty((rows, W, 3), np.float64)
        o8 = np.empty((rows, W, 4), np.uint8) if rgba else None
        st = oracle_stats()
        rc = lib().oracle_render(self._h, camera_index, chunk_first, chunk_step, threads,
                                 out.ctypes.data_as(C.POINTER(C.c_double)),
                                 o8.ctypes.data_as(C.POINTER(C.c_uint8)) if rgba else None, C.byref(st))
        if rc != 0:
            raise RuntimeError(f"oracle_render: {rc} {lib().oracle_last_error().decode()}")
        return (out, o8, st) if rgba else (out, st)

    def bvh_hash(self, instance):
        return int(lib().oracle_bvh_hash(self._h, instance))

    def num_instances(self):
        return int(lib().oracle_num_instances(self._h))

    @staticmethod
    def _rays(origins, dirs, tlim, time):
        o = np.ascontiguousarray(origins, dtype=np.float64).reshape(-1, 3)
        d = np.ascontiguousarray(dirs, dtype=np.float64).reshape(-1, 3)
        n = o.shape[0]
        tl = np.zeros(n) if tlim is None else np.ascontiguousarray(np.broadcast_to(tlim, (n,)), dtype=np.float64)
        tm = np.zeros(n) if time is None else np.ascontiguousarray(np.broadcast_to(time, (n,)), dtype=np.float64)
        return o, d, n, tl, tm

    def trace_rays(self, origins, dirs, tmin=None, time=None):
        """intersectTLAS on explicit rays: (t, world point, world normal, material)."""
        o, d, n, tl, tm = self._rays(origins, dirs, tmin, time)
        t = np.empty(n); p = np.empty((n, 3)); nn = np.empty((n, 3)); mat = np.empty(n, np.int32)
        dp = lambda a: a.ctypes.data_as(C.POINTER(C.c_double))
        lib().oracle_trace_rays(self._h, n, dp(o), dp(d), dp(tl), dp(tm), dp(t), dp(p), dp(nn),
                                mat.ctypes.data_as(C.POINTER(C.c_int32)))
        return t, p, nn, mat

    def occluded_rays(self, origins, dirs, tmax, time=None):
        """occludedTLAS on explicit segments: bool per ray."""
        o, d, n, tl, tm = self._rays(origins, dirs, tmax, time)
        out = np.empty(n, np.uint8)
        dp = lambda a: a.ctypes.data_as(C.POINTER(C.c_double))
        lib().oracle_occluded_rays(self._h, n, dp(o), dp(d), dp(tl), dp(tm), out.ctypes.data_as(C.POINTER(C.c_uint8)))
        return out.astype(bool)


def pcg32_stream(seed: int, n: int):
    out = (C.c_uint32 * n)()
    lib().oracle_pcg32_stream(seed, n, out)
    return list(out)


def hit_aabb(bmin, bmax, origin, direction, eps):
    return lib().oracle_hit_aabb(_dp(bmin), _dp(bmax), _dp(origin), _dp(direction), eps)


def intersect_triangle(v0, v1, v2, origin, direction, tmin=0.0, eps=1e-6):
    p = np.zeros(3)
    n = np.zeros(3)
    t = lib().oracle_intersect_triangle(_dp(v0), _dp(v1), _dp(v2), _dp(origin), _dp(direction), tmin, eps,
                                        p.ctypes.data_as(C.POINTER(C.c_double)),
                                        n.ctypes.data_as(C.POINTER(C.c_double)))
    return t, p, n


# ---------------------------------------------------------------- reference CPly
class RefCPly:
    """Drives the reference's own compiled CPly exactly like PLYLoader.load
    (Sources/RayTracer/Helpers/PLYReader.swift:54-210)."""

    def __init__(self, path=REF_CPLY):
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing (oracle/build_ref.sh needs /root/reference)")
        L = C.CDLL(path)
        vp, u32p = C.c_void_p, C.POINTER(C.c_uint32)
        sig = {
            "ply_reader_create": ([C.c_char_p], vp), "ply_reader_destroy": ([vp], None),
            "ply_reader_valid": ([vp], C.c_bool), "ply_reader_has_element": ([vp], C.c_bool),
            "ply_reader_load_element": ([vp], C.c_bool), "ply_reader_next_element": ([vp], None),
            "ply_reader_element_is": ([vp, C.c_char_p], C.c_bool), "ply_reader_num_rows": ([vp], C.c_uint32),
            "ply_reader_find_pos": ([vp, u32p], C.c_bool), "ply_reader_find_normals": ([vp, u32p], C.c_bool),
            "ply_reader_find_texcoord": ([vp, u32p], C.c_bool), "ply_reader_find_indices": ([vp, u32p], C.c_bool),
            "ply_reader_extract_properties": ([vp, u32p, C.c_uint32, C.c_int, vp], C.c_bool),
            "ply_reader_sum_of_list_counts": ([vp, C.c_uint32], C.c_uint32),
            "ply_reader_extract_list_property": ([vp, C.c_uint32, C.c_int, vp], C.c_bool),
            "ply_reader_requires_triangulation": ([vp, C.c_uint32], C.c_bool),
            "ply_reader_num_triangles": ([vp, C.c_uint32], C.c_uint32),
            "ply_reader_extract_triangles": ([vp, C.c_uint32, C.POINTER(C.c_float), C.c_uint32, C.c_int, vp], C.c_bool),
        }
        for name, (args, res) in sig.items():
            f = getattr(L, name)
            f.argtypes, f.restype = args, res
        self.L = L

    def load(self, path: str):
        """Returns dict like PlyMesh, or raises ValueError(<PlyError case>)."""
        L = self.L
        r = L.ply_reader_create(path.encode())
        if not r:
            raise ValueError("fileOpenFailed")
        try:
            if not L.ply_reader_valid(r):
                raise ValueError("corrupted")
            props = (C.c_uint32 * 3)()
            pos, nrm, uv, idx = None, None, None, None
            got_v = got_f = False
            while L.ply_reader_has_element(r):
                if L.ply_reader_element_is(r, b"vertex") and L.ply_reader_load_element(r) and \
                        L.ply_reader_find_pos(r, props):
                    n = L.ply_reader_num_rows(r)
                    buf = np.zeros(n * 3, np.float32)
                    L.ply_reader_extract_properties(r, props, 3, 6, buf.ctypes.data_as(C.c_void_p))
                    pos = buf.astype(np.float64).reshape(-1, 3)
                    if L.ply_reader_find_normals(r, props):
                        nb = np.zeros(n * 3, np.float32)
                        L.ply_reader_extract_properties(r, props, 3, 6, nb.ctypes.data_as(C.c_void_p))
                        v = nb.astype(np.float64).reshape(-1, 3)
                        s = 1.0 / np.sqrt((v[:, 0] * v[:, 0] + v[:, 1] * v[:, 1]) + v[:, 2] * v[:, 2])
                        nrm = v * s[:, None]
                    if L.ply_reader_find_texcoord(r, props):
                        tb = np.zeros(n * 2, np.float32)
                        L.ply_reader_extract_properties(r, props, 2, 6, tb.ctypes.data_as(C.c_void_p))
                        uv = tb.reshape(-1, 2)
                    got_v = True
                elif L.ply_reader_element_is(r, b"face") and L.ply_reader_load_element(r) and \
                        L.ply_reader_find_indices(r, props):
                    ip = props[0]
                    need = L.ply_reader_requires_triangulation(r, ip)
                    if need and not got_v:
                        raise ValueError("triangulationNeedsVerts")
                    if need:
                        posF = np.ascontiguousarray(pos.reshape(-1), dtype=np.float32)
                        tc = L.ply_reader_num_triangles(r, ip)
                        # slack past the end: miniply's n>4 path can write beyond triCount*3
                        tri = np.zeros(tc * 3 + 64, np.int32)
                        L.ply_reader_extract_triangles(r, ip, posF.ctypes.data_as(C.POINTER(C.c_float)),
                                                       len(pos), 4, tri.ctypes.data_as(C.c_void_p))
                        idx = tri[:tc * 3].copy()
                    else:
                        tot = L.ply_reader_sum_of_list_counts(r, ip)
                        raw = np.zeros(tot, np.int32)
                        L.ply_reader_extract_list_property(r, ip, 4, raw.ctypes.data_as(C.c_void_p))
                        idx = raw
                    got_f = True
                L.ply_reader_next_element(r)
            if not got_v:
                raise ValueError("vertexDataMissing")
            if not got_f:
                raise ValueError("faceDataMissing")
            return {"positions": pos, "normals": nrm, "texcoords": uv, "indices": idx}
        finally:
            L.ply_reader_destroy(r)
