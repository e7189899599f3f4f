"""Python host mirror of the reference's public engine API.

`RayTracerEngine` mirrors `RayTracerEngine` (RT/RayTracer.swift:25-228): it is built
from a scene (init(from:data:) :30-49), answers `inspect` (:52-67) and renders one
camera (`render`, :115-131) or all cameras (`render_all`, :70-102), returning
`RenderResult`s with RGBA8 pixels (:186-195) and `RenderStats` (Models/RenderStats.swift).

Every render goes through libmyrt.so's C ABI (include/rtcore.h) into the HIP kernels;
there is no CPU fallback — if the library or a GPU is missing, construction fails.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence

import numpy as np

from . import _abi as A
from .scene import Scene

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libmyrt.so")
_lib = None


class RenderError(RuntimeError):
    """Raised for a negative rtcore status (NSError equivalents, RayTracer.swift:121,141-154)."""

    def __init__(self, code: int, message: str):
        super().__init__(f"[{code}] {message}")
        self.code = code


def load_library() -> C.CDLL:
    """Load the in-tree HIP library.  torch is imported first so the process has ONE HIP
    runtime (libmyrt.so then binds to torch's libamdhip64.so.7 by SONAME)."""
    global _lib
    if _lib is not None:
        return _lib
    path = os.environ.get("MYRT_LIB") or LIB_PATH      # MYRT_LIB: A/B a tuning variant (tools/build_variants.sh)
    if not os.path.exists(path):
        raise RenderError(A.RT_ERR_NO_RENDERER,
                          f"{path} is missing: run `python -c 'import __graft_entry__ as g; g.build()'`")
    try:
        import torch  # noqa: F401  (shared HIP runtime)
    except Exception:  # pragma: no cover - torch is part of the image
        pass
    _lib = A.bind(C.CDLL(path))
    return _lib


def _check(rc: int):
    if rc != A.RT_OK:
        msg = load_library().rt_last_error()
        raise RenderError(rc, msg.decode() if msg else "")


@dataclass
class RenderStats:                       # Models/RenderStats.swift:8-24 (+ ray counts)
    meshes: int
    triangles: int
    spheres: int
    planes: int
    rays: int                            # primary + shadow (the reference always reported 0)
    primary_rays: int
    shadow_rays: int
    secondary_rays: int
    milliseconds: float
    kernel_ms: float
    shadow_rays_traced: int = 0          # shadow rays whose any-hit walk ran (<= shadow_rays)
    rewalked: int = 0                    # closest-hit rays re-walked in reference order (equal-t ties)

    @property
    def rays_traced(self) -> int:
        return self.primary_rays + self.shadow_rays_traced


@dataclass
class CameraSpec:                        # Models/RenderConfig.swift:19-25
    index: int
    id: Optional[str]
    image_name: Optional[str]
    width: int
    height: int


@dataclass
class SceneInfo:                         # Models/RenderConfig.swift:27-33
    cameras: List[CameraSpec]
    meshes: int
    triangles: int
    spheres: int
    planes: int


@dataclass
class RenderResult:                      # Models/RenderResult.swift:10-15 (CGImage -> arrays)
    file_name: Optional[str]
    rgba8: np.ndarray                    # (H, W, 4) uint8, row 0 = top
    rgb: np.ndarray                      # (H, W, 3) float64 — Renderer.render's [Vec3]
    camera: CameraSpec
    stats: RenderStats


@dataclass
class RenderProgress:                    # Models/RenderProgress.swift:8-14
    fraction: float
    message: Optional[str] = None


class RayTracerEngine:
    """Device-resident scene + renderer (one full replica per listed GPU)."""

    def __init__(self, scene: Scene, devices: Optional[Sequence[int]] = None):
        lib = load_library()
        self.scene = scene
        self._packed = scene.to_desc()
        handle = C.c_void_p()
        devs = list(devices) if devices else [0]
        arr = (C.c_int32 * len(devs))(*devs)
        _check(lib.rt_scene_create(self._packed.ptr, arr, len(devs), C.byref(handle)))
        self._h = handle
        self.devices = devs

    @classmethod
    def from_file(cls, path, format: str = "auto", devices: Optional[Sequence[int]] = None) -> "RayTracerEngine":
        """RayTracerEngine.init(from: url) (RayTracer.swift:30-34): JSON or XML scene file."""
        from . import sceneio
        return cls(sceneio.load(path, format), devices)

    @classmethod
    def from_data(cls, data, format: str = "auto", devices: Optional[Sequence[int]] = None,
                  base_dir: Optional[str] = None) -> "RayTracerEngine":
        """RayTracerEngine.init(data:) (RayTracer.swift:35-36)."""
        from . import sceneio
        return cls(sceneio.loads(data, format, base_dir), devices)

    # -- lifecycle
    def close(self):
        if getattr(self, "_h", None):
            load_library().rt_scene_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @property
    def handle(self):
        return self._h

    # -- render options (rt_scene_set_option; defaults are the production settings)
    def set_option(self, name: str, value: int):
        _check(load_library().rt_scene_set_option(self._h, name.encode(), int(value)))

    def set_unsafe_option(self, name: str, value: int):
        """Test hooks (debug_fail_replica, wide_delta_scale) through the non-production
        rt_scene_set_unsafe_option; set_option refuses them."""
        _check(load_library().rt_scene_set_unsafe_option(self._h, name.encode(), int(value)))

    def get_option(self, name: str) -> int:
        v = C.c_int64()
        _check(load_library().rt_scene_get_option(self._h, name.encode(), C.byref(v)))
        return int(v.value)

    # -- introspection (RayTracer.swift:52-67)
    def info(self) -> A.rt_scene_info:
        out = A.rt_scene_info()
        _check(load_library().rt_scene_info_get(self._h, C.byref(out)))
        return out

    def camera_spec(self, index: int) -> CameraSpec:
        c = self.scene.cameras[index]
        return CameraSpec(index, c.id, c.image_name, int(c.image_resolution[0]), int(c.image_resolution[1]))

    def inspect(self) -> SceneInfo:
        i = self.info()
        return SceneInfo([self.camera_spec(k) for k in range(len(self.scene.cameras))],
                         int(i.meshes), int(i.triangles), int(i.spheres), int(i.planes))

    # -- rendering
    def alloc_frame(self, camera_index: int = 0, chunk_first: int = 0, chunk_step: int = 1, rgba: bool = True):
        """Page-locked (rgb, rgba) output arrays for a chunk selection (rt_host_alloc): passed to
        render_rows as out/out_rgba, finished rows are DMA'd into them with no host copy."""
        cam = self.scene.cameras[camera_index]
        W, H = max(1, int(cam.image_resolution[0])), max(1, int(cam.image_resolution[1]))
        rows = load_library().rt_rows_for_chunks(H, chunk_first, chunk_step)
        rgb = pinned_array((rows, W, 3), np.float64)
        return rgb, (pinned_array((rows, W, 4), np.uint8) if rgba else None)

    def render_rows(self, camera_index: int = 0, chunk_first: int = 0, chunk_step: int = 1,
                    want_rgba: bool = True, progress: Optional[Callable[[RenderProgress], bool]] = None,
                    out: Optional[np.ndarray] = None, out_rgba: Optional[np.ndarray] = None):
        """Render the selected 8-row chunks; returns (rgb[rows,W,3] f64, rgba[rows,W,4] u8, RenderStats).
        `out` / `out_rgba`: optional reusable C-contiguous (rows, W, 3) float64 / (rows, W, 4) uint8
        arrays for the results (page-locked ones from alloc_frame take the direct-DMA path)."""
        lib = load_library()
        if not (0 <= camera_index < len(self.scene.cameras)):
            raise RenderError(A.RT_ERR_INVALID_CAMERA, "Invalid camera index")
        cam = self.scene.cameras[camera_index]
        W, H = max(1, int(cam.image_resolution[0])), max(1, int(cam.image_resolution[1]))
        rows = lib.rt_rows_for_chunks(H, chunk_first, chunk_step)
        if out is not None and out.shape == (rows, W, 3) and out.dtype == np.float64 and out.flags.c_contiguous:
            rgb = out
        else:
            rgb = np.empty((rows, W, 3), dtype=np.float64)
        if not want_rgba:
            rgba = None
        elif out_rgba is not None and out_rgba.shape == (rows, W, 4) and out_rgba.dtype == np.uint8 \
                and out_rgba.flags.c_contiguous:
            rgba = out_rgba
        else:
            rgba = np.empty((rows, W, 4), dtype=np.uint8)
        stats = self.render_into(camera_index, chunk_first, chunk_step, rgb, rgba, progress=progress)
        return rgb, rgba, stats

    def render_into(self, camera_index: int = 0, chunk_first: int = 0, chunk_step: int = 1,
                    rgb: Optional[np.ndarray] = None, rgba: Optional[np.ndarray] = None,
                    frame_layout: bool = False,
                    progress: Optional[Callable[[RenderProgress], bool]] = None) -> RenderStats:
        """rt_render_ex into caller-owned arrays (either may be None).  Shapes: the selected
        rows packed, (rows, W, 3|4); with frame_layout the whole frame (H, W, 3|4), the
        selected chunks' rows written at their image rows (RT_RENDER_FRAME_LAYOUT)."""
        lib = load_library()
        if not (0 <= camera_index < len(self.scene.cameras)):
            raise RenderError(A.RT_ERR_INVALID_CAMERA, "Invalid camera index")
        cam = self.scene.cameras[camera_index]
        W, H = max(1, int(cam.image_resolution[0])), max(1, int(cam.image_resolution[1]))
        rows = H if frame_layout else lib.rt_rows_for_chunks(H, chunk_first, chunk_step)
        for a, ch, dt in ((rgb, 3, np.float64), (rgba, 4, np.uint8)):
            if a is not None and (a.shape != (rows, W, ch) or a.dtype != dt or not a.flags.c_contiguous):
                raise ValueError(f"output array must be C-contiguous {dt.__name__}{(rows, W, ch)}, got "
                                 f"{a.dtype}{a.shape}")
        st = A.rt_stats()

        def _cb(user, done, total):
            if progress is None:
                return 1
            return 1 if progress(RenderProgress(done / max(total, 1), f"Row {done}/{total}")) else 0

        cb = A.RT_PROGRESS_FN(_cb) if progress is not None else A.RT_PROGRESS_FN()
        _check(lib.rt_render_ex(self._h, camera_index, chunk_first, chunk_step,
                                rgb.ctypes.data_as(A.c_double_p) if rgb is not None else None,
                                rgba.ctypes.data_as(C.POINTER(C.c_uint8)) if rgba is not None else None,
                                A.RT_RENDER_FRAME_LAYOUT if frame_layout else 0, C.byref(st), cb, None))
        return _stats(st)

    def submit_into(self, camera_index: int = 0, chunk_first: int = 0, chunk_step: int = 1,
                    rgb: Optional[np.ndarray] = None, rgba: Optional[np.ndarray] = None,
                    frame_layout: bool = False, kernel_time: bool = False) -> int:
        """rt_render_submit: enqueue a render into page-locked arrays (pinned_array /
        register_host) and return its ticket at once; the arrays must stay alive until
        wait(ticket).  At most A.RT_MAX_IN_FLIGHT renders may be pending (RenderError -32).
        kernel_time: time the kernels with HIP events (RenderStats.kernel_ms, else 0)."""
        lib = load_library()
        if not (0 <= camera_index < len(self.scene.cameras)):
            raise RenderError(A.RT_ERR_INVALID_CAMERA, "Invalid camera index")
        cam = self.scene.cameras[camera_index]
        W, H = max(1, int(cam.image_resolution[0])), max(1, int(cam.image_resolution[1]))
        rows = H if frame_layout else lib.rt_rows_for_chunks(H, chunk_first, chunk_step)
        for a, ch, dt in ((rgb, 3, np.float64), (rgba, 4, np.uint8)):
            if a is not None and (a.shape != (rows, W, ch) or a.dtype != dt or not a.flags.c_contiguous):
                raise ValueError(f"output array must be C-contiguous {dt.__name__}{(rows, W, ch)}, got "
                                 f"{a.dtype}{a.shape}")
        t = C.c_int64(-1)
        _check(lib.rt_render_submit(self._h, camera_index, chunk_first, chunk_step,
                                    rgb.ctypes.data_as(A.c_double_p) if rgb is not None else None,
                                    rgba.ctypes.data_as(C.POINTER(C.c_uint8)) if rgba is not None else None,
                                    (A.RT_RENDER_FRAME_LAYOUT if frame_layout else 0) |
                                    (A.RT_RENDER_KERNEL_TIME if kernel_time else 0), C.byref(t)))
        return int(t.value)

    def wait(self, ticket: int) -> RenderStats:
        """rt_render_wait: block until the submitted render is complete in its arrays."""
        st = A.rt_stats()
        _check(load_library().rt_render_wait(self._h, ticket, C.byref(st)))
        return _stats(st)

    def frame_pipeline(self, camera_index: int, chunk_first: int, chunk_step: int, rgbas, frame_layout: bool = True):
        """Frames rendered with len(rgbas) renders in flight (rt_render_submit / rt_render_wait),
        frame k into rgbas[k % len(rgbas)], arguments marshalled once.  Returns (submit, wait):
        submit(k) enqueues frame k and returns its ticket; wait(ticket) returns the raw rt_stats."""
        for a in rgbas:                                      # validates every buffer once
            self.wait(self.submit_into(camera_index, chunk_first, chunk_step, None, a, frame_layout))
        lib = load_library()
        h = self._h
        fs, fw = lib.rt_render_submit, lib.rt_render_wait
        ptrs = [a.ctypes.data_as(C.POINTER(C.c_uint8)) for a in rgbas]
        flags = A.RT_RENDER_FRAME_LAYOUT if frame_layout else 0
        t = C.c_int64(-1)
        pt = C.byref(t)
        st = A.rt_stats()
        pst = C.byref(st)
        keep = list(rgbas)

        def submit(k: int) -> int:
            rc = fs(h, camera_index, chunk_first, chunk_step, None, ptrs[k % len(ptrs)], flags, pt)
            if rc != A.RT_OK:
                _check(rc)
            assert keep
            return t.value

        def wait(ticket: int) -> A.rt_stats:
            rc = fw(h, ticket, pst)
            if rc != A.RT_OK:
                _check(rc)
            return st
        return submit, wait

    def frame_renderer(self, camera_index: int = 0, chunk_first: int = 0, chunk_step: int = 1,
                       rgb: Optional[np.ndarray] = None, rgba: Optional[np.ndarray] = None,
                       frame_layout: bool = False) -> Callable[[], A.rt_stats]:
        """render_into with the arguments checked and marshalled once: returns a callable that
        renders one frame into the same arrays (one rt_render_ex call, no progress callback)
        and returns the raw rt_stats.  For frame loops whose per-call Python cost should not
        count as render time (bench.py)."""
        self.render_into(camera_index, chunk_first, chunk_step, rgb, rgba, frame_layout)   # validates
        lib = load_library()
        fn = lib.rt_render_ex
        h = self._h
        prgb = rgb.ctypes.data_as(A.c_double_p) if rgb is not None else None
        prgba = rgba.ctypes.data_as(C.POINTER(C.c_uint8)) if rgba is not None else None
        flags = A.RT_RENDER_FRAME_LAYOUT if frame_layout else 0
        st = A.rt_stats()
        pst = C.byref(st)
        cb = A.RT_PROGRESS_FN()
        keep = (rgb, rgba)

        def one() -> A.rt_stats:
            rc = fn(h, camera_index, chunk_first, chunk_step, prgb, prgba, flags, pst, cb, None)
            if rc != A.RT_OK:
                _check(rc)
            assert keep is not None
            return st
        return one

    def render(self, camera_index: int = 0, progress: Optional[Callable[[RenderProgress], bool]] = None) -> RenderResult:
        """RayTracerEngine.render(format:cameraIndex:progress:) (RayTracer.swift:115-131)."""
        rgb, rgba, stats = self.render_rows(camera_index, 0, 1, True, progress)
        spec = self.camera_spec(camera_index)
        return RenderResult(self.scene.cameras[camera_index].image_name, rgba, rgb, spec, stats)

    def save_png(self, path: str, camera_index: int = 0,
                 progress: Optional[Callable[[RenderProgress], bool]] = None) -> RenderResult:
        """renderCGImage + ImageHelper.savePNG (RayTracer.swift:105-112, Helpers/Image.swift:14-42)."""
        from . import sceneio
        res = self.render(camera_index, progress)
        sceneio.save_png(res.rgba8, path)
        return res

    def render_all(self, progress: Optional[Callable[[RenderProgress], bool]] = None) -> List[RenderResult]:
        """renderAll (RayTracer.swift:70-102)."""
        return [self.render(k, progress) for k in range(len(self.scene.cameras))]

    # -- device-resident path (bench / multi-GPU ranks)
    def render_device(self, out_rgb_ptr: int, camera_index: int = 0, chunk_first: int = 0, chunk_step: int = 1,
                      slot: int = 0, stream: int = 0, out_rgba_ptr: int = 0):
        """Enqueue a render into device buffers on `stream` (no host sync)."""
        _check(load_library().rt_render_device(self._h, slot, camera_index, chunk_first, chunk_step,
                                               C.c_void_p(out_rgb_ptr), C.c_void_p(out_rgba_ptr or None),
                                               C.c_void_p(stream or None)))

    def collect_stats(self, slot: int = 0) -> A.rt_stats:
        st = A.rt_stats()
        _check(load_library().rt_stats_collect(self._h, slot, C.byref(st)))
        return st

    def work_counters(self, out_rgb_ptr: int, camera_index: int = 0, chunk_first: int = 0, chunk_step: int = 1,
                      slot: int = 0, stream: int = 0) -> A.rt_work_counters:
        wc = A.rt_work_counters()
        _check(load_library().rt_render_device_counted(self._h, slot, camera_index, chunk_first, chunk_step,
                                                       C.c_void_p(out_rgb_ptr), C.c_void_p(stream or None),
                                                       C.byref(wc)))
        return wc

    def trace_rays(self, origins, dirs, tmin=None, time=None, slot: int = 0):
        """Closest hits of explicit rays through the render kernels' traversal
        (rt_debug_trace_rays): returns t (+inf = miss), world point, world normal, material."""
        o, d, n, tl, tm = _ray_arrays(origins, dirs, tmin, time)
        t = np.empty(n); p = np.empty((n, 3)); nn = np.empty((n, 3)); mat = np.empty(n, np.int32)
        _check(load_library().rt_debug_trace_rays(
            self._h, slot, n, o.ctypes.data_as(A.c_double_p), d.ctypes.data_as(A.c_double_p),
            tl.ctypes.data_as(A.c_double_p), tm.ctypes.data_as(A.c_double_p), t.ctypes.data_as(A.c_double_p),
            p.ctypes.data_as(A.c_double_p), nn.ctypes.data_as(A.c_double_p), mat.ctypes.data_as(A.c_int32_p)))
        return t, p, nn, mat

    def occluded_rays(self, origins, dirs, tmax, time=None, slot: int = 0):
        """Any-hit of explicit segments (rt_debug_occluded_rays): bool per ray."""
        o, d, n, tl, tm = _ray_arrays(origins, dirs, tmax, time)
        out = np.empty(n, np.uint8)
        _check(load_library().rt_debug_occluded_rays(
            self._h, slot, n, o.ctypes.data_as(A.c_double_p), d.ctypes.data_as(A.c_double_p),
            tl.ctypes.data_as(A.c_double_p), tm.ctypes.data_as(A.c_double_p), out.ctypes.data_as(C.POINTER(C.c_uint8))))
        return out.astype(bool)

    def bvh_hash(self, instance: int) -> int:
        return int(load_library().rt_debug_bvh_hash(self._h, instance))


def _stats(st: A.rt_stats) -> RenderStats:
    return RenderStats(int(st.meshes), int(st.triangles), int(st.spheres), int(st.planes),
                       int(st.primary_rays + st.shadow_rays), int(st.primary_rays), int(st.shadow_rays),
                       int(st.secondary_rays), float(st.milliseconds), float(st.kernel_ms),
                       int(st.shadow_rays_traced), int(st.rewalked))


def register_host(arr: np.ndarray):
    """Page-lock an existing host array (rt_host_register; e.g. a framebuffer in shared memory
    that several processes fill).  Call unregister_host(arr) before the memory goes away."""
    _check(load_library().rt_host_register(C.c_void_p(arr.ctypes.data), arr.nbytes))


def unregister_host(arr: np.ndarray):
    _check(load_library().rt_host_unregister(C.c_void_p(arr.ctypes.data)))


def _ray_arrays(origins, dirs, tlim, time):
    o = np.ascontiguousarray(origins, dtype=np.float64).reshape(-1, 3)
    d = np.ascontiguousarray(dirs, dtype=np.float64).reshape(-1, 3)
    n = o.shape[0]
    if d.shape[0] != n:
        raise ValueError("origins and dirs differ in length")
    tl = np.zeros(n) if tlim is None else np.ascontiguousarray(np.broadcast_to(tlim, (n,)), dtype=np.float64)
    tm = np.zeros(n) if time is None else np.ascontiguousarray(np.broadcast_to(time, (n,)), dtype=np.float64)
    return o, d, n, tl, tm


def pinned_array(shape, dtype) -> np.ndarray:
    """numpy array over page-locked host memory (rt_host_alloc); freed with the array."""
    import weakref
    lib = load_library()
    dt = np.dtype(dtype)
    nbytes = int(np.prod(shape)) * dt.itemsize
    if nbytes == 0:
        return np.empty(shape, dt)
    p = C.c_void_p()
    _check(lib.rt_host_alloc(nbytes, C.byref(p)))
    buf = (C.c_uint8 * nbytes).from_address(p.value)
    arr = np.frombuffer(buf, dtype=dt).reshape(shape)
    weakref.finalize(buf, lib.rt_host_free, C.c_void_p(p.value))
    return arr


def rows_for_chunks(height: int, chunk_first: int, chunk_step: int) -> int:
    """Pure-Python restatement of rt_rows_for_chunks (used by host-side sharding logic)."""
    height = max(1, height)
    n = (height + 7) // 8
    return sum(min(8, height - 8 * c) for c in range(chunk_first, n, chunk_step)) if chunk_step >= 1 else 0


def ply_load(path: str):
    """PLYLoader.load (PLYReader.swift:54-210) through the product's C ABI.
    Returns dict(positions (V,3) f64, normals (V,3) f64 | None, texcoords (V,2) f32 | None, indices (T,3) i32)."""
    lib = load_library()
    m = A.rt_ply_mesh()
    _check(lib.rt_ply_load(path.encode(), C.byref(m)))
    try:
        pos = np.ctypeslib.as_array(m.positions, shape=(m.num_positions * 3,)).reshape(-1, 3).copy() \
            if m.num_positions else np.zeros((0, 3))
        nrm = np.ctypeslib.as_array(m.normals, shape=(m.num_normals * 3,)).reshape(-1, 3).copy() \
            if m.num_normals else None
        uv = np.ctypeslib.as_array(m.texcoords, shape=(m.num_texcoords * 2,)).reshape(-1, 2).copy() \
            if m.num_texcoords else None
        idx = np.ctypeslib.as_array(m.indices, shape=(m.num_indices,)).copy() if m.num_indices else \
            np.zeros((0,), np.int32)
    finally:
        lib.rt_ply_free(C.byref(m))
    return {"positions": pos, "normals": nrm, "texcoords": uv, "indices": idx.reshape(-1, 3) if idx.size % 3 == 0 else idx}
