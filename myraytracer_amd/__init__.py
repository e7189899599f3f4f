"""myraytracer_amd — MI355X-native (gfx950) renderer core with the behaviour of
erndmrcn/MyRayTracer's per-pixel trace path.

The hot path (primary rays, TLAS/BLAS traversal, Moeller-Trumbore, Whitted shading
with shadow rays and mirror bounces) runs in hand-written FP64 HIP kernels in
libmyrt.so (C ABI: include/rtcore.h).  PLY parsing, scene flattening and the SAH BVH
build are host C++ in the same library.  This package is the Python host mirror of
the reference's `RayTracerEngine` API.
"""
from .scene import (AreaLight, Camera, Material, Mesh, MeshInstance, Plane, PointLight, Scene, Sphere,  # noqa: F401
                    Triangle, translation)
from .sceneio import SceneLoadError, load as load_scene, loads as loads_scene, save_png  # noqa: F401
from .engine import (CameraSpec, RayTracerEngine, RenderError, RenderProgress, RenderResult,  # noqa: F401
                     RenderStats, SceneInfo, load_library, pinned_array, ply_load, register_host,
                     rows_for_chunks, unregister_host)

__all__ = ["RayTracerEngine", "Scene", "Camera", "Material", "Mesh", "MeshInstance", "Triangle", "Sphere", "Plane",
           "PointLight", "AreaLight", "RenderResult", "RenderStats", "RenderProgress", "RenderError", "SceneInfo",
           "CameraSpec", "load_library", "ply_load", "rows_for_chunks", "translation", "load_scene", "loads_scene",
           "save_png", "SceneLoadError", "pinned_array", "register_host", "unregister_host"]
