"""ctypes mirror of include/rtcore.h (the C ABI of libmyrt.so).

Field order and types follow the header exactly; `tests/test_abi.py` checks the
struct sizes against the compiled library.
"""
from __future__ import annotations

import ctypes as C

c_double_p = C.POINTER(C.c_double)
c_int32_p = C.POINTER(C.c_int32)


class rt_vec3(C.Structure):
    _fields_ = [("x", C.c_double), ("y", C.c_double), ("z", C.c_double)]


class rt_material(C.Structure):
    _fields_ = [("ambient", rt_vec3), ("diffuse", rt_vec3), ("specular", rt_vec3), ("mirror", rt_vec3),
                ("absorption", rt_vec3), ("phong", C.c_double), ("ior", C.c_double),
                ("absorption_index", C.c_double), ("roughness", C.c_double), ("type", C.c_int32),
                ("_pad", C.c_int32)]


class rt_point_light(C.Structure):
    _fields_ = [("position", rt_vec3), ("intensity", rt_vec3)]


class rt_area_light(C.Structure):
    _fields_ = [("position", rt_vec3), ("normal", rt_vec3), ("radiance", rt_vec3), ("size", C.c_double)]


class rt_camera(C.Structure):
    _fields_ = [("type", C.c_int32), ("width", C.c_int32), ("height", C.c_int32), ("num_samples", C.c_int32),
                ("position", rt_vec3), ("gaze_point", rt_vec3), ("gaze", rt_vec3), ("up", rt_vec3),
                ("fovy", C.c_double), ("near_distance", C.c_double), ("near_plane", C.c_double * 4),
                ("aperture_size", C.c_double), ("focus_distance", C.c_double)]


class rt_object(C.Structure):
    _fields_ = [("kind", C.c_int32), ("material_id", C.c_int32), ("smooth", C.c_int32), ("id", C.c_int32),
                ("base_mesh_id", C.c_int32), ("indices_one_based", C.c_int32),
                ("transform", C.c_double * 16), ("motion_blur", rt_vec3),
                ("ply_path", C.c_char_p),
                ("positions", c_double_p), ("num_positions", C.c_int64),
                ("indices", c_int32_p), ("num_indices", C.c_int64),
                ("normals", c_double_p),
                ("v", rt_vec3 * 3), ("center", rt_vec3), ("normal", rt_vec3), ("radius", C.c_double),
                ("num_normals", C.c_int64)]


class rt_scene_desc(C.Structure):
    _fields_ = [("background_color", rt_vec3), ("ambient_light", rt_vec3),
                ("shadow_ray_epsilon", C.c_double), ("intersection_test_epsilon", C.c_double),
                ("max_recursion_depth", C.c_int32), ("num_materials", C.c_int32),
                ("materials", C.POINTER(rt_material)),
                ("num_point_lights", C.c_int32), ("num_area_lights", C.c_int32),
                ("point_lights", C.POINTER(rt_point_light)), ("area_lights", C.POINTER(rt_area_light)),
                ("num_objects", C.c_int32), ("num_cameras", C.c_int32),
                ("objects", C.POINTER(rt_object)), ("cameras", C.POINTER(rt_camera))]


RT_RENDER_FRAME_LAYOUT = 1
RT_RENDER_KERNEL_TIME = 2
RT_SCENE_FORMAT_AUTO, RT_SCENE_FORMAT_JSON, RT_SCENE_FORMAT_XML = 0, 1, 2


class rt_stats(C.Structure):
    _fields_ = [("meshes", C.c_int64), ("triangles", C.c_int64), ("spheres", C.c_int64), ("planes", C.c_int64),
                ("primary_rays", C.c_int64), ("shadow_rays", C.c_int64), ("secondary_rays", C.c_int64),
                ("milliseconds", C.c_double), ("kernel_ms", C.c_double),
                ("shadow_rays_traced", C.c_int64), ("rewalked", C.c_int64)]


class rt_scene_info(C.Structure):
    _fields_ = [("meshes", C.c_int64), ("triangles", C.c_int64), ("spheres", C.c_int64), ("planes", C.c_int64),
                ("instances", C.c_int64), ("blas_nodes", C.c_int64), ("tlas_nodes", C.c_int64),
                ("max_depth", C.c_int64), ("build_ms", C.c_double), ("upload_ms", C.c_double),
                ("device_bytes", C.c_int64), ("scratch_bytes", C.c_int64)]


class rt_work_counters(C.Structure):
    _fields_ = [("records_fetched", C.c_int64), ("tri_tests", C.c_int64), ("normal_fetches", C.c_int64),
                ("instance_entries", C.c_int64), ("pixels", C.c_int64),
                ("ref_node_fetches", C.c_int64), ("ref_tri_tests", C.c_int64),
                ("ref_smooth_hits", C.c_int64), ("ref_pixels", C.c_int64),
                ("lane_steps_closest", C.c_int64), ("wave_steps_closest", C.c_int64),
                ("lane_steps_shadow", C.c_int64), ("wave_steps_shadow", C.c_int64),
                ("divergent_lane_loads", C.c_int64), ("divergent_distinct_records", C.c_int64),
                ("iter_wave_inner", C.c_int64 * 2), ("iter_wave_leaf", C.c_int64 * 2),
                ("iter_wave_scalar", C.c_int64 * 2), ("iter_lane_inner", C.c_int64 * 2),
                ("iter_lane_leaf", C.c_int64 * 2)]


class rt_ply_mesh(C.Structure):
    _fields_ = [("positions", c_double_p), ("num_positions", C.c_int64),
                ("normals", c_double_p), ("num_normals", C.c_int64),
                ("texcoords", C.POINTER(C.c_float)), ("num_texcoords", C.c_int64),
                ("indices", c_int32_p), ("num_indices", C.c_int64)]


RT_PROGRESS_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int32, C.c_int32)

# status codes (rtcore.h)
RT_OK = 0
RT_ERR_INVALID_CAMERA = -10
RT_ERR_NO_SCENE = -20
RT_ERR_BUSY = -32
RT_MAX_IN_FLIGHT = 16
RT_ERR_NO_RENDERER = -21
RT_ERR_INVALID_ARG = -30
RT_ERR_UNSUPPORTED = -31
RT_ERR_PLY = -40
RT_ERR_SCENE_FILE = -41
RT_ERR_DEVICE = -50
RT_ERR_OOM = -51
RT_ERR_CANCELLED = -60
RT_ERR_STACK = -61

RT_MAT = {"": 0, "default": 0, "mirror": 1, "dielectric": 2, "conductor": 3}
RT_CAM_LOOKAT, RT_CAM_NEARPLANE = 0, 1
RT_OBJ_MESH, RT_OBJ_TRIANGLE, RT_OBJ_SPHERE, RT_OBJ_PLANE, RT_OBJ_MESH_INSTANCE = 0, 1, 2, 3, 4

# every symbol include/rtcore.h declares (tests check the .so exports them all)
EXPORTED_SYMBOLS = [
    "rt_scene_create", "rt_scene_destroy", "rt_scene_info_get", "rt_render", "rt_render_device",
    "rt_stats_collect", "rt_rows_for_chunks", "rt_render_device_counted", "rt_last_error", "rt_version",
    "rt_ply_load", "rt_ply_free", "rt_debug_bvh_hash", "rt_debug_host_build", "rt_debug_fit_build",
    "rt_debug_trace_rays", "rt_debug_occluded_rays", "rt_host_alloc", "rt_host_free", "rt_debug_wave_times",
    "rt_debug_rcp", "rt_render_submit", "rt_render_wait",
    "rt_render_ex", "rt_host_register", "rt_host_unregister",
    "rt_scene_file_load", "rt_scene_file_parse", "rt_scene_file_desc", "rt_scene_file_image_name",
    "rt_scene_file_last_error", "rt_scene_file_destroy", "rt_scene_set_option", "rt_scene_get_option",
    "rt_scene_set_unsafe_option",
]
RT_ABI_VERSION = 4


def bind(lib: C.CDLL) -> C.CDLL:
    """Attach argtypes/restype to every exported function."""
    P = C.POINTER
    lib.rt_scene_create.argtypes = [P(rt_scene_desc), c_int32_p, C.c_int32, P(C.c_void_p)]
    lib.rt_scene_create.restype = C.c_int32
    lib.rt_scene_destroy.argtypes = [C.c_void_p]
    lib.rt_scene_destroy.restype = None
    lib.rt_scene_info_get.argtypes = [C.c_void_p, P(rt_scene_info)]
    lib.rt_scene_info_get.restype = C.c_int32
    lib.rt_render.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, c_double_p, P(C.c_uint8),
                              P(rt_stats), RT_PROGRESS_FN, C.c_void_p]
    lib.rt_render.restype = C.c_int32
    lib.rt_render_ex.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, c_double_p, P(C.c_uint8),
                                 C.c_uint32, P(rt_stats), RT_PROGRESS_FN, C.c_void_p]
    lib.rt_render_ex.restype = C.c_int32
    lib.rt_scene_file_load.argtypes = [C.c_char_p, C.c_int32, P(C.c_void_p)]
    lib.rt_scene_file_load.restype = C.c_int32
    lib.rt_scene_file_parse.argtypes = [C.c_void_p, C.c_uint64, C.c_int32, C.c_char_p, P(C.c_void_p)]
    lib.rt_scene_file_parse.restype = C.c_int32
    lib.rt_scene_file_desc.argtypes = [C.c_void_p]
    lib.rt_scene_file_desc.restype = P(rt_scene_desc)
    lib.rt_scene_file_image_name.argtypes = [C.c_void_p, C.c_int32]
    lib.rt_scene_file_image_name.restype = C.c_char_p
    lib.rt_scene_file_last_error.argtypes = []
    lib.rt_scene_file_last_error.restype = C.c_char_p
    lib.rt_scene_file_destroy.argtypes = [C.c_void_p]
    lib.rt_scene_file_destroy.restype = None
    lib.rt_host_register.argtypes = [C.c_void_p, C.c_uint64]
    lib.rt_host_register.restype = C.c_int32
    lib.rt_host_unregister.argtypes = [C.c_void_p]
    lib.rt_host_unregister.restype = C.c_int32
    lib.rt_render_device.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_void_p,
                                     C.c_void_p, C.c_void_p]
    lib.rt_render_device.restype = C.c_int32
    lib.rt_stats_collect.argtypes = [C.c_void_p, C.c_int32, P(rt_stats)]
    lib.rt_stats_collect.restype = C.c_int32
    lib.rt_rows_for_chunks.argtypes = [C.c_int32, C.c_int32, C.c_int32]
    lib.rt_rows_for_chunks.restype = C.c_int32
    lib.rt_render_device_counted.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_void_p,
                                             C.c_void_p, P(rt_work_counters)]
    lib.rt_render_device_counted.restype = C.c_int32
    lib.rt_last_error.argtypes = []
    lib.rt_last_error.restype = C.c_char_p
    lib.rt_version.argtypes = []
    lib.rt_version.restype = C.c_char_p
    lib.rt_ply_load.argtypes = [C.c_char_p, P(rt_ply_mesh)]
    lib.rt_ply_load.restype = C.c_int32
    lib.rt_ply_free.argtypes = [P(rt_ply_mesh)]
    lib.rt_ply_free.restype = None
    lib.rt_host_alloc.argtypes = [C.c_uint64, P(C.c_void_p)]
    lib.rt_host_alloc.restype = C.c_int32
    lib.rt_host_free.argtypes = [C.c_void_p]
    lib.rt_host_free.restype = None
    lib.rt_debug_wave_times.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_void_p,
                                        P(C.c_uint64), C.c_int64, P(C.c_int64)]
    lib.rt_debug_wave_times.restype = C.c_int32
    lib.rt_debug_rcp.argtypes = [C.c_int32, c_double_p, c_double_p, c_double_p]
    lib.rt_debug_rcp.restype = C.c_int32
    lib.rt_render_submit.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, c_double_p, C.POINTER(C.c_uint8),
                                     C.c_uint32, C.POINTER(C.c_int64)]
    lib.rt_render_submit.restype = C.c_int32
    lib.rt_render_wait.argtypes = [C.c_void_p, C.c_int64, C.POINTER(rt_stats)]
    lib.rt_render_wait.restype = C.c_int32
    lib.rt_debug_bvh_hash.argtypes = [C.c_void_p, C.c_int32]
    lib.rt_debug_bvh_hash.restype = C.c_uint64
    lib.rt_debug_host_build.argtypes = [P(rt_scene_desc), P(C.c_uint64), C.c_int32, c_int32_p, P(rt_scene_info)]
    lib.rt_debug_host_build.restype = C.c_int32
    if hasattr(lib, "rt_debug_fit_build"):   # round 6 (an older build may be loaded for an A/B, MYRT_LIB)
        lib.rt_debug_fit_build.argtypes = [P(rt_scene_desc), P(C.c_int64)]
        lib.rt_debug_fit_build.restype = C.c_int32
    lib.rt_debug_trace_rays.argtypes = [C.c_void_p, C.c_int32, C.c_int32, c_double_p, c_double_p, c_double_p,
                                        c_double_p, c_double_p, c_double_p, c_double_p, c_int32_p]
    lib.rt_debug_trace_rays.restype = C.c_int32
    lib.rt_debug_occluded_rays.argtypes = [C.c_void_p, C.c_int32, C.c_int32, c_double_p, c_double_p, c_double_p,
                                           c_double_p, P(C.c_uint8)]
    lib.rt_debug_occluded_rays.restype = C.c_int32
    if hasattr(lib, "rt_scene_set_option"):   # ABI >= 3 (an older build may be loaded for an A/B, MYRT_LIB)
        lib.rt_scene_set_option.argtypes = [C.c_void_p, C.c_char_p, C.c_int64]
        lib.rt_scene_set_option.restype = C.c_int32
        lib.rt_scene_get_option.argtypes = [C.c_void_p, C.c_char_p, P(C.c_int64)]
        lib.rt_scene_get_option.restype = C.c_int32
    if hasattr(lib, "rt_scene_set_unsafe_option"):   # ABI >= 4 (test hooks, not for production)
        lib.rt_scene_set_unsafe_option.argtypes = [C.c_void_p, C.c_char_p, C.c_int64]
        lib.rt_scene_set_unsafe_option.restype = C.c_int32
    return lib
