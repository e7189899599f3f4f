/*
 * rtcore.h — C ABI of the MI355X-native renderer core (libmyrt.so).
 *
 * This is the drop-in boundary for the reference's per-pixel trace path
 * (erndmrcn/MyRayTracer).  A host (the Swift `RayTracerEngine`, or the Python
 * mirror in myraytracer_amd/engine.py) describes a scene with plain C structs,
 * creates a device-resident scene once, and renders cameras from it.
 *
 * Each entry point cites the reference interface it replaces
 * (paths relative to Sources/ of the reference):
 *
 *   rt_scene_create   <- RayTracerEngine.init(from:data:)  RayTracer/RayTracer.swift:30-49
 *                        + RTContext.init(scene:)         RayTracer/Models/RTContext.swift:94-418
 *   rt_render         <- RayTracerEngine.render(format:cameraIndex:progress:)
 *                                                          RayTracer/RayTracer.swift:115-131
 *                        -> renderRGBA8Async               RayTracer/RayTracer.swift:137-205
 *                        -> Renderer.render(scene:cameraIndex:progressRow:)
 *                                                          RayTracer/Extensions/Object+Extension.swift:52-379
 *   rt_render_device  <- same path, output left in device memory (bench / multi-GPU)
 *   rt_scene_info     <- RayTracerEngine.inspect / sceneMeshAndTriangleCounts
 *                                                          RayTracer/RayTracer.swift:52-67,208-227
 *   rt_scene_file_*   <- SceneLoader.load (ParsingKit) in RayTracerEngine.init(from:data:)
 *                                                          RayTracer/RayTracer.swift:30-49
 *   rt_ply_load       <- PLYLoader.load(from:)             RayTracer/Helpers/PLYReader.swift:54-210
 *                        (which drives CPly's ply_reader_* C ABI, CPly/include/PLYReaderWrapper.h:26-69)
 *
 * Conventions mirror the reference's only C ABI (CPly/include/PLYReaderWrapper.h:22-69,
 * CPly/wrapper.cpp:17-27): opaque handle + create/destroy pair, caller-allocated
 * outputs, no C++ exception ever crosses the boundary.  Status codes: 0 = OK,
 * negative = error; the reference's NSError codes are reused (-10, -20, -21,
 * RayTracer.swift:121,141-154).  rt_last_error() returns a thread-local message.
 *
 * All arithmetic is IEEE binary64 (the reference's Vec3 = SIMD3<Double>,
 * RTContext.swift:13-16).  Matrices are column-major 4x4 (simd_double4x4 layout:
 * m[c*4 + r] = column c, row r).
 */
#ifndef MYRT_RTCORE_H
#define MYRT_RTCORE_H

#include <stdint.h>

/* ABI version of this header (rt_version() reports it).
 *   1: round-1/2 layout.
 *   2: rt_object gained `num_normals` (sizeof(rt_object), the stride of rt_scene_desc.objects,
 *      changed: callers built against version 1 must be rebuilt).  A non-NULL `normals` now
 *      requires num_normals == num_positions; version-1 callers that left it 0 get
 *      RT_ERR_INVALID_ARG instead of an unchecked read.
 *   3: rt_stats gained `rewalked` and rt_scene_info `scratch_bytes` (both appended: the
 *      structs grew); rt_scene_set_option / rt_scene_get_option replace the MYRT_*
 *      environment switches (the library reads no environment variable on the render path).
 *   4: the test hooks debug_fail_replica / wide_delta_scale moved behind the non-production
 *      rt_scene_set_unsafe_option; rt_scene_set_option refuses them. */
#define RT_ABI_VERSION 4

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ------------------------------------------------------ */
#define RT_OK                    0
#define RT_ERR_INVALID_CAMERA  (-10)  /* RayTracer.swift:151-154 "Invalid camera index" */
#define RT_ERR_NO_SCENE        (-20)  /* RayTracer.swift:141-144 "No scene loaded"      */
#define RT_ERR_NO_RENDERER     (-21)  /* RayTracer.swift:145-148 "Renderer not initialized" */
#define RT_ERR_INVALID_ARG     (-30)
#define RT_ERR_UNSUPPORTED     (-31)  /* feature outside the implemented hot path      */
#define RT_ERR_PLY             (-40)  /* PLYReader.swift:24-40 PlyError                */
#define RT_ERR_SCENE_FILE      (-41)  /* SceneLoader / PKDecodingError (scene file decode) */
#define RT_ERR_DEVICE          (-50)  /* HIP runtime failure                           */
#define RT_ERR_OOM             (-51)
#define RT_ERR_CANCELLED       (-60)  /* progress callback returned 0                  */
#define RT_ERR_STACK           (-61)  /* BVH deeper than the traversal stack           */
#define RT_ERR_BUSY            (-32)  /* RT_MAX_IN_FLIGHT renders submitted and not waited for */

/* ---- scene description (ParsingKit Scene stand-in) ----------------------- */
typedef struct rt_vec3 { double x, y, z; } rt_vec3;

/* Material.type strings of the reference (Object+Extension.swift:189,207,252) */
#define RT_MAT_DEFAULT     0
#define RT_MAT_MIRROR      1   /* "mirror"     */
#define RT_MAT_DIELECTRIC  2   /* "dielectric" */
#define RT_MAT_CONDUCTOR   3   /* "conductor"  */

typedef struct rt_material {   /* ParsingKit Material, fields read in trace() */
    rt_vec3 ambient, diffuse, specular, mirror, absorption;
    double  phong;              /* Phong exponent, clamped to >= 1 (:131)      */
    double  ior;                /* refraction index; > 0 disables direct light on back faces (:112-115) */
    double  absorption_index;   /* conductor k (:254)                           */
    double  roughness;          /* glossy perturbation (:191-197)               */
    int32_t type;               /* RT_MAT_*                                     */
    int32_t _pad;
} rt_material;

typedef struct rt_point_light { rt_vec3 position, intensity; } rt_point_light;

typedef struct rt_area_light {  /* Object+Extension.swift:145-186 */
    rt_vec3 position, normal, radiance;
    double  size;
} rt_area_light;

#define RT_CAM_LOOKAT     0     /* cam.type == "lookAt" (Object+Extension.swift:394)   */
#define RT_CAM_NEARPLANE  1     /* explicit nearPlane + gaze (:415-426)                */

typedef struct rt_camera {      /* ParsingKit Camera */
    int32_t type;               /* RT_CAM_*                                            */
    int32_t width, height;      /* imageResolution                                     */
    int32_t num_samples;        /* numSamples                                          */
    rt_vec3 position, gaze_point, gaze, up;
    double  fovy;               /* degrees; NaN = absent (Camera.fovy: Double?)        */
    double  near_distance;
    double  near_plane[4];      /* l, r, b, t                                          */
    double  aperture_size, focus_distance;
} rt_camera;

#define RT_OBJ_MESH           0
#define RT_OBJ_TRIANGLE       1
#define RT_OBJ_SPHERE         2
#define RT_OBJ_PLANE          3
#define RT_OBJ_MESH_INSTANCE  4

/* One entry of Scene.objects, in scene order (RTContext.swift:120-378). */
typedef struct rt_object {
    int32_t kind;               /* RT_OBJ_*                                            */
    int32_t material_id;        /* materialIndex(for:) = Int(id) or -1 (RTContext.swift:423-426), 1-based */
    int32_t smooth;             /* Mesh.shadingMode == "smooth" (RTContext.swift:245)  */
    int32_t id;                 /* object id (MeshInstance.baseMeshID refers to it)    */
    int32_t base_mesh_id;       /* RT_OBJ_MESH_INSTANCE only                           */
    int32_t indices_one_based;  /* inline faces.data are 1-based (RTContext.swift:300-301) */
    double  transform[16];      /* composed localToWorld (Scene.composeTransform result), column-major */
    rt_vec3 motion_blur;        /* Mesh.motionBlur / MeshInstance.motionBlur           */
    /* mesh payload: either a PLY path or inline arrays                               */
    const char*    ply_path;
    const double*  positions;   int64_t num_positions;   /* xyz triples               */
    const int32_t* indices;     int64_t num_indices;     /* triangle list             */
    const double*  normals;     /* optional per-vertex normals (PLY branch, RTContext.swift:267-297);
                                 * length in num_normals below                            */
    /* analytic payloads (RT_OBJ_TRIANGLE / SPHERE / PLANE)                           */
    rt_vec3 v[3];               /* triangle vertices                                   */
    rt_vec3 center;             /* sphere / plane center                               */
    rt_vec3 normal;             /* plane normal                                        */
    double  radius;             /* sphere radius                                       */
    int64_t num_normals;        /* xyz triples behind `normals`; must equal num_positions */
} rt_object;

typedef struct rt_scene_desc {
    rt_vec3 background_color;
    rt_vec3 ambient_light;             /* scene.lights.ambient                         */
    double  shadow_ray_epsilon;
    double  intersection_test_epsilon;
    int32_t max_recursion_depth;
    int32_t num_materials;
    const rt_material*    materials;
    int32_t num_point_lights;
    int32_t num_area_lights;
    const rt_point_light* point_lights;
    const rt_area_light*  area_lights;
    int32_t num_objects;
    int32_t num_cameras;
    const rt_object*      objects;
    const rt_camera*      cameras;
} rt_scene_desc;

/* ---- results -------------------------------------------------------------- */
typedef struct rt_stats {       /* RenderStats (Models/RenderStats.swift:8-24) + ray counts */
    int64_t meshes, triangles, spheres, planes;
    int64_t primary_rays;       /* W*H*n^2 actually cast                               */
    int64_t shadow_rays;        /* one per point light per directly-lit hit            */
    int64_t secondary_rays;     /* reflection rays                                     */
    double  milliseconds;       /* wall time of the render call                        */
    double  kernel_ms;          /* device time of the render kernels                   */
    int64_t shadow_rays_traced; /* shadow rays whose any-hit walk actually ran: the walk is
                                 * skipped when !(N.L > 0), where the reference discards the
                                 * occlusion result (Object+Extension.swift:123-141)      */
    int64_t rewalked;           /* closest-hit rays the four-wide walk handed to the reference-
                                 * order walk because two candidates met their final t    */
} rt_stats;

typedef struct rt_scene_info {
    int64_t meshes, triangles, spheres, planes, instances;
    int64_t blas_nodes, tlas_nodes, max_depth;
    double  build_ms;           /* PLY load + flatten + BVH build + layout            */
    double  upload_ms;          /* host -> device copies                               */
    int64_t device_bytes;       /* per-device resident scene bytes                     */
    int64_t scratch_bytes;      /* device scratch held now by replica 0 (render outputs, pass
                                 * scratch of full trace() renders, queues, deep frames) */
} rt_scene_info;

typedef struct rt_scene rt_scene;   /* opaque */

/* progress: rows finished so far; return 0 to cancel (RayTracer.swift:172-181). */
typedef int (*rt_progress_fn)(void* user, int32_t rows_done, int32_t rows_total);

/* ---- lifecycle ------------------------------------------------------------- */
/* Builds the scene on the host (PLY load, flattening, SAH BVH) and uploads a full
 * replica to each listed device (HIP ordinals; n_devices <= 0 means device 0). */
int32_t rt_scene_create(const rt_scene_desc* desc, const int32_t* devices, int32_t n_devices,
                        rt_scene** out);
void    rt_scene_destroy(rt_scene* scene);
int32_t rt_scene_info_get(const rt_scene* scene, rt_scene_info* out);

/* Render options: tuning and test switches, each default being the production setting.
 *   wide (1)             conservative FP32 four-wide walk of identity scenes (exact: wide.h)
 *   unified (1)          one-stack TLAS+BLAS walks; 0 = the nested walk of intersectTLAS
 *   unified_transformed (1)  one-stack walk of instanced scenes (device.h ut_walk)
 *   compact_records (1), compact_tris (1)   float32 records / triangles when exact
 *   xcd_group (0 = auto) tiles per XCD run      queue (1)  compacted bounce render (0 = megakernel)
 *   queue_levels (-1)    timing probe           hitlog (-1 = auto) logged hits per pixel
 *   nodeshade (1), levels (1), tree_ppw (4),
 *   node_lists (1)                              full trace() pass structure
 *   full_flights (4)     full trace() renders overlapping on slot streams
 *   deep_cap_mb (8192)   deep trace() frames per launch batch
 *   batches (0 = auto), zerocopy (1)            rt_render delivery
 *   submit_events (1), submit_counters (1), submit_dma (0)   rt_render_submit delivery
 *   tile_order (0)       % of tile groups dispatched slowest first
 *   fit (1)              transformed scenes: the flattened instance tree (wide.h fit_walk);
 *                        0 = the TLAS / per-BLAS four-wide walk (tw_walk)
 *   queue_tail (2)       compacted bounce render: levels >= this one traced depth-first in one
 *                        launch (render.hip k_bounce_tail); 0 = one launch per level
 * Unknown names and out-of-range values return RT_ERR_INVALID_ARG.  Set options between
 * renders (not while renders of the scene are in flight).  The test hooks below are refused
 * here (RT_ERR_INVALID_ARG); rt_scene_get_option reads every option. */
int32_t rt_scene_set_option(rt_scene* scene, const char* name, int64_t value);
int32_t rt_scene_get_option(const rt_scene* scene, const char* name, int64_t* value);

/* NOT FOR PRODUCTION (ABI 4).  Sets any option, including the test hooks that
 * rt_scene_set_option refuses because they void the library's guarantees:
 *   debug_fail_replica (-1)   inject a launch failure on that replica
 *   wide_delta_scale (1000)   the four-wide walk's widening in 1/1000 of the proven bound
 *                             (wide.h); below 1000 exactness is no longer guaranteed
 * Used only by the parity tests that show the exactness proof has teeth. */
int32_t rt_scene_set_unsafe_option(rt_scene* scene, const char* name, int64_t value);

/* ---- rendering -------------------------------------------------------------- */
/* Renders 8-row chunks chunk_first, chunk_first+chunk_step, ... of camera
 * `camera_index` (chunk c covers rows [8c, min(8c+8, H)) as in
 * Object+Extension.swift:75-82; row 0 = top).  Outputs are caller-owned HOST
 * buffers holding the selected chunks' rows packed in chunk order:
 * out_rgb = rows*W*3 doubles (the [Vec3] of Renderer.render), out_rgba8 =
 * rows*W*4 bytes (RayTracer.swift:186-195).  Either may be NULL.  chunk_step = 1,
 * chunk_first = 0 renders the whole image.  Work is spread over all devices of
 * the scene. */
int32_t rt_render(rt_scene* scene, int32_t camera_index, int32_t chunk_first, int32_t chunk_step,
                  double* out_rgb, uint8_t* out_rgba8, rt_stats* stats,
                  rt_progress_fn progress, void* user);

/* rt_render with flags.  RT_RENDER_FRAME_LAYOUT: out_rgb / out_rgba8 are whole W x H
 * frames (W*H*3 doubles / W*H*4 bytes) and the selected chunks' rows are written at
 * their image rows; other rows are left untouched.  Several renders of disjoint chunk
 * selections (other devices, other processes sharing one registered buffer) thereby
 * gather one image with no copy.  rt_render(...) == rt_render_ex(..., 0, ...). */
#define RT_RENDER_FRAME_LAYOUT  1u
/* rt_render_submit: time the render kernels with HIP events (rt_stats.kernel_ms of
 * rt_render_wait; 0 without the flag).  rt_render / rt_render_ex always time them. */
#define RT_RENDER_KERNEL_TIME   2u
int32_t rt_render_ex(rt_scene* scene, int32_t camera_index, int32_t chunk_first, int32_t chunk_step,
                     double* out_rgb, uint8_t* out_rgba8, uint32_t flags, rt_stats* stats,
                     rt_progress_fn progress, void* user);

/* Asynchronous render: RayTracerEngine.render is `async` (RayTracer.swift:115-131, 137-205),
 * so a Swift caller may keep several renders in flight (renderAll, BatchRender).
 * rt_render_submit enqueues the render rt_render_ex(..., flags, ...) would do into PAGE-LOCKED
 * outputs (rt_host_alloc / rt_host_register; RT_ERR_INVALID_ARG otherwise), returns at once
 * with *ticket, and the kernels store the image straight into the buffers.  At most
 * RT_MAX_IN_FLIGHT renders per scene may be submitted and not yet waited for (RT_ERR_BUSY).
 * Renders in flight overlap on the GPUs: the next frame's tiles fill the compute units the
 * previous frame's slowest tiles leave idle.  rt_render_wait blocks until that render's
 * image is complete in the buffers and fills stats (milliseconds from submit to completion).
 * Scenes with dielectrics, area lights or maxRecursionDepth > 16 are rendered in submission
 * order.  rt_render_ex with page-locked outputs and no progress callback is submit + wait. */
#define RT_MAX_IN_FLIGHT 16
int32_t rt_render_submit(rt_scene* scene, int32_t camera_index, int32_t chunk_first, int32_t chunk_step,
                         double* out_rgb, uint8_t* out_rgba8, uint32_t flags, int64_t* ticket);
int32_t rt_render_wait(rt_scene* scene, int64_t ticket, rt_stats* stats);

/* Page-locked host buffers for rt_render outputs (hipHostMalloc, mapped + portable).
 * When out_rgb / out_rgba8 lie inside one such allocation (or a range registered with
 * rt_host_register), the render kernels of every device replica store their rows
 * straight into them over PCIe; other host memory goes through pinned staging and a
 * host memcpy.  rt_host_register pins existing host memory (e.g. a shared-memory
 * framebuffer mapped by several processes); unregister before unmapping it. */
int32_t rt_host_alloc(uint64_t bytes, void** out);
void    rt_host_free(void* ptr);
int32_t rt_host_register(void* ptr, uint64_t bytes);
int32_t rt_host_unregister(void* ptr);

/* Same as rt_render on ONE device slot, but outputs are DEVICE pointers on that
 * device and the work is enqueued on `stream` (a hipStream_t, NULL = default)
 * without host synchronisation.  Ray counters are only valid after rt_stats_collect()
 * once the stream has drained.  Device renders have their own counters, pass scratch and
 * queues, so they may overlap rt_render / rt_render_submit renders of the same scene;
 * exception: scenes with maxRecursionDepth > 16 share one deep-frame buffer per replica,
 * and a device render of such a scene must not overlap another render of it.
 * Device renders of ONE slot share those counters and scratch among themselves: issue them
 * on one stream (or order them externally); two concurrent device renders of a slot on
 * different streams race.  Scratch that grows is never freed under a render still queued
 * (the old buffer is retired until rt_scene_destroy), and the call itself reads the scene's
 * options under the scene's lock. */
int32_t rt_render_device(rt_scene* scene, int32_t device_slot, int32_t camera_index,
                         int32_t chunk_first, int32_t chunk_step,
                         double* d_out_rgb, uint8_t* d_out_rgba8, void* stream);
int32_t rt_stats_collect(rt_scene* scene, int32_t device_slot, rt_stats* stats);

/* Number of output rows rt_render writes for a chunk selection. */
int32_t rt_rows_for_chunks(int32_t height, int32_t chunk_first, int32_t chunk_step);

/* Traversal work counters of the last rt_render_device on a slot (instrumented
 * kernel variant; used to price algorithmic bytes for the roofline). */
typedef struct rt_work_counters {
    int64_t records_fetched;    /* 128-B two-child node records loaded                */
    int64_t tri_tests;          /* 80-B triangle records tested                       */
    int64_t normal_fetches;     /* 72-B smooth-normal triples loaded (final hits)     */
    int64_t instance_entries;   /* world->local transforms                            */
    int64_t pixels;             /* pixels written                                     */
    /* The same frame walked in the REFERENCE's order (no t-pruning; any-hit visits L
     * before R and stops at the first occluder; RTContext.swift:544-829), tallied as
     * SURVEY.md §8(d) defines algorithmic work: B = 56*N_nodeFetch + 72*N_triTest +
     * 72*N_smoothHit + 24*N_pixelWrite.  Equal to the oracle's counts (tests/test_gpu_parity.py). */
    int64_t ref_node_fetches;   /* node bounds loaded (roots + both children of each popped inner node; every any-hit pop) */
    int64_t ref_tri_tests;      /* Moeller-Trumbore tests                             */
    int64_t ref_smooth_hits;    /* closer smooth hits (normal triple interpolated)    */
    int64_t ref_pixels;         /* pixels written                                     */
    /* SIMD efficiency of the traversal loops (megakernel, identity scenes): iterations run
     * by lanes vs iterations run by their waves (64 x the max over the wave's lanes).     */
    int64_t lane_steps_closest, wave_steps_closest;
    int64_t lane_steps_shadow, wave_steps_shadow;
    /* Vector-memory redundancy of the inner steps that take per-lane loads (the wave's lanes
     * at more than one record): active lanes vs distinct records among them.             */
    int64_t divergent_lane_loads, divergent_distinct_records;
    /* Per-iteration divergence of the unified walks ([0] closest hit, [1] any hit): wave
     * iterations in which some lane took an inner step / a leaf run / the wave-uniform
     * scalar-cache inner step, and lane iterations that took an inner step / a leaf run.  */
    int64_t iter_wave_inner[2], iter_wave_leaf[2], iter_wave_scalar[2];
    int64_t iter_lane_inner[2], iter_lane_leaf[2];
} rt_work_counters;
int32_t rt_render_device_counted(rt_scene* scene, int32_t device_slot, int32_t camera_index,
                                 int32_t chunk_first, int32_t chunk_step,
                                 double* d_out_rgb, void* stream, rt_work_counters* out);

const char* rt_last_error(void);
const char* rt_version(void);

/* ---- PLY (host) --------------------------------------------------------------- */
typedef struct rt_ply_mesh {            /* PlyMesh (PLYReader.swift:14-19)           */
    double*  positions;  int64_t num_positions;   /* float32 widened to double (:96-102) */
    double*  normals;    int64_t num_normals;     /* normalized (:105-123), 0 if absent  */
    float*   texcoords;  int64_t num_texcoords;
    int32_t* indices;    int64_t num_indices;     /* triangulated, 0-based (:149-198)    */
} rt_ply_mesh;
int32_t rt_ply_load(const char* path, rt_ply_mesh* out);
void    rt_ply_free(rt_ply_mesh* mesh);

/* ---- scene files (host) --------------------------------------------------------
 * RayTracerEngine.init(from: url) / init(data:)  RayTracer/RayTracer.swift:30-49, which read
 * the scene through ParsingKit's SceneLoader.load(.url / .data(format:)) (SceneFormat
 * Models/SceneFormat.swift:8-10).  The decoded scene owns every array rt_scene_file_desc()
 * points into; pass that descriptor to rt_scene_create, then destroy the file.  JSON and XML
 * follow ParsingKit's flexible conventions (myraytracer_amd/csrc/sceneio.cpp); a mesh's PLY
 * path resolves against the scene file's directory (base_dir for in-memory data; NULL = the
 * current directory).  Errors: RT_ERR_SCENE_FILE with rt_scene_file_last_error().           */
#define RT_SCENE_FORMAT_AUTO  0
#define RT_SCENE_FORMAT_JSON  1
#define RT_SCENE_FORMAT_XML   2
typedef struct rt_scene_file rt_scene_file;   /* opaque */
int32_t rt_scene_file_load(const char* path, int32_t format, rt_scene_file** out);
int32_t rt_scene_file_parse(const void* data, uint64_t size, int32_t format, const char* base_dir,
                            rt_scene_file** out);
const rt_scene_desc* rt_scene_file_desc(const rt_scene_file* file);
const char* rt_scene_file_image_name(const rt_scene_file* file, int32_t camera_index);  /* Camera.imageName */
const char* rt_scene_file_last_error(void);
void    rt_scene_file_destroy(rt_scene_file* file);

/* ---- debug / test hooks (not part of the reference surface) -------------------- */
/* Canonical hash of instance `instance`'s BLAS (instance = -1: the TLAS); equal to the
 * oracle's oracle_bvh_hash when the topology, bounds and leaf order match BVH.swift. */
uint64_t rt_debug_bvh_hash(const rt_scene* scene, int32_t instance);
/* Host-only build (no device): hashes[0..n) per instance, hashes[n] = TLAS. */
int32_t  rt_debug_host_build(const rt_scene_desc* desc, uint64_t* hashes, int32_t max_hashes,
                             int32_t* n_instances, rt_scene_info* info);
/* Host-only build of a transformed scene's flattened instance tree (wide.h fit_walk): out[0] =
 * pairs (0: no tree), out[1] = nodes, out[2] = depth, out[3] = leaf runs over all instances,
 * out[4] = a hash of the pairs and the nodes (octant copy 0). */
int32_t  rt_debug_fit_build(const rt_scene_desc* desc, int64_t* out);

/* Explicit-ray queries on device `slot` through the render kernels' traversal (host
 * arrays, n rays; o/d: 3 doubles per ray).  rt_debug_trace_rays = intersectTLAS
 * (RTContext.swift:619-720) with tMin: out_t (+inf on a miss), world hit point, world
 * geometric normal (before facing), materialOverride (-1 on a miss).
 * rt_debug_occluded_rays = occludedTLAS (:724-781) with tMax: out[i] = 1 if blocked.   */
int32_t rt_debug_trace_rays(rt_scene* scene, int32_t slot, int32_t n, const double* o, const double* d,
                            const double* tmin, const double* time, double* out_t, double* out_p,
                            double* out_n, int32_t* out_mat);
int32_t rt_debug_occluded_rays(rt_scene* scene, int32_t slot, int32_t n, const double* o, const double* d,
                               const double* tmax, const double* time, uint8_t* out);
/* Reciprocals on device 0 (host arrays, n values): out_fast[i] = the traversal's 1/x
 * (device.h rcp_rn, used when RenderParams::fast_rcp holds), out_div[i] = IEEE 1.0/x.
 * Equal bit for bit for 2^-700 <= |x| <= 2^1000 (tests/test_gpu_rays.py).  No scene. */
int32_t rt_debug_rcp(int32_t n, const double* x, double* out_fast, double* out_div);
/* Per-wave timeline of one megakernel launch (identity scenes without dielectrics or area
 * lights) into device buffer d_out_rgb: out[3*k..3*k+2] = {start, end, tile} of wave k in
 * 100 MHz ticks (s_memrealtime); the tile word also holds the wave's largest lane iteration
 * counts of the closest-hit walks (bits 24-43) and the any-hit walks (bits 44-63).  *n_waves = waves launched; at most max_waves are copied.
 * Returns RT_ERR_UNSUPPORTED unless the library was built with -DMYRT_WAVE_TIMES=1. */
int32_t rt_debug_wave_times(rt_scene* scene, int32_t slot, int32_t camera_index, int32_t chunk_first,
                            int32_t chunk_step, double* d_out_rgb, uint64_t* out, int64_t max_waves,
                            int64_t* n_waves);

#ifdef __cplusplus
}
#endif
#endif /* MYRT_RTCORE_H */
