/*
 * rt_engine.hpp — C++17 host mirror of the reference's public engine API over the C ABI
 * (include/rtcore.h).  Header-only; link with -lmyrt.
 *
 * The reference's host is Swift (`public final class RayTracerEngine`,
 * Sources/RayTracer/RayTracer.swift:25-228), which cannot run on Linux.  This is the same
 * surface for compiled C++ hosts, with the same names, argument meaning and error
 * behaviour:
 *
 *   RayTracerEngine(scene)          <- init(from:data:) after SceneLoader.load      RayTracer.swift:30-49
 *   inspect()                       <- inspect(scene:format:)                       RayTracer.swift:52-67
 *   render(format, cameraIndex, p)  <- render(format:cameraIndex:progress:)         RayTracer.swift:115-131
 *   renderAll(p)                    <- renderAll(progress:)                         RayTracer.swift:70-102
 *   RenderResult / RenderStats / RenderProgress / CameraSpec / SceneInfo            Models/*.swift
 *   RenderError{code}               <- NSError(domain:"Render"/"Ray", code: -10/-20/-21)
 *
 * Differences, all deliberate: RenderResult carries the RGBA8 pixels (and the FP64
 * [Vec3] buffer Renderer.render returns) instead of a CGImage; RenderStats.rays is the
 * number of primary + shadow rays actually cast (the reference always reported 0,
 * RayTracer.swift:167,200) and milliseconds is a double; returning false from the
 * progress callback really cancels (RT_ERR_CANCELLED; the reference's cancel was a
 * no-op on an unstructured task).  Scene files are decoded by the host (ParsingKit's
 * role); this class takes the decoded scene as an rt_scene_desc.
 */
#ifndef MYRT_RT_ENGINE_HPP
#define MYRT_RT_ENGINE_HPP

#include <algorithm>
#include <cstdint>
#include <functional>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "rtcore.h"

namespace myrt {

/* NSError equivalent: `code` is the rtcore status (-10 invalid camera, -20 no scene,
 * -21 renderer not initialised, -50 device, -60 cancelled, ...). */
class RenderError : public std::runtime_error {
public:
    RenderError(int32_t code, const std::string& msg)
        : std::runtime_error("[" + std::to_string(code) + "] " + msg), code(code) {}
    int32_t code;
};

inline void check(int32_t rc) {
    if (rc != RT_OK) {
        const char* m = rt_last_error();
        throw RenderError(rc, m ? m : "");
    }
}

enum class SceneFormat { Auto, Json, Xml };           /* Models/SceneFormat.swift:8-10 */

struct RenderProgress {                                 /* Models/RenderProgress.swift:8-14 */
    double fraction;                                    /* 0...1 */
    std::string message;
};

struct RenderStats {                                    /* Models/RenderStats.swift:8-24 */
    int64_t meshes = 0, triangles = 0, spheres = 0, planes = 0;
    int64_t rays = 0;                                   /* primary + shadow */
    int64_t primary_rays = 0, shadow_rays = 0, secondary_rays = 0;
    int64_t shadow_rays_traced = 0;                     /* any-hit walks that ran (<= shadow_rays) */
    int64_t rewalked = 0;                               /* closest-hit rays re-walked in reference order (ties) */
    double milliseconds = 0, kernel_ms = 0;
};

struct CameraSpec {                                     /* Models/RenderConfig.swift:19-25 */
    int32_t index = 0;
    std::string id, imageName;
    int32_t width = 0, height = 0;
};

struct SceneInfo {                                      /* Models/RenderConfig.swift:27-33 */
    std::vector<CameraSpec> cameras;
    int64_t meshes = 0, triangles = 0, spheres = 0, planes = 0;
};

struct RenderResult {                                   /* Models/RenderResult.swift:10-15 */
    std::string fileName;
    std::vector<uint8_t> rgba8;                         /* H*W*4, row 0 = top (RayTracer.swift:186-195) */
    std::vector<double> rgb;                            /* H*W*3, Renderer.render's [Vec3] */
    CameraSpec camera;
    RenderStats stats;
};

/* Camera metadata the C ABI does not carry (Camera.id / imageName). */
struct CameraMeta {
    std::string id, imageName;
};

using ProgressFn = std::function<bool(const RenderProgress&)>;

class RayTracerEngine {
public:
    /* Builds the scene on the host (PLY, flattening, SAH BVH) and uploads a replica to
     * every listed device (empty = device 0).  The descriptor is copied. */
    explicit RayTracerEngine(const rt_scene_desc& desc, std::vector<int32_t> devices = {},
                             std::vector<CameraMeta> cameraMeta = {})
        : meta_(std::move(cameraMeta)) {
        for (int32_t i = 0; i < desc.num_cameras; ++i) cams_.push_back(desc.cameras[i]);
        check(rt_scene_create(&desc, devices.empty() ? nullptr : devices.data(), (int32_t)devices.size(), &scene_));
    }
    /* RayTracerEngine.init(from: url) / init(data:) (RayTracer.swift:30-49): the scene file is
     * decoded by rt_scene_file_* (JSON or XML, ParsingKit's conventions), then built like the
     * descriptor constructor.  Throws RenderError(RT_ERR_SCENE_FILE) on a decode error. */
    static RayTracerEngine fromFile(const std::string& path, SceneFormat format = SceneFormat::Auto,
                                    std::vector<int32_t> devices = {}) {
        rt_scene_file* f = nullptr;
        if (const int32_t rc = rt_scene_file_load(path.c_str(), fileFormat(format), &f))
            throw RenderError(rc, rt_scene_file_last_error());
        return fromSceneFile(f, std::move(devices));
    }
    static RayTracerEngine fromData(const std::string& data, SceneFormat format = SceneFormat::Auto,
                                    const std::string& baseDir = "", std::vector<int32_t> devices = {}) {
        rt_scene_file* f = nullptr;
        if (const int32_t rc = rt_scene_file_parse(data.data(), data.size(), fileFormat(format),
                                                   baseDir.empty() ? nullptr : baseDir.c_str(), &f))
            throw RenderError(rc, rt_scene_file_last_error());
        return fromSceneFile(f, std::move(devices));
    }
    ~RayTracerEngine() { if (scene_) rt_scene_destroy(scene_); }
    RayTracerEngine(const RayTracerEngine&) = delete;
    RayTracerEngine& operator=(const RayTracerEngine&) = delete;
    RayTracerEngine(RayTracerEngine&& o) noexcept : scene_(o.scene_), cams_(std::move(o.cams_)), meta_(std::move(o.meta_)) {
        o.scene_ = nullptr;
    }

    rt_scene* handle() const { return scene_; }

    /* Render options (rt_scene_set_option; defaults are the production settings). */
    void setOption(const std::string& name, int64_t value) { check(rt_scene_set_option(scene_, name.c_str(), value)); }
    /* Test hooks (rt_scene_set_unsafe_option: not for production, rtcore.h). */
    void setUnsafeOption(const std::string& name, int64_t value) {
        check(rt_scene_set_unsafe_option(scene_, name.c_str(), value));
    }
    int64_t option(const std::string& name) const {
        int64_t v = 0;
        check(rt_scene_get_option(scene_, name.c_str(), &v));
        return v;
    }

private:
    static int32_t fileFormat(SceneFormat f) {
        return f == SceneFormat::Json ? RT_SCENE_FORMAT_JSON : f == SceneFormat::Xml ? RT_SCENE_FORMAT_XML
                                                                                     : RT_SCENE_FORMAT_AUTO;
    }
    static RayTracerEngine fromSceneFile(rt_scene_file* f, std::vector<int32_t> devices) {
        std::unique_ptr<rt_scene_file, void (*)(rt_scene_file*)> own(f, rt_scene_file_destroy);
        const rt_scene_desc* d = rt_scene_file_desc(f);
        std::vector<CameraMeta> meta;
        for (int32_t k = 0; k < d->num_cameras; ++k) {
            const char* n = rt_scene_file_image_name(f, k);
            meta.push_back(CameraMeta{"", n ? n : ""});
        }
        return RayTracerEngine(*d, std::move(devices), std::move(meta));
    }

public:

    CameraSpec cameraSpec(int32_t index) const {
        CameraSpec c;
        c.index = index;
        if (index >= 0 && index < (int32_t)meta_.size()) { c.id = meta_[index].id; c.imageName = meta_[index].imageName; }
        c.width = cams_.at(index).width;
        c.height = cams_.at(index).height;
        return c;
    }

    SceneInfo inspect() const {
        rt_scene_info i{};
        check(rt_scene_info_get(scene_, &i));
        SceneInfo s;
        for (int32_t k = 0; k < (int32_t)cams_.size(); ++k) s.cameras.push_back(cameraSpec(k));
        s.meshes = i.meshes; s.triangles = i.triangles; s.spheres = i.spheres; s.planes = i.planes;
        return s;
    }

    /* render(format:cameraIndex:progress:).  `format` is accepted for signature parity (the
     * reference ignores it too once the scene is loaded).  Throws RenderError. */
    RenderResult render(SceneFormat /*format*/, int32_t cameraIndex, const ProgressFn& progress = {}) {
        if (!scene_) throw RenderError(RT_ERR_NO_SCENE, "No scene loaded. Can't render.");
        if (cameraIndex < 0 || cameraIndex >= (int32_t)cams_.size())
            throw RenderError(RT_ERR_INVALID_CAMERA, "Invalid camera index");
        RenderResult r;
        r.camera = cameraSpec(cameraIndex);
        r.fileName = r.camera.imageName;
        const int64_t W = std::max<int32_t>(1, r.camera.width), H = std::max<int32_t>(1, r.camera.height);
        r.rgb.resize((size_t)(W * H * 3));
        r.rgba8.resize((size_t)(W * H * 4));
        rt_stats st{};
        struct Ctx { const ProgressFn* fn; };
        Ctx ctx{&progress};
        rt_progress_fn cb = nullptr;
        if (progress) {
            cb = [](void* user, int32_t done, int32_t total) -> int {
                const Ctx* c = static_cast<const Ctx*>(user);
                RenderProgress p{double(done) / double(total > 0 ? total : 1),
                                 "Row " + std::to_string(done) + "/" + std::to_string(total)};
                return (*c->fn)(p) ? 1 : 0;
            };
        }
        check(rt_render(scene_, cameraIndex, 0, 1, r.rgb.data(), r.rgba8.data(), &st, cb, &ctx));
        r.stats = toStats(st);
        return r;
    }

    /* The render is `async` in the reference (renderRGBA8Async, RayTracer.swift:137-205): a
     * caller may keep several in flight.  submit() enqueues a render of camera `cameraIndex`
     * into page-locked buffers (PinnedBuffer; W*H*4 bytes RGBA8, and/or W*H*3 doubles) that
     * must stay alive until wait(ticket) returns; at most RT_MAX_IN_FLIGHT renders may be
     * pending (RenderError RT_ERR_BUSY).  Renders in flight overlap on the GPUs.
     * kernelTime: time the kernels with HIP events (RenderStats::kernel_ms, else 0). */
    int64_t submit(int32_t cameraIndex, uint8_t* pinnedRgba8, double* pinnedRgb = nullptr, bool kernelTime = false) {
        if (!scene_) throw RenderError(RT_ERR_NO_SCENE, "No scene loaded. Can't render.");
        if (cameraIndex < 0 || cameraIndex >= (int32_t)cams_.size())
            throw RenderError(RT_ERR_INVALID_CAMERA, "Invalid camera index");
        int64_t t = -1;
        check(rt_render_submit(scene_, cameraIndex, 0, 1, pinnedRgb, pinnedRgba8,
                               kernelTime ? RT_RENDER_KERNEL_TIME : 0u, &t));
        return t;
    }
    RenderStats wait(int64_t ticket) {
        rt_stats st{};
        check(rt_render_wait(scene_, ticket, &st));
        return toStats(st);
    }

    /* renderAll(progress:): every camera in order, progress as one fraction over all rows. */
    std::vector<RenderResult> renderAll(const ProgressFn& progress = {}) {
        std::vector<RenderResult> out;
        int64_t totalRows = 0, offset = 0;
        for (const auto& c : cams_) totalRows += std::max(1, c.height);
        for (int32_t k = 0; k < (int32_t)cams_.size(); ++k) {
            const int64_t h = std::max(1, cams_[k].height);
            ProgressFn sub;
            if (progress) {
                sub = [&, h](const RenderProgress& p) {
                    return progress(RenderProgress{(double(offset) + p.fraction * double(h)) / double(totalRows),
                                                   "Camera " + std::to_string(k + 1) + "/" + std::to_string(cams_.size())});
                };
            }
            out.push_back(render(SceneFormat::Auto, k, sub));
            offset += h;
        }
        if (progress) progress(RenderProgress{1.0, "Done"});
        return out;
    }

private:
    static RenderStats toStats(const rt_stats& st) {
        RenderStats r;
        r.meshes = st.meshes; r.triangles = st.triangles; r.spheres = st.spheres; r.planes = st.planes;
        r.primary_rays = st.primary_rays; r.shadow_rays = st.shadow_rays; r.secondary_rays = st.secondary_rays;
        r.rays = st.primary_rays + st.shadow_rays;
        r.milliseconds = st.milliseconds; r.kernel_ms = st.kernel_ms;
        r.shadow_rays_traced = st.shadow_rays_traced;
        r.rewalked = st.rewalked;
        return r;
    }
    rt_scene* scene_ = nullptr;
    std::vector<rt_camera> cams_;
    std::vector<CameraMeta> meta_;
};

/* Page-locked output buffer (rt_host_alloc): rt_render writes such buffers directly. */
template <class T>
class PinnedBuffer {
public:
    explicit PinnedBuffer(size_t n) : n_(n) {
        void* p = nullptr;
        check(rt_host_alloc((uint64_t)(n * sizeof(T)), &p));
        p_ = static_cast<T*>(p);
    }
    ~PinnedBuffer() { rt_host_free(p_); }
    PinnedBuffer(const PinnedBuffer&) = delete;
    PinnedBuffer& operator=(const PinnedBuffer&) = delete;
    T* data() { return p_; }
    const T* data() const { return p_; }
    size_t size() const { return n_; }
    T& operator[](size_t i) { return p_[i]; }

private:
    T* p_ = nullptr;
    size_t n_ = 0;
};

}  // namespace myrt

#endif /* MYRT_RT_ENGINE_HPP */
