// C++ host driving the renderer core through include/rt_engine.hpp (the RayTracerEngine
// mirror) and the C ABI, as SURVEY.md §8(b) asks ("tests drive the shim from C++").
// Test infrastructure: the GPU mode checks every render against the CPU oracle
// (oracle/liboracle.so, a restatement of the reference) on the same rt_scene_desc.
//
//   engine_test cpu   no GPU: scene creation and pinned allocation fail with RenderError
//                     carrying the rtcore code (no CPU fallback exists)
//   engine_test gpu   render / renderAll / inspect / progress / cancel / invalid camera /
//                     page-locked output, parity <= 1e-5 L-inf, exact RGBA8, equal ray counts
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "rt_engine.hpp"

extern "C" {
typedef struct oracle_stats {
    int64_t primary_rays, shadow_rays, secondary_rays, node_visits;
    int64_t node_fetches, tri_tests, smooth_hits, pixels;
    double milliseconds;
    int32_t threads;
    int64_t shadow_rays_used;
} oracle_stats;
int32_t oracle_scene_create(const rt_scene_desc* desc, void** out);
void oracle_scene_destroy(void* s);
int32_t oracle_render(void* scene, int32_t camera_index, int32_t chunk_first, int32_t chunk_step,
                      int32_t nthreads, double* out_rgb, uint8_t* out_rgba8, oracle_stats* stats);
}

static int g_fail = 0;
#define EXPECT(c, ...)                                                   \
    do {                                                                 \
        if (!(c)) {                                                      \
            std::fprintf(stderr, "FAIL %s:%d: %s | ", __FILE__, __LINE__, #c); \
            std::fprintf(stderr, __VA_ARGS__);                           \
            std::fprintf(stderr, "\n");                                  \
            ++g_fail;                                                    \
        }                                                                \
    } while (0)

static rt_vec3 V(double x, double y, double z) { return rt_vec3{x, y, z}; }

// Scene storage (rt_scene_desc points into it).
struct SceneData {
    std::vector<rt_material> mats;
    std::vector<rt_point_light> lights;
    std::vector<rt_camera> cams;
    std::vector<rt_object> objs;
    std::vector<std::vector<double>> pos;
    std::vector<std::vector<int32_t>> idx;
    rt_scene_desc desc{};
    void finish(rt_vec3 bg, rt_vec3 ambient, int depth) {
        desc = rt_scene_desc{};
        desc.background_color = bg;
        desc.ambient_light = ambient;
        desc.shadow_ray_epsilon = 1e-3;
        desc.intersection_test_epsilon = 1e-6;
        desc.max_recursion_depth = depth;
        desc.num_materials = (int32_t)mats.size(); desc.materials = mats.data();
        desc.num_point_lights = (int32_t)lights.size(); desc.point_lights = lights.data();
        desc.num_objects = (int32_t)objs.size(); desc.objects = objs.data();
        desc.num_cameras = (int32_t)cams.size(); desc.cameras = cams.data();
    }
};

static rt_camera lookat(int w, int h, rt_vec3 pos, rt_vec3 at, double fovy) {
    rt_camera c{};
    c.type = RT_CAM_LOOKAT; c.width = w; c.height = h; c.num_samples = 1;
    c.position = pos; c.gaze_point = at; c.gaze = V(0, 0, -1); c.up = V(0, 1, 0);
    c.fovy = fovy; c.near_distance = 1.0;
    c.near_plane[0] = -1; c.near_plane[1] = 1; c.near_plane[2] = -1; c.near_plane[3] = 1;
    return c;
}

static rt_object mesh_obj(int id, int mat, int smooth, const std::vector<double>& p, const std::vector<int32_t>& ix) {
    rt_object o{};
    o.kind = RT_OBJ_MESH; o.material_id = mat; o.smooth = smooth; o.id = id; o.indices_one_based = 1;
    for (int k = 0; k < 16; ++k) o.transform[k] = (k % 5 == 0) ? 1.0 : 0.0;
    o.positions = p.data(); o.num_positions = (int64_t)p.size() / 3;
    o.indices = ix.data(); o.num_indices = (int64_t)ix.size();
    return o;
}

// C1: one triangle, lookAt camera, one point light.
static void scene_c1(SceneData& s, int w, int h) {
    s.pos.push_back({-1, -1, -3, 1, -1, -3, 0, 1, -3});
    s.idx.push_back({1, 2, 3});
    rt_material m{};
    m.ambient = V(1, 1, 1); m.diffuse = V(0.8, 0.5, 0.3); m.specular = V(0.5, 0.5, 0.5); m.phong = 32;
    s.mats.push_back(m);
    s.lights.push_back(rt_point_light{V(2, 2, 0), V(3e3, 3e3, 3e3)});
    s.cams.push_back(lookat(w, h, V(0, 0, 0), V(0, 0, -1), 60.0));
    s.objs.push_back(mesh_obj(1, 1, 0, s.pos[0], s.idx[0]));
    s.finish(V(10, 20, 30), V(25, 25, 25), 6);
}

// A smooth displaced grid under a flat mirror box; two cameras, two lights, bounces.
static void scene_grid(SceneData& s) {
    const int n = 40;
    std::vector<double> p;
    std::vector<int32_t> ix;
    for (int j = 0; j <= n; ++j)
        for (int i = 0; i <= n; ++i) {
            const double x = -3.0 + 6.0 * i / n, z = -6.0 + 6.0 * j / n;
            const float y = (float)(-1.0 + 0.25 * std::sin(1.7 * x) * std::cos(1.3 * z));
            p.insert(p.end(), {(double)(float)x, (double)y, (double)(float)z});
        }
    for (int j = 0; j < n; ++j)
        for (int i = 0; i < n; ++i) {
            const int a = j * (n + 1) + i + 1, b = a + 1, c = a + n + 1, d = c + 1;
            ix.insert(ix.end(), {a, c, b, b, c, d});
        }
    s.pos.push_back(p);
    s.idx.push_back(ix);
    // unit cube, 12 triangles
    std::vector<double> cp;
    for (int k = 0; k < 8; ++k) cp.insert(cp.end(), {(k & 1) ? 0.6 : -0.6, (k & 2) ? 0.6 : -0.6, (k & 4) ? -2.4 : -3.6});
    std::vector<int32_t> ci = {1, 3, 2, 2, 3, 4, 5, 6, 7, 6, 8, 7, 1, 2, 5, 2, 6, 5,
                               3, 7, 4, 4, 7, 8, 1, 5, 3, 3, 5, 7, 2, 4, 6, 4, 8, 6};
    s.pos.push_back(cp);
    s.idx.push_back(ci);
    rt_material g{};
    g.ambient = V(0.1, 0.1, 0.1); g.diffuse = V(0.5, 0.6, 0.4); g.specular = V(0.3, 0.3, 0.3); g.phong = 16;
    rt_material m{};
    m.ambient = V(0.05, 0.05, 0.05); m.diffuse = V(0.2, 0.2, 0.2); m.specular = V(0.6, 0.6, 0.6); m.phong = 64;
    m.mirror = V(0.7, 0.7, 0.75); m.type = RT_MAT_MIRROR;
    s.mats = {g, m};
    s.lights.push_back(rt_point_light{V(3, 5, 1), V(9000, 9000, 9000)});
    s.lights.push_back(rt_point_light{V(-4, 2, -1), V(3000, 2500, 2000)});
    s.cams.push_back(lookat(120, 90, V(0, 1.2, 2.5), V(0, -0.6, -3.0), 55.0));
    rt_camera np{};
    np.type = RT_CAM_NEARPLANE; np.width = 64; np.height = 52; np.num_samples = 4;
    np.position = V(0.5, 0.8, 2.0); np.gaze = V(-0.1, -0.3, -1.0); np.up = V(0, 1, 0);
    np.fovy = NAN; np.near_distance = 1.0;
    np.near_plane[0] = -0.5; np.near_plane[1] = 0.5; np.near_plane[2] = -0.4; np.near_plane[3] = 0.4;
    s.cams.push_back(np);
    s.objs.push_back(mesh_obj(1, 1, 1, s.pos[0], s.idx[0]));
    s.objs.push_back(mesh_obj(2, 2, 0, s.pos[1], s.idx[1]));
    s.finish(V(8, 12, 20), V(20, 20, 20), 4);
}

static void compare_with_oracle(const rt_scene_desc& desc, const myrt::RenderResult& r, int cam, const char* what) {
    void* o = nullptr;
    EXPECT(oracle_scene_create(&desc, &o) == RT_OK, "%s: oracle scene", what);
    const size_t px = (size_t)r.camera.width * r.camera.height;
    std::vector<double> ref(px * 3);
    std::vector<uint8_t> ref8(px * 4);
    oracle_stats st{};
    EXPECT(oracle_render(o, cam, 0, 1, 0, ref.data(), ref8.data(), &st) == RT_OK, "%s: oracle render", what);
    oracle_scene_destroy(o);
    double linf = 0;
    for (size_t i = 0; i < ref.size(); ++i) linf = std::max(linf, std::fabs(ref[i] - r.rgb[i]));
    EXPECT(linf <= 1e-5, "%s: L-inf %.3e", what, linf);
    EXPECT(std::memcmp(ref8.data(), r.rgba8.data(), ref8.size()) == 0, "%s: RGBA8 differs", what);
    EXPECT(r.stats.primary_rays == st.primary_rays && r.stats.shadow_rays == st.shadow_rays &&
               r.stats.secondary_rays == st.secondary_rays,
           "%s: rays %lld/%lld/%lld vs oracle %lld/%lld/%lld", what, (long long)r.stats.primary_rays,
           (long long)r.stats.shadow_rays, (long long)r.stats.secondary_rays, (long long)st.primary_rays,
           (long long)st.shadow_rays, (long long)st.secondary_rays);
    std::printf("%s: L-inf %.3e, rays %lld (+%lld secondary)\n", what, linf, (long long)r.stats.rays,
                (long long)r.stats.secondary_rays);
}

// The C1 scene as a scene file (RayTracerEngine.init(data:), RayTracer.swift:35-36)
static const char* kC1Json = R"({"Scene": {
  "MaxRecursionDepth": "6", "BackgroundColor": "10 20 30", "ShadowRayEpsilon": "1e-3",
  "IntersectionTestEpsilon": "1e-6",
  "Cameras": {"Camera": {"_id": "1", "_type": "lookAt", "Position": "0 0 0", "GazePoint": "0 0 -1",
              "Up": "0 1 0", "FovY": "60", "NearDistance": "1", "ImageResolution": "80 60",
              "ImageName": "c1_file.png"}},
  "Lights": {"AmbientLight": "25 25 25", "PointLight": {"_id": "1", "Position": "2 2 0", "Intensity": "3e3 3e3 3e3"}},
  "Materials": {"Material": {"_id": "1", "AmbientReflectance": "1 1 1", "DiffuseReflectance": "0.8 0.5 0.3",
                "SpecularReflectance": "0.5 0.5 0.5", "PhongExponent": "32"}},
  "VertexData": "-1 -1 -3 1 -1 -3 0 1 -3",
  "Objects": {"Mesh": {"_id": "1", "_shadingMode": "flat", "Material": "1", "Faces": "1 2 3"}}}})";

static int run_cpu() {
    // scene files: a decode error is RT_ERR_SCENE_FILE; a good file then needs the device
    try {
        auto e = myrt::RayTracerEngine::fromData("{\"Scene\": {\"BackgroundColor\": \"1 2\"}}");
        EXPECT(false, "bad scene file accepted");
    } catch (const myrt::RenderError& e) {
        EXPECT(e.code == RT_ERR_SCENE_FILE && std::string(e.what()).find("requires 3") != std::string::npos,
               "code %d (%s)", e.code, e.what());
    }
    try {
        auto e = myrt::RayTracerEngine::fromData(kC1Json);
        EXPECT(false, "scene creation succeeded without a GPU");
    } catch (const myrt::RenderError& e) {
        EXPECT(e.code == RT_ERR_DEVICE, "code %d (%s)", e.code, e.what());
    }
    SceneData s;
    scene_c1(s, 32, 32);
    try {
        myrt::RayTracerEngine eng(s.desc);
        EXPECT(false, "scene creation succeeded without a GPU");
    } catch (const myrt::RenderError& e) {
        EXPECT(e.code == RT_ERR_DEVICE, "code %d (%s)", e.code, e.what());
    }
    try {
        myrt::PinnedBuffer<double> b(1024);
        EXPECT(false, "pinned allocation succeeded without a GPU");
    } catch (const myrt::RenderError& e) {
        EXPECT(e.code == RT_ERR_OOM, "code %d", e.code);
    }
    EXPECT(rt_rows_for_chunks(1080, 0, 1) == 1080 && rt_rows_for_chunks(20, 1, 2) == 8, "rows_for_chunks");
    return g_fail;
}

static int run_gpu() {
    {   // C1 through render(), with progress
        SceneData s;
        scene_c1(s, 96, 64);
        myrt::RayTracerEngine eng(s.desc, {0}, {{"1", "c1.png"}});
        std::vector<double> seen;
        auto r = eng.render(myrt::SceneFormat::Auto, 0, [&](const myrt::RenderProgress& p) {
            seen.push_back(p.fraction);
            return true;
        });
        EXPECT(r.fileName == "c1.png" && r.camera.width == 96 && r.camera.height == 64, "camera spec");
        EXPECT(!seen.empty() && seen.back() == 1.0, "progress did not reach 1");
        for (size_t i = 1; i < seen.size(); ++i) EXPECT(seen[i] >= seen[i - 1], "progress not monotone");
        compare_with_oracle(s.desc, r, 0, "c1");
        const auto info = eng.inspect();
        EXPECT(info.meshes == 1 && info.triangles == 1 && info.cameras.size() == 1, "inspect");
        // invalid camera index -> NSError code -10 (RayTracer.swift:151-154)
        try {
            eng.render(myrt::SceneFormat::Json, 3);
            EXPECT(false, "invalid camera accepted");
        } catch (const myrt::RenderError& e) {
            EXPECT(e.code == RT_ERR_INVALID_CAMERA, "code %d", e.code);
        }
        // cancellation from the progress callback
        try {
            eng.render(myrt::SceneFormat::Auto, 0, [](const myrt::RenderProgress&) { return false; });
            EXPECT(false, "cancel ignored");
        } catch (const myrt::RenderError& e) {
            EXPECT(e.code == RT_ERR_CANCELLED, "code %d", e.code);
        }
        // page-locked output: rt_render writes it directly; same pixels
        myrt::PinnedBuffer<double> pin((size_t)96 * 64 * 3);
        rt_stats st{};
        myrt::check(rt_render(eng.handle(), 0, 0, 1, pin.data(), nullptr, &st, nullptr, nullptr));
        EXPECT(std::memcmp(pin.data(), r.rgb.data(), r.rgb.size() * sizeof(double)) == 0, "pinned output differs");
        // renders in flight (submit / wait): every one delivers the same image, waits out of order
        std::vector<std::unique_ptr<myrt::PinnedBuffer<uint8_t>>> bufs;
        std::vector<int64_t> tickets;
        for (int k = 0; k < RT_MAX_IN_FLIGHT; ++k) {
            bufs.emplace_back(new myrt::PinnedBuffer<uint8_t>((size_t)96 * 64 * 4));
            std::memset(bufs.back()->data(), 0, bufs.back()->size());
            tickets.push_back(eng.submit(0, bufs.back()->data()));
        }
        try {
            myrt::PinnedBuffer<uint8_t> more((size_t)96 * 64 * 4);
            eng.submit(0, more.data());
            EXPECT(false, "a render past RT_MAX_IN_FLIGHT was accepted");
        } catch (const myrt::RenderError& e) {
            EXPECT(e.code == RT_ERR_BUSY, "busy code %d", e.code);
        }
        for (int k = RT_MAX_IN_FLIGHT - 1; k >= 0; --k) {
            const auto ws = eng.wait(tickets[k]);
            EXPECT(std::memcmp(bufs[k]->data(), r.rgba8.data(), r.rgba8.size()) == 0, "in-flight render %d differs", k);
            EXPECT(ws.shadow_rays == r.stats.shadow_rays && ws.primary_rays == r.stats.primary_rays,
                   "in-flight render %d counts", k);
        }
    }
    {   // a scene file decoded by the library (RayTracerEngine.init(data:)) renders like its descriptor
        auto eng = myrt::RayTracerEngine::fromData(kC1Json, myrt::SceneFormat::Json);
        auto r = eng.render(myrt::SceneFormat::Auto, 0);
        EXPECT(r.fileName == "c1_file.png" && r.camera.width == 80 && r.camera.height == 60, "file camera spec");
        rt_scene_file* f = nullptr;
        myrt::check(rt_scene_file_parse(kC1Json, std::strlen(kC1Json), RT_SCENE_FORMAT_AUTO, nullptr, &f));
        compare_with_oracle(*rt_scene_file_desc(f), r, 0, "c1 scene file");
        rt_scene_file_destroy(f);
    }
    {   // two cameras (lookAt + nearPlane with 4 spp), mirror bounces, renderAll
        SceneData s;
        scene_grid(s);
        myrt::RayTracerEngine eng(s.desc, {0}, {{"a", "grid_a.png"}, {"b", "grid_b.png"}});
        std::vector<std::string> msgs;
        double last = -1;
        auto all = eng.renderAll([&](const myrt::RenderProgress& p) {
            EXPECT(p.fraction >= last, "renderAll progress not monotone");
            last = p.fraction;
            msgs.push_back(p.message);
            return true;
        });
        EXPECT(all.size() == 2 && !msgs.empty() && msgs.back() == "Done" && last == 1.0, "renderAll progress");
        compare_with_oracle(s.desc, all[0], 0, "grid cam0");
        compare_with_oracle(s.desc, all[1], 1, "grid cam1 (nearPlane, 4 spp)");
        EXPECT(all[0].stats.secondary_rays > 0, "no mirror bounces traced");
        const auto info = eng.inspect();
        EXPECT(info.meshes == 2 && info.triangles == 2 * 40 * 40 + 12, "inspect triangles %lld",
               (long long)info.triangles);
    }
    return g_fail;
}

int main(int argc, char** argv) {
    const std::string mode = argc > 1 ? argv[1] : "cpu";
    int rc = 0;
    try {
        rc = mode == "gpu" ? run_gpu() : run_cpu();
    } catch (const std::exception& e) {
        std::fprintf(stderr, "FAIL: uncaught %s\n", e.what());
        rc = 1;
    }
    std::printf("%s: %s\n", mode.c_str(), rc ? "FAILED" : "ok");
    return rc ? 1 : 0;
}
