// scene.h — host-side scene construction for the MI355X renderer core.
//
// Restates what RTContext.init(scene:) (RT/Models/RTContext.swift:94-418) and
// BVHBuilder (RT/Accelearion/BVH.swift:67-250) produce, then re-lays the result
// into the device layout of layout.h.  BVH topology, node bounds and leaf
// primitive order are bit-identical to the reference builder (they decide the
// traversal order); node numbering is free.
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/rtcore.h"
#include "layout.h"

namespace myrt {

// Reference-form BVH (BVH.swift:16-30): node bounds, leftFirst/primitiveCount,
// primitiveIdx permutation.  Nodes are numbered exactly as the Swift builder does.
struct RefBVH {
    std::vector<double> lo, hi;            // 3 per node
    std::vector<int64_t> leftFirst, count; // count > 0 => leaf
    std::vector<int64_t> primIdx;
    int64_t nodesUsed = 0;
    bool isLeaf(int64_t n) const { return count[n] > 0; }
};

// Primitive set handed to the builder (PrimitiveInfo bounds + centroid).
struct PrimSet {
    int64_t n = 0;
    std::vector<double> bmin, bmax, cen;   // 3 per prim, xyz interleaved
};

RefBVH build_ref_bvh(const PrimSet& prims, int maxLeaf = 2, int binCount = 12);
uint64_t ref_bvh_hash(const RefBVH& b, const std::vector<int64_t>& primIndexOf);
int64_t ref_bvh_depth(const RefBVH& b);   // max number of inner nodes on a root-to-leaf path

struct HostCamera { rt_camera c; };

struct HostScene {
    // ---- scene-level parameters
    double eps = 0, shadow_eps = 0;
    double background[3] = {0, 0, 0}, ambient[3] = {0, 0, 0};
    int32_t max_depth = 0;
    std::vector<DMaterial> mats;
    std::vector<DPointLight> plights;
    std::vector<DAreaLight> alights;
    std::vector<double> jitter;            // 2 x kJitterCells (buildStratifiedJitter)
    int32_t num_area_lights = 0;
    bool has_special = false;              // sphere / plane objects present
    std::vector<rt_camera> cams;
    bool has_dielectric = false;
    // ---- device layout (host copies)
    std::vector<WRec> recs;
    std::vector<CRec> crecs;               // float32-bound copy of the BLAS records (if exact)
    int64_t compact_records = 0;           // crecs.size() (kept after the host copy is dropped)
    std::vector<TriRec> tris;
    std::vector<CTri> ctris;               // float32-vertex copy of tris (if every vertex is exact)
    bool compact_tris = false;
    std::vector<double> normals;           // 9 per TriRec
    std::vector<DInstance> insts;
    std::vector<DTlasLeafEntry> tlas_leaf;
    double tlas_root_lo[3] = {0, 0, 0}, tlas_root_hi[3] = {0, 0, 0};
    int32_t tlas_root_ref = 0;
    int64_t tlas_leaf_base = 0;            // TLAS leaf refs are ~(tlas_leaf_base + entry)
    bool has_tlas = false;
    bool identity = false;                 // all instances identity & static (unified walk)
    int64_t blas_records = 0, tlas_records = 0;
    int64_t max_stack = 0;                 // traversal stack entries the general walk needs
    int64_t max_stack_unified = 0;         // ... and the unified identity walk
    double scene_extent = 1.0;             // world bounds diagonal (pruning margin scale)
    double scene_center[3] = {0, 0, 0};    // world bounds center
    double prune_k = 0.0;                  // MT t-error constant (scene.cpp, "pruning margin")
    double max_motion = 0.0;               // largest instance + triangle motion-blur offset
    double det_scale = 0.0;                // >= |e1||e2| * ||A||_F over triangle instances: every
                                           // Moeller-Trumbore |det| <= det_scale * |d_world|
    // ---- conservative FP32 four-wide walk (identity scenes, scene.cpp build_wide)
    std::vector<W4Node> wnodes;
    std::vector<double> lbox;              // 6 per TriRec index: exact box of the leaf run starting there
    int64_t wide_leaves = 0;               // reference leaves under the wide tree
    int32_t wide_root = -1;                // -1: no wide tree
    int64_t wide_copy = 0;                 // nodes per octant copy (wnodes holds eight, layout.h W4Node)
    double wide_coord = 0.0;               // largest |coordinate| of any box (wdelta scale; TLAS boxes
                                           // for transformed scenes)
    // transformed scenes (static, triangles only): TLAS nodes first, then every BLAS's nodes
    std::vector<DWideInst> winst;          // per instance (layout.h DWideInst); empty: identity tree
    int64_t tw_tlas_nodes = 0;
    // flattened instance tree (scene.cpp build_fit): world-space nodes over (leaf run, instance)
    // pairs, appended to wnodes; fit_root < 0: none (tw_walk only)
    std::vector<DFitPair> fpairs;
    int32_t fit_root = -1;
    int64_t fit_nodes = 0, fit_depth = 0;
    double fit_coord = 0.0;                // bound on every magnitude the fit widening covers
    double fit_ms = 0.0;                   // host time of build_fit
    // ---- bookkeeping / debug
    int64_t n_meshes = 0, n_tris = 0, n_spheres = 0, n_planes = 0;
    std::vector<uint64_t> inst_bvh_hash;   // per instance: canonical hash of its BLAS
    uint64_t tlas_hash = 0;
    double build_ms = 0;
};

// Returns RT_OK or a negative status with `err` set.
int32_t build_host_scene(const rt_scene_desc* desc, HostScene& out, std::string& err);

// PLY loading (ply.cpp).  Mirrors PLYLoader.load (RT/Helpers/PLYReader.swift:54-210).
int32_t ply_load(const char* path, std::vector<double>& positions, std::vector<double>& normals,
                 std::vector<float>& texcoords, std::vector<int32_t>& indices, std::string& err);

}  // namespace myrt
