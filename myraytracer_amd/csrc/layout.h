// layout.h — device-resident scene layout shared by the host builder (scene.cpp)
// and the HIP kernels (render.hip).  Everything is IEEE binary64 like the
// reference (RTContext.swift:13-16).
//
// HBM layout (per device replica):
//   recs    : WRec[]    128-B two-child BVH records, one per INNER node of every
//             BLAS and of the TLAS (RT/Accelearion/BVH.swift:16-30 nodes, re-laid so
//             that a parent holds both children's bounds -> one cache line per
//             visited inner node instead of two 56-B node reads + a re-test).
//   tris    : TriRec[]  80-B {v0, e1, e2, last-in-leaf} in BVH LEAF order, so a leaf
//             is a contiguous run (removes primIdx -> prims -> triangles indirection,
//             RTContext.swift:573-581).
//   normals : double[9] per TriRec (n0, n1, n2), read only for the final hit.
//   insts   : DInstance[] (RTContext.swift:43-61) + TLAS leaf instance lists.
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace myrt {

// Child reference encoding used in WRec.ref[], stack entries and instance roots:
//   ref >= 0 : inner node -> index of its WRec
//   ref <  0 : leaf       -> ~ref = index of its first TriRec (BLAS leaf), or
//                            tlas_leaf_base + index of its first TLAS leaf-list entry;
//                            the run ends at the entry whose `last` flag is set.
struct alignas(128) WRec {
    double lo[2][3];      // child c aabbMin (x,y,z)
    double hi[2][3];      // child c aabbMax
    int32_t ref[2];       // child refs (c = 0 is the reference's L = leftFirst, c = 1 is R)
    int32_t pad[6];
};
static_assert(sizeof(WRec) == 128, "WRec must be one 128-B line");

// BLAS record with float32 bounds, used when every BLAS bound is exactly a float (always
// true for PLY meshes without motion blur: positions are float32 widened to double,
// PLYReader.swift:85-102, and node bounds are min/max of vertex coordinates).  Widening
// back to double is exact, so the FP64 slab test sees the same values from half the bytes.
struct alignas(64) CRec {
    float lo[2][3], hi[2][3];
    int32_t ref[2];
    int32_t pad[2];
};
static_assert(sizeof(CRec) == 64, "CRec is one 64-B half line");

struct alignas(16) TriRec {
    double v0[3], e1[3], e2[3];
    int32_t last;         // 1 = last triangle of its leaf
    int32_t prim;         // identity mode: owning instance; otherwise the reference `triangles[]` index
};
static_assert(sizeof(TriRec) == 80, "TriRec is 80 B");

// Leaf-ordered triangle with float32 vertices, used when every vertex is exactly a float
// (PLY meshes).  The kernel rebuilds e1 = v1 - v0 and e2 = v2 - v0 in FP64 from the
// widened vertices - the same operation on the same values as the host's TriRec edges
// (RTContext.swift:204-208), so the MT test sees identical edges from 48 B instead of 80 B.
struct alignas(16) CTri {
    float v0[3], v1[3], v2[3];
    int32_t last;
    int32_t prim;
    int32_t pad;
};
static_assert(sizeof(CTri) == 48, "CTri is 48 B");

// Four-wide node of the conservative FP32 walk (wide.h), built for identity scenes by collapsing
// the unified TLAS + BLAS tree (scene.cpp build_wide).  Only the reference's LEAVES matter to
// the result: with every 1/d finite, child boxes nest inside parent boxes (node bounds are
// min/max over a subset of the parent's primitives, BVH.swift:108-124, 184-185) and the FP64
// slab test is monotone in the bounds, so intersectBLAS tests exactly the triangles whose leaf
// box passes hitAABB.  Inner boxes here are rounded outward to float; the walk widens them
// further per render (RenderParams::wdelta) so a conservative FP32 test passes whenever the
// reference's FP64 test of any leaf below passes.  Leaf boxes are then checked exactly (FP64,
// lbox) before a hit is accepted.  Slots [axis][child], SoA per axis.
// The node array holds EIGHT copies of the tree, one per ray-direction octant o (bit a of o set:
// d[a] < 0; copy o starts at node o * RenderParams::wide_copy): in copy o a node's rows are
// already the near and far planes of that octant (near = the box minimum along a when d[a] >= 0,
// the maximum otherwise) and its slots are in front-to-back order for directions of that octant
// (scene.cpp wide_octant_copies), so a lane reads fixed rows and visits slots in memory order.
struct alignas(128) W4Node {
    float pnear[3][4];    // slot c's near plane along axis a: pnear[a][c] (rounded outward)
    int32_t ref[4];       // >= 0: node index within the copy; < 0: ~first TriRec of a reference leaf run
    float pfar[3][4];     // ... far plane; an empty slot has pnear = pfar = +inf (never hit)
    int32_t pad[4];
};
static_assert(sizeof(W4Node) == 128, "W4Node is one 128-B line");
static_assert(offsetof(W4Node, pfar) == offsetof(W4Node, pnear) + 64, "near/far rows 64 B apart");

// Per instance of a transformed scene's four-wide walk (wide.h tw_walk): the exact FP64 box of
// the TLAS leaf holding the instance (world space: tested when the walk enters the instance,
// the reference's intersectTLAS leaf test, RTContext.swift:632-646), the largest |coordinate| of
// its BLAS's boxes (local space: the per-ray widening bound) and its BLAS's four-wide root.
struct DWideInst {
    double tbox[6];       // lo x, y, z, hi x, y, z
    double bcoord;
    int32_t wroot;        // >= 0 node index, < 0 a single leaf run (~first TriRec)
    int32_t pad;
};
static_assert(sizeof(DWideInst) == 64, "DWideInst is 64 B");

// Flattened instance tree of a transformed scene (scene.cpp build_fit, wide.h fit_walk): one
// world-space four-wide tree over every (instance, BLAS leaf run) pair; its terminal slot ~p names
// pair p: the leaf run's first TriRec (shared by the instances of one mesh) and the instance.
struct DFitPair {
    int32_t t0;
    int32_t inst;
};

struct DMaterial {        // ParsingKit Material fields used by trace()
    double ambient[3], diffuse[3], specular[3], mirror[3], absorption[3];
    double phong, ior, absorption_index, roughness;
    int32_t type, pad;
};

struct DPointLight { double position[3], intensity[3]; };

struct DInstance {        // Instance (RTContext.swift:43-61) + its BLAS entry point
    double w2l[16];       // worldToLocal, column-major
    double l2w[16];       // localToWorld
    double nmat[9];       // normalMatrix = inverse(M3)^T, column-major
    double motion[3];     // instanceMotion
    double tri_motion[3]; // Triangle.motionBlur of the mesh (uniform per BLAS)
    double root_lo[3], root_hi[3];   // BLAS root node bounds (tested first, RTContext.swift:567-571)
    int32_t root_ref;     // BLAS root ref (global)
    int32_t material;     // materialOverride (always set by makeInstance callers)
    int32_t smooth;       // prim shadingMode == .smooth
    int32_t det_neg;      // simd_determinant(M3) < 0
    int32_t kind;         // BLAS primitive kind: kPrimTriangles / kPrimSphere / kPrimPlane
    int32_t pad;
};

// Single-primitive BLASes of Sphere / Plane objects (RTContext.swift:122-192) keep their
// primitive in one TriRec: sphere = {v0 = center, e1.x = radius}, plane = {v0 = center,
// e1 = normal}.  Every sphere/plane is its own instance, so the kind lives in DInstance.
constexpr int32_t kPrimTriangles = 0, kPrimSphere = 1, kPrimPlane = 2;

struct DAreaLight { double position[3], normal[3], radiance[3], size; };   // ParsingKit AreaLight
constexpr int kJitterCells = 100;    // buildStratifiedJitter 10x10 table (Object+Extension.swift:646-659)

struct DTlasLeafEntry { int32_t inst; int32_t last; };

// Area-light frames (render_full.h): k_events walks every path once to count the jitterIndex
// increments; it also logs each closest hit, so render_full shades the same paths without
// walking them again.  Walk k of pixel q (packed selection index) sits at [k * stride + q].
struct DHitRec { double t, u, v; int32_t tri, inst; };
// A logged walk's ray, for the node-parallel shading pass (render_full.h k_shade): its origin,
// direction and time, and the pixel's jitterIndex when the node is shaded (from the pixel's start).
struct DNodeRec { double o[3], d[3], time; int32_t jofs, hit; };

// A queued mirror/conductor bounce ray (compacted bounce render, render.hip k_bounce): the
// child trace(depth + 1) of one sample plus what its parent level adds back,
// Lo_parent + M_parent * trace(depth + 1) (Object+Extension.swift:189-206, 252-275).
// Records are compacted per level (render.hip q_reserve: a level holds only its rays); `parent`
// is the index of the record one level up (-1 at level 1), so a ray that ends resolves its sample
// backward along the parents.
struct alignas(128) BounceRec {
    double o[3], d[3];        // the reflected ray (origin p + N * shadowRayEpsilon, tMin 0)
    double Lo[3], M[3];       // the parent level's radiance and its mirror/Fresnel multiplier
    unsigned long long rng;   // the sample's PCG32 state after the parent's draws (roughness)
    double time;              // the sample's ray time (instance motion)
    int32_t i, j;             // pixel
    int32_t parent;           // the parent level's record (index into RenderParams::bounce), -1 at level 1
    int32_t pad;
};
static_assert(sizeof(BounceRec) == 128, "BounceRec is one 128-B line");

// Camera + frame constants precomputed on the host (Object+Extension.swift:58-93)
struct DCamera {
    double eye[3], u[3], v[3], w[3];
    double q00[3];
    double du, dv, nd;
    double aperture, focus;
    int32_t width, height, samples, n;   // samples = max(1, numSamples); n = Int(sqrt(samples))
};

struct RenderParams {
    const WRec* recs;
    const CRec* crecs;               // compact copy of records [0, compact_limit)
    const CTri* ctris;               // compact triangles (nullptr = use tris)
    const TriRec* tris;
    const double* normals;
    const DInstance* insts;
    const DTlasLeafEntry* tlas_leaf;
    const DMaterial* mats;
    const DPointLight* plights;
    double tlas_root_lo[3], tlas_root_hi[3];
    int32_t tlas_root_ref;
    int32_t has_tlas;
    int32_t tlas_leaf_base;          // TriRec count: ~ref >= base means a TLAS leaf
    int32_t identity;                // unified TLAS+BLAS walk allowed (scene.h HostScene::identity)
    int32_t num_mats;
    int32_t num_plights;
    DCamera cam;
    double eps, shadow_eps;
    double prune_rel, prune_abs;     // conservative t-pruning margins (DESIGN.md "H3")
    double background[3], ambient[3];
    int32_t max_depth;
    int32_t chunk_first, chunk_step, num_chunks;   // selected 8-row chunks
    // output row of chunk c, row r: ((c - out_first) / out_step) * 8 + r.  Packed selection
    // rows: out_first = chunk_first, out_step = chunk_step; full-frame layout (rows at their
    // image positions, RT_RENDER_FRAME_LAYOUT): out_first = 0, out_step = 1.
    int32_t out_first, out_step;
    int32_t stack_depth;             // LDS stack entries per lane
    int32_t count_ref;               // COUNT launches: walk + tally in reference order (device.h Counts)
    int32_t xcd_remap;               // megakernel: tiles per XCD run (device.h xcd_tile; <= 1 = identity)
    int32_t compact_limit;           // records below this index are read from crecs
    int32_t fast_rcp;                // every Moeller-Trumbore |det| >= eps lies in [2^-700, 2^1000]
                                     // (host bound): 1/det by device.h rcp_rn, bit-identical
    const DAreaLight* alights;
    const double* jitter;            // [0..99] jitterX, [100..199] jitterY
    const long long* jstart;         // area lights: per-pixel first jitterIndex (packed rows)
    long long* events;               // k_events output: per-pixel area-light evaluations
    int32_t num_alights;
    int32_t has_special;             // spheres / planes present (general walk tests kinds)
    // maxRecursionDepth > kMaxDepthGPU (render_full<.., DEEP>): trace() levels beyond the
    // per-lane private frames live in `deep`, [level - kMaxDepthGPU - 1][lane of the launch];
    // a launch covers selected chunks [slot_base, slot_base + gridDim.x / tiles-per-chunk)
    void* deep;
    int32_t slot_base;
    // compacted bounce render (render.hip k_bounce); bounce == nullptr: the bounce megakernel.
    // Level L's rays sit in kQRegions regions of qhdr[kQHdrCap + L] records from record qhdr[L]
    // on; region r's count is the counter q_counter(L, r) (wave-level atomic reservation,
    // q_reserve).  qneed (host-mapped, or null): each level's largest region count, written by
    // k_queue_done, so the host can grow the arena and render an overflowed frame again.
    BounceRec* bounce;
    unsigned long long* qhdr;
    unsigned long long* qneed;
    int64_t qrecs;                   // records in the arena
    int32_t qlevels;                 // levels the arena holds
    double* out_rgb;                 // packed rows of the selected chunks
    uint8_t* out_rgba8;
    unsigned long long* counters;    // [0] shadow rays cast, [1] secondary rays, [2..12] work counters,
                                     // [13] shadow rays traversed, [16..25] per-iteration divergence
                                     // breakdown (rt_work_counters; kCounterWords)
    unsigned long long* wave_times;  // debug (rt_debug_wave_times): per wave {start, end, tile} in 100 MHz ticks
    // Unified transformed walk (kept at the end, so the fields above keep their kernel-argument
    // offsets and scalar-load grouping; profiles/r03y_bisect.txt)
    int32_t ut;                      // unified transformed walk allowed (device.h ut_walk; stack bound)
    int32_t tlas_rec_base;           // records [tlas_rec_base, ...) are TLAS records (ut_walk)
    int32_t ut_marker_base;          // leaf refs ~e with e >= this are instance markers (ut_walk)
    int32_t hit_slots;               // logged walks per pixel (DHitRec; 0 = render_full walks them all)
    DHitRec* hits;
    int64_t hit_stride;              // pixels of the selection
    // node-parallel shading of the logged walks (render_full.h k_shade): k_events records each
    // logged walk's ray (nodes) and each pixel's walk count (walks); k_shade writes the direct
    // light of every logged hit (node_lo, 3 doubles, [k * hit_stride + q]); render_full reads it.
    // nullptr = render_full shades every hit itself.
    DNodeRec* nodes;
    double* node_lo;
    int32_t* walks;
    // breadth-first events passes (render_full.h k_level): the log indexed by tree node
    // (1 = chain, 2 = heap; 0 = the k-th walk), nodes per traced sample, per-node flags
    int32_t hit_tree;
    int32_t tree_size;
    uint8_t* nflags;
    int32_t tree_ppw;                // node positions per wave in k_level / k_shade
    // compacted node lists (render.hip k_clist; option compact): the flag-log entries a level pass
    // or the node shading has work for, ascending; per-block counts; list lengths by word
    // (level L: word L, node shading: word kCListShade)
    uint32_t* clist;
    uint32_t* cblk;
    uint32_t* cword;
    // conservative FP32 four-wide walk (wide.h; identity scenes): nodes, the root node, the exact
    // FP64 box of every reference leaf by its first TriRec (6 doubles), the per-render widening of
    // every box (wdelta, world units: covers the FP32 rounding of o*inv for every ray origin of
    // the render) and the FP32 form of eps rounded down.  wide == 0: the binary FP64 walk.
    const W4Node* wnodes;
    const double* lbox;
    int32_t wide;
    int32_t wide_root;
    double wdelta;
    float weps;
    uint32_t wide_copy_bytes;        // bytes of one octant copy of the node array (W4Node)
    // transformed scenes' four-wide walk (wide.h tw_walk; wide_root is then the TLAS's root):
    // nodes [0, tw_tlas_nodes) of each copy are the TLAS's (world space), the rest the BLASes'
    // (local space); TLAS leaves became instance markers ~(ut_marker_base + instance)
    const DWideInst* winst;
    int32_t tw_tlas_nodes;
    float tw_wscale;                 // the local rays' widening factor (option wide_delta_scale / 1000)
    // tile order (render.hip TileOrder; option tile_order): block -> tile of the megakernels, or
    // null = row-major XCD groups (device.h xcd_tile); tile_cost: per tile {start, end} of its
    // wave (s_memrealtime), recorded by the first render of a camera and chunk selection
    const uint32_t* tile_order;
    unsigned long long* tile_cost;
    // flattened instance tree (wide.h fit_walk; option fit): its root node in the same node array
    // and the (leaf run, instance) pairs its terminal slots name; fit == 0: tw_walk
    const DFitPair* fpairs;
    int32_t fit_root;
    int32_t fit;
};

constexpr int kCounterWords = 64;   // u64 words behind RenderParams::counters
// Compacted bounce render arena header (u64 words at RenderParams::qhdr): [L] the first record of
// level L (1..kMaxQueueLevels), [kQHdrCap + L] the records per region of level L, and from word
// kQHdrCnt the (level, region) counters, 128 B apart; k_queue_done zeroes the counters after
// the last level.
constexpr int kMaxQueueLevels = 15;
#ifndef MYRT_QREGION_BITS
#define MYRT_QREGION_BITS 5
#endif
constexpr int kQRegionBits = MYRT_QREGION_BITS;    // <= 6: k_bounce holds one region per lane
constexpr int kQRegions = 1 << kQRegionBits;
constexpr int kQHdrCap = 16, kQHdrCnt = 64, kQCntStride = 16;
constexpr int kQHdrWords = kQHdrCnt + kMaxQueueLevels * kQRegions * kQCntStride;
constexpr int kCounterShadowTraced = 13;
constexpr int kCounterTies = 26;     // wide walks re-walked in reference order (equal-t candidates, wide.h)
constexpr int kMaxDepthGPU = 16;     // trace() levels kept in private memory per lane (deeper: RenderParams::deep)
constexpr int64_t kDeepBytesCap = 8ll << 30;   // device bytes of deep frames per launch batch

// Per-lane traversal stack capacity (device.h Stack: kLds LDS entries + the private rest).
// The reference gives the TLAS walk and each BLAS walk their own 64-entry stacks
// (RTContext.swift:550, 623); one shared stack of 128 holds both at their limits.
constexpr int kStackCap = 128;

}  // namespace myrt
