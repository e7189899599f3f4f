// render.hip — MI355X (gfx950) kernels of the renderer core + the rtcore.h C ABI.
//
// Hot path (reference: RT/Extensions/Object+Extension.swift:52-379 render loop +
// trace(); RT/Models/RTContext.swift:476-870 traversal and intersectors):
//   one lane per pixel, one wave per 8x8 pixel tile (8-row chunks, :75-82),
//   primary ray with the per-pixel PCG32 jitter -> TLAS/BLAS closest-hit traversal
//   with FP64 slab tests -> Moeller-Trumbore -> Whitted shading with any-hit shadow
//   rays -> mirror/conductor bounces, all IEEE binary64 (build with -ffp-contract=off).
//
// Traversal visits the surviving nodes in exactly the reference's order (near child
// first, ties to L; RTContext.swift:600-606).  It additionally prunes nodes whose
// entry distance exceeds the current closest hit by a conservative margin
// (tmin > t*(1+prune_rel)+prune_abs), which cannot remove a node holding a hit the
// reference would accept (DESIGN.md "Pruning").
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/rtcore.h"
#include "device.h"
#include "layout.h"
#include "scene.h"

namespace myrt {
namespace dev {
// Per-pixel PCG32 seed (Object+Extension.swift:294)
__device__ __forceinline__ unsigned long long pixel_seed(int i, int j) {
    return (((unsigned long long)j << 32) ^ (unsigned long long)i) + 0x9E3779B97F4A7C15ull;
}

// The reference-order transformed walk as the four-wide transformed walk's fallback (ties, local
// rays out of its FP32 range): out of line, so its registers do not weigh on the wide walk's.
#ifndef MYRT_TW_CALL
#define MYRT_TW_CALL 0
#endif
#if MYRT_TW_CALL
#define MYRT_TW_INLINE __noinline__
#else
#define MYRT_TW_INLINE __forceinline__
#endif
__device__ MYRT_TW_INLINE void ut_closest_call(const RenderParams& P, const V3 o, const V3 d, const V3 inv, double tlo,
                                            double time, Hit& h, Stack& st) {
    h.t = DINF; h.inst = -1; h.tri = -1; h.u = 0; h.v = 0;
    (void)ut_walk<false>(P, o, d, inv, tlo, DINF, time, h, st);
}
__device__ MYRT_TW_INLINE bool ut_occluded_call(const RenderParams& P, const V3 o, const V3 d, double tmax, double time,
                                             Stack& st) {
    Hit hu;
    return ut_walk<true>(P, o, d, rcp(d), 0.0, tmax, time, hu, st);
}

// The flattened instance tree's fallbacks (equal-t ties, world rays out of the FP32 range): the
// reference-order transformed walk.  (Out of line, __noinline__, the megakernel went to 212 VGPRs
// and 144 spills: a call costs the kernel its register budget.)
__device__ __forceinline__ void fit_closest_fallback(const RenderParams& P, const V3 o, const V3 d, double tlo, double time,
                                                  Hit& h, Stack& st) {
    h.t = DINF; h.inst = -1; h.tri = -1; h.u = 0; h.v = 0;
    (void)ut_walk<false>(P, o, d, rcp(d), tlo, DINF, time, h, st);
}
__device__ __forceinline__ bool fit_occluded_fallback(const RenderParams& P, const V3 o, const V3 d, double tmax,
                                                   double time, Stack& st) {
    Hit hu;
    return ut_walk<true>(P, o, d, rcp(d), 0.0, tmax, time, hu, st);
}

// Closest hit of one ray by the scene's walk (WALK, render_kernel).
template <bool COUNT, int WALK, bool WIDE = true>
__device__ __forceinline__ void walk_closest(const RenderParams& P, const V3& o, const V3& d, const V3& inv, double tlo,
                                             double time, Hit& h, Stack& st, Counts& c) {
    if (WALK == kWalkIdentity) {
        uni_closest<COUNT, WIDE>(P, o, d, inv, tlo, h, st, c);
    } else if (WALK == kWalkFit) {
        h.t = DINF; h.inst = -1; h.tri = -1; h.u = 0; h.v = 0;
        if (WIDE && __all(wide_ok(inv))) {
            // the flattened instance tree (wide.h fit_walk); equal-t candidates re-walked in order
            bool tie = false;
            (void)wide_walk<COUNT, false, true>(P, TwWorld{o, d}, inv, tlo, DINF, h, tie, st, c);
            if (__any(tie) && tie) {
                c.ties++;
                fit_closest_fallback(P, o, d, tlo, time, h, st);
            }
            return;
        }
        fit_closest_fallback(P, o, d, tlo, time, h, st);
    } else if (WALK == kWalkTransformed) {
        h.t = DINF; h.inst = -1; h.tri = -1; h.u = 0; h.v = 0;
        if (WIDE && P.wide && P.winst && __all(wide_ok(inv))) {
            // the four-wide walk of transformed scenes (wide.h tw_walk); equal-t candidates and
            // local rays out of its range are re-walked in the reference's order
            bool tie = false, redo = false;
            (void)tw_walk<false>(P, TwWorld{o, d}, tlo, DINF, h, tie, redo, st);
            if (__any(tie || redo) && (tie || redo)) {
                if (tie) c.ties++;
                ut_closest_call(P, o, d, inv, tlo, time, h, st);
            }
            return;
        }
        (void)ut_walk<false>(P, o, d, inv, tlo, DINF, time, h, st);
    } else {
        intersect_closest<COUNT>(P, o, d, inv, tlo, time, h, st, c);
    }
}

// The megakernel's closest hit of a transformed scene with the world ray parked (wide.h
// TwParked): the caller stores it before and reads it back after, so it is not live across the
// walk (MYRT_TW_PARK).
#ifndef MYRT_TW_PARK
#define MYRT_TW_PARK 1
#endif
#ifndef MYRT_FIT_PARK
#define MYRT_FIT_PARK 1      // the flattened-tree walks park the world ray too (read back at each pair)
#endif
template <bool COUNT, class Park>
__device__ __forceinline__ void walk_closest_tw_parked(const RenderParams& P, const Park& pk, double tlo,
                                                       double time, Hit& h, Stack& st, Counts& c) {
    h.t = DINF; h.inst = -1; h.tri = -1; h.u = 0; h.v = 0;
    if (P.wide && P.winst && __all(wide_ok(rcp(pk.d())))) {
        bool tie = false, redo = false;
        (void)tw_walk<false>(P, pk, tlo, DINF, h, tie, redo, st);
        if (__any(tie || redo) && (tie || redo)) {
            if (tie) c.ties++;
            ut_closest_call(P, pk.o(), pk.d(), rcp(pk.d()), tlo, time, h, st);
        }
        return;
    }
    (void)ut_walk<false>(P, pk.o(), pk.d(), rcp(pk.d()), tlo, DINF, time, h, st);
}

// ... and through the flattened instance tree (kWalkFit): the walk reads the parked world ray back
// at each pair, where it forms the local ray
template <bool COUNT, class Park>
__device__ __forceinline__ void walk_closest_fit_parked(const RenderParams& P, const Park& pk, double tlo,
                                                        double time, Hit& h, Stack& st, Counts& c) {
    h.t = DINF; h.inst = -1; h.tri = -1; h.u = 0; h.v = 0;
    if (__all(wide_ok(rcp(pk.d())))) {
        bool tie = false;
        (void)wide_walk<COUNT, false, true>(P, pk, rcp(pk.d()), tlo, DINF, h, tie, st, c);
        if (__any(tie) && tie) {
            c.ties++;
            fit_closest_fallback(P, pk.o(), pk.d(), tlo, time, h, st);
        }
        return;
    }
    fit_closest_fallback(P, pk.o(), pk.d(), tlo, time, h, st);
}

// Any hit of one shadow ray (tMin 0, tMax) by the scene's walk.
template <bool COUNT, int WALK, bool WIDE = true, bool PARK = (MYRT_TW_PARK != 0), class WPark = TwParked>
__device__ __forceinline__ bool walk_occluded(const RenderParams& P, const V3& o, const V3& d, double tmax, double time,
                                              Stack& st, Counts& c) {
    if (WALK == kWalkIdentity) return uni_occluded<COUNT, WIDE>(P, o, d, tmax, st, c);
    if (WALK == kWalkFit) {
        if (!P.has_tlas) return false;
        Hit hu;
        const V3 inv = rcp(d);
        if (WIDE && __all(wide_ok(inv))) {
            bool tie = false;
            if (PARK && MYRT_FIT_PARK) {
                WPark pk;                                 // private memory, or the megakernel's LDS slots
                pk.store(o, d);
                return wide_walk<COUNT, true, true>(P, pk, inv, 0.0, tmax, hu, tie, st, c);
            }
            return wide_walk<COUNT, true, true>(P, TwWorld{o, d}, inv, 0.0, tmax, hu, tie, st, c);
        }
        return fit_occluded_fallback(P, o, d, tmax, time, st);
    }
    if (WALK == kWalkTransformed) {
        if (!P.has_tlas) return false;
        Hit hu;
        const V3 inv = rcp(d);
        if (WIDE && P.wide && P.winst && __all(wide_ok(inv))) {
            bool tie = false, redo = false;
            bool occ;
            if (PARK) {
                WPark pk;                                 // private memory, or the megakernel's LDS slots
                pk.store(o, d);
                occ = tw_walk<true>(P, pk, 0.0, tmax, hu, tie, redo, st);
            } else {
                occ = tw_walk<true>(P, TwWorld{o, d}, 0.0, tmax, hu, tie, redo, st);
            }
            if (!redo) return occ;
            return ut_occluded_call(P, o, d, tmax, time, st);
        }
        return ut_walk<true>(P, o, d, inv, 0.0, tmax, time, hu, st);
    }
    return occluded<COUNT>(P, o, d, tmax, time, st, c);
}

// Point lights at a hit (Object+Extension.swift:116-143): adds the unoccluded Blinn-Phong
// terms to Lo.  With !(N.L > 0) the reference discards the occlusion result, so that walk is
// skipped; the ray is still counted as cast.
// park/unpark: the caller's PCG32 state moves to LDS around each walk (trace_path BOUNCE).
template <bool COUNT, int WALK, bool WIDE, class WPark = TwParked, class Park, class Unpark>
__device__ __forceinline__ void point_lights(const RenderParams& P, const DMaterial& M, const V3& N, const V3& p,
                                             const V3& d, double time, Stack& st, Counts& c, V3& Lo, Park park,
                                             Unpark unpark, bool count_shadow = true) {
    for (int li = 0; li < P.num_plights; ++li) {
        const DPointLight& PL = P.plights[li];
        V3 wi = ld3(PL.position) - p;
        const double dist = length(wi);
        wi = normalize(wi);
        const V3 so = p + wi * P.shadow_eps;
        if (count_shadow) c.shadow++;
        // The contribution is formed before the shadow walk (same expressions, same
        // values) so that only it - not N, wi, view, material - stays live across the walk.
        const double NdotL = smax(0.0, dot(N, wi));
        V3 contrib = v3(0, 0, 0);
        if (NdotL > 0) {
            const double shininess = smax(1.0, M.phong);
            const V3 Ld = ld3(M.diffuse) * NdotL;
            const V3 view = normalize(-d);
            const V3 hv = normalize(wi + view);
            const double NdotH = smax(0.0, dot(N, hv));
            const V3 Ls = ld3(M.specular) * phong_pow(NdotH, shininess);
            const V3 atten = ld3(PL.intensity) / smax(dist * dist, 1e-12);
            contrib = (Ld + Ls) * atten;
        }
        // pin it here: otherwise the compiler sinks the whole computation below the
        // walk, into the one branch that uses it, and spills its inputs across the walk
        asm volatile("" : "+v"(contrib.x), "+v"(contrib.y), "+v"(contrib.z));
        if (NdotL > 0 || MYRT_REF(P)) {
            c.shadow_traced++;
            park();
            const bool blocked = walk_occluded<COUNT, WALK, WIDE, (MYRT_TW_PARK != 0), WPark>(P, so, wi, dist, time, st, c);
            unpark();
            if (!blocked && NdotL > 0) Lo = Lo + contrib;
        }
    }
}

// ---- compacted bounce render (mirror/conductor scenes, one traced sample per pixel) --------
// The primary pass renders every pixel's primary ray and shadow rays in the spill-free
// primary instantiation; a lane whose hit is a mirror or conductor below maxRecursionDepth
// writes its reflected ray to a level-1 record instead of tracing it.  Records are compacted per
// level: a wave reserves consecutive records for its reflecting lanes with ONE atomic on one of
// kQRegions counters (q_reserve; region = the wave's block mod kQRegions, so no counter is hit
// by more than 1/32 of the waves: returning atomics on one address serialize, ~85 ns each,
// measured), so a level holds only its rays (C5's scratch was 16 slots x 4
// levels x one 128-B record per pixel = 68 GB).  Per level, k_bounce traces the level's rays in
// batches of 64 consecutive records (one tile's reflecting pixels are consecutive: coherent
// walks) and reserves the next level the same way, each record keeping its parent's index.  A
// ray that ends resolves its sample backward along the parents with the per-level NaN guard,
// Lo_k + M_k * L_(k+1) (Object+Extension.swift:189-206, 252-283), and stores the pixel: the
// operations of the recursion on the same values, so frames are identical.  A region that
// overflows its capacity drops the records (k_queue_done reports each level's largest region
// count; the host grows the arena and renders that frame again, render.hip wait_impl).

__device__ __forceinline__ unsigned long long* q_counter(const RenderParams& P, int level, int region) {
    return P.qhdr + kQHdrCnt + ((size_t)(level - 1) * kQRegions + (size_t)region) * kQCntStride;
}
// Wave-level reservation of level `level` records in `region`: the active lanes of `m` (the ballot
// of `want`) get consecutive records with ONE atomic.  q_issue sends it (the first active lane
// holds the old count); the caller forms the records meanwhile and q_index reads the result:
// the lane's record, or -1 (no want, or the region is full: the frame is rendered again with a
// larger arena).
struct QTicket { unsigned long long base; int first; };
__device__ __forceinline__ QTicket q_issue(const RenderParams& P, int level, int region, unsigned long long m) {
    QTicket t;
    t.first = __builtin_ctzll(__ballot(1));
    t.base = 0;
    if ((int)(threadIdx.x & 63) == t.first) t.base = atomicAdd(q_counter(P, level, region), (unsigned long long)__popcll(m));
    return t;
}
__device__ __forceinline__ long long q_index(const RenderParams& P, int level, int region, unsigned long long m,
                                             bool want, const QTicket& t) {
    const int lane = (int)(threadIdx.x & 63);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)t.base, t.first);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(t.base >> 32), t.first);
    const unsigned long long idx =
        ((unsigned long long)lo | ((unsigned long long)hi << 32)) + (unsigned long long)__popcll(m & ((1ull << lane) - 1ull));
    const unsigned long long cap = P.qhdr[kQHdrCap + level];
    if (!want || idx >= cap) return -1;
    return (long long)(P.qhdr[level] + (unsigned long long)region * cap + idx);
}

// The reflected ray of a mirror/conductor hit and its multiplier (Object+Extension.swift:
// 189-206, 252-275): the record's ray; the parent's Lo follows after its shadow walks.
struct QRay { V3 o, d, mult; unsigned long long rng; };
__device__ __forceinline__ QRay queue_ray(const RenderParams& P, const DMaterial& M, const V3& d, const V3& N,
                                          const V3& p, PCG32& rng) {
    QRay r;
    if (M.type == RT_MAT_MIRROR) {
        r.mult = ld3(M.mirror);
    } else {
        const double cosI = smax(0.0, -dot(d, N));
        r.mult = fresnel_conductor(M.ior, M.absorption_index, cosI) * ld3(M.mirror);
    }
    V3 rd = normalize(reflect(d, N));
    if (M.roughness != 0.0) {
        V3 t, b;
        onb(rd, t, b);
        const double r1 = rng.nextFloat() - 0.5;
        const double r2 = rng.nextFloat() - 0.5;
        rd = (rd + (M.roughness * r1) * b) + (M.roughness * r2) * t;
        rd = normalize(rd);
    }
    r.d = rd;
    r.o = p + N * P.shadow_eps;
    r.rng = rng.state;
    return r;
}
__device__ __forceinline__ void queue_store(const RenderParams& P, long long q, const QRay& r, double time, int i,
                                            int j, long long parent) {
    BounceRec& R = P.bounce[q];
    R.o[0] = r.o.x; R.o[1] = r.o.y; R.o[2] = r.o.z;
    R.d[0] = r.d.x; R.d[1] = r.d.y; R.d[2] = r.d.z;
    R.M[0] = r.mult.x; R.M[1] = r.mult.y; R.M[2] = r.mult.z;
    R.rng = r.rng;
    R.time = time;
    R.i = i; R.j = j;
    R.parent = (int32_t)parent;
}
__device__ __forceinline__ void queue_write_lo(const RenderParams& P, long long q, const V3& Lo) {
    BounceRec& R = P.bounce[q];
    R.Lo[0] = Lo.x; R.Lo[1] = Lo.y; R.Lo[2] = Lo.z;
}

// The pixel of one traced sample (RayTracer.swift:186-195 for RGBA8): px = (0 + col) / spp.
__device__ __forceinline__ void store_pixel(const RenderParams& P, int i, int j, const V3& px) {
    const size_t o = out_row_of(P, j >> 3, j & 7) * (size_t)P.cam.width + i;
    if (P.out_rgb) {
        P.out_rgb[o * 3 + 0] = px.x;
        P.out_rgb[o * 3 + 1] = px.y;
        P.out_rgb[o * 3 + 2] = px.z;
    }
    if (P.out_rgba8) {
        const double cx = fmin(fmax(px.x, 0.0), 255.0), cy = fmin(fmax(px.y, 0.0), 255.0),
                     cz = fmin(fmax(px.z, 0.0), 255.0);
        const unsigned packed = (unsigned)(unsigned char)cx | ((unsigned)(unsigned char)cy << 8) |
                                ((unsigned)(unsigned char)cz << 16) | (255u << 24);
        reinterpret_cast<unsigned*>(P.out_rgba8)[o] = packed;
    }
}

constexpr int kPixSlots = 4;   // per lane: pixel sum x/y/z and the parked PCG32 state, after the stacks
// then, with MYRT_TW_LDS, kParkSlots doubles per lane where a transformed walk parks its world ray
#ifndef MYRT_TW_LDS
#define MYRT_TW_LDS 1     // C3i 4,535 -> 4,956 Mrays/s against the private-memory park (profiles/r05m_ab_c3i.txt)
#endif
constexpr int kParkSlots = MYRT_TW_LDS ? 6 : 0;
constexpr int kTileW = 8;      // 8x8 pixel tiles (16x4 / 32x2 measured slower: DESIGN.md §4)
typedef __attribute__((address_space(3))) double lds_f64;
// This lane's index in its (one-wave) block, computed afresh: the empty asm keeps the compiler from
// reusing an earlier value, which it would otherwise keep live - spilled - across the walks.
__device__ __forceinline__ int pix_lane() {
    int l = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
    asm volatile("" : "+v"(l));
    return l;
}
// this lane's pixel slot k (0-2 pixel sum, 3 PCG32 state) of the megakernel's LDS: the [kLds][64]
// stack slab of the block's one wave, then [kPixSlots][64] doubles
__device__ __forceinline__ lds_f64* pix_slot(int k) {
    extern __shared__ unsigned long long lds_stack[];
    return (lds_f64*)(lds_u64*)(lds_stack + 64 * kLds) + k * 64 + pix_lane();
}

// The megakernel's world-ray park in LDS (MYRT_TW_LDS): the slots after the pixel slots, read
// back where the transformed walk needs the world ray (wide.h tw_walk, TwParked's interface).
struct TwParkedLds {
    __device__ __forceinline__ static lds_f64* at(int k) { return pix_slot(kPixSlots + k); }
    __device__ __forceinline__ void store(const V3& o, const V3& d) const {
        *at(0) = o.x; *at(1) = o.y; *at(2) = o.z; *at(3) = d.x; *at(4) = d.y; *at(5) = d.z;
        asm volatile("" ::: "memory");
    }
    __device__ __forceinline__ V3 o() const { asm volatile("" ::: "memory"); return v3(*at(0), *at(1), *at(2)); }
    __device__ __forceinline__ V3 d() const { asm volatile("" ::: "memory"); return v3(*at(3), *at(4), *at(5)); }
    static constexpr bool kParked = true;
};
#if MYRT_TW_LDS
typedef TwParkedLds TwPark;
#else
typedef TwParked TwPark;
#endif

// trace() (Object+Extension.swift:96-283) for diffuse/mirror/conductor materials and
// point lights.  The recursion Lo + M*trace(depth+1) is run forward and combined
// backward with the same per-level NaN guard, so the result is the recursive one.
// `park_rng`: the PCG32 state waits in this lane's LDS pixel slot 3 while the rays are traced
// (BOUNCE) instead of being live - spilled - across the walks
// QUEUE (primary pass of the compacted bounce render, !BOUNCE): a mirror/conductor hit writes
// its reflected ray to a level-1 record (q_reserve, region = its block's) and sets `deferred`;
// k_bounce delivers that pixel.  The record index waits in pixel slot 0 (the sample sum, written
// only after trace_path) across the shadow walks.  The PCG32 state is read from pixel slot 3
// (the caller parks it there) and (i0, j0) + the lane give its stream.
// The bounce megakernel (C5's mirror scenes) walks the four-wide tree too, at 4 waves/SIMD
// (MYRT_BOUNCE_WPE): C5 5020 vs 4733 Mrays/s for the binary walk at 6 waves, which was the binary
// walk's best occupancy; the wide walk at 5 waves spills (4142), DESIGN.md §4.
#ifndef MYRT_BOUNCE_WIDE
#define MYRT_BOUNCE_WIDE 1
#endif
template <bool COUNT, bool BOUNCE, int WALK, bool QUEUE = false>
__device__ V3 trace_path(const RenderParams& P, V3 o, V3 d, double tlo, double time, PCG32& rng, Stack& st,
                         Counts& c, bool park_rng, int i0 = 0, int j0 = 0,
                         bool* deferred = nullptr) {
    static_assert(!(QUEUE && BOUNCE), "the queued primary pass has no bounce loop");
    // flattened-tree scenes are static (scene.cpp build_wide_tw): motion * time == 0 for every time in
    // [0, 1), so the ray time need not stay live (the caller still draws it: the PCG32 sequence)
    if (WALK == kWalkFit) time = 0.0;
    auto park = [&]() { if (BOUNCE && park_rng) *pix_slot(3) = __builtin_bit_cast(double, rng.state); };
    auto unpark = [&]() {
        if (BOUNCE && park_rng) {
            asm volatile("" ::: "memory");
            rng.state = __builtin_bit_cast(unsigned long long, (double)*pix_slot(3));
        }
    };
    V3 Lst[BOUNCE ? kMaxDepthGPU : 1], Mst[BOUNCE ? kMaxDepthGPU : 1];
    int depth = 0;
    V3 L;
    for (;;) {
        if (!P.has_tlas) { L = v3(0, 0, 0); break; }
        const V3 inv = rcp(d);
        Hit h;
        park();
        if ((WALK == kWalkTransformed || (WALK == kWalkFit && MYRT_FIT_PARK)) && MYRT_TW_PARK &&
            (!BOUNCE || MYRT_BOUNCE_WIDE)) {
            TwPark pk;                                    // the world ray waits in private memory / LDS
            pk.store(o, d);
            if (WALK == kWalkFit) walk_closest_fit_parked<COUNT>(P, pk, tlo, time, h, st, c);
            else walk_closest_tw_parked<COUNT>(P, pk, tlo, time, h, st, c);
            o = pk.o();
            d = pk.d();
        } else {
            walk_closest<COUNT, WALK, !BOUNCE || MYRT_BOUNCE_WIDE>(P, o, d, inv, tlo, time, h, st, c);
        }
        unpark();
        if (h.inst < 0) { L = ld3(P.background); break; }
        V3 p, Ngeo;
        // identity scenes do not move (scene.cpp): motion*time == motion*0 for every time in
        // [0, 1), so `time` need not stay live across the walk
        hit_geometry<COUNT>(P, o, d, WALK == kWalkIdentity ? 0.0 : time, h, p, Ngeo, c);
        const DInstance& I = P.insts[h.inst];
        const int matIndex = max(0, min(P.num_mats - 1, I.material - 1));
        const DMaterial& M = P.mats[matIndex];
        const bool frontFacing = dot(d, Ngeo) < 0;
        const V3 N = frontFacing ? Ngeo : -Ngeo;
        const bool computeDirect = !(M.ior > 0) || frontFacing;
        V3 Lo = computeDirect ? ld3(P.ambient) * ld3(M.ambient) : v3(0, 0, 0);
        bool queued = false;
        if (QUEUE) {     // the bounce ray is formed before the shadow walks: only a flag stays live
            const bool want = (M.type == RT_MAT_MIRROR || M.type == RT_MAT_CONDUCTOR) && P.max_depth > 0;
            const unsigned long long m = __ballot(want);
            if (m) {
                // the wave's records with one atomic in its region (the block's, recomputed: a
                // region kept live from the caller, or the ray formed while the atomic returns,
                // spilled - 417 vs 180 MB of writes per C5 frame); the secondary-ray count is
                // k_queue_done's
                const int region = (int)(blockIdx.x % kQRegions);
                const QTicket tk = q_issue(P, 1, region, m);
                const long long q = q_index(P, 1, region, m, want, tk);
                if (want) {
                    queued = true;
                    *pix_slot(0) = __builtin_bit_cast(double, q);  // not live across the shadow walks
                    if (q >= 0) {
                        const int l = pix_lane();                 // the lane's pixel, recomputed
                        const int i = i0 + l % kTileW, j = j0 + l / kTileW;
                        PCG32 r = PCG32::resume(__builtin_bit_cast(unsigned long long, (double)*pix_slot(3)),
                                                pixel_seed(i, j));
                        const QRay qr = queue_ray(P, M, d, N, p, r);
                        queue_store(P, q, qr, time, i, j, -1);
                    }
                }
            }
        }
        if (QUEUE) {     // the wave counts its shadow rays here: no per-lane counter across the walks
            const unsigned long long m = __ballot(computeDirect);
            if (m && pix_lane() == __builtin_ctzll(__ballot(1)))
                atomicAdd(&P.counters[0], (unsigned long long)__builtin_popcountll(m) * (unsigned)P.num_plights);
        }
        if (computeDirect)
            point_lights<COUNT, WALK, !BOUNCE || MYRT_BOUNCE_WIDE, TwPark>(P, M, N, p, d, time, st, c, Lo, park, unpark,
                                                                          !QUEUE);
        if (QUEUE && queued) {
            asm volatile("" ::: "memory");
            const long long q = __builtin_bit_cast(long long, (double)*pix_slot(0));
            if (q >= 0) queue_write_lo(P, q, Lo);
            *deferred = true;
            L = v3(0, 0, 0);
            break;
        }
        if (BOUNCE && (M.type == RT_MAT_MIRROR || M.type == RT_MAT_CONDUCTOR) && depth < P.max_depth &&
            depth < kMaxDepthGPU) {
            V3 mult;
            if (M.type == RT_MAT_MIRROR) {
                mult = ld3(M.mirror);
            } else {
                const double cosI = smax(0.0, -dot(d, N));
                mult = fresnel_conductor(M.ior, M.absorption_index, cosI) * ld3(M.mirror);
            }
            V3 rd = normalize(reflect(d, N));
            if (M.roughness != 0.0) {
                V3 t, b;
                onb(rd, t, b);
                const double r1 = rng.nextFloat() - 0.5;
                const double r2 = rng.nextFloat() - 0.5;
                rd = (rd + (M.roughness * r1) * b) + (M.roughness * r2) * t;
                rd = normalize(rd);
            }
            Lst[depth] = Lo; Mst[depth] = mult;
            depth++;
            c.secondary++;
            o = p + N * P.shadow_eps;
            d = rd;
            tlo = 0.0;
            continue;
        }
        L = isfin(Lo) ? Lo : v3(0, 0, 0);
        break;
    }
    if (BOUNCE) {
        for (int q = depth - 1; q >= 0; --q) {
            const V3 Lo = Lst[q] + Mst[q] * L;
            L = isfin(Lo) ? Lo : v3(0, 0, 0);
        }
    }
    return L;
}


// One wave renders an 8x8 tile of one 8-row chunk; one wave per block (kRenderBlock).
#ifndef MYRT_MEGA_WPE
#define MYRT_MEGA_WPE 4      // amdgpu_waves_per_eu for the megakernel (0 = compiler default = 2 waves at ~200 VGPRs)
#endif
#ifndef MYRT_BOUNCE_WPE
#define MYRT_BOUNCE_WPE 4   // the bounce (mirror/conductor) instantiation: 4 waves/SIMD with the wide walk
#endif
#ifndef MYRT_QPRIM_WPE
#define MYRT_QPRIM_WPE 4    // the queued primary pass of the compacted bounce render
#endif
#ifndef MYRT_TW_WPE
#define MYRT_TW_WPE 4       // the transformed-walk primary instantiation (C3i, option fit = 0)
#endif
#ifndef MYRT_FIT_WPE
#define MYRT_FIT_WPE 4      // the flattened-instance-tree primary instantiation (C3i)
#endif
#if MYRT_MEGA_WPE > 0
#define MYRT_MEGA_ATTR \
    __attribute__((amdgpu_waves_per_eu(BOUNCE ? MYRT_BOUNCE_WPE : QUEUE ? MYRT_QPRIM_WPE : \
                                       WALK == kWalkTransformed ? MYRT_TW_WPE : WALK == kWalkFit ? MYRT_FIT_WPE : \
                                       MYRT_MEGA_WPE)))
#else
#define MYRT_MEGA_ATTR
#endif
}  // namespace dev
}  // namespace myrt
#include "render_full.h"
namespace myrt {
namespace dev {
// WALK: kWalkIdentity = identity scenes walk TLAS + BLAS as one tree (device.h unified_step);
// kWalkTransformed = the same with per-instance ray switches (device.h ut_walk); kWalkGeneral =
// the nested TLAS/BLAS walks (intersect_closest / occluded; reference-order counting).
// QUEUE: primary pass of the compacted bounce render (one traced sample per pixel, host-checked):
// mirror/conductor hits queue their reflected rays and their pixels are stored by k_bounce.
template <bool COUNT, bool BOUNCE, int WALK, bool QUEUE = false>
__global__ __launch_bounds__(256) MYRT_MEGA_ATTR void render_kernel(RenderParams P) {
    extern __shared__ unsigned long long lds_stack[];
#if MYRT_WAVE_TIMES
    const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
#endif
    // One wave per block (kRenderBlock = 64) renders one kTileW x 8 tile of one selected chunk;
    // tiles are row-major over (slot in the chunk list, column).  Everything but the lane is
    // wave-uniform: the lane's pixel is (lane % kTileW, lane / kTileW) in the tile, and it is
    // recomputed from a fresh lane id where it is needed after the walks (pix_lane), not kept
    // live - spilled - across them.
    const int gx = (P.cam.width + kTileW - 1) / kTileW;
    const int tile = P.tile_order ? (int)P.tile_order[blockIdx.x] : xcd_tile((int)blockIdx.x, (int)gridDim.x, P.xcd_remap);
    // tile order measurement (option tile_order): the wave's start and end by block
    if (P.tile_cost && pix_lane() == 0) P.tile_cost[2 * (size_t)blockIdx.x] = __builtin_amdgcn_s_memrealtime();
    const int chunk = P.chunk_first + (tile / gx) * P.chunk_step;     // slot = tile / gx
    // the tile's corner in VGPRs: the kernel's SGPRs are at the 106 limit, and uniform values
    // live across the walks there are spilled to VGPR lanes and restored with v_readlane
    int i0 = (tile % gx) * kTileW, j0 = chunk * 8;
    // (the queued pass keeps only the row there: both in VGPRs 6,061, neither 5,940, the row alone
    // 6,152 Mrays/s on C5, profiles/r05v_ab_c5.txt)
    if (!QUEUE) asm volatile("" : "+v"(i0), "+v"(j0));
    else asm volatile("" : "+v"(j0));
    const DCamera& C = P.cam;
    Counts cnt{};
    bool valid;
    {
        const int lane = pix_lane();
        valid = (i0 + lane % kTileW < C.width) && (j0 + lane / kTileW < C.height);
    }
    if (valid) {
        MYRT_STACK(st, lds_stack);
        st.uni_spill = !BOUNCE;     // the LDS-only fast path raised the bounce kernel's spills
        const int l0 = pix_lane();
        PCG32 rng(pixel_seed(i0 + l0 % kTileW, j0 + l0 / kTileW));
        const V3 eye = ld3(C.eye), u = ld3(C.u), v = ld3(C.v), w = ld3(C.w), q00 = ld3(C.q00);
        const int n = C.n;
        // the reference's sy / sx loops (Object+Extension.swift:298-354): sample s is (sx, sy) =
        // (s % n, s / n), up to C.samples
        const int ns = min(C.samples, n * n);
        bool deferred = false;
        // (one flattened loop over s measured 3.5 % slower on C3: profiles/r04q_ab_flat.txt)
        int s = 0;
        for (int sy = 0; sy < n && s < ns; ++sy)
        for (int sx = 0; sx < n && s < ns; ++sx, ++s) {
            const double xi1 = rng.nextFloat();
            const double xi2 = rng.nextFloat();
            const double iOffset = ((double)sx + xi1) / (double)n;
            const double jOffset = ((double)sy + xi2) / (double)n;
            // per-sample values the compiler cannot hoist: otherwise (double)i, (double)j and
            // eye - w*nd are computed once before the sample loop and spilled across the walks
            const int lane = pix_lane();
            const int ii = i0 + lane % kTileW, jj = j0 + lane / kTileW;
            // nd + 0 * sample index: a per-sample value (no fast-math, so not folded; the same
            // value for every nd but -0).  An empty "+v" asm on nd instead made its VGPR copy once,
            // in the prologue, and spilled it to scratch: 8 B per lane, 16.6 MB of HBM writes per
            // C3 frame.
            double nd;
            if (!BOUNCE && !QUEUE && WALK == kWalkIdentity) {
                nd = C.nd;
                asm volatile("" : "+s"(nd));
            } else {
                nd = C.nd + 0.0 * (double)s;
            }
            const double currentI = (double)ii + iOffset;
            const double currentJ = (double)jj + jOffset;
            const V3 vOff = v * (currentJ * C.dv);
            const V3 rowTopLeft = q00 - vOff;
            const V3 uOff = u * (currentI * C.du);
            const V3 sp = rowTopLeft + uOff;
            const V3 dir0 = normalize(sp - eye);
            V3 dir = dir0, camEye = eye;
            if (C.aperture > 0 && C.focus > 0) {                  // DOF (:325-338)
                const V3 forward = -w;
                const double denom = dot(dir0, forward);
                const double tFocus = fabs(denom) < 1e-6 ? C.focus : (C.focus / denom);
                const V3 pFocus = eye + dir0 * tFocus;
                const double uRand = rng.nextFloat() - 0.5;
                const double vRand = rng.nextFloat() - 0.5;
                const V3 lensOffset = ((uRand * u) + (vRand * v)) * C.aperture;
                const V3 a = eye + lensOffset;
                dir = normalize(pFocus - a);
                camEye = a;
            }
            const double time = rng.nextFloat();
            const double denom = dot(dir, w);
            const double tImg = dot((eye - w * nd) - camEye, w) / (denom == 0.0 ? 4.9406564584124654e-324 : denom);
            const double tlo = smax(tImg, 0.0);
            // The pixel sum and (when the walk does not draw from it) the PCG32 state wait in the
            // wave's LDS pixel slots while the rays are traced, so they are not live - spilled -
            // across the walks; the memory clobber makes the reloads real loads.
            if (!BOUNCE) *pix_slot(3) = __builtin_bit_cast(double, rng.state);
            const V3 col = trace_path<COUNT, BOUNCE, WALK, QUEUE>(P, camEye, dir, tlo, time, rng, st, cnt, true,
                                                                 i0, j0, &deferred);
            asm volatile("" ::: "memory");
            if (!BOUNCE) {
                const int l2 = pix_lane();
                rng.state = __builtin_bit_cast(unsigned long long, (double)*pix_slot(3));
                rng.inc = (pixel_seed(i0 + l2 % kTileW, j0 + l2 / kTileW) << 1) | 1ull;   // PCG32(seed): inc = seed<<1 | 1
            }
            lds_f64* pacc = pix_slot(0);
            if (s == 0) {
                pacc[0] = 0.0 + col.x; pacc[64] = 0.0 + col.y; pacc[128] = 0.0 + col.z;
            } else {
                pacc[0] = pacc[0] + col.x; pacc[64] = pacc[64] + col.y; pacc[128] = pacc[128] + col.z;
            }
        }
        const lds_f64* pacc = pix_slot(0);
        const V3 pixel = ns > 0 ? v3(pacc[0], pacc[64], pacc[128]) : v3(0, 0, 0);
        const V3 px = pixel / (double)C.samples;
        const int lane = pix_lane();
        if (!(QUEUE && deferred)) store_pixel(P, i0 + lane % kTileW, j0 + lane / kTileW, px);   // RayTracer.swift:186-195
#if MYRT_WAVE_TIMES >= 2
        const size_t o = out_row_of(P, chunk, lane / kTileW) * (size_t)C.width + i0 + lane % kTileW;
        if (P.wave_times && P.out_rgb) {        // debug: per-lane walk iterations instead of the colour
            P.out_rgb[o * 3 + 0] = (double)cnt.it_closest;
            P.out_rgb[o * 3 + 1] = (double)cnt.it_shadow;
        }
#endif
    }
    const int lane = pix_lane();
#if MYRT_WAVE_TIMES
    if (P.wave_times) {                                              // debug timeline
        const unsigned long long t_end = __builtin_amdgcn_s_memrealtime();
        // the wave's walk iterations: its longest lane's, closest hit and any hit
        const unsigned long long mc = wave_max(cnt.it_closest), ms = wave_max(cnt.it_shadow);
        if (lane == 0) {
            unsigned long long* w = P.wave_times + 3 * (size_t)blockIdx.x;
            w[0] = t_start; w[1] = t_end;
            w[2] = (unsigned long long)tile | (std::min(mc, 0xFFFFFull) << 24) | (std::min(ms, 0xFFFFFull) << 44);
        }
    }
#endif
    if (P.tile_cost && lane == 0) P.tile_cost[2 * (size_t)blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
    // ray / work counters: one atomic per wave
    const unsigned long long s0 = wave_sum(cnt.shadow), s1 = wave_sum(cnt.secondary),
                             s2 = wave_sum(cnt.shadow_traced), s3 = wave_sum(cnt.ties);
    if (lane == 0) {
        if (s0) atomicAdd(&P.counters[0], s0);
        if (s1) atomicAdd(&P.counters[1], s1);
        if (s2) atomicAdd(&P.counters[kCounterShadowTraced], s2);
        if (s3) atomicAdd(&P.counters[kCounterTies], s3);
    }
    if (COUNT) {
        const unsigned long long a = wave_sum(cnt.recs), b = wave_sum(cnt.tris), cc = wave_sum(cnt.normals),
                                 dd = wave_sum(cnt.insts), ee = wave_sum(valid ? 1ull : 0ull);
        if (lane == 0) {
            atomicAdd(&P.counters[2], a); atomicAdd(&P.counters[3], b); atomicAdd(&P.counters[4], cc);
            atomicAdd(&P.counters[5], dd); atomicAdd(&P.counters[6], ee);
        }
        const unsigned long long ff = wave_sum(cnt.nodes), gg = wave_sum(cnt.smooth);
        if (lane == 0 && P.count_ref) { atomicAdd(&P.counters[7], ff); atomicAdd(&P.counters[8], gg); }
        // divergence study: lane iterations vs the wave's (max over lanes) iterations
        const unsigned long long lc = wave_sum(cnt.it_closest), wc = wave_max(cnt.it_closest);
        const unsigned long long ls = wave_sum(cnt.it_shadow), ws = wave_max(cnt.it_shadow);
        if (lane == 0 && !P.count_ref) {
            atomicAdd(&P.counters[9], lc); atomicAdd(&P.counters[10], wc);
            atomicAdd(&P.counters[11], ls); atomicAdd(&P.counters[12], ws);
        }
        const unsigned long long dl = wave_sum(cnt.div_lanes), dd2 = wave_sum(cnt.div_distinct);
        if (lane == 0 && !P.count_ref && dl) {
            atomicAdd(&P.counters[14], dl); atomicAdd(&P.counters[15], dd2);
        }
        for (int k = 0; k < 2; ++k) {
            const unsigned long long v0 = wave_sum(cnt.it_wave_inner[k]), v1 = wave_sum(cnt.it_wave_leaf[k]),
                                     v2 = wave_sum(cnt.it_wave_scalar[k]), v3 = wave_sum(cnt.it_lane_inner[k]),
                                     v4 = wave_sum(cnt.it_lane_leaf[k]);
            if (lane == 0 && !P.count_ref) {
                atomicAdd(&P.counters[16 + 5 * k], v0); atomicAdd(&P.counters[17 + 5 * k], v1);
                atomicAdd(&P.counters[18 + 5 * k], v2); atomicAdd(&P.counters[19 + 5 * k], v3);
                atomicAdd(&P.counters[20 + 5 * k], v4);
            }
        }
    }
}

}  // namespace dev
}  // namespace myrt

namespace myrt {
namespace dev {
// Block sum of one u64 per thread over kSumThreads threads (the node-list passes below).
constexpr int kSumThreads = 256;
__device__ __forceinline__ unsigned long long block_sum_u64(unsigned long long x, unsigned long long* s_w) {
    x = wave_sum(x);
    if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = x;
    __syncthreads();
    unsigned long long t = 0;
#pragma unroll
    for (int w = 0; w < kSumThreads / 64; ++w) t += s_w[w];
    __syncthreads();
    return t;
}

// A sample whose ray of record g (level `level`) ended with radiance L: back along the parents,
// Lo_k + M_k * L_(k+1) with the NaN guard per level, and the pixel stored.
__device__ __forceinline__ void q_resolve(const RenderParams& P, long long g, int level, V3 L) {
    int pi = 0, pj = 0;
    for (int lev = level; lev >= 1; --lev) {
        const BounceRec& Q = P.bounce[g];
        const V3 Lq = ld3(Q.Lo) + ld3(Q.M) * L;
        L = isfin(Lq) ? Lq : v3(0, 0, 0);
        pi = Q.i; pj = Q.j;
        g = Q.parent;
    }
    const V3 pixel = v3(0.0 + L.x, 0.0 + L.y, 0.0 + L.z);   // the sample sum (one sample)
    store_pixel(P, pi, pj, pixel / (double)P.cam.samples);
}

// One level of the compacted bounce render: the rays trace(depth = level), one lane per ray;
// wave w of the grid takes the batches of 64 consecutive records w, w + G, ... of the level's
// regions laid end to end (lane r < kQRegions holds region r's count, clamped to the capacity,
// and the exclusive prefix).  A mirror/conductor hit below maxRecursionDepth reserves a
// level + 1 record (q_reserve, in its own record's region: a region holds at most the rays of
// ceil(tiles / kQRegions) primary-pass tiles), writes its reflected ray there with this record as the
// parent, and its own Lo after the shadow walks; any other end resolves the sample backward
// along the parents and stores the pixel.
#ifndef MYRT_QUEUE_WPE
#define MYRT_QUEUE_WPE 4
#endif
// A level's records as one list: lane r < kQRegions holds region r's count (k_bounce(level - 1) /
// the primary pass), clamped to the capacity, and its exclusive prefix `ex`; T = the level's rays.
struct QLevel { unsigned long long cap, lbase; unsigned ex, T; };
__device__ __forceinline__ QLevel q_level(const RenderParams& P, int level) {
    const int lane = threadIdx.x & 63;
    QLevel Q;
    Q.cap = P.qhdr[kQHdrCap + level];
    Q.lbase = P.qhdr[level];
    const unsigned long long cr = lane < kQRegions ? *q_counter(P, level, lane) : 0ull;
    const unsigned c = (unsigned)(cr < Q.cap ? cr : Q.cap);
    unsigned inc = c;                                    // inclusive prefix over the regions
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const unsigned y = (unsigned)__shfl_up((int)inc, off, 64);
        if (lane >= off) inc += y;
    }
    Q.ex = inc - c;
    Q.T = (unsigned)__shfl((int)inc, 63, 64);
    return Q;
}
// ray b of the list (every lane of the wave calls it): its record and region jl, the last region
// with ex <= b
__device__ __forceinline__ long long q_record(const QLevel& Q, unsigned b, int& jl) {
    jl = 0;
    int jh = kQRegions;
#pragma unroll
    for (int s = 0; s < kQRegionBits; ++s) {
        const int mid = (jl + jh) >> 1;
        if ((unsigned)__shfl((int)Q.ex, mid, 64) <= b) jl = mid; else jh = mid;
    }
    return (long long)(Q.lbase + (unsigned long long)jl * Q.cap + (unsigned long long)(b - (unsigned)__shfl((int)Q.ex, jl, 64)));
}
template <int WALK>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(MYRT_QUEUE_WPE))) void k_bounce(RenderParams P,
                                                                                                    int level) {
    extern __shared__ unsigned long long lds_stack[];
    const int lane = threadIdx.x & 63;
    Counts cnt{};
    const QLevel ql = q_level(P, level);
    MYRT_STACK(st, lds_stack);
    st.uni_spill = true;
    for (unsigned x0 = blockIdx.x * 64u; x0 < ql.T; x0 += gridDim.x * 64u) {
        const unsigned b = x0 + (unsigned)lane;          // this lane's ray
        int jl;
        const long long g = q_record(ql, b, jl);
        if (b >= ql.T) continue;
        const BounceRec& R = P.bounce[g];
        const V3 o = ld3(R.o), d = ld3(R.d);
        const double time = (WALK == kWalkIdentity || WALK == kWalkFit) ? 0.0 : R.time;
        V3 L = v3(0, 0, 0);
        bool hit = false, want = false, computeDirect = false;
        V3 p, N, Lo;
        const DMaterial* Mp = nullptr;
        if (P.has_tlas) {
            const V3 inv = rcp(d);
            Hit h;
            walk_closest<false, WALK>(P, o, d, inv, 0.0, time, h, st, cnt);
            if (h.inst < 0) {
                L = ld3(P.background);
            } else {
                hit = true;
                V3 Ngeo;
                hit_geometry<false>(P, o, d, time, h, p, Ngeo, cnt);
                const DInstance& I = P.insts[h.inst];
                Mp = &P.mats[max(0, min(P.num_mats - 1, I.material - 1))];
                const bool frontFacing = dot(d, Ngeo) < 0;
                N = frontFacing ? Ngeo : -Ngeo;
                computeDirect = !(Mp->ior > 0) || frontFacing;
                Lo = computeDirect ? ld3(P.ambient) * ld3(Mp->ambient) : v3(0, 0, 0);
                want = (Mp->type == RT_MAT_MIRROR || Mp->type == RT_MAT_CONDUCTOR) && level < P.max_depth;
            }
        }
        // The next level's records go to this record's own region (jl): a region's rays at every
        // level are then the descendants of a fixed set of primary-pass waves, so its count is the
        // same every frame (with the batch's region it varied with the atomics' order, and the
        // by-need arenas kept growing - a hipMalloc inside the pipelined loop).  One atomic per
        // region the wave's reflecting lanes are in (one, at most a few at sparse levels).
        unsigned long long pend = __ballot(want);
        long long q = -1;
        if (pend) {
            QRay qr{};
            if (want) {
                PCG32 r = PCG32::resume(R.rng, pixel_seed(R.i, R.j));
                qr = queue_ray(P, *Mp, d, N, p, r);
            }
            while (pend) {
                const int r0 = __shfl(jl, __builtin_ctzll(pend), 64);
                const bool mine = want && jl == r0;
                const unsigned long long m = __ballot(mine);
                const QTicket tk = q_issue(P, level + 1, r0, m);
                const long long qq = q_index(P, level + 1, r0, m, mine, tk);
                if (mine) q = qq;
                pend &= ~m;
            }
            if (q >= 0) queue_store(P, q, qr, R.time, R.i, R.j, g);
        }
        if (hit) {
            auto none = []() {};
            if (computeDirect) point_lights<false, WALK, true>(P, *Mp, N, p, d, time, st, cnt, Lo, none, none);
            if (!want) L = isfin(Lo) ? Lo : v3(0, 0, 0);
            else if (q >= 0) queue_write_lo(P, q, Lo);
        }
        if (!want) q_resolve(P, g, level, L);
    }
    const unsigned long long s0 = wave_sum(cnt.shadow), s2 = wave_sum(cnt.shadow_traced), s3 = wave_sum(cnt.ties);
    if (lane == 0) {
        if (s0) atomicAdd(&P.counters[0], s0);
        if (s2) atomicAdd(&P.counters[kCounterShadowTraced], s2);
        if (s3) atomicAdd(&P.counters[kCounterTies], s3);
    }
}

// The sparse last levels of the compacted bounce render in one launch (option queue_tail): each
// lane takes one ray of `level` and traces its whole subtree depth-first - the reflected ray of a
// mirror/conductor hit below maxRecursionDepth is traced by the same lane, its Lo and multiplier
// kept per level - instead of a level launch each (at C5's levels 2-4 a launch is ~0.2 ms of one
// ray's latency for a few thousand rays).  The values and operations are k_bounce's: the PCG32
// stream continues from the record, the sample is combined backward with the per-level NaN
// guard, then along the parent records (q_resolve).  Its bounces count as secondary rays here
// (k_queue_done counts the reserved records).
template <int WALK>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(MYRT_QUEUE_WPE))) void k_bounce_tail(
    RenderParams P, int level) {
    extern __shared__ unsigned long long lds_stack[];
    const int lane = threadIdx.x & 63;
    Counts cnt{};
    const QLevel ql = q_level(P, level);
    MYRT_STACK(st, lds_stack);
    st.uni_spill = true;
    for (unsigned x0 = blockIdx.x * 64u; x0 < ql.T; x0 += gridDim.x * 64u) {
        const unsigned b = x0 + (unsigned)lane;
        int jl;
        const long long g = q_record(ql, b, jl);
        if (b >= ql.T) continue;
        const BounceRec& R = P.bounce[g];
        V3 o = ld3(R.o), d = ld3(R.d);
        const double time = (WALK == kWalkIdentity || WALK == kWalkFit) ? 0.0 : R.time;
        PCG32 rng = PCG32::resume(R.rng, pixel_seed(R.i, R.j));
        V3 Lst[kMaxQueueLevels], Mst[kMaxQueueLevels];
        int k = 0;                                       // levels below `level` traced by this lane
        V3 L = v3(0, 0, 0);
        for (;;) {
            if (!P.has_tlas) break;
            const V3 inv = rcp(d);
            Hit h;
            walk_closest<false, WALK>(P, o, d, inv, 0.0, time, h, st, cnt);
            if (h.inst < 0) { L = ld3(P.background); break; }
            V3 p, Ngeo;
            hit_geometry<false>(P, o, d, time, h, p, Ngeo, cnt);
            const DInstance& I = P.insts[h.inst];
            const DMaterial& M = P.mats[max(0, min(P.num_mats - 1, I.material - 1))];
            const bool frontFacing = dot(d, Ngeo) < 0;
            const V3 N = frontFacing ? Ngeo : -Ngeo;
            const bool computeDirect = !(M.ior > 0) || frontFacing;
            V3 Lo = computeDirect ? ld3(P.ambient) * ld3(M.ambient) : v3(0, 0, 0);
            const bool want = (M.type == RT_MAT_MIRROR || M.type == RT_MAT_CONDUCTOR) && level + k < P.max_depth &&
                              k < kMaxQueueLevels;
            QRay qr{};
            if (want) qr = queue_ray(P, M, d, N, p, rng);
            auto none = []() {};
            if (computeDirect) point_lights<false, WALK, true>(P, M, N, p, d, time, st, cnt, Lo, none, none);
            if (!want) { L = isfin(Lo) ? Lo : v3(0, 0, 0); break; }
            Lst[k] = Lo;
            Mst[k] = qr.mult;
            ++k;
            cnt.secondary++;
            o = qr.o;
            d = qr.d;
        }
        for (int q = k - 1; q >= 0; --q) {
            const V3 Lq = Lst[q] + Mst[q] * L;
            L = isfin(Lq) ? Lq : v3(0, 0, 0);
        }
        q_resolve(P, g, level, L);
    }
    const unsigned long long s0 = wave_sum(cnt.shadow), s1 = wave_sum(cnt.secondary),
                             s2 = wave_sum(cnt.shadow_traced), s3 = wave_sum(cnt.ties);
    if (lane == 0) {
        if (s0) atomicAdd(&P.counters[0], s0);
        if (s1) atomicAdd(&P.counters[1], s1);
        if (s2) atomicAdd(&P.counters[kCounterShadowTraced], s2);
        if (s3) atomicAdd(&P.counters[kCounterTies], s3);
    }
}

// After the last level (one wave): every level's largest region count to the host (qneed: the
// arena a frame needs), the records reserved over all levels (= the secondary rays) to the
// counters, and the region counters back at zero for the next launch.
__global__ void k_queue_done(RenderParams P, int levels) {
    const int lane = threadIdx.x & 63;
    unsigned long long tot = 0;
    for (int L = 1; L <= levels; ++L) {
        const unsigned long long c = lane < kQRegions ? *q_counter(P, L, lane) : 0ull;
        tot += c;
        const unsigned long long mx = wave_max(c);
        if (lane < kQRegions) *q_counter(P, L, lane) = 0ull;
        if (lane == 0 && P.qneed) P.qneed[L] = mx;
    }
    tot = wave_sum(tot);
    if (lane == 0 && tot) atomicAdd(&P.counters[1], tot);
}

// ---- compacted node lists (option node_lists; render_full.h level / shading passes) ----------
// k_level and k_shade give a wave one node position of a tile: a lane idles where its pixel's
// trace() tree has no node there, and on C3g most do past level 0 (lane utilisation 0.34 / 0.41,
// profiles/r04z_c3g_valu.txt).  Instead each pass after level 0 runs over a dense list of the
// flag-log entries it has work for (flags holding `bits`), in the per-tile passes' order: by log
// entry k, then 8x8 pixel tile, then pixel within the tile - a wave's lanes hold one node position
// of 64 neighbouring pixels (row order instead of tiles measured 12 % slower node shading: lane
// utilisation 0.36, profiles/r05x_shade_roofline.json).  The walks are the same (no PCG32 draw
// inside these trees), only their assignment to lanes changes.
// A level's entries are k = s per + first ... s per + first + width - 1 per traced sample s;
// node shading takes every k.  Two passes over groups of 64 flags (one (k, tile) per thread):
// k_ccount writes each block's count, k_clist prefixes the blocks before its own, writes the list
// and its length.
constexpr int kCListThreads = 256, kCListShade = 7;
static_assert(kCListThreads == kSumThreads, "block_sum_u64 sums kSumThreads lanes");
// the log entries [k_lo, k_hi) the groups of `level` run over (level < 0: the whole log, also
// k_events' walk-indexed log: tree 0)
__host__ __device__ inline void clist_span(int tree, int per, int slots, int level, int& k_lo, int& k_hi) {
    if (level < 0) { k_lo = 0; k_hi = slots; return; }
    k_lo = tree_first(tree, level);
    k_hi = (slots / per - 1) * per + tree_first(tree, level) + tree_width(tree, level);
}
__host__ __device__ inline int clist_tiles(int width, int num_chunks) { return num_chunks * ((width + 7) / 8); }
// group g of `level`: its log entry k, tile row base q0 (row 0, column 0 of the tile) and the flags
// of its 64 pixels holding `bits` (bit r * 8 + c: row r, column c of the tile)
__device__ __forceinline__ unsigned long long clist_group(const RenderParams& P, size_t g, int level, unsigned bits,
                                                          size_t& k, size_t& q0) {
    const int W = P.cam.width, tiles = clist_tiles(W, P.num_chunks), gx = (W + 7) / 8;
    int k_lo, k_hi;
    clist_span(P.hit_tree, P.tree_size, P.hit_slots, level, k_lo, k_hi);
    k = (size_t)k_lo + g / (size_t)tiles;
    const int t = (int)(g % (size_t)tiles), slot = t / gx, tx = t % gx;
    q0 = (size_t)slot * 8 * W + (size_t)tx * 8;
    if (k >= (size_t)k_hi) return 0ull;
    if (level >= 0) {
        const int h = (int)(k % (size_t)P.tree_size), first = tree_first(P.hit_tree, level);
        if (h < first || h >= first + tree_width(P.hit_tree, level)) return 0ull;
    }
    const uint8_t* f = P.nflags + k * (size_t)P.hit_stride + q0;
    unsigned long long m = 0;
    if ((W & 7) == 0) {                                  // 8-byte aligned rows of the tile
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            const uint2 v = *reinterpret_cast<const uint2*>(f + (size_t)r * W);
#pragma unroll
            for (int c = 0; c < 8; ++c)
                if ((((c < 4 ? v.x : v.y) >> (8 * (c & 3))) & bits) == bits) m |= 1ull << (r * 8 + c);
        }
    } else {
        const int cols = min(8, W - tx * 8);
        for (int r = 0; r < 8; ++r)
            for (int c = 0; c < cols; ++c)
                if ((f[(size_t)r * W + c] & bits) == bits) m |= 1ull << (r * 8 + c);
    }
    return m;
}
__global__ __launch_bounds__(kCListThreads) void k_ccount(RenderParams P, int level, unsigned bits) {
    __shared__ unsigned long long s_w[kCListThreads / 64];
    size_t k, q0;
    const size_t g = (size_t)blockIdx.x * kCListThreads + threadIdx.x;
    const unsigned long long c = (unsigned long long)__popcll(clist_group(P, g, level, bits, k, q0));
    const unsigned long long t = block_sum_u64(c, s_w);
    if (threadIdx.x == 0) P.cblk[blockIdx.x] = (uint32_t)t;
}
__global__ __launch_bounds__(kCListThreads) void k_clist(RenderParams P, int level, unsigned bits, int word) {
    __shared__ unsigned long long s_w[kCListThreads / 64];
    const int t = threadIdx.x, lane = t & 63;
    unsigned long long before = 0;                       // the blocks before this one
    for (int b = t; b < (int)blockIdx.x; b += kCListThreads) before += P.cblk[b];
    before = block_sum_u64(before, s_w);
    size_t k, q0;
    const size_t g = (size_t)blockIdx.x * kCListThreads + t;
    unsigned long long m = clist_group(P, g, level, bits, k, q0);
    const unsigned mine = (unsigned)__popcll(m);
    unsigned inc = mine;                                 // inclusive scan over the wave, then the block
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const unsigned y = (unsigned)__shfl_up((int)inc, off, 64);
        if (lane >= off) inc += y;
    }
    if (lane == 63) s_w[t >> 6] = inc;
    __syncthreads();
    unsigned at = (unsigned)before + inc - mine;
    for (int w = 0; w < (t >> 6); ++w) at += (unsigned)s_w[w];
    const unsigned end = at + mine;
    const size_t base = k * (size_t)P.hit_stride + q0;
    const int W = P.cam.width;
    while (m) {
        const int b = __builtin_ctzll(m);
        P.clist[at++] = (uint32_t)(base + (size_t)(b >> 3) * W + (b & 7));
        m &= m - 1ull;
    }
    if (blockIdx.x == gridDim.x - 1 && t == kCListThreads - 1) P.cword[word] = end;
}

// Level `level` (>= 1) over its list: one lane per existing node (level_node, as k_level).  A
// fixed grid of waves strides over the list in batches of 64 (its length is on the device).
#ifndef MYRT_LEVELC_WPE
#define MYRT_LEVELC_WPE 4   // waves/SIMD of k_level_c (grid: cus x 4 x MYRT_LEVELC_WPE)
#endif
template <int WALK>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(MYRT_LEVELC_WPE))) void k_level_c(RenderParams P,
                                                                                                   int level) {
    extern __shared__ unsigned long long lds_stack[];
    const unsigned T = P.cword[level];
    const unsigned S = (unsigned)P.hit_stride, per = (unsigned)P.tree_size;
    const unsigned lane = threadIdx.x & 63;
    Counts cnt{};
    MYRT_STACK(st, lds_stack);
    for (unsigned x0 = blockIdx.x * 64u; x0 < T; x0 += gridDim.x * 64u) {
        if (x0 + lane < T) {
            const unsigned at = P.clist[x0 + lane];
            const unsigned k = at / S, q = at - k * S, s = k / per;
            const DNodeRec n = P.nodes[at];
            level_node<WALK>(P, q, (int)s, (int)(k - s * per), level, v3(n.o[0], n.o[1], n.o[2]),
                             v3(n.d[0], n.d[1], n.d[2]), 0.0, n.time, st, cnt);
        }
    }
    flush_ties(P, cnt);
}

// Node shading over its list: one lane per logged walk that hit (shade_node, as k_shade).
#ifndef MYRT_SHADE_WPE
#define MYRT_SHADE_WPE 5    // waves/SIMD of k_shade_c (its grid fills them: cus x 4 x MYRT_SHADE_WPE);
                            // 5 with 36 VGPR spills beat 4 without: C3g 3.22 -> 3.14 ms per frame,
                            // C3r 3.78 -> 3.74 (6: 3.21 / 3.77; profiles/r05zc_ab_c3{g,r}.txt)
#endif
template <int WALK>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(MYRT_SHADE_WPE))) void k_shade_c(RenderParams P) {
    extern __shared__ unsigned long long lds_stack[];
    const unsigned T = P.cword[kCListShade];
    const unsigned S = (unsigned)P.hit_stride;
    const unsigned lane = threadIdx.x & 63;
    Counts cnt{};
    MYRT_STACK(st, lds_stack);
    for (unsigned x0 = blockIdx.x * 64u; x0 < T; x0 += gridDim.x * 64u) {
        if (x0 + lane < T) {
            const unsigned at = P.clist[x0 + lane];
            const unsigned k = at / S;
            shade_node<WALK>(P, at - k * S, (int)k, st, cnt);
        }
    }
    const unsigned long long s0 = wave_sum(cnt.shadow), s2 = wave_sum(cnt.shadow_traced);
    if (lane == 0) {
        if (s0) atomicAdd(&P.counters[0], s0);
        if (s2) atomicAdd(&P.counters[kCounterShadowTraced], s2);
    }
}
}  // namespace dev
}  // namespace myrt

namespace myrt {
namespace dev {
// Explicit-ray queries (rt_debug_trace_rays / rt_debug_occluded_rays): the render kernels'
// walks on caller-given rays, one lane per ray.
struct RayBatch {
    const double *o, *d, *tlim, *time;
    double *out_t, *out_p, *out_n;
    int32_t* out_mat;
    uint8_t* out_occ;
    int32_t n, uni;
};
__global__ __launch_bounds__(256) void k_trace_rays(RenderParams P, RayBatch B) {
    extern __shared__ unsigned long long lds_stack[];
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= B.n) return;
    MYRT_STACK(st, lds_stack);
    Counts c{};
    const V3 o = v3(B.o[3 * i], B.o[3 * i + 1], B.o[3 * i + 2]), d = v3(B.d[3 * i], B.d[3 * i + 1], B.d[3 * i + 2]);
    const double time = B.time[i];
    Hit h;
    h.t = DINF; h.inst = -1; h.tri = -1; h.u = 0; h.v = 0;
    if (P.has_tlas) {
        if (B.uni == 1) uni_closest<false>(P, o, d, rcp(d), B.tlim[i], h, st, c);
        else if (B.uni == 2) walk_closest<false, kWalkTransformed>(P, o, d, rcp(d), B.tlim[i], time, h, st, c);
        else if (B.uni == 3) walk_closest<false, kWalkFit>(P, o, d, rcp(d), B.tlim[i], time, h, st, c);
        else intersect_closest<false>(P, o, d, rcp(d), B.tlim[i], time, h, st, c);
    }
    V3 p = v3(0, 0, 0), n = v3(0, 0, 0);
    if (h.inst >= 0) hit_geometry<false>(P, o, d, time, h, p, n, c);
    B.out_t[i] = h.inst >= 0 ? h.t : DINF;
    B.out_p[3 * i] = p.x; B.out_p[3 * i + 1] = p.y; B.out_p[3 * i + 2] = p.z;
    B.out_n[3 * i] = n.x; B.out_n[3 * i + 1] = n.y; B.out_n[3 * i + 2] = n.z;
    B.out_mat[i] = h.inst >= 0 ? P.insts[h.inst].material : -1;
}
__global__ __launch_bounds__(256) void k_occluded_rays(RenderParams P, RayBatch B) {
    extern __shared__ unsigned long long lds_stack[];
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= B.n) return;
    MYRT_STACK(st, lds_stack);
    Counts c{};
    const V3 o = v3(B.o[3 * i], B.o[3 * i + 1], B.o[3 * i + 2]), d = v3(B.d[3 * i], B.d[3 * i + 1], B.d[3 * i + 2]);
    const bool hit = B.uni == 1 ? uni_occluded<false>(P, o, d, B.tlim[i], st, c)
                     : B.uni == 2 ? walk_occluded<false, kWalkTransformed, true, false>(P, o, d, B.tlim[i], B.time[i], st, c)
                     : B.uni == 3 ? walk_occluded<false, kWalkFit, true, false>(P, o, d, B.tlim[i], B.time[i], st, c)
                           : occluded<false>(P, o, d, B.tlim[i], B.time[i], st, c);
    B.out_occ[i] = hit ? 1 : 0;
}
}  // namespace dev
}  // namespace myrt

// ================================================================== host side / C ABI
using namespace myrt;

namespace {

thread_local std::string g_err;
static int32_t fail(int32_t code, const std::string& msg) { g_err = msg; return code; }

#define HIP_TRY(expr)                                                                    \
    do {                                                                                 \
        hipError_t _e = (expr);                                                          \
        if (_e != hipSuccess) return fail(RT_ERR_DEVICE, std::string(#expr ": ") + hipGetErrorString(_e)); \
    } while (0)

// Threads per render block: one wave.  A block's LDS and wave slots are released only when ALL
// of its waves finish, and wave durations vary ~4x across neighbouring 8x8 tiles: with 4-wave
// blocks ~25% of the wave slots sat idle behind a block's slowest wave (tools/probe_timeline.py).
constexpr int kRenderBlock = 64;
constexpr int kRenderBatches = 8;   // rt_render: chunk batches per replica (progress / overlap granularity)
// rt_render_submit: renders in flight per scene.  Each has its own stream, counters and events
// on every replica, so consecutive frames overlap on the GPU: the next frame's tiles fill the
// compute units the previous frame's slowest tiles leave idle (tools/probe_overlap.py).
constexpr int kInFlight = RT_MAX_IN_FLIGHT;
// Queued bounce rays of one stream's renders (queue_arena): the header (kQHdrWords u64: level
// bases, capacities, region counters), then the records, level by level, kQRegions regions each.
// In-flight slots size their arenas by the need measured on earlier frames (by_need: a frame that
// overflows is rendered again, wait_impl); the replica's and the device path's arenas take the
// worst case (every pixel reflects), since nothing waits for their renders to check.
struct BounceArena {
    void* base = nullptr;
    int64_t levels = 0;
    int64_t cap[kMaxQueueLevels + 1] = {};         // records per region of each level
    int64_t recs = 0;                              // records behind the header
    unsigned long long hdr[kQHdrCnt] = {};         // host image of the header's bases and capacities
    bool by_need = false;
    unsigned long long* qneed = nullptr;           // host-mapped (by_need): k_queue_done's need per level
    unsigned long long* qneed_dev = nullptr;
    bool check = false;                            // a render on this arena reported qneed, unchecked
    int64_t check_levels = 0;
};
// Compacted bounce render: device bytes one launch may take for its queues (else the megakernel)
constexpr int64_t kQueueBytesCap = 16ll << 30;
// (The compacted bounce render is the default since round 4, option queue: faster pipelined than
// the bounce megakernel on C5, slower one frame alone, DESIGN.md §4 "Compacted bounce render".)
// Scratch of the full trace() passes (render_full.h), grown on demand: per-pixel area-light
// event counts and jitter prefixes, the closest-hit log, the node-parallel shading records and
// the level passes' node flags.  The replica has one (rt_render, in-order renders) and each
// of the first `full_flights` in-flight slots one (option, default 4; rt_render_submit:
// overlapping full renders, C3g: ~7.8 GB of scratch per slot).
struct FullScratch {
    long long* events = nullptr;
    long long* jstart = nullptr;
    int64_t cap_px = 0;
    DHitRec* hitlog = nullptr;                // records
    int64_t hitlog_cap = 0;
    DNodeRec* nodes = nullptr;                // node-parallel shading: logged rays + direct light
    double* node_lo = nullptr;
    int32_t* walks = nullptr;
    int64_t nodes_cap = 0, walks_cap = 0;     // records (nodes, node_lo); pixels (walks)
    uint8_t* nflags = nullptr;                // level passes: per-node flags
    int64_t nflags_cap = 0;
    uint32_t* clist = nullptr;                // compacted node lists: entries, then block counts,
    int64_t clist_cap = 0;                    // then 8 list lengths (k_clist)
    void release() {
        (void)hipFree(events); (void)hipFree(jstart); (void)hipFree(hitlog);
        (void)hipFree(nodes); (void)hipFree(node_lo); (void)hipFree(walks); (void)hipFree(nflags);
        (void)hipFree(clist);
        *this = FullScratch{};
    }
};
struct Flight {
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr, done = nullptr;
    unsigned long long* counters = nullptr;        // device, kCounterWords
    unsigned long long* host_counters = nullptr;   // pinned (mapped) copy, valid once `done`
    unsigned long long* host_counters_dev = nullptr;   // its device address
    bool timed = false;                            // ev0/ev1 recorded for the slot's current render
    double* stage_rgb = nullptr;                   // device staging of this replica's rows (DMA delivery)
    uint8_t* stage_rgba = nullptr;
    int64_t stage_px = 0;
    bool counters_zero = false;
    bool counters_valid = false;                   // host_counters hold this render's counts (k_counters_out ran)
    bool used = false;                             // this replica took part in the render
    std::function<int32_t()> relaunch;             // this replica's launches of the slot's render, again
    BounceArena arena;                             // compacted bounce render queues of this slot
    FullScratch full;                              // full trace() passes of the renders on this slot's stream
};

// ---- tile order (render option tile_order): the longest tiles dispatched first ------------------
// A frame lasts as long as its slowest tiles: a wave whose lanes walk ~300 steps
// (grazing rays over the terrain) takes 0.3-0.5 ms alone against 0.07 ms for the median tile, and
// in row-major order some of them start late and form the frame's tail - the tail of the last
// frame of a pipelined run, and the whole latency of a strong split's share.  The first render of
// a (camera, chunk selection) records every wave's start and end (RenderParams::tile_cost); the
// next renders of it dispatch the slowest XCD tile groups first (longest-processing-time order),
// the rest in row-major order behind them.  Which wave renders a pixel does not change the pixel
// (each pixel seeds its own PCG32, Object+Extension.swift:294), so frames are identical.
struct TileOrderKey {
    double eye[3], w[3];
    int32_t width, height, first, step, chunks, group;
    bool operator==(const TileOrderKey& o) const { return std::memcmp(this, &o, sizeof(*this)) == 0; }
};
struct TileOrder {
    TileOrderKey key{};
    int state = 0;                            // 1: costs being measured (ev), 2: order ready
    int64_t n = 0;                            // tiles (blocks of the launch)
    uint32_t* order = nullptr;                // block -> tile
    unsigned long long* cost = nullptr;       // per tile {start, end} (s_memrealtime)
    hipEvent_t ev = nullptr;
    int64_t used = 0;                         // last use (eviction)
};

struct DeviceReplica {
    int device = 0;
    WRec* recs = nullptr;
    CRec* crecs = nullptr;
    CTri* ctris = nullptr;
    TriRec* tris = nullptr;
    W4Node* wnodes = nullptr;                 // conservative four-wide walk (wide.h)
    DWideInst* winst = nullptr;               // ... of transformed scenes: per instance (tw_walk)
    DFitPair* fpairs = nullptr;               // ... their flattened instance tree's pairs (fit_walk)
    double* lbox = nullptr;
    double* normals = nullptr;
    DInstance* insts = nullptr;
    DTlasLeafEntry* tlas_leaf = nullptr;
    DMaterial* mats = nullptr;
    DPointLight* plights = nullptr;
    DAreaLight* alights = nullptr;
    double* jitter = nullptr;
    FullScratch full;                         // full trace() passes on the replica stream
    void* deep = nullptr; int64_t deep_cap = 0;   // deep trace() frames (render_full<.., true>)
    std::vector<void*> retired;               // grown scratch's predecessors (retire(), freed by reclaim())
    int64_t retired_bytes = 0;
    unsigned long long* counters = nullptr;   // kCounterWords x u64
    unsigned long long* wave_times = nullptr; int64_t wave_times_cap = 0;   // rt_debug_wave_times
    hipStream_t stream = nullptr;
    hipStream_t copy_stream = nullptr;        // rt_render: D2H of finished batches
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    // rt_render: the frame's ray counters come back with one async copy into pinned memory
    // (ready = counters_ready) and are zeroed behind it, off the next frame's critical path
    unsigned long long* host_counters = nullptr;
    hipEvent_t counters_ready = nullptr;
    bool counters_zero = false;               // r.counters hold zeros (rt_render's trailing memset)
    // rt_render staging (grown on demand, reused across calls)
    double* out_d = nullptr; uint8_t* out8_d = nullptr; int64_t out_cap_px = 0;
    double* host_rgb = nullptr; uint8_t* host_rgba = nullptr; int64_t host_cap_px = 0;   // pinned
    std::vector<hipEvent_t> batch_done, batch_copied;
    int64_t bytes = 0;
    int cus = 256;                            // compute units (k_bounce grid)
    BounceArena arena;                        // compacted bounce queues of the replica stream
    int64_t qhint[kMaxQueueLevels + 1] = {};  // largest region count seen per level (by_need arenas)
    // rt_render_device / rt_render_device_counted (the caller's stream): counters, pass scratch and
    // queues of their own, so device renders may overlap the replica-stream and slot renders
    unsigned long long* dev_counters = nullptr;
    FullScratch dev_full;
    BounceArena dev_arena;
    Flight fl[kInFlight];                     // rt_render_submit slots
    std::vector<TileOrder> orders;            // tile orders by camera and chunk selection (option tile_order)
    int64_t order_clock = 0;
};

}  // namespace

// ---- render options (rt_scene_set_option, rtcore.h): tuning and test switches whose defaults are
// the production settings.  They replace the MYRT_* environment switches of earlier rounds: the
// library reads no environment variable on the render path.
enum OptId {
    kOptWide, kOptUnified, kOptUnifiedTransformed, kOptCompactRecords, kOptCompactTris, kOptXcdGroup,
    kOptQueue, kOptQueueLevels, kOptHitlog, kOptNodeshade, kOptLevels, kOptTreePpw, kOptFullFlights,
    kOptDeepCapMb, kOptBatches, kOptZerocopy, kOptSubmitEvents, kOptSubmitCounters, kOptSubmitDma,
    kOptDebugFailReplica, kOptWideDeltaScale, kOptNodeLists, kOptTileOrder, kOptFit, kOptQueueTail, kOptCount
};
// `unsafe` options are test hooks: rt_scene_set_option refuses them (RT_ERR_INVALID_ARG); only the
// non-production entry point rt_scene_set_unsafe_option sets them (rtcore.h).
struct OptDef { const char* name; int64_t def, lo, hi; bool unsafe = false; };
static const OptDef kOptDefs[kOptCount] = {
    {"wide", 1, 0, 1},                    // conservative FP32 four-wide walk on identity scenes (wide.h)
    {"unified", 1, 0, 1},                 // one-stack TLAS+BLAS walks (0: the nested general walk)
    {"unified_transformed", 1, 0, 1},     // the unified transformed walk for instanced scenes (device.h ut_walk)
    {"compact_records", 1, 0, 1},         // float32-bound BLAS records when exact (layout.h CRec)
    {"compact_tris", 1, 0, 1},            // float32-vertex triangles when exact (layout.h CTri)
    {"xcd_group", 0, 0, 64},              // tiles per XCD run (device.h xcd_tile); 0 = max(2, width / 960)
    {"queue", 1, 0, 1},                   // compacted bounce render for mirror scenes (k_bounce per level)
    {"queue_levels", -1, -1, 15},         // timing probe: bounce levels of the compacted render (-1 = all)
    {"hitlog", -1, -1, 64},               // closest hits logged per pixel for render_full (-1 = sized automatically)
    {"nodeshade", 1, 0, 1},               // node-parallel shading of logged hits (render_full.h k_shade)
    {"levels", 1, 0, 1},                  // breadth-first events passes (render_full.h k_level)
    {"tree_ppw", 4, 1, 64},               // trace() tree node positions per wave in k_level / k_shade
    {"full_flights", 4, 0, RT_MAX_IN_FLIGHT},  // full trace() renders overlapping on slot streams
    {"deep_cap_mb", 8192, 1, 1 << 20},    // device MB of deep trace() frames per launch batch
    {"batches", 0, 0, 8},                 // rt_render launches per replica (0 = automatic)
    {"zerocopy", 1, 0, 1},                // kernels store page-locked outputs directly (0: staged copies)
    {"submit_events", 1, 0, 1},           // kernel-timing events on renders that ask for them
    {"submit_counters", 1, 0, 1},         // ray counters delivered per submitted render
    {"submit_dma", 0, 0, 2},              // submitted delivery: 0 kernel stores, 1 staging + DMA, 2 staging only
    {"debug_fail_replica", -1, -1, 1 << 20, true},   // test hook: launch failure injected on this replica
    {"wide_delta_scale", 1000, 0, 1000000, true},    // test hook: the four-wide walk's widening (wdelta)
                                                     // in 1/1000 of the exact bound; < 1000 voids wide.h's
                                                     // exactness proof (tests show that it has teeth)
    {"node_lists", 1, 0, 1},              // level passes past 0 and node shading over compacted node lists
    {"tile_order", 0, 0, 100},            // % of XCD tile groups dispatched first, slowest first (TileOrder; 0 = row-major)
    {"fit", 1, 0, 1},                     // transformed scenes: the flattened instance tree (wide.h fit_walk; 0 = tw_walk)
    {"queue_tail", 2, 0, 15},             // compacted bounce render: levels >= this one in one k_bounce_tail launch (0 = a launch per level;
                                          // C5 one frame 3.49 -> 3.23 ms, pipelined +0.2 %: profiles/r06t_ab_c5_tail.txt, r06u_ab_c5_tail.txt)
};

struct rt_scene {
    HostScene host;
    int64_t opt[kOptCount];
    rt_scene() { for (int k = 0; k < kOptCount; ++k) opt[k] = kOptDefs[k].def; }
    std::vector<DeviceReplica> devs;
    std::mutex mu;
    double upload_ms = 0;
    // rt_render_submit bookkeeping: ticket t uses slot t % kInFlight
    struct Pending {
        int64_t ticket = -1;
        bool pending = false;
        std::chrono::steady_clock::time_point t0;
        int64_t primary = 0;
        bool concurrent = true;                   // on the slot's own stream (else the replica stream)
        bool waiting = false;                     // a thread is blocked in rt_render_wait on it
    } flights[RT_MAX_IN_FLIGHT];
    int64_t next_ticket = 0;
};

static int64_t full_scratch_bytes(const FullScratch& f) {
    return f.cap_px * 16 + f.hitlog_cap * (int64_t)sizeof(DHitRec) +
           f.nodes_cap * (int64_t)(sizeof(DNodeRec) + 3 * sizeof(double)) + f.walks_cap * 4 + f.nflags_cap +
           f.clist_cap * (int64_t)sizeof(uint32_t);
}
static int64_t arena_bytes(const BounceArena& a) {
    return a.base ? (int64_t)kQHdrWords * 8 + a.recs * (int64_t)sizeof(BounceRec) : 0;
}
// device scratch a replica holds now (rt_scene_info.scratch_bytes): grown on demand, kept for reuse
static int64_t scratch_bytes(const DeviceReplica& r) {
    int64_t b = full_scratch_bytes(r.full) + full_scratch_bytes(r.dev_full) + arena_bytes(r.arena) +
                arena_bytes(r.dev_arena) + r.deep_cap + r.out_cap_px * 28 + r.wave_times_cap * 24 + r.retired_bytes;
    for (const Flight& f : r.fl) b += full_scratch_bytes(f.full) + arena_bytes(f.arena) + f.stage_px * 28;
    for (const TileOrder& o : r.orders) b += o.n * (int64_t)(sizeof(uint32_t) + 2 * sizeof(unsigned long long));
    return b;
}

template <class T>
static int32_t upload(const std::vector<T>& v, T** dst, int64_t& bytes) {
    const size_t n = std::max<size_t>(1, v.size());
    HIP_TRY(hipMalloc((void**)dst, n * sizeof(T)));
    if (!v.empty()) HIP_TRY(hipMemcpy(*dst, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    bytes += (int64_t)(n * sizeof(T));
    return RT_OK;
}

// Scratch grows on demand (a larger chunk selection, a deeper scene), but a grown buffer's
// predecessor is never freed beside renders in flight: hipFree may wait for the whole device
// (stalling every in-flight render), and a render still queued on another stream - a caller's
// stream for rt_render_device, an in-flight slot - may still read it.  It is retired instead
// (rt_scene_info.scratch_bytes counts it) and freed by reclaim() once the scene has no render in
// flight (after a device synchronisation), or with the replica; the new buffer is zeroed, where
// needed, on the growing render's own stream.  Every growing buffer takes at least 1.5x its old
// capacity (grow_buf), so a scene whose selections keep creeping up retires O(log) buffers.
static void retire(DeviceReplica& r, void* p, int64_t bytes) {
    if (p) { r.retired.push_back(p); r.retired_bytes += bytes; }
}
static int64_t grown(int64_t need, int64_t cap) { return std::max(need, cap + cap / 2); }
// Grow *p to hold `need` elements (capacity `cap`, in elements): the old buffer is retired and the
// new one takes grown(need, cap) elements, or exactly `need` when that much is not available.
// Returns false (and leaves *p null, cap 0) when not even `need` fits.
template <class T>
static bool grow_buf(DeviceReplica& r, T** p, int64_t& cap, int64_t need, size_t elem = sizeof(T)) {
    if (need <= cap && *p) return true;
    const int64_t old = cap;
    retire(r, *p, old * (int64_t)elem);
    *p = nullptr; cap = 0;
    const int64_t want = grown(need, old);
    if (hipMalloc((void**)p, (size_t)want * elem) == hipSuccess) { cap = want; return true; }
    (void)hipGetLastError();
    if (want > need && hipMalloc((void**)p, (size_t)need * elem) == hipSuccess) { cap = need; return true; }
    (void)hipGetLastError();
    *p = nullptr;
    return false;
}
static void free_retired(DeviceReplica& r) {
    for (void* p : r.retired) (void)hipFree(p);
    r.retired.clear();
    r.retired_bytes = 0;
}
// Free the retired scratch once no submitted render of the scene is in flight (the scene lock is
// held): a device synchronisation first, so a render still queued on a caller's stream
// (rt_render_device) has finished with it.  Growth is rare, so is the synchronisation.
static void reclaim(rt_scene* s) {
    bool any = false;
    for (const DeviceReplica& r : s->devs) any = any || !r.retired.empty();
    if (!any) return;
    for (const rt_scene::Pending& fp : s->flights)
        if (fp.pending) return;
    for (DeviceReplica& r : s->devs) {
        if (r.retired.empty()) continue;
        if (hipSetDevice(r.device) == hipSuccess && hipDeviceSynchronize() == hipSuccess) free_retired(r);
        else (void)hipGetLastError();
    }
}
static void free_replica(DeviceReplica& r) {
    (void)hipSetDevice(r.device);
    (void)hipDeviceSynchronize();
    free_retired(r);
    (void)hipFree(r.wnodes); (void)hipFree(r.lbox); (void)hipFree(r.winst); (void)hipFree(r.fpairs);
    (void)hipFree(r.recs); (void)hipFree(r.crecs); (void)hipFree(r.ctris); (void)hipFree(r.tris); (void)hipFree(r.normals); (void)hipFree(r.insts);
    (void)hipFree(r.tlas_leaf); (void)hipFree(r.mats); (void)hipFree(r.plights); (void)hipFree(r.counters);
    (void)hipFree(r.alights); (void)hipFree(r.jitter); (void)hipFree(r.wave_times);
    (void)hipFree(r.deep);
    r.full.release();
    r.dev_full.release();
    (void)hipFree(r.arena.base);
    (void)hipFree(r.dev_arena.base);
    (void)hipFree(r.dev_counters);
    if (r.ev0) (void)hipEventDestroy(r.ev0);
    if (r.ev1) (void)hipEventDestroy(r.ev1);
    if (r.counters_ready) (void)hipEventDestroy(r.counters_ready);
    if (r.host_counters) (void)hipHostFree(r.host_counters);
    for (Flight& f : r.fl) {
        if (f.stream) (void)hipStreamSynchronize(f.stream);
        if (f.ev0) (void)hipEventDestroy(f.ev0);
        if (f.ev1) (void)hipEventDestroy(f.ev1);
        if (f.done) (void)hipEventDestroy(f.done);
        if (f.stream) (void)hipStreamDestroy(f.stream);
        (void)hipFree(f.counters);
        f.full.release();
        (void)hipFree(f.stage_rgb);
        (void)hipFree(f.stage_rgba);
        (void)hipFree(f.arena.base);
        if (f.arena.qneed) (void)hipHostFree(f.arena.qneed);
        if (f.host_counters) (void)hipHostFree(f.host_counters);
    }
    if (r.stream) (void)hipStreamDestroy(r.stream);
    if (r.copy_stream) (void)hipStreamDestroy(r.copy_stream);
    (void)hipFree(r.out_d); (void)hipFree(r.out8_d);
    if (r.host_rgb) (void)hipHostFree(r.host_rgb);
    if (r.host_rgba) (void)hipHostFree(r.host_rgba);
    for (auto e : r.batch_done) (void)hipEventDestroy(e);
    for (auto e : r.batch_copied) (void)hipEventDestroy(e);
    for (TileOrder& o : r.orders) {
        (void)hipFree(o.order); (void)hipFree(o.cost);
        if (o.ev) (void)hipEventDestroy(o.ev);
    }
    r = DeviceReplica();
}

// Triangle arrays get one zeroed record past the end (a guard record after the last run).
template <class T>
static int32_t upload_padded(const std::vector<T>& v, T** dst, int64_t& bytes) {
    const size_t n = v.size() + 1;
    HIP_TRY(hipMalloc((void**)dst, n * sizeof(T)));
    HIP_TRY(hipMemset(*dst, 0, n * sizeof(T)));
    if (!v.empty()) HIP_TRY(hipMemcpy(*dst, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    bytes += (int64_t)(n * sizeof(T));
    return RT_OK;
}

// Replica from another replica's device buffers: device-to-device over xGMI (or a local
// copy when both live on one GPU) instead of a second PCIe upload from the host.
template <class T>
static int32_t replicate(const std::vector<T>& v, const T* src, int src_dev, T** dst, int dst_dev, int64_t& bytes,
                         bool padded = false) {
    const size_t n = padded ? v.size() + 1 : std::max<size_t>(1, v.size());
    HIP_TRY(hipMalloc((void**)dst, n * sizeof(T)));
    if (padded) HIP_TRY(hipMemcpyPeer(*dst, dst_dev, src, src_dev, n * sizeof(T)));   // the zeroed record too
    else if (!v.empty()) HIP_TRY(hipMemcpyPeer(*dst, dst_dev, src, src_dev, v.size() * sizeof(T)));
    bytes += (int64_t)(n * sizeof(T));
    return RT_OK;
}

static int32_t make_replica(const HostScene& S, int device, DeviceReplica& r, const DeviceReplica* src = nullptr) {
    r.device = device;
    HIP_TRY(hipSetDevice(device));
    int32_t rc;
    if (src) {   // the bulk arrays (records, triangles, normals) come from `src` over the fabric
        const int sd = src->device;
        if ((rc = replicate(S.recs, src->recs, sd, &r.recs, device, r.bytes)) != RT_OK) return rc;
        if ((rc = replicate(S.crecs, src->crecs, sd, &r.crecs, device, r.bytes)) != RT_OK) return rc;
        if ((rc = replicate(S.ctris, src->ctris, sd, &r.ctris, device, r.bytes, true)) != RT_OK) return rc;
        if ((rc = replicate(S.tris, src->tris, sd, &r.tris, device, r.bytes, true)) != RT_OK) return rc;
        if ((rc = replicate(S.normals, src->normals, sd, &r.normals, device, r.bytes)) != RT_OK) return rc;
        if ((rc = replicate(S.wnodes, src->wnodes, sd, &r.wnodes, device, r.bytes)) != RT_OK) return rc;
        if ((rc = replicate(S.lbox, src->lbox, sd, &r.lbox, device, r.bytes)) != RT_OK) return rc;
    } else {
        if ((rc = upload(S.recs, &r.recs, r.bytes)) != RT_OK) return rc;
        if ((rc = upload(S.crecs, &r.crecs, r.bytes)) != RT_OK) return rc;
        if ((rc = upload_padded(S.ctris, &r.ctris, r.bytes)) != RT_OK) return rc;
        if ((rc = upload_padded(S.tris, &r.tris, r.bytes)) != RT_OK) return rc;
        if ((rc = upload(S.normals, &r.normals, r.bytes)) != RT_OK) return rc;
        if ((rc = upload(S.wnodes, &r.wnodes, r.bytes)) != RT_OK) return rc;
        if ((rc = upload(S.lbox, &r.lbox, r.bytes)) != RT_OK) return rc;
    }
    if ((rc = upload(S.winst, &r.winst, r.bytes)) != RT_OK) return rc;
    if ((rc = upload(S.fpairs, &r.fpairs, r.bytes)) != RT_OK) return rc;
    if ((rc = upload(S.insts, &r.insts, r.bytes)) != RT_OK) return rc;
    if ((rc = upload(S.tlas_leaf, &r.tlas_leaf, r.bytes)) != RT_OK) return rc;
    if ((rc = upload(S.mats, &r.mats, r.bytes)) != RT_OK) return rc;
    if ((rc = upload(S.plights, &r.plights, r.bytes)) != RT_OK) return rc;
    if ((rc = upload(S.alights, &r.alights, r.bytes)) != RT_OK) return rc;
    if ((rc = upload(S.jitter, &r.jitter, r.bytes)) != RT_OK) return rc;
    HIP_TRY(hipMalloc((void**)&r.counters, kCounterWords * sizeof(unsigned long long)));
    HIP_TRY(hipMemset(r.counters, 0, kCounterWords * sizeof(unsigned long long)));
    HIP_TRY(hipMalloc((void**)&r.dev_counters, kCounterWords * sizeof(unsigned long long)));
    HIP_TRY(hipMemset(r.dev_counters, 0, kCounterWords * sizeof(unsigned long long)));
    if (hipDeviceGetAttribute(&r.cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || r.cus <= 0) {
        (void)hipGetLastError();
        r.cus = 256;
    }
    HIP_TRY(hipStreamCreateWithFlags(&r.stream, hipStreamNonBlocking));
    HIP_TRY(hipStreamCreateWithFlags(&r.copy_stream, hipStreamNonBlocking));
    r.batch_done.resize(kRenderBatches);
    r.batch_copied.resize(kRenderBatches);
    for (int b = 0; b < kRenderBatches; ++b) {
        HIP_TRY(hipEventCreateWithFlags(&r.batch_done[b], hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&r.batch_copied[b], hipEventDisableTiming));
    }
    HIP_TRY(hipEventCreate(&r.ev0));
    HIP_TRY(hipEventCreate(&r.ev1));
    HIP_TRY(hipEventCreateWithFlags(&r.counters_ready, hipEventDisableTiming));
    HIP_TRY(hipHostMalloc((void**)&r.host_counters, kCounterWords * sizeof(unsigned long long), hipHostMallocDefault));
    for (Flight& f : r.fl) {
        HIP_TRY(hipStreamCreateWithFlags(&f.stream, hipStreamNonBlocking));
        HIP_TRY(hipEventCreate(&f.ev0));
        HIP_TRY(hipEventCreate(&f.ev1));
        HIP_TRY(hipEventCreateWithFlags(&f.done, hipEventDisableTiming));
        HIP_TRY(hipMalloc((void**)&f.counters, kCounterWords * sizeof(unsigned long long)));
        HIP_TRY(hipMemset(f.counters, 0, kCounterWords * sizeof(unsigned long long)));
        f.counters_zero = true;
        HIP_TRY(hipHostMalloc((void**)&f.host_counters, kCounterWords * sizeof(unsigned long long),
                              hipHostMallocMapped));
        HIP_TRY(hipHostGetDevicePointer((void**)&f.host_counters_dev, f.host_counters, 0));
        HIP_TRY(hipHostMalloc((void**)&f.arena.qneed, (kMaxQueueLevels + 1) * sizeof(unsigned long long),
                              hipHostMallocMapped));
        HIP_TRY(hipHostGetDevicePointer((void**)&f.arena.qneed_dev, f.arena.qneed, 0));
        f.arena.by_need = true;
    }
    // the zeroing above ran on the null stream, which does not order against the non-blocking
    // render streams: finish it before any render can start
    HIP_TRY(hipDeviceSynchronize());
    return RT_OK;
}

// makeCameraBasis + frame constants (Object+Extension.swift:58-93, 382-427), on the host
static DCamera camera_constants(const rt_camera& cam) {
    auto nrm = [](const double a[3], double o[3]) {
        const double r = 1.0 / std::sqrt((a[0] * a[0] + a[1] * a[1]) + a[2] * a[2]);
        o[0] = a[0] * r; o[1] = a[1] * r; o[2] = a[2] * r;
    };
    auto crs = [](const double a[3], const double b[3], double o[3]) {
        o[0] = a[1] * b[2] - a[2] * b[1]; o[1] = a[2] * b[0] - a[0] * b[2]; o[2] = a[0] * b[1] - a[1] * b[0];
    };
    DCamera C{};
    const int width = std::max(1, cam.width), height = std::max(1, cam.height);
    const double aspect = double(width) / double(height);
    const double e[3] = {cam.position.x, cam.position.y, cam.position.z};
    const double nd = cam.near_distance;
    double l, r, b, t, w[3], u[3], v[3], gn[3], un[3], tmp[3];
    const double up[3] = {cam.up.x, cam.up.y, cam.up.z};
    if (cam.type == RT_CAM_LOOKAT) {
        const double gaze[3] = {cam.gaze_point.x - cam.position.x, cam.gaze_point.y - cam.position.y,
                                cam.gaze_point.z - cam.position.z};
        nrm(gaze, gn);
        if (!std::isnan(cam.fovy)) {
            const double fovYRad = (cam.fovy * M_PI) / (2.0 * 180.0);
            t = nd * std::tan(fovYRad);
        } else {
            t = nd * 0.5;
        }
        b = -t; r = t * aspect; l = -r;
    } else {
        const double gaze[3] = {cam.gaze.x, cam.gaze.y, cam.gaze.z};
        nrm(gaze, gn);
        l = cam.near_plane[0]; r = cam.near_plane[1]; b = cam.near_plane[2]; t = cam.near_plane[3];
    }
    w[0] = -gn[0]; w[1] = -gn[1]; w[2] = -gn[2];
    nrm(up, un);
    crs(un, w, tmp); nrm(tmp, u);
    crs(w, u, tmp); nrm(tmp, v);
    const double du = (r - l) / double(width), dv = (t - b) / double(height);
    double m[3], q00[3];
    for (int k = 0; k < 3; ++k) m[k] = e[k] - w[k] * nd;
    for (int k = 0; k < 3; ++k) q00[k] = (m[k] + u[k] * l) + v[k] * t;
    for (int k = 0; k < 3; ++k) { C.eye[k] = e[k]; C.u[k] = u[k]; C.v[k] = v[k]; C.w[k] = w[k]; C.q00[k] = q00[k]; }
    C.du = du; C.dv = dv; C.nd = nd;
    C.aperture = cam.aperture_size; C.focus = cam.focus_distance;
    C.width = width; C.height = height;
    C.samples = std::max(1, cam.num_samples);
    C.n = (int)std::sqrt((double)C.samples);
    return C;
}

// Device bytes of deep frames per launch batch (option deep_cap_mb; default kDeepBytesCap)
static double deep_cap(const rt_scene* s) { return (double)s->opt[kOptDeepCapMb] * 1048576.0; }
// Lanes of one selected 8-row chunk (render_grid) times the deep trace() levels per lane.
static double deep_bytes_per_chunk(int32_t max_depth, int32_t width) {
    const int bt = kRenderBlock, px = 8 * (bt / 64);
    const double lanes = (double)((std::max(1, width) + px - 1) / px) * bt;
    return lanes * (double)std::max(0, max_depth - kMaxDepthGPU) * (double)sizeof(dev::Frame);
}
static int32_t check_renderable(const rt_scene* s, int32_t cam) {
    const HostScene& S = s->host;
    if (cam < 0 || cam >= (int32_t)S.cams.size()) return fail(RT_ERR_INVALID_CAMERA, "Invalid camera index");
    // trace() levels beyond kMaxDepthGPU live in a device buffer, one Frame per level and lane
    // of a launch batch (render_full<.., DEEP>); one 8-row chunk's lanes must fit kDeepBytesCap
    if (S.max_depth > kMaxDepthGPU && deep_bytes_per_chunk(S.max_depth, S.cams[cam].width) > deep_cap(s))
        return fail(RT_ERR_UNSUPPORTED, "maxRecursionDepth too deep for the device frame buffer");
    return RT_OK;
}

static int32_t num_chunks_total(int32_t height) { return (std::max(1, height) + 7) / 8; }

extern "C" int32_t rt_rows_for_chunks(int32_t height, int32_t chunk_first, int32_t chunk_step) {
    if (chunk_step < 1 || chunk_first < 0) return 0;
    height = std::max(1, height);
    int32_t rows = 0;
    for (int32_t c = chunk_first; c < num_chunks_total(height); c += chunk_step) rows += std::min(8, height - 8 * c);
    return rows;
}


// Absolute pruning margin for rays whose origins lie within `origin_dist` of the scene
// center (or inside the scene bounds): prune_k * (|o - v0| + t|d|) with both terms bounded
// by the origin's distance plus the scene diagonal (scene.cpp, "pruning margin").
static double prune_abs_for(const HostScene& S, double origin_dist) {
    const double half = 0.5 * S.scene_extent;
    const double rmax = std::max(origin_dist, half) + half + S.max_motion;
    const double mt = 2.0 * S.prune_k * (2.0 * rmax + S.scene_extent);
    const double a = std::max(1e-9 * S.scene_extent, mt);
    return std::isfinite(a) ? a : HUGE_VAL;                          // eps <= 0: no pruning
}
// RenderParams::fast_rcp: every determinant the triangle tests divide by satisfies
// 2^-700 <= eps <= |det| <= det_scale * |d| <= 2^1000 for directions with |d| <= dmax
// (device.h rcp_rn is then bit-identical to 1.0/det).
static int32_t fast_rcp_for(const HostScene& S, double dmax) {
    return (S.eps >= 0x1p-700 && std::isfinite(S.det_scale) && std::isfinite(dmax) &&
            S.det_scale * dmax <= 0x1p1000) ? 1 : 0;
}
static double dist_to_center(const HostScene& S, const double p[3]) {
    double d = 0.0;
    for (int k = 0; k < 3; ++k) d += (p[k] - S.scene_center[k]) * (p[k] - S.scene_center[k]);
    return std::sqrt(d);
}

// The conservative four-wide walk (wide.h) for this render: every ray origin has coordinates of
// magnitude <= origin_coord (camera + lens) or lies inside the scene bounds (hit points, offset by
// shadowRayEpsilon; triangle hit points only: scene.cpp build_wide builds no tree for scenes with
// spheres or planes, whose hit points can lie outside every box).  wdelta = 8 * 2^-24 * max(|box coordinate|, |origin coordinate|) bounds the
// FP32 rounding of the slab terms (wide.h header); weps = eps rounded down to float.
// Transformed scenes with a flattened instance tree (option fit): R also covers the tree's
// magnitudes (fit_coord) and wdelta carries 2^-27 R more for the world <-> local rounding (wide.h
// fit_walk header); the larger widening only loosens tw_walk's TLAS filter.
static void set_wide(const HostScene& S, const DeviceReplica& r, RenderParams& P, double origin_coord, bool on,
                     int64_t scale_permille, bool fit) {
    P.wnodes = r.wnodes; P.lbox = r.lbox; P.wide_root = S.wide_root;
    P.wide_copy_bytes = (uint32_t)(S.wide_copy * (int64_t)sizeof(W4Node));
    P.winst = S.winst.empty() ? nullptr : r.winst;          // transformed scenes (wide.h tw_walk)
    P.tw_tlas_nodes = (int32_t)S.tw_tlas_nodes;
    P.tw_wscale = (float)((double)scale_permille * 1e-3);
    const bool has_fit = S.fit_root >= 0 && !S.fpairs.empty() && r.fpairs;
    const double R = std::max({S.wide_coord, has_fit ? S.fit_coord : 0.0, origin_coord}) + std::fabs(S.shadow_eps) +
                     std::fabs(S.eps);
    P.wdelta = R * (has_fit ? 0x1p-21 + 0x1p-27 : 0x1p-21) * ((double)scale_permille * 1e-3);
    float we = (float)S.eps;
    if ((double)we > S.eps) we = std::nextafter(we, -HUGE_VALF);
    P.weps = we;
    P.wide = (S.wide_root >= 0 && r.wnodes && !S.has_special && R < 0x1p27 && R > 0x1p-60 && std::isfinite(R) &&
              on) ? 1 : 0;
    P.fpairs = has_fit ? r.fpairs : nullptr;
    P.fit_root = has_fit ? S.fit_root : -1;
    P.fit = (P.wide && has_fit && fit) ? 1 : 0;
}

static RenderParams make_params(const rt_scene* s, const DeviceReplica& r, int32_t cam, int32_t first, int32_t step,
                                double* out_rgb, uint8_t* out_rgba8) {
    const HostScene& S = s->host;
    RenderParams P{};
    P.recs = r.recs; P.crecs = r.crecs; P.tris = r.tris; P.normals = r.normals; P.insts = r.insts; P.tlas_leaf = r.tlas_leaf;
    P.mats = r.mats; P.plights = r.plights;
    for (int k = 0; k < 3; ++k) { P.tlas_root_lo[k] = S.tlas_root_lo[k]; P.tlas_root_hi[k] = S.tlas_root_hi[k]; }
    P.tlas_root_ref = S.tlas_root_ref;
    P.has_tlas = S.has_tlas ? 1 : 0;
    P.tlas_leaf_base = (int32_t)S.tlas_leaf_base;
    P.identity = S.identity ? 1 : 0;
    // one stack for TLAS + BLAS + a TLAS leaf's markers (HostScene::max_stack_unified)
    P.ut = (S.has_tlas && S.max_stack_unified <= kStackCap && s->opt[kOptUnifiedTransformed] != 0) ? 1 : 0;
    P.tlas_rec_base = (int32_t)S.blas_records;
    P.ut_marker_base = (int32_t)(S.tlas_leaf_base + (int64_t)S.tlas_leaf.size());
    P.num_mats = (int32_t)S.mats.size();
    P.num_plights = (int32_t)S.plights.size();
    P.cam = camera_constants(S.cams[cam]);
    P.eps = S.eps; P.shadow_eps = S.shadow_eps;
    // Pruning margin (DESIGN.md "Pruning", scene.cpp): relative 1e-7 covers the rounding of
    // slab entries and sphere roots; the absolute part bounds Moeller-Trumbore's t error,
    // prune_k * (|o - v0| + t|d|), for every ray origin of this render: the camera (plus the
    // lens) or a hit point inside the scene bounds.
    P.prune_rel = 1.0 + 1e-7;
    {
        const rt_camera& cam0 = S.cams[cam];
        const double ce[3] = {cam0.position.x, cam0.position.y, cam0.position.z};
        P.prune_abs = prune_abs_for(S, dist_to_center(S, ce) + std::fabs(cam0.aperture_size));
    }
    P.fast_rcp = fast_rcp_for(S, 2.0);   // rendered directions are normalized (|d| <= 1 + 2^-50)
    for (int k = 0; k < 3; ++k) { P.background[k] = S.background[k]; P.ambient[k] = S.ambient[k]; }
    P.max_depth = S.max_depth;
    P.chunk_first = first; P.chunk_step = step;
    P.out_first = first; P.out_step = step;          // packed selection rows (callers may remap)
    int32_t nsel = 0;
    for (int32_t c = first; c < num_chunks_total(P.cam.height); c += step) nsel++;
    P.num_chunks = nsel;
    P.stack_depth = dev::kLds;
    {
        // runs of G neighbouring 8x8 tiles per XCD (device.h xcd_tile); measured best: G = 2 at
        // 1920 px (C3), G = 4 at 3840 px (C5), i.e. about one run per 960 px of image width
        const int64_t xg = s->opt[kOptXcdGroup];
        P.xcd_remap = xg > 0 ? (int32_t)xg : std::max(2, P.cam.width / 960);
        P.compact_limit = s->opt[kOptCompactRecords] ? (int32_t)S.compact_records : 0;
        P.ctris = (S.compact_tris && s->opt[kOptCompactTris]) ? r.ctris : nullptr;
    }
    P.out_rgb = out_rgb; P.out_rgba8 = out_rgba8;
    P.counters = r.counters;
    P.wave_times = nullptr;
    P.alights = r.alights;
    P.jitter = r.jitter;
    P.num_alights = (int32_t)S.alights.size();
    P.has_special = S.has_special ? 1 : 0;
    {
        const rt_camera& cam0 = S.cams[cam];
        const double ce[3] = {cam0.position.x, cam0.position.y, cam0.position.z};
        set_wide(S, r, P, std::max({std::fabs(ce[0]), std::fabs(ce[1]), std::fabs(ce[2])}) + std::fabs(cam0.aperture_size),
                 s->opt[kOptWide] != 0, s->opt[kOptWideDeltaScale], s->opt[kOptFit] != 0);
    }
    return P;
}

// a material some instance shades with (hits take the instance's material, clamped) is rough
static bool scene_is_rough(const HostScene& S) {
    if (S.mats.empty()) return false;
    for (const auto& I : S.insts) {
        const int mi = std::max(0, std::min((int)S.mats.size() - 1, (int)I.material - 1));
        if (S.mats[mi].roughness != 0.0) return true;
    }
    return false;
}
// (Option tree_ppw, the node positions of a tree level one wave of k_level / k_shade runs: one
// per wave dispatches mostly empty waves at the deep levels, all in one wave makes a tile's
// positions a serial chain, the slowest tile bounding a pass; 4 is measured best.)
static bool scene_has_bounce(const HostScene& S) {
    for (const auto& m : S.mats) if (m.type == RT_MAT_MIRROR || m.type == RT_MAT_CONDUCTOR) return true;
    return false;
}

// blocks of `threads` lanes over the selected chunks, one tw x (64/tw) tile per wave
static dim3 render_grid(const RenderParams& P, int threads, int tw = 8) {
    const int px = tw * (threads / 64);                  // pixels per block along a row
    return dim3((unsigned)(((P.cam.width + px - 1) / px) * (8 / (64 / tw)) * P.num_chunks), 1, 1);
}

// Walks logged per pixel by k_events (hit + ray + direct light: 120 B each): every walk of a
// pixel's paths when they fit - n*n traced samples, each a trace() tree of at most 2^(D+1) - 1
// walks with dielectrics (reflection + transmission per level) or D + 1 without - capped at 64 and
// at kHitLogBytes; walks past the log are walked and shaded by render_full itself.
constexpr int64_t kHitLogBytes = 16ll << 30;
static int64_t hit_slots_for(const RenderParams& P, bool dielectric, int64_t px) {
    const int64_t d = std::min<int64_t>(std::max(0, P.max_depth), 6);
    const int64_t per_sample = dielectric ? ((int64_t(2) << d) - 1) : d + 1;
    const int64_t traced = std::max(1, std::min(P.cam.samples, P.cam.n * P.cam.n));
    const int64_t by_mem = kHitLogBytes / std::max<int64_t>(1, px * (int64_t)(sizeof(DHitRec) + sizeof(DNodeRec) + 24));
    return std::max<int64_t>(0, std::min<int64_t>({per_sample * traced, 64, by_mem}));
}
// The list of level `level`'s entries (level < 0: every logged walk) whose flags hold `bits`,
// its length into list word `word` (render.hip k_ccount / k_clist).
static void clist_launch(const RenderParams& P, int level, unsigned bits, int word, hipStream_t stream) {
    int k_lo, k_hi;
    dev::clist_span(P.hit_tree, P.tree_size, P.hit_slots, level, k_lo, k_hi);
    const unsigned long long groups = (unsigned long long)(k_hi - k_lo) * dev::clist_tiles(P.cam.width, P.num_chunks);
    const dim3 grid((unsigned)((groups + dev::kCListThreads - 1) / dev::kCListThreads));
    hipLaunchKernelGGL(dev::k_ccount, grid, dim3(dev::kCListThreads), 0, stream, P, level, bits);
    hipLaunchKernelGGL(dev::k_clist, grid, dim3(dev::kCListThreads), 0, stream, P, level, bits, word);
}
static int32_t launch_full(const rt_scene* s, DeviceReplica& r, FullScratch& fs, RenderParams P, hipStream_t stream,
                           bool count, bool dielectric, bool rough) {
    const int bt = kRenderBlock;
    dim3 block((unsigned)bt, 1, 1);
    const size_t lds = (size_t)dev::kLds * bt * sizeof(unsigned long long);
    const unsigned per_slot = render_grid(P, bt).x / (unsigned)std::max(1, P.num_chunks);   // blocks per chunk
    // maxRecursionDepth > kMaxDepthGPU: batches of chunks whose deep frames fit kDeepBytesCap
    const bool deep = P.max_depth > kMaxDepthGPU;
    int32_t batch = P.num_chunks;
    if (deep) {
        const double per_chunk = deep_bytes_per_chunk(P.max_depth, P.cam.width);
        batch = (int32_t)std::max(1.0, std::min((double)P.num_chunks, std::floor(deep_cap(s) / per_chunk)));
        const int64_t need = (int64_t)(per_chunk * batch);
        if (need > r.deep_cap) {
            char* d = static_cast<char*>(r.deep);
            const bool ok = grow_buf(r, &d, r.deep_cap, need, 1);
            r.deep = d;
            if (!ok) return fail(RT_ERR_OOM, "device allocation of deep trace() frames failed");
        }
        P.deep = r.deep;
    }
    const bool unified = P.has_tlas && !P.count_ref && s->opt[kOptUnified] != 0;
    const int walk = (unified && P.identity) ? dev::kWalkIdentity
                     : (unified && P.ut && !count) ? (P.fit ? dev::kWalkFit : dev::kWalkTransformed) : dev::kWalkGeneral;
#define MYRT_BY_WALK(M_)                                                    \
    do {                                                                    \
        if (walk == dev::kWalkIdentity) M_(dev::kWalkIdentity);             \
        else if (walk == dev::kWalkFit) M_(dev::kWalkFit);                  \
        else if (walk == dev::kWalkTransformed) M_(dev::kWalkTransformed);  \
        else M_(dev::kWalkGeneral);                                         \
    } while (0)
    // Area-light frames need the events passes (jitterIndex prefixes); dielectric frames without
    // area lights take the same level passes + node shading when they apply (no rough
    // material, whole trees logged), else render_full alone walks and shades every tree.
    const bool alights = P.num_alights > 0;
    bool lists = false;                       // compacted node lists (k_level_c / k_shade_c)
    // their passes: a fixed grid of one-wave blocks striding over the list, one block per wave
    // slot of the chip at the kernel's occupancy (MYRT_LEVELC_WPE, MYRT_SHADE_WPE)
    const size_t clds = (size_t)dev::kLds * 64 * sizeof(unsigned long long);
    if (alights || (dielectric && !count && !deep)) {
        const int64_t px = (int64_t)P.num_chunks * 8 * P.cam.width;
        if (px > fs.cap_px) {
            const int64_t cap = grown(px, fs.cap_px);
            retire(r, fs.events, fs.cap_px * 8); retire(r, fs.jstart, fs.cap_px * 8);
            fs.events = nullptr; fs.jstart = nullptr; fs.cap_px = 0;
            if (hipMalloc((void**)&fs.events, cap * sizeof(long long)) != hipSuccess ||
                hipMalloc((void**)&fs.jstart, cap * sizeof(long long)) != hipSuccess) {
                (void)hipFree(fs.events); (void)hipFree(fs.jstart);      // never used: safe to free
                fs.events = nullptr; fs.jstart = nullptr;
                if (alights) return fail(RT_ERR_OOM, "device allocation of area-light jitter buffers failed");
                (void)hipGetLastError();
            } else {
                fs.cap_px = cap;
            }
        }
        P.events = fs.events;
        P.jstart = fs.jstart;
        // the closest-hit log: render_full reads the first `slots` walks of every pixel back
        // instead of walking them again (option hitlog = K overrides, 0 = off; counting launches walk)
        const int64_t hl = s->opt[kOptHitlog];
        const int64_t slots = count ? 0 : (hl >= 0 ? hl : hit_slots_for(P, dielectric, px));
        if (slots > 0 && slots * px > fs.hitlog_cap)
            (void)grow_buf(r, &fs.hitlog, fs.hitlog_cap, slots * px);   // none: render_full walks every ray
        const bool log = slots > 0 && slots * px <= fs.hitlog_cap;
        P.hits = log ? fs.hitlog : nullptr;
        P.hit_slots = log ? (int32_t)slots : 0;
        P.hit_stride = px;
        // node-parallel shading of the logged hits (render_full.h k_shade; option nodeshade = 0: render_full
        // shades them).  Every pointer a pass writes through is set here, before the first launch:
        // kernels take RenderParams by value.
        bool nodeshade = log && s->opt[kOptNodeshade] != 0;
        if (nodeshade && (slots * px > fs.nodes_cap || px > fs.walks_cap)) {
            const int64_t recs = slots * px > fs.nodes_cap ? grown(slots * px, fs.nodes_cap) : fs.nodes_cap;
            const int64_t pxs = px > fs.walks_cap ? grown(px, fs.walks_cap) : fs.walks_cap;
            retire(r, fs.nodes, fs.nodes_cap * (int64_t)sizeof(DNodeRec));
            retire(r, fs.node_lo, fs.nodes_cap * 24); retire(r, fs.walks, fs.walks_cap * 4);
            fs.nodes = nullptr; fs.node_lo = nullptr; fs.walks = nullptr; fs.nodes_cap = fs.walks_cap = 0;
            if (hipMalloc((void**)&fs.nodes, (size_t)recs * sizeof(DNodeRec)) == hipSuccess &&
                hipMalloc((void**)&fs.node_lo, (size_t)recs * 3 * sizeof(double)) == hipSuccess &&
                hipMalloc((void**)&fs.walks, (size_t)pxs * sizeof(int32_t)) == hipSuccess) {
                fs.nodes_cap = recs;
                fs.walks_cap = pxs;
            } else {
                (void)hipGetLastError();              // render_full shades every hit (never used: safe to free)
                (void)hipFree(fs.nodes); (void)hipFree(fs.node_lo); (void)hipFree(fs.walks);
                fs.nodes = nullptr; fs.node_lo = nullptr; fs.walks = nullptr;
            }
        }
        nodeshade = nodeshade && slots * px <= fs.nodes_cap && px <= fs.walks_cap;
        P.nodes = nodeshade ? fs.nodes : nullptr;
        P.node_lo = nodeshade ? fs.node_lo : nullptr;
        P.walks = nodeshade ? fs.walks : nullptr;
        // Breadth-first events passes (render_full.h k_level) when the log holds every pixel's
        // whole trace() trees and no material is rough (no PCG32 draw inside trace(), so the
        // order of the walks is free); option levels = 0 keeps the depth-first k_events.
        const int32_t tree = dielectric ? 2 : 1;
        const int64_t traced = std::max(1, std::min(P.cam.samples, P.cam.n * P.cam.n));
        const int64_t tree_size = P.max_depth >= 0 && P.max_depth <= 5
                                      ? (tree == 2 ? (int64_t(2) << P.max_depth) - 1 : P.max_depth + 1) : 0;
        bool levels = nodeshade && !deep && P.has_tlas && tree_size > 0 && slots == tree_size * traced &&
                      !rough && s->opt[kOptLevels] != 0;
        // node lists (option node_lists): over the level passes' flags, or - depth-first k_events
        // with area lights - over hit flags k_events writes for node shading
        const bool want_lists = nodeshade && s->opt[kOptNodeLists] != 0 && slots * px < (int64_t(1) << 32);
        bool flags_ev = want_lists && !levels && alights;
        if ((levels || flags_ev) && slots * px > fs.nflags_cap)
            (void)grow_buf(r, &fs.nflags, fs.nflags_cap, slots * px);   // none: depth-first k_events
        levels = levels && slots * px <= fs.nflags_cap && px <= fs.cap_px;
        flags_ev = flags_ev && slots * px <= fs.nflags_cap;
        // compacted node lists: entry indices are u32; list + block counts + lengths
        const int64_t cgroups = slots * dev::clist_tiles(P.cam.width, P.num_chunks);
        const int64_t cblocks = (cgroups + dev::kCListThreads - 1) / dev::kCListThreads;
        const int64_t cwords = slots * px + cblocks + 8;
        lists = want_lists && (levels || flags_ev);
        if (lists && cwords > fs.clist_cap)
            (void)grow_buf(r, &fs.clist, fs.clist_cap, cwords);          // none: the per-tile passes
        lists = lists && cwords <= fs.clist_cap;
        P.clist = lists ? fs.clist : nullptr;
        P.cblk = lists ? fs.clist + slots * px : nullptr;
        P.cword = lists ? fs.clist + slots * px + cblocks : nullptr;
        if (!alights && !levels) {                     // dielectrics only: render_full does it all
            P.hits = nullptr; P.hit_slots = 0;
            P.nodes = nullptr; P.node_lo = nullptr; P.walks = nullptr;
            nodeshade = false;
        }
        P.hit_tree = levels ? tree : 0;
        P.tree_ppw = (int32_t)s->opt[kOptTreePpw];
        P.tree_size = levels ? (int32_t)tree_size : 0;
        P.nflags = (levels || lists) ? fs.nflags : nullptr;
        if (lists && !levels) HIP_TRY(hipMemsetAsync(fs.nflags, 0, (size_t)(slots * px), stream));
        if (levels) {
            HIP_TRY(hipMemsetAsync(fs.nflags, 0, (size_t)(slots * px), stream));
            P.slot_base = 0;
            const unsigned g0 = per_slot * (unsigned)P.num_chunks;
#define MYRT_LV(W_) hipLaunchKernelGGL((dev::k_level<W_>), dim3(g0, ly, 1), block, lds, stream, P, level)
#define MYRT_LVC(W_) hipLaunchKernelGGL((dev::k_level_c<W_>), dim3((unsigned)(r.cus * 4 * MYRT_LEVELC_WPE)), dim3(64), clds, stream, P, level)
            for (int32_t level = 0; level <= P.max_depth; ++level) {
                if (lists && level > 0) {
                    clist_launch(P, level, dev::kNodeExists, level, stream);
                    MYRT_BY_WALK(MYRT_LVC);
                    continue;
                }
                const unsigned ly = level == 0 ? 1u : (unsigned)(traced * dev::tree_rows(tree, level, P.tree_ppw));
                MYRT_BY_WALK(MYRT_LV);
            }
#undef MYRT_LV
#undef MYRT_LVC
            hipLaunchKernelGGL(dev::k_jofs, dim3(g0), block, 0, stream, P);
        }
        for (int32_t base = 0; base < P.num_chunks && !levels && alights; base += batch) {
            P.slot_base = base;
            dim3 grid(per_slot * (unsigned)std::min(batch, P.num_chunks - base), 1, 1);
#define MYRT_EV1(W_) hipLaunchKernelGGL((dev::k_events<true, W_>), grid, block, lds, stream, P)
#define MYRT_EV0(W_) hipLaunchKernelGGL((dev::k_events<false, W_>), grid, block, lds, stream, P)
            if (deep) MYRT_BY_WALK(MYRT_EV1);
            else MYRT_BY_WALK(MYRT_EV0);
#undef MYRT_EV1
#undef MYRT_EV0
        }
        if (alights) hipLaunchKernelGGL(dev::k_jscan, dim3((unsigned)P.num_chunks), dim3(256, 1, 1), 0, stream, P);
        if (nodeshade) {
            int64_t shade_rows = 0;                            // per traced sample (k_shade)
            for (int32_t L = 0; P.hit_tree && L <= P.max_depth; ++L) shade_rows += dev::tree_rows(tree, L, P.tree_ppw);
            P.slot_base = 0;                                   // one launch over every chunk
            const dim3 sgrid(per_slot * (unsigned)P.num_chunks,
                             P.hit_tree ? (unsigned)(traced * shade_rows) : (unsigned)slots, 1);
#define MYRT_SH(W_) hipLaunchKernelGGL((dev::k_shade<W_>), sgrid, block, lds, stream, P)
#define MYRT_SHC(W_) hipLaunchKernelGGL((dev::k_shade_c<W_>), dim3((unsigned)(r.cus * 4 * MYRT_SHADE_WPE)), dim3(64), clds, stream, P)
            if (lists) {
                clist_launch(P, -1, dev::kNodeHit, dev::kCListShade, stream);
                MYRT_BY_WALK(MYRT_SHC);
            } else {
                MYRT_BY_WALK(MYRT_SH);
            }
#undef MYRT_SH
#undef MYRT_SHC
        }
    }
    for (int32_t base = 0; base < P.num_chunks; base += batch) {
        P.slot_base = base;
        dim3 grid(per_slot * (unsigned)std::min(batch, P.num_chunks - base), 1, 1);
        const bool u = walk == dev::kWalkIdentity;
        if (count) {
            if (deep) {
                if (u) hipLaunchKernelGGL((dev::render_full<true, true, dev::kWalkIdentity>), grid, block, lds, stream, P);
                else hipLaunchKernelGGL((dev::render_full<true, true, dev::kWalkGeneral>), grid, block, lds, stream, P);
            } else {
                if (u) hipLaunchKernelGGL((dev::render_full<true, false, dev::kWalkIdentity>), grid, block, lds, stream, P);
                else hipLaunchKernelGGL((dev::render_full<true, false, dev::kWalkGeneral>), grid, block, lds, stream, P);
            }
        } else {
#define MYRT_RF1(W_) hipLaunchKernelGGL((dev::render_full<false, true, W_>), grid, block, lds, stream, P)
#define MYRT_RF0(W_) hipLaunchKernelGGL((dev::render_full<false, false, W_>), grid, block, lds, stream, P)
            if (deep) MYRT_BY_WALK(MYRT_RF1);
            else MYRT_BY_WALK(MYRT_RF0);
#undef MYRT_RF1
#undef MYRT_RF0
        }
    }
#undef MYRT_BY_WALK
    HIP_TRY(hipGetLastError());
    return RT_OK;
}

// Compacted bounce render for this launch (render.hip k_bounce): mirror/conductor scenes whose
// pixels trace one sample (Int(sqrt(spp)) == 1) with maxRecursionDepth <= kMaxQueueLevels.  A
// region of level L takes at most ceil(tiles / kQRegions) * 64 records (the worst case: every
// pixel reflects; render.hip q_reserve); by_need arenas take 1.25x the largest region count seen
// (DeviceReplica::qhint; 1/16 of the worst case before any is known) and grow when that rises.
// (false: allocation refused or failed -> the bounce megakernel.)
static bool queue_arena(const rt_scene* s, DeviceReplica& r, BounceArena* arena, RenderParams& P, int64_t tiles,
                        hipStream_t stream) {
    if (!arena || s->opt[kOptQueue] == 0) return false;
    if (P.cam.n != 1 || P.max_depth < 1 || P.max_depth > kMaxQueueLevels) return false;
    const int64_t levels = P.max_depth;
    const int64_t worst = (tiles + kQRegions - 1) / kQRegions * 64;
    // levels past k_bounce_tail's (option queue_tail) are traced in its lanes: no records
    const int64_t tail = s->opt[kOptQueueTail];
    const int64_t top = tail > 0 ? std::min(levels, tail) : levels;
    int64_t want[kMaxQueueLevels + 1] = {};
    bool grow = arena->base == nullptr || levels > arena->levels;
    for (int64_t L = 1; L <= levels; ++L) {
        const int64_t h = r.qhint[L];
        want[L] = L > top ? 0 : !arena->by_need ? worst : std::min(worst, h > 0 ? h + h / 4 + 64 : worst / 16 + 64);
        grow = grow || arena->cap[L] < want[L];
    }
    if (grow) {
        const int64_t lv = std::max(levels, arena->levels);
        int64_t cap[kMaxQueueLevels + 1] = {};
        int64_t recs = 0;
        for (int64_t L = 1; L <= lv; ++L) {
            cap[L] = std::max(L <= levels ? want[L] : 0, L <= arena->levels ? arena->cap[L] : 0);
            recs += kQRegions * cap[L];
        }
        const size_t bytes = (size_t)kQHdrWords * 8 + (size_t)recs * sizeof(BounceRec);
        if ((int64_t)bytes > kQueueBytesCap) return false;
        retire(r, arena->base, arena_bytes(*arena));
        arena->base = nullptr;
        arena->levels = 0;
        arena->recs = 0;
        std::memset(arena->hdr, 0, sizeof(arena->hdr));
        int64_t at = 0;
        for (int64_t L = 1; L <= lv; ++L) {
            arena->hdr[L] = (unsigned long long)at;
            arena->hdr[kQHdrCap + L] = (unsigned long long)cap[L];
            at += kQRegions * cap[L];
        }
        // header written and counters zeroed on the render's own stream: a plain hipMemset runs on
        // the null stream, which does not order against the library's non-blocking streams
        if (hipMalloc(&arena->base, bytes) != hipSuccess ||
            hipMemsetAsync(arena->base, 0, (size_t)kQHdrWords * 8, stream) != hipSuccess ||
            hipMemcpyAsync(arena->base, arena->hdr, sizeof(arena->hdr), hipMemcpyHostToDevice, stream) != hipSuccess) {
            (void)hipGetLastError();
            (void)hipFree(arena->base);
            arena->base = nullptr;
            return false;
        }
        arena->levels = lv;
        arena->recs = recs;
        for (int64_t L = 0; L <= kMaxQueueLevels; ++L) arena->cap[L] = L <= lv ? cap[L] : 0;
    }
    char* b = static_cast<char*>(arena->base);
    P.qhdr = reinterpret_cast<unsigned long long*>(b);
    P.bounce = reinterpret_cast<BounceRec*>(b + (size_t)kQHdrWords * 8);
    P.qneed = arena->by_need ? arena->qneed_dev : nullptr;
    P.qrecs = arena->recs;
    P.qlevels = (int32_t)arena->levels;
    arena->check = arena->by_need;
    arena->check_levels = levels;
    return true;
}

// After a by_need arena's render: fold its need into the replica's hint; true when a level
// overflowed (some of its rays were dropped: the render must run again on a larger arena).
static bool queue_overflowed(DeviceReplica& r, BounceArena& a) {
    if (!a.check) return false;
    a.check = false;
    bool over = false;
    for (int64_t L = 1; L <= a.check_levels; ++L) {
        const int64_t need = (int64_t)a.qneed[L];
        r.qhint[L] = std::max(r.qhint[L], need);
        over = over || need > a.cap[L];
    }
    return over;
}

// device.h xcd_tile on the host: block b -> tile of the row-major XCD-group mapping
static int64_t xcd_tile_host(int64_t b, int64_t nb, int64_t G) {
    if (G <= 1) return b;
    const int64_t round = 8 * G, full = nb / round * round;
    if (b >= full) return b;
    const int64_t x = b & 7, k = b >> 3;
    return ((k / G) * 8 + x) * G + (k % G);
}

// From the measured wave times: the XCD tile groups (G consecutive tiles, device.h xcd_tile) by
// their slowest tile, the top `pct` % of them first, slowest first, the rest in row-major order;
// then the same block -> position mapping as xcd_tile, so a group's tiles still share an XCD.
static int32_t build_tile_order(TileOrder& e, int64_t pct) {
    const int64_t n = e.n, G = std::max<int64_t>(1, e.key.group);
    std::vector<unsigned long long> c((size_t)(2 * n));
    HIP_TRY(hipMemcpy(c.data(), e.cost, c.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    std::vector<unsigned long long> dur((size_t)n, 0);
    for (int64_t b = 0; b < n; ++b) {
        const unsigned long long t0 = c[2 * b], t1 = c[2 * b + 1];
        dur[(size_t)xcd_tile_host(b, n, G)] = t1 > t0 ? t1 - t0 : 0;
    }
    const int64_t ng = n / G;                            // full groups; a partial last group stays last
    std::vector<unsigned long long> gc((size_t)ng, 0);
    for (int64_t g = 0; g < ng; ++g)
        for (int64_t t = g * G; t < g * G + G; ++t) gc[(size_t)g] = std::max(gc[(size_t)g], dur[(size_t)t]);
    std::vector<int64_t> byc((size_t)ng);
    for (int64_t g = 0; g < ng; ++g) byc[(size_t)g] = g;
    std::stable_sort(byc.begin(), byc.end(), [&](int64_t a, int64_t b) { return gc[(size_t)a] > gc[(size_t)b]; });
    const int64_t npro = (ng * pct + 99) / 100;
    std::vector<char> pro((size_t)ng, 0);
    std::vector<uint32_t> seq;
    seq.reserve((size_t)n);
    for (int64_t k = 0; k < npro; ++k) {
        const int64_t g = byc[(size_t)k];
        pro[(size_t)g] = 1;
        for (int64_t t = g * G; t < g * G + G; ++t) seq.push_back((uint32_t)t);
    }
    for (int64_t g = 0; g < ng; ++g)
        if (!pro[(size_t)g])
            for (int64_t t = g * G; t < g * G + G; ++t) seq.push_back((uint32_t)t);
    for (int64_t t = ng * G; t < n; ++t) seq.push_back((uint32_t)t);
    std::vector<uint32_t> ord((size_t)n);
    for (int64_t b = 0; b < n; ++b) ord[(size_t)b] = seq[(size_t)xcd_tile_host(b, n, G)];
    HIP_TRY(hipMemcpy(e.order, ord.data(), ord.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
    e.state = 2;
    return RT_OK;
}

// Before a megakernel launch of n blocks: the order of its (camera, chunk selection) when known
// (P.tile_order), else, the first time, its wave times are recorded (P.tile_cost; the returned
// entry's event is recorded behind the launch).  Renders while the first one runs use row-major
// order.  At most kMaxTileOrders selections are kept (least recently used out).
constexpr size_t kMaxTileOrders = 32;
static TileOrder* tile_order_for(const rt_scene* s, DeviceReplica& r, RenderParams& P, int64_t n) {
    const int64_t pct = s->opt[kOptTileOrder];
    if (pct <= 0 || n < 2) return nullptr;
    TileOrderKey k{};
    std::memcpy(k.eye, P.cam.eye, sizeof(k.eye));
    std::memcpy(k.w, P.cam.w, sizeof(k.w));
    k.width = P.cam.width; k.height = P.cam.height;
    k.first = P.chunk_first; k.step = P.chunk_step; k.chunks = P.num_chunks; k.group = P.xcd_remap;
    TileOrder* e = nullptr;
    for (TileOrder& o : r.orders)
        if (o.key == k && o.n == n) { e = &o; break; }
    if (!e) {
        if (r.orders.size() >= kMaxTileOrders) {
            auto lru = std::min_element(r.orders.begin(), r.orders.end(),
                                        [](const TileOrder& a, const TileOrder& b) { return a.used < b.used; });
            if (lru->state == 1) return nullptr;              // still being measured: keep it
            retire(r, lru->order, lru->n * 4); retire(r, lru->cost, lru->n * 16);
            if (lru->ev) (void)hipEventDestroy(lru->ev);
            r.orders.erase(lru);
        }
        TileOrder o;
        o.key = k;
        o.n = n;
        if (hipMalloc((void**)&o.order, (size_t)n * sizeof(uint32_t)) != hipSuccess ||
            hipMalloc((void**)&o.cost, (size_t)(2 * n) * sizeof(unsigned long long)) != hipSuccess ||
            hipEventCreateWithFlags(&o.ev, hipEventDisableTiming) != hipSuccess) {
            (void)hipGetLastError();
            (void)hipFree(o.order); (void)hipFree(o.cost);
            return nullptr;
        }
        r.orders.push_back(o);
        e = &r.orders.back();
    }
    e->used = ++r.order_clock;
    if (e->state == 1) {
        if (hipEventQuery(e->ev) != hipSuccess) { (void)hipGetLastError(); return nullptr; }
        if (build_tile_order(*e, pct) != RT_OK) { (void)hipGetLastError(); e->state = 0; return nullptr; }
    }
    if (e->state == 2) { P.tile_order = e->order; return nullptr; }
    P.tile_cost = e->cost;                                // state 0: this launch measures
    e->state = 1;
    return e;
}

static int32_t launch(const rt_scene* s, DeviceReplica& r, const RenderParams& P0, hipStream_t stream, bool count,
                      BounceArena* arena = nullptr, FullScratch* full_scratch = nullptr) {
    RenderParams P = P0;
    if (P.num_chunks == 0) return RT_OK;
    // dielectrics, area lights and maxRecursionDepth > kMaxDepthGPU: the full trace()
    // (render_full.h); it and spheres/planes exist only as megakernels
    const bool full = s->host.has_dielectric || P.num_alights > 0 || P.max_depth > kMaxDepthGPU;
    if (full) return launch_full(s, r, full_scratch ? *full_scratch : r.full, P, stream, count, s->host.has_dielectric,
                                 scene_is_rough(s->host));
    const int bt = kRenderBlock;
    dim3 grid = render_grid(P, bt, dev::kTileW);
    dim3 block((unsigned)bt, 1, 1);
    const size_t lds = (size_t)dev::kLds * bt * sizeof(unsigned long long) +
                       (size_t)(dev::kPixSlots + dev::kParkSlots) * bt * sizeof(double);
    const bool bounce = scene_has_bounce(s->host) && P.max_depth > 0;
    // The walk: identity scenes walk TLAS + BLAS as one tree; other scenes the unified transformed
    // walk (per-instance ray switches), or the nested general walk when the stack bound does not
    // allow one stack or for counting launches (reference-order counting needs the general walk)
    const bool unified = P.has_tlas && !P.count_ref && s->opt[kOptUnified] != 0;
    const int walk = (unified && P.identity) ? dev::kWalkIdentity
                     : (unified && P.ut && !count) ? (P.fit ? dev::kWalkFit : dev::kWalkTransformed) : dev::kWalkGeneral;
#define MYRT_LAUNCH(C_, B_, W_) hipLaunchKernelGGL((dev::render_kernel<C_, B_, W_>), grid, block, lds, stream, P)
#define MYRT_BY_WALK(M_)                                                    \
    do {                                                                    \
        if (walk == dev::kWalkIdentity) M_(dev::kWalkIdentity);             \
        else if (walk == dev::kWalkFit) M_(dev::kWalkFit);                  \
        else if (walk == dev::kWalkTransformed) M_(dev::kWalkTransformed);  \
        else M_(dev::kWalkGeneral);                                         \
    } while (0)
    if (bounce && !count && queue_arena(s, r, arena, P, (int64_t)grid.x * (bt / 64), stream)) {
        // primary + shadow rays of every pixel in the spill-free primary instantiation, then per
        // level the level's rays in coherent batches (k_bounce), then the need (k_queue_done)
        TileOrder* measuring = tile_order_for(s, r, P, (int64_t)grid.x);
#define MYRT_QPRIM(W_) hipLaunchKernelGGL((dev::render_kernel<false, false, W_, true>), grid, block, lds, stream, P)
        MYRT_BY_WALK(MYRT_QPRIM);
#undef MYRT_QPRIM
        if (measuring) HIP_TRY(hipEventRecord(measuring->ev, stream));
        const dim3 qgrid((unsigned)(r.cus * 4 * MYRT_QUEUE_WPE)), qblock(64);
        const size_t qlds = (size_t)dev::kLds * 64 * sizeof(unsigned long long);
        // option queue_levels (timing probe only: frames are incomplete below max_depth)
        const int64_t ql = s->opt[kOptQueueLevels];
        const int32_t levels = ql >= 0 ? (int32_t)std::min<int64_t>(ql, P.max_depth) : P.max_depth;
        const int64_t tail = s->opt[kOptQueueTail];
        for (int32_t level = 1; level <= levels; ++level) {
            // (a grid sized by the level's ray-count hint measured neutral: profiles/r06q_ab_c5.txt)
#define MYRT_QB(W_) hipLaunchKernelGGL((dev::k_bounce<W_>), qgrid, qblock, qlds, stream, P, level)
#define MYRT_QT(W_) hipLaunchKernelGGL((dev::k_bounce_tail<W_>), qgrid, qblock, qlds, stream, P, level)
            if (tail > 0 && level >= tail) {
                MYRT_BY_WALK(MYRT_QT);
                break;
            }
            MYRT_BY_WALK(MYRT_QB);
#undef MYRT_QT
#undef MYRT_QB
        }
        hipLaunchKernelGGL(dev::k_queue_done, dim3(1), dim3(64), 0, stream, P, (int)P.max_depth);
    } else if (count) {
        const bool u = walk == dev::kWalkIdentity;
        if (bounce) { if (u) MYRT_LAUNCH(true, true, dev::kWalkIdentity); else MYRT_LAUNCH(true, true, dev::kWalkGeneral); }
        else { if (u) MYRT_LAUNCH(true, false, dev::kWalkIdentity); else MYRT_LAUNCH(true, false, dev::kWalkGeneral); }
    } else {
        TileOrder* measuring = tile_order_for(s, r, P, (int64_t)grid.x);
#define MYRT_B1(W_) MYRT_LAUNCH(false, true, W_)
#define MYRT_B0(W_) MYRT_LAUNCH(false, false, W_)
        if (bounce) MYRT_BY_WALK(MYRT_B1);
        else MYRT_BY_WALK(MYRT_B0);
#undef MYRT_B1
#undef MYRT_B0
        if (measuring) HIP_TRY(hipEventRecord(measuring->ev, stream));
    }
#undef MYRT_BY_WALK
#undef MYRT_LAUNCH
    HIP_TRY(hipGetLastError());
    return RT_OK;
}

extern "C" {

const char* rt_last_error(void) { return g_err.c_str(); }
#define MYRT_STR2(x) #x
#define MYRT_STR(x) MYRT_STR2(x)
const char* rt_version(void) { return "myraytracer_amd 0.2 (abi " MYRT_STR(RT_ABI_VERSION) ", gfx950, fp64)"; }

int32_t rt_scene_create(const rt_scene_desc* desc, const int32_t* devices, int32_t n_devices, rt_scene** out) {
    if (!out) return fail(RT_ERR_INVALID_ARG, "out is NULL");
    *out = nullptr;
    if (!desc) return fail(RT_ERR_NO_SCENE, "No scene loaded. Can't render.");
    try {
        auto* s = new rt_scene();
        std::string err;
        int32_t rc = build_host_scene(desc, s->host, err);
        if (rc != RT_OK) { delete s; return fail(rc, err); }
        std::vector<int> devs;
        if (n_devices <= 0 || !devices) devs.push_back(0);
        else for (int k = 0; k < n_devices; ++k) devs.push_back(devices[k]);
        auto t0 = std::chrono::steady_clock::now();
        s->devs.resize(devs.size());
        for (size_t k = 0; k < devs.size(); ++k) {
            // replicas after the first copy from replica 0 when the fabric allows it
            const DeviceReplica* src = nullptr;
            if (k > 0) {
                int can = (devs[k] == devs[0]) ? 1 : 0;
                if (!can && hipDeviceCanAccessPeer(&can, devs[k], devs[0]) != hipSuccess) can = 0;
                if (can && devs[k] != devs[0]) {
                    (void)hipSetDevice(devs[k]);
                    const hipError_t pe = hipDeviceEnablePeerAccess(devs[0], 0);
                    if (pe != hipSuccess && pe != hipErrorPeerAccessAlreadyEnabled) can = 0;
                    (void)hipGetLastError();
                }
                if (can) src = &s->devs[0];
            }
            rc = make_replica(s->host, devs[k], s->devs[k], src);
            if (rc != RT_OK) {
                std::string e = g_err;
                for (auto& r : s->devs) free_replica(r);
                delete s;
                return fail(rc, e);
            }
        }
        s->upload_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        // device copies are authoritative; drop the large host arrays
        s->host.recs.clear(); s->host.recs.shrink_to_fit();
        s->host.crecs.clear(); s->host.crecs.shrink_to_fit();
        s->host.ctris.clear(); s->host.ctris.shrink_to_fit();
        s->host.tris.clear(); s->host.tris.shrink_to_fit();
        s->host.normals.clear(); s->host.normals.shrink_to_fit();
        s->host.wnodes.clear(); s->host.wnodes.shrink_to_fit();
        s->host.lbox.clear(); s->host.lbox.shrink_to_fit();
        *out = s;
        return RT_OK;
    } catch (const std::bad_alloc&) {
        return fail(RT_ERR_OOM, "host allocation failed");
    } catch (const std::exception& e) {
        return fail(RT_ERR_INVALID_ARG, e.what());
    }
}

void rt_scene_destroy(rt_scene* s) {
    if (!s) return;
    for (auto& r : s->devs) free_replica(r);
    delete s;
}

int32_t rt_scene_info_get(const rt_scene* s, rt_scene_info* out) {
    if (!s) return fail(RT_ERR_NO_SCENE, "No scene loaded.");
    if (!out) return fail(RT_ERR_INVALID_ARG, "out is NULL");
    const HostScene& S = s->host;
    out->meshes = S.n_meshes; out->triangles = S.n_tris; out->spheres = S.n_spheres; out->planes = S.n_planes;
    out->instances = (int64_t)S.insts.size();
    out->blas_nodes = S.blas_records; out->tlas_nodes = S.tlas_records; out->max_depth = S.max_stack;
    out->build_ms = S.build_ms; out->upload_ms = s->upload_ms;
    out->device_bytes = s->devs.empty() ? 0 : s->devs[0].bytes;
    out->scratch_bytes = s->devs.empty() ? 0 : scratch_bytes(s->devs[0]);
    return RT_OK;
}

static int32_t set_option(rt_scene* s, const char* name, int64_t value, bool unsafe_ok) {
    if (!s) return fail(RT_ERR_NO_SCENE, "No scene loaded.");
    if (!name) return fail(RT_ERR_INVALID_ARG, "option name is NULL");
    for (int k = 0; k < kOptCount; ++k) {
        if (std::strcmp(name, kOptDefs[k].name) != 0) continue;
        if (kOptDefs[k].unsafe && !unsafe_ok)
            return fail(RT_ERR_INVALID_ARG, std::string("option ") + name +
                                                " is a test hook (rt_scene_set_unsafe_option, not for production)");
        if (value < kOptDefs[k].lo || value > kOptDefs[k].hi)
            return fail(RT_ERR_INVALID_ARG, std::string("option ") + name + " out of range [" +
                                                std::to_string(kOptDefs[k].lo) + ", " + std::to_string(kOptDefs[k].hi) + "]");
        std::lock_guard<std::mutex> lock(s->mu);
        s->opt[k] = value;
        return RT_OK;
    }
    return fail(RT_ERR_INVALID_ARG, std::string("unknown option ") + name);
}

int32_t rt_scene_set_option(rt_scene* s, const char* name, int64_t value) { return set_option(s, name, value, false); }

int32_t rt_scene_set_unsafe_option(rt_scene* s, const char* name, int64_t value) {
    return set_option(s, name, value, true);
}

int32_t rt_scene_get_option(const rt_scene* s, const char* name, int64_t* value) {
    if (!s) return fail(RT_ERR_NO_SCENE, "No scene loaded.");
    if (!name || !value) return fail(RT_ERR_INVALID_ARG, "NULL argument");
    for (int k = 0; k < kOptCount; ++k)
        if (std::strcmp(name, kOptDefs[k].name) == 0) { *value = s->opt[k]; return RT_OK; }
    return fail(RT_ERR_INVALID_ARG, std::string("unknown option ") + name);
}

int32_t rt_render_device(rt_scene* s, int32_t slot, int32_t cam, int32_t first, int32_t step, double* d_rgb,
                         uint8_t* d_rgba8, void* stream) {
    if (!s) return fail(RT_ERR_NO_SCENE, "No scene loaded. Can't render.");
    if (slot < 0 || slot >= (int32_t)s->devs.size()) return fail(RT_ERR_INVALID_ARG, "bad device slot");
    if (step < 1 || first < 0) return fail(RT_ERR_INVALID_ARG, "bad chunk selection");
    int32_t rc = check_renderable(s, cam);
    if (rc != RT_OK) return rc;
    // the scene's lock: options, scratch growth and its retire list are shared with the submit path
    // (enqueueing only; rt_render_wait releases the lock while it blocks)
    std::lock_guard<std::mutex> lock(s->mu);
    DeviceReplica& r = s->devs[slot];
    HIP_TRY(hipSetDevice(r.device));
    hipStream_t st = (hipStream_t)stream;   // NULL = the default (null) stream, as torch's
    HIP_TRY(hipMemsetAsync(r.dev_counters, 0, kCounterWords * sizeof(unsigned long long), st));
    RenderParams P = make_params(s, r, cam, first, step, d_rgb, d_rgba8);
    P.counters = r.dev_counters;
    return launch(s, r, P, st, false, &r.dev_arena, &r.dev_full);
}

int32_t rt_stats_collect(rt_scene* s, int32_t slot, rt_stats* stats) {
    if (!s) return fail(RT_ERR_NO_SCENE, "No scene loaded.");
    if (slot < 0 || slot >= (int32_t)s->devs.size()) return fail(RT_ERR_INVALID_ARG, "bad device slot");
    DeviceReplica& r = s->devs[slot];
    HIP_TRY(hipSetDevice(r.device));
    unsigned long long c[kCounterWords];
    HIP_TRY(hipMemcpy(c, r.dev_counters, sizeof(c), hipMemcpyDeviceToHost));
    if (stats) {
        stats->shadow_rays = (int64_t)c[0]; stats->secondary_rays = (int64_t)c[1];
        stats->shadow_rays_traced = (int64_t)c[kCounterShadowTraced];
        stats->rewalked = (int64_t)c[kCounterTies];
    }
    return RT_OK;
}

int32_t rt_render_device_counted(rt_scene* s, int32_t slot, int32_t cam, int32_t first, int32_t step, double* d_rgb,
                                 void* stream, rt_work_counters* out) {
    if (!s) return fail(RT_ERR_NO_SCENE, "No scene loaded. Can't render.");
    if (slot < 0 || slot >= (int32_t)s->devs.size()) return fail(RT_ERR_INVALID_ARG, "bad device slot");
    int32_t rc = check_renderable(s, cam);
    if (rc != RT_OK) return rc;
    // the scene's lock: options, scratch growth and its retire list are shared with the submit path
    // (enqueueing only; rt_render_wait releases the lock while it blocks)
    std::lock_guard<std::mutex> lock(s->mu);
    DeviceReplica& r = s->devs[slot];
    HIP_TRY(hipSetDevice(r.device));
    hipStream_t st = (hipStream_t)stream;   // NULL = the default (null) stream, as torch's
    HIP_TRY(hipMemsetAsync(r.dev_counters, 0, kCounterWords * sizeof(unsigned long long), st));
    RenderParams P = make_params(s, r, cam, first, step, d_rgb, nullptr);
    P.counters = r.dev_counters;
    rc = launch(s, r, P, st, true, &r.dev_arena, &r.dev_full);   // 1) work this path executes
    if (rc != RT_OK) return rc;
    HIP_TRY(hipStreamSynchronize(st));
    unsigned long long c[kCounterWords];
    HIP_TRY(hipMemcpy(c, r.dev_counters, sizeof(c), hipMemcpyDeviceToHost));
    HIP_TRY(hipMemsetAsync(r.dev_counters, 0, kCounterWords * sizeof(unsigned long long), st));
    P.count_ref = 1;                                 // 2) the reference's work
    rc = launch(s, r, P, st, true, &r.dev_arena, &r.dev_full);
    if (rc != RT_OK) return rc;
    HIP_TRY(hipStreamSynchronize(st));
    unsigned long long q[kCounterWords];
    HIP_TRY(hipMemcpy(q, r.dev_counters, sizeof(q), hipMemcpyDeviceToHost));
    if (out) {
        out->records_fetched = (int64_t)c[2]; out->tri_tests = (int64_t)c[3]; out->normal_fetches = (int64_t)c[4];
        out->instance_entries = (int64_t)c[5]; out->pixels = (int64_t)c[6];
        out->ref_node_fetches = (int64_t)q[7]; out->ref_tri_tests = (int64_t)q[3];
        out->ref_smooth_hits = (int64_t)q[8]; out->ref_pixels = (int64_t)q[6];
        out->lane_steps_closest = (int64_t)c[9]; out->wave_steps_closest = (int64_t)c[10];
        out->lane_steps_shadow = (int64_t)c[11]; out->wave_steps_shadow = (int64_t)c[12];
        out->divergent_lane_loads = (int64_t)c[14]; out->divergent_distinct_records = (int64_t)c[15];
        for (int k = 0; k < 2; ++k) {
            out->iter_wave_inner[k] = (int64_t)c[16 + 5 * k]; out->iter_wave_leaf[k] = (int64_t)c[17 + 5 * k];
            out->iter_wave_scalar[k] = (int64_t)c[18 + 5 * k]; out->iter_lane_inner[k] = (int64_t)c[19 + 5 * k];
            out->iter_lane_leaf[k] = (int64_t)c[20 + 5 * k];
        }
    }
    reclaim(s);
    return RT_OK;
}

// True when [p, p+bytes) lies inside ONE page-locked host allocation (hipHostMalloc /
// hipHostRegister): the DMA engine can then write it directly.  NULL counts as true.
static bool pinned_range(const void* p, size_t bytes) {
    if (!p || bytes == 0) return true;
    const void* ends[2] = {p, static_cast<const char*>(p) + bytes - 1};
    unsigned long long id[2] = {0, 0};
    for (int k = 0; k < 2; ++k) {
        hipPointerAttribute_t a{};
        if (hipPointerGetAttributes(&a, ends[k]) != hipSuccess) { (void)hipGetLastError(); return false; }
        if (a.type != hipMemoryTypeHost) return false;
        if (hipPointerGetAttribute(&id[k], HIP_POINTER_ATTRIBUTE_BUFFER_ID,
                                   reinterpret_cast<hipDeviceptr_t>(const_cast<void*>(ends[k]))) != hipSuccess) {
            (void)hipGetLastError();
            return false;
        }
    }
    return id[0] == id[1];
}

int32_t rt_host_alloc(uint64_t bytes, void** out) {
    if (!out) return fail(RT_ERR_INVALID_ARG, "null output pointer");
    *out = nullptr;
    if (bytes == 0) return RT_OK;
    const unsigned fl = hipHostMallocMapped | hipHostMallocPortable;
    if (hipHostMalloc(out, bytes, fl) != hipSuccess) {
        (void)hipGetLastError();
        *out = nullptr;
        return fail(RT_ERR_OOM, "hipHostMalloc failed");
    }
    return RT_OK;
}

void rt_host_free(void* ptr) {
    if (ptr) (void)hipHostFree(ptr);
}


namespace myrt {
namespace dev {
// A render's ray counters to page-locked host memory, zeroed behind for the slot's next render:
// one tiny kernel on the render's stream (a D2H copy + memset would cross to the DMA engine
// and back between consecutive frames of a stream).
__global__ void k_counters_out(unsigned long long* counters, unsigned long long* host) {
    const int i = threadIdx.x;
    if (i < kCounterWords) {
        host[i] = counters[i];
        counters[i] = 0ull;
    }
}
}  // namespace dev
}  // namespace myrt

// ---- asynchronous renders into page-locked buffers (rt_render_submit / rt_render_wait).
// One launch per replica on slot (ticket mod kInFlight)'s stream; the kernels store the rows
// straight into the caller's buffers; the frame's ray counters follow in one async copy into
// pinned memory and are zeroed behind it.  Called with s->mu held.  *not_pinned: the outputs
// are not page-locked (rt_render_ex then takes its staged path).
static int32_t submit_impl(rt_scene* s, int32_t cam, int32_t first, int32_t step, double* out_rgb,
                           uint8_t* out_rgba8, uint32_t flags, int64_t* ticket, bool* not_pinned) {
    *not_pinned = false;
    // kernel timing events only when asked for (rt_render_ex always asks): each is a packet
    // on the stream, ~1 us of a C4/8 share's 85 us per frame (tools/probe_shares.py)
    const bool timing = (flags & RT_RENDER_KERNEL_TIME) != 0 && s->opt[kOptSubmitEvents] != 0;
    const rt_camera& C = s->host.cams[cam];
    const int32_t W = std::max(1, C.width), H = std::max(1, C.height);
    const bool frame = (flags & RT_RENDER_FRAME_LAYOUT) != 0;
    const int32_t rows = frame ? H : rt_rows_for_chunks(H, first, step);
    if (!pinned_range(out_rgb, (size_t)rows * W * 3 * sizeof(double)) || !pinned_range(out_rgba8, (size_t)rows * W * 4)) {
        *not_pinned = true;
        return fail(RT_ERR_INVALID_ARG, "rt_render_submit needs page-locked outputs (rt_host_alloc / rt_host_register)");
    }
    const int q = (int)(s->next_ticket % kInFlight);
    rt_scene::Pending& fp = s->flights[q];
    if (fp.pending)
        return fail(RT_ERR_BUSY, "too many renders in flight: wait for ticket " + std::to_string(fp.ticket) + " first");
    const int32_t D = (int32_t)s->devs.size();
    // Full trace() renders (dielectrics, area lights: render_full) take the stream and pass
    // scratch of slot q % full_flights, so up to full_flights of them overlap; deep recursion (one
    // deep-frame buffer per replica) stay on the replica's own stream, in order.
    const bool full = s->host.has_dielectric || !s->host.alights.empty() || s->host.max_depth > kMaxDepthGPU;
    const int32_t full_flights = (int32_t)s->opt[kOptFullFlights];
    const bool full_slots = full && s->host.max_depth <= kMaxDepthGPU && full_flights > 0;
    const bool concurrent = full ? full_slots : true;
    const int qs = full_slots ? q % full_flights : q;  // the slot whose stream (and full scratch) it takes
    const auto t0 = std::chrono::steady_clock::now();
    // the caller's buffers mapped for every replica BEFORE anything is launched: a replica
    // that cannot map them must not leave the others' kernels writing into them
    std::vector<double*> zrgb(D, nullptr);
    std::vector<uint8_t*> zrgba(D, nullptr);
    for (int32_t k = 0; k < D; ++k) {
        if (first + k * step >= num_chunks_total(H)) continue;
        HIP_TRY(hipSetDevice(s->devs[k].device));
        if ((out_rgb && hipHostGetDevicePointer((void**)&zrgb[k], out_rgb, 0) != hipSuccess) ||
            (out_rgba8 && hipHostGetDevicePointer((void**)&zrgba[k], out_rgba8, 0) != hipSuccess)) {
            (void)hipGetLastError();
            *not_pinned = true;
            return fail(RT_ERR_INVALID_ARG, "page-locked outputs are not mapped for this device");
        }
    }
    for (int32_t k = 0; k < D; ++k) s->devs[k].fl[q].used = false;
    // delivery: 0 = the kernel stores the rows into the host buffer; 1 = rows rendered into
    // device staging and copied by the DMA engine; 2 = staging only, not delivered
    // (measurement option submit_dma)
    const int dma = (int)s->opt[kOptSubmitDma];
    const bool counters_out = s->opt[kOptSubmitCounters] != 0;
    const int64_t fail_at = s->opt[kOptDebugFailReplica];   // test hook
    // replica k's launches, kept by value in the slot (Flight::relaunch): wait_impl runs them again
    // when the compacted bounce render's arena overflowed
    auto make_launch = [s, q, qs, first, step, D, H, W, cam, frame, dma, timing, counters_out, concurrent, full_slots,
                        fail_at, out_rgb, out_rgba8](int32_t k, double* zr, uint8_t* za) -> std::function<int32_t()> {
      return [s, q, qs, first, step, D, H, W, cam, frame, dma, timing, counters_out, concurrent, full_slots, fail_at,
              out_rgb, out_rgba8, k, zr, za]() -> int32_t {
        DeviceReplica& r = s->devs[k];
        Flight& f = r.fl[q];
        const int32_t myFirst = first + k * step, myStep = step * D;
        HIP_TRY(hipSetDevice(r.device));
        if (k == fail_at) return fail(RT_ERR_DEVICE, "injected launch failure (option debug_fail_replica)");
        hipStream_t st = concurrent ? r.fl[qs].stream : r.stream;
        int32_t nq = 0;
        for (int32_t c = myFirst; c < num_chunks_total(H); c += myStep) nq++;
        if (dma) {
            const int64_t px = (int64_t)nq * 8 * W;
            if (px > f.stage_px) {
                const int64_t cap = grown(px, f.stage_px);
                retire(r, f.stage_rgb, f.stage_px * 24); retire(r, f.stage_rgba, f.stage_px * 4);
                f.stage_rgb = nullptr; f.stage_rgba = nullptr; f.stage_px = 0;
                HIP_TRY(hipMalloc((void**)&f.stage_rgb, cap * 3 * sizeof(double)));
                HIP_TRY(hipMalloc((void**)&f.stage_rgba, cap * 4));
                f.stage_px = cap;
            }
        }
        if (!f.counters_zero) HIP_TRY(hipMemsetAsync(f.counters, 0, kCounterWords * sizeof(unsigned long long), st));
        f.counters_zero = false;
        f.used = true;                                   // work may be queued on its stream from here on
        if (timing) HIP_TRY(hipEventRecord(f.ev0, st));
        f.timed = timing;
        RenderParams P = make_params(s, r, cam, myFirst, myStep, dma ? (out_rgb ? f.stage_rgb : nullptr) : zr,
                                     dma ? (out_rgba8 ? f.stage_rgba : nullptr) : za);
        P.counters = f.counters;
        if (!dma) {                                      // rows at their places in the caller's buffer
            P.out_first = frame ? 0 : first;
            P.out_step = frame ? 1 : step;
        }                                                // else packed rows of this replica's chunks
        const int32_t rc = launch(s, r, P, st, false, concurrent ? &f.arena : &r.arena,
                                  full_slots ? &r.fl[qs].full : nullptr);
        if (rc != RT_OK) return rc;
        if (dma == 1) {
            // chunk q of this replica = selection entry k + q*D = image chunk myFirst + q*myStep;
            // its 8 rows go to output row 8*(base + q*stride): one 2-D copy for the full chunks
            const int32_t base = frame ? myFirst : k, stride = frame ? myStep : D;
            const bool lastPartial = (H % 8) != 0 && myFirst + (nq - 1) * myStep == num_chunks_total(H) - 1;
            const int32_t nfull = nq - (lastPartial ? 1 : 0);
            auto copy = [&](void* dst, const void* src, size_t bpp) -> hipError_t {
                const size_t rowB = (size_t)W * bpp, chunkB = 8 * rowB;
                hipError_t e = hipSuccess;
                if (nfull > 0)
                    e = hipMemcpy2DAsync(static_cast<char*>(dst) + (size_t)base * chunkB, (size_t)stride * chunkB, src,
                                         chunkB, chunkB, (size_t)nfull, hipMemcpyDeviceToHost, st);
                if (e == hipSuccess && lastPartial)
                    e = hipMemcpyAsync(static_cast<char*>(dst) + (size_t)(base + nfull * stride) * chunkB,
                                       static_cast<const char*>(src) + (size_t)nfull * chunkB, (size_t)(H % 8) * rowB,
                                       hipMemcpyDeviceToHost, st);
                return e;
            };
            if (out_rgb) HIP_TRY(copy(out_rgb, f.stage_rgb, 3 * sizeof(double)));
            if (out_rgba8) HIP_TRY(copy(out_rgba8, f.stage_rgba, 4));
        }
        if (timing) HIP_TRY(hipEventRecord(f.ev1, st));
        if (counters_out) {
            hipLaunchKernelGGL(dev::k_counters_out, dim3(1), dim3(64), 0, st, f.counters, f.host_counters_dev);
            HIP_TRY(hipGetLastError());
        }
        HIP_TRY(hipEventRecord(f.done, st));
        // the counters are zero again only when k_counters_out ran (it zeroes them behind its copy)
        f.counters_zero = counters_out;
        f.counters_valid = counters_out;
        return RT_OK;
      };
    };
    for (int32_t k = 0; k < D; ++k) {
        if (first + k * step >= num_chunks_total(H)) continue;
        Flight& fk = s->devs[k].fl[q];
        fk.relaunch = make_launch(k, zrgb[k], zrgba[k]);
        const int32_t rc = fk.relaunch();
        if (rc != RT_OK) {
            // replicas already launched write into the caller's buffers: drain them before the
            // error returns (the caller may free the buffers), and leave the slot free
            const std::string err = g_err;
            for (int32_t j = 0; j <= k; ++j) {
                Flight& f = s->devs[j].fl[q];
                if (!f.used) continue;
                (void)hipSetDevice(s->devs[j].device);
                (void)hipStreamSynchronize(concurrent ? s->devs[j].fl[qs].stream : s->devs[j].stream);
                f.used = false;
                f.counters_zero = false;
            }
            (void)hipGetLastError();
            return fail(rc, err);
        }
    }
    const int64_t n = (int64_t)std::sqrt((double)std::max(1, C.num_samples));
    fp.ticket = s->next_ticket++;
    fp.pending = true;
    fp.t0 = t0;
    fp.primary = (int64_t)rt_rows_for_chunks(H, first, step) * W * n * n;
    fp.concurrent = concurrent;
    if (ticket) *ticket = fp.ticket;
    return RT_OK;
}

// Wait for `ticket`; the scene lock is released while the host blocks on the GPU.
static int32_t wait_impl(rt_scene* s, std::unique_lock<std::mutex>& lock, int64_t ticket, rt_stats* stats) {
    const int q = (int)(((ticket % kInFlight) + kInFlight) % kInFlight);
    rt_scene::Pending& fp = s->flights[q];
    if (ticket < 0 || !fp.pending || fp.ticket != ticket)
        return fail(RT_ERR_INVALID_ARG, "unknown ticket, or already waited for");
    // one waiter per ticket: the slot stays pending (no submit can reuse it) until that waiter
    // has re-locked and read its counters; a second concurrent wait is refused
    if (fp.waiting) return fail(RT_ERR_INVALID_ARG, "ticket is already being waited for by another thread");
    fp.waiting = true;
    std::vector<std::pair<int, hipEvent_t>> evs;
    for (auto& r : s->devs)
        if (r.fl[q].used) evs.emplace_back(r.device, r.fl[q].done);
    lock.unlock();
    hipError_t e = hipSuccess;
    for (auto& de : evs) {
        if (e == hipSuccess) e = hipSetDevice(de.first);
        if (e == hipSuccess) e = hipEventSynchronize(de.second);
    }
    lock.lock();
    fp.waiting = false;
    // Compacted bounce render: a replica whose by_need arena overflowed (rays were dropped) renders
    // its share again on an arena grown to the need its render reported; a frame's need does not
    // change between runs, so one retry suffices (the third check is an error).
    for (int attempt = 0; e == hipSuccess; ++attempt) {
        std::vector<std::pair<int, hipEvent_t>> redo;
        for (auto& r : s->devs) {
            Flight& f = r.fl[q];
            if (!f.used || !queue_overflowed(r, f.arena)) continue;
            if (attempt == 2 || !f.relaunch) {
                fp.pending = false;
                return fail(RT_ERR_DEVICE, "compacted bounce queues overflowed again after growing");
            }
            const int32_t rc = f.relaunch();
            if (rc != RT_OK) {
                (void)hipStreamSynchronize(r.fl[q].stream);
                fp.pending = false;
                return rc;
            }
            redo.emplace_back(r.device, f.done);
        }
        if (redo.empty()) break;
        for (auto& de : redo) {
            if (e == hipSuccess) e = hipSetDevice(de.first);
            if (e == hipSuccess) e = hipEventSynchronize(de.second);
        }
    }
    fp.pending = false;
    if (e != hipSuccess) return fail(RT_ERR_DEVICE, std::string("render failed: ") + hipGetErrorString(e));
    double km = 0;
    int64_t sh = 0, se = 0, stc = 0, rw = 0;
    for (auto& r : s->devs) {
        Flight& f = r.fl[q];
        if (!f.used) continue;
        // with option submit_counters = 0 no counts came back: shadow/secondary stats are reported as 0
        const unsigned long long* c = f.host_counters;
        if (f.counters_valid) {
            sh += (int64_t)c[0]; se += (int64_t)c[1]; stc += (int64_t)c[kCounterShadowTraced]; rw += (int64_t)c[kCounterTies];
        }
        float ms = 0;
        if (f.timed && hipEventElapsedTime(&ms, f.ev0, f.ev1) != hipSuccess) (void)hipGetLastError();
        km = std::max(km, (double)ms);
    }
    if (stats) {
        stats->meshes = s->host.n_meshes; stats->triangles = s->host.n_tris;
        stats->spheres = s->host.n_spheres; stats->planes = s->host.n_planes;
        stats->primary_rays = fp.primary;
        stats->shadow_rays = sh; stats->secondary_rays = se; stats->kernel_ms = km;
        stats->shadow_rays_traced = stc;
        stats->rewalked = rw;
        stats->milliseconds = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - fp.t0).count();
    }
    reclaim(s);
    return RT_OK;
}

int32_t rt_render_submit(rt_scene* s, int32_t cam, int32_t first, int32_t step, double* out_rgb, uint8_t* out_rgba8,
                         uint32_t flags, int64_t* ticket) {
    if (!s) return fail(RT_ERR_NO_SCENE, "No scene loaded. Can't render.");
    if (s->devs.empty()) return fail(RT_ERR_NO_RENDERER, "Renderer not initialized.");
    if (step < 1 || first < 0) return fail(RT_ERR_INVALID_ARG, "bad chunk selection");
    if (flags & ~(uint32_t)(RT_RENDER_FRAME_LAYOUT | RT_RENDER_KERNEL_TIME))
        return fail(RT_ERR_INVALID_ARG, "unknown render flags");
    if (!ticket) return fail(RT_ERR_INVALID_ARG, "ticket is NULL");
    int32_t rc = check_renderable(s, cam);
    if (rc != RT_OK) return rc;
    std::lock_guard<std::mutex> lock(s->mu);
    bool not_pinned = false;
    return submit_impl(s, cam, first, step, out_rgb, out_rgba8, flags, ticket, &not_pinned);
}

int32_t rt_render_wait(rt_scene* s, int64_t ticket, rt_stats* stats) {
    if (!s) return fail(RT_ERR_NO_SCENE, "No scene loaded. Can't render.");
    std::unique_lock<std::mutex> lock(s->mu);
    return wait_impl(s, lock, ticket, stats);
}

// Host-buffer render across all device replicas (Renderer.render + renderRGBA8Async,
// Object+Extension.swift:52-379, RayTracer.swift:137-205).  Chunk k of the selection goes to
// replica (k mod D).  Outputs in page-locked memory (rt_host_alloc / rt_host_register) are
// written by the kernels themselves over PCIe (host-mapped, no copy); other host memory is
// filled from batches that render on the compute stream while a copy stream moves the
// previous batch into pinned staging and the calling thread scatters it.  Progress is
// reported after every batch and cancellation is honoured at batch granularity (SURVEY.md
// §8b; the reference's cancel was a no-op).  No collective is involved.
// flags & RT_RENDER_FRAME_LAYOUT: outputs are whole W x H frames and the selected chunks'
// rows land at their image rows (several processes can fill disjoint rows of one shared
// framebuffer: bench.py's multi-GPU gather).
int32_t rt_render_ex(rt_scene* s, int32_t cam, int32_t first, int32_t step, double* out_rgb, uint8_t* out_rgba8,
                     uint32_t flags, rt_stats* stats, rt_progress_fn progress, void* user) {
    if (!s) return fail(RT_ERR_NO_SCENE, "No scene loaded. Can't render.");
    if (s->devs.empty()) return fail(RT_ERR_NO_RENDERER, "Renderer not initialized.");
    if (step < 1 || first < 0) return fail(RT_ERR_INVALID_ARG, "bad chunk selection");
    if (flags & ~(uint32_t)RT_RENDER_FRAME_LAYOUT) return fail(RT_ERR_INVALID_ARG, "unknown render flags");
    int32_t rc = check_renderable(s, cam);
    if (rc != RT_OK) return rc;
    std::unique_lock<std::mutex> lock(s->mu);
    if (!progress && s->opt[kOptZerocopy] != 0) {
        // page-locked outputs: one submitted render (the kernels store the rows themselves)
        int64_t t = -1;
        bool not_pinned = false;
        rc = submit_impl(s, cam, first, step, out_rgb, out_rgba8, flags | RT_RENDER_KERNEL_TIME, &t, &not_pinned);
        if (rc == RT_OK) return wait_impl(s, lock, t, stats);
        if (!not_pinned && rc != RT_ERR_BUSY) return rc;
        (void)hipGetLastError();               // pageable outputs (or every slot busy): staged path
    }
    auto t0 = std::chrono::steady_clock::now();
    const rt_camera& C = s->host.cams[cam];
    const int32_t W = std::max(1, C.width), H = std::max(1, C.height);
    const bool frame = (flags & RT_RENDER_FRAME_LAYOUT) != 0;
    std::vector<int32_t> sel;
    for (int32_t c = first; c < num_chunks_total(H); c += step) sel.push_back(c);
    const int32_t D = (int32_t)s->devs.size();
    // output row of selection entry e: packed (rowOff) or its image row (frame layout)
    std::vector<int32_t> rowOff(sel.size() + 1, 0);
    for (size_t q = 0; q < sel.size(); ++q) rowOff[q + 1] = rowOff[q] + std::min(8, H - 8 * sel[q]);
    const int32_t rowsTotal = rowOff.back();
    auto dstRow = [&](size_t e) -> int32_t { return frame ? 8 * sel[e] : rowOff[e]; };
    const int32_t outRows = frame ? H : rowsTotal;
    // outputs in page-locked memory: finished rows go straight into the caller's buffer
    const bool direct = pinned_range(out_rgb, (size_t)outRows * W * 3 * sizeof(double)) &&
                        pinned_range(out_rgba8, (size_t)outRows * W * 4);
    // ... and the kernels can store them there themselves (host-mapped), for any number of
    // replicas: each maps the buffer and writes its own chunks' rows
    std::vector<double*> zc_rgb(D, nullptr);
    std::vector<uint8_t*> zc_rgba(D, nullptr);
    bool zerocopy = direct && s->opt[kOptZerocopy] != 0;
    for (int32_t k = 0; k < D && zerocopy; ++k) {
        HIP_TRY(hipSetDevice(s->devs[k].device));
        zerocopy = (!out_rgb || hipHostGetDevicePointer((void**)&zc_rgb[k], out_rgb, 0) == hipSuccess) &&
                   (!out_rgba8 || hipHostGetDevicePointer((void**)&zc_rgba[k], out_rgba8, 0) == hipSuccess);
    }
    (void)hipGetLastError();
    // Launches per replica.  Each batch ends on its slowest tile, so batches cost time
    // (~0.1-0.2 ms each on C3): they are used for progress granularity when a callback is
    // given, and otherwise only to overlap the copy of batch b with the render of b+1.
    const int32_t nBatches = s->opt[kOptBatches] > 0 ? (int32_t)s->opt[kOptBatches]
                                                    : (progress ? kRenderBatches : (zerocopy ? 1 : 2));

    // ---- per replica: its chunk list, batch plan, buffers; enqueue everything
    struct Plan { int32_t myFirst, myStep, nChunks, rows, nb, per; std::vector<int32_t> batchRow; };
    std::vector<Plan> plan(D);
    for (int32_t k = 0; k < D; ++k) {
        DeviceReplica& r = s->devs[k];
        Plan& pl = plan[k];
        pl.myFirst = first + k * step; pl.myStep = step * D;
        pl.nChunks = 0;
        for (int32_t c = pl.myFirst; c < num_chunks_total(H); c += pl.myStep) pl.nChunks++;
        pl.rows = rt_rows_for_chunks(H, pl.myFirst, pl.myStep);
        if (pl.nChunks == 0) { pl.nb = 0; continue; }
        pl.per = (pl.nChunks + nBatches - 1) / nBatches;
        pl.nb = (pl.nChunks + pl.per - 1) / pl.per;
        pl.batchRow.assign(pl.nb + 1, 0);
        for (int32_t b = 0; b < pl.nb; ++b) {
            const int32_t c0 = pl.myFirst + b * pl.per * pl.myStep;
            const int32_t nc = std::min(pl.per, pl.nChunks - b * pl.per);
            pl.batchRow[b + 1] = pl.batchRow[b] + rt_rows_for_chunks(H, c0, pl.myStep) -
                                 rt_rows_for_chunks(H, c0 + nc * pl.myStep, pl.myStep);
        }
        HIP_TRY(hipSetDevice(r.device));
        const int64_t px = (int64_t)pl.rows * W;
        if (!zerocopy && px > r.out_cap_px) {
            const int64_t cap = grown(px, r.out_cap_px);
            retire(r, r.out_d, r.out_cap_px * 24); retire(r, r.out8_d, r.out_cap_px * 4);
            r.out_d = nullptr; r.out8_d = nullptr; r.out_cap_px = 0;
            HIP_TRY(hipMalloc((void**)&r.out_d, cap * 3 * sizeof(double)));
            HIP_TRY(hipMalloc((void**)&r.out8_d, cap * 4));
            r.out_cap_px = cap;
        }
        if (!direct && px > r.host_cap_px) {
            if (r.host_rgb) (void)hipHostFree(r.host_rgb);
            if (r.host_rgba) (void)hipHostFree(r.host_rgba);
            r.host_rgb = nullptr; r.host_rgba = nullptr; r.host_cap_px = 0;
            HIP_TRY(hipHostMalloc((void**)&r.host_rgb, px * 3 * sizeof(double), hipHostMallocDefault));
            HIP_TRY(hipHostMalloc((void**)&r.host_rgba, px * 4, hipHostMallocDefault));
            r.host_cap_px = px;
        }
        if (!r.counters_zero)
            HIP_TRY(hipMemsetAsync(r.counters, 0, kCounterWords * sizeof(unsigned long long), r.stream));
        r.counters_zero = false;
        HIP_TRY(hipEventRecord(r.ev0, r.stream));
    }
    // batch b of every replica is enqueued before batch b-1 is drained: one batch renders
    // while the previous one is copied and scattered; cancellation stops further launches
    int32_t maxNb = 0;
    for (const auto& pl : plan) maxNb = std::max(maxNb, pl.nb);
    auto enqueue = [&](int32_t b) -> int32_t {
        for (int32_t k = 0; k < D; ++k) {
            const Plan& pl = plan[k];
            if (b >= pl.nb) continue;
            DeviceReplica& r = s->devs[k];
            HIP_TRY(hipSetDevice(r.device));
            const int32_t c0 = pl.myFirst + b * pl.per * pl.myStep;
            const int32_t nc = std::min(pl.per, pl.nChunks - b * pl.per);
            double* drgb;
            uint8_t* drgba;
            if (zerocopy) {          // the caller's buffer, addressed by the global row mapping
                drgb = zc_rgb[k];
                drgba = zc_rgba[k];
            } else {                 // this batch's rows, packed, in device staging
                drgb = out_rgb ? r.out_d + (size_t)pl.batchRow[b] * W * 3 : nullptr;
                drgba = out_rgba8 ? r.out8_d + (size_t)pl.batchRow[b] * W * 4 : nullptr;
            }
            RenderParams P = make_params(s, r, cam, c0, pl.myStep, drgb, drgba);
            P.num_chunks = nc;
            if (zerocopy) {
                P.out_first = frame ? 0 : first;
                P.out_step = frame ? 1 : step;
            }
            const int32_t lrc = launch(s, r, P, r.stream, false, &r.arena);
            if (lrc != RT_OK) return lrc;
            HIP_TRY(hipEventRecord(r.batch_done[b], r.stream));
            if (b == pl.nb - 1) {
                // last launch of this replica: kernel time ends here; its counters follow
                // in one async copy and are zeroed behind it (the next frame skips its memset)
                HIP_TRY(hipEventRecord(r.ev1, r.stream));
                HIP_TRY(hipMemcpyAsync(r.host_counters, r.counters, kCounterWords * sizeof(unsigned long long),
                                       hipMemcpyDeviceToHost, r.stream));
                HIP_TRY(hipEventRecord(r.counters_ready, r.stream));
                HIP_TRY(hipMemsetAsync(r.counters, 0, kCounterWords * sizeof(unsigned long long), r.stream));
                r.counters_zero = true;
            }
            const size_t nrows = (size_t)(pl.batchRow[b + 1] - pl.batchRow[b]);
            if (zerocopy) {                                  // rows already in the caller's buffer
                HIP_TRY(hipEventRecord(r.batch_copied[b], r.stream));
                continue;
            }
            HIP_TRY(hipStreamWaitEvent(r.copy_stream, r.batch_done[b], 0));
            if (direct) {
                // replica k's q-th chunk is selection entry k + q*D; its rows follow the
                // batch's earlier chunks in drgb.  Runs of adjacent output rows are one copy.
                int32_t q = b * pl.per;
                const int32_t qEnd = q + nc;
                size_t srcRow = 0;
                while (q < qEnd) {
                    const size_t e0 = (size_t)k + (size_t)q * D;
                    int32_t nr = rowOff[e0 + 1] - rowOff[e0];
                    int32_t q1 = q + 1;
                    while (q1 < qEnd) {
                        const size_t e = (size_t)k + (size_t)q1 * D;
                        if (dstRow(e) != dstRow(e0) + nr) break;
                        nr += rowOff[e + 1] - rowOff[e];
                        ++q1;
                    }
                    const size_t d0 = (size_t)dstRow(e0);
                    if (out_rgb)
                        HIP_TRY(hipMemcpyAsync(out_rgb + d0 * W * 3, drgb + srcRow * W * 3,
                                               (size_t)nr * W * 3 * sizeof(double), hipMemcpyDeviceToHost,
                                               r.copy_stream));
                    if (out_rgba8)
                        HIP_TRY(hipMemcpyAsync(out_rgba8 + d0 * W * 4, drgba + srcRow * W * 4,
                                               (size_t)nr * W * 4, hipMemcpyDeviceToHost, r.copy_stream));
                    srcRow += (size_t)nr;
                    q = q1;
                }
            } else {
                if (out_rgb)
                    HIP_TRY(hipMemcpyAsync(r.host_rgb + (size_t)pl.batchRow[b] * W * 3, drgb,
                                           nrows * W * 3 * sizeof(double), hipMemcpyDeviceToHost, r.copy_stream));
                if (out_rgba8)
                    HIP_TRY(hipMemcpyAsync(r.host_rgba + (size_t)pl.batchRow[b] * W * 4, drgba, nrows * W * 4,
                                           hipMemcpyDeviceToHost, r.copy_stream));
            }
            HIP_TRY(hipEventRecord(r.batch_copied[b], r.copy_stream));
        }
        return RT_OK;
    };
    if (maxNb > 0 && (rc = enqueue(0)) != RT_OK) return rc;
    int32_t enqueued = maxNb > 0 ? 1 : 0;
    // ---- drain: scatter each finished batch, report progress, honour cancellation
    int32_t rowsDone = 0;
    bool cancelled = false;
    for (int32_t b = 0; b < enqueued; ++b) {
        if (!cancelled && enqueued < maxNb) {
            if ((rc = enqueue(enqueued)) != RT_OK) return rc;
            enqueued++;
        }
        for (int32_t k = 0; k < D; ++k) {
            const Plan& pl = plan[k];
            if (b >= pl.nb) continue;
            DeviceReplica& r = s->devs[k];
            HIP_TRY(hipSetDevice(r.device));
            HIP_TRY(hipEventSynchronize(r.batch_copied[b]));
            if (cancelled) continue;
            if (direct) {
                rowsDone += pl.batchRow[b + 1] - pl.batchRow[b];
                if (progress && !progress(user, rowsDone, rowsTotal)) cancelled = true;
                continue;
            }
            // replica k's q-th chunk is selection entry k + q*D; chunks are scattered by
            // several threads (host memcpy bandwidth, not PCIe, bounds this step)
            const int32_t q0 = b * pl.per, q1 = std::min(pl.nChunks, q0 + pl.per);
            std::vector<int32_t> src(q1 - q0 + 1, pl.batchRow[b]);
            for (int32_t q = q0; q < q1; ++q) {
                const size_t e = (size_t)k + (size_t)q * D;
                src[q - q0 + 1] = src[q - q0] + (rowOff[e + 1] - rowOff[e]);
            }
            auto copy_chunks = [&](int32_t qa, int32_t qb) {
                for (int32_t q = qa; q < qb; ++q) {
                    const size_t e = (size_t)k + (size_t)q * D;
                    const int32_t nr = rowOff[e + 1] - rowOff[e];
                    const int32_t sr = src[q - q0];
                    const size_t dr = (size_t)dstRow(e);
                    if (out_rgb) std::memcpy(out_rgb + dr * W * 3, r.host_rgb + (size_t)sr * W * 3,
                                             (size_t)nr * W * 3 * sizeof(double));
                    if (out_rgba8) std::memcpy(out_rgba8 + dr * W * 4, r.host_rgba + (size_t)sr * W * 4,
                                               (size_t)nr * W * 4);
                }
            };
            const int32_t nq = q1 - q0;
            const int32_t nt = std::max(1, std::min<int32_t>(nq, (int32_t)std::min(8u, std::thread::hardware_concurrency())));
            if (nt <= 1 || (int64_t)nq * 8 * W < 65536) {
                copy_chunks(q0, q1);
            } else {
                std::vector<std::thread> th;
                for (int32_t t = 1; t < nt; ++t)
                    th.emplace_back(copy_chunks, q0 + nq * t / nt, q0 + nq * (t + 1) / nt);
                copy_chunks(q0, q0 + nq / nt);
                for (auto& x : th) x.join();
            }
            rowsDone += src.back() - src.front();
            if (progress && !progress(user, rowsDone, rowsTotal)) cancelled = true;
        }
    }
    double km = 0;
    int64_t sh = 0, se = 0, st = 0, rw = 0;
    for (int32_t k = 0; k < D; ++k) {
        if (plan[k].nb == 0) continue;
        DeviceReplica& r = s->devs[k];
        HIP_TRY(hipSetDevice(r.device));
        if (enqueued < plan[k].nb) {            // cancelled before the last batch: drain, count
            HIP_TRY(hipEventRecord(r.ev1, r.stream));
            HIP_TRY(hipMemcpyAsync(r.host_counters, r.counters, kCounterWords * sizeof(unsigned long long),
                                   hipMemcpyDeviceToHost, r.stream));
            HIP_TRY(hipEventRecord(r.counters_ready, r.stream));
        }
        HIP_TRY(hipEventSynchronize(r.counters_ready));
        const unsigned long long* c = r.host_counters;
        sh += (int64_t)c[0]; se += (int64_t)c[1]; st += (int64_t)c[kCounterShadowTraced]; rw += (int64_t)c[kCounterTies];
        float ms = 0; (void)hipEventElapsedTime(&ms, r.ev0, r.ev1);
        km = std::max(km, (double)ms);
    }
    if (cancelled) return fail(RT_ERR_CANCELLED, "cancelled");
    if (stats) {
        stats->meshes = s->host.n_meshes; stats->triangles = s->host.n_tris;
        stats->spheres = s->host.n_spheres; stats->planes = s->host.n_planes;
        const int64_t n = (int64_t)std::sqrt((double)std::max(1, C.num_samples));
        stats->primary_rays = (int64_t)rowsTotal * W * n * n;
        stats->shadow_rays = sh; stats->secondary_rays = se; stats->kernel_ms = km;
        stats->shadow_rays_traced = st;
        stats->rewalked = rw;
        stats->milliseconds = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    reclaim(s);
    return RT_OK;
}

int32_t rt_render(rt_scene* s, int32_t cam, int32_t first, int32_t step, double* out_rgb, uint8_t* out_rgba8,
                  rt_stats* stats, rt_progress_fn progress, void* user) {
    return rt_render_ex(s, cam, first, step, out_rgb, out_rgba8, 0u, stats, progress, user);
}

int32_t rt_host_register(void* ptr, uint64_t bytes) {
    if (!ptr || bytes == 0) return fail(RT_ERR_INVALID_ARG, "null or empty host range");
    const hipError_t e = hipHostRegister(ptr, bytes, hipHostRegisterMapped | hipHostRegisterPortable);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return fail(RT_ERR_DEVICE, std::string("hipHostRegister: ") + hipGetErrorString(e));
    }
    return RT_OK;
}

int32_t rt_host_unregister(void* ptr) {
    if (!ptr) return RT_OK;
    const hipError_t e = hipHostUnregister(ptr);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return fail(RT_ERR_DEVICE, std::string("hipHostUnregister: ") + hipGetErrorString(e));
    }
    return RT_OK;
}

// ---- PLY
int32_t rt_ply_load(const char* path, rt_ply_mesh* out) {
    if (!out) return fail(RT_ERR_INVALID_ARG, "out is NULL");
    std::memset(out, 0, sizeof(*out));
    std::vector<double> pos, nrm; std::vector<float> uv; std::vector<int32_t> idx;
    std::string err;
    try {
        int32_t rc = ply_load(path, pos, nrm, uv, idx, err);
        if (rc != RT_OK) return fail(rc, err);
    } catch (const std::exception& e) {
        return fail(RT_ERR_PLY, e.what());
    }
    auto dup = [](const auto& v, auto** dst) {
        using T = typename std::decay_t<decltype(v)>::value_type;
        *dst = v.empty() ? nullptr : static_cast<T*>(std::malloc(v.size() * sizeof(T)));
        if (*dst) std::memcpy(*dst, v.data(), v.size() * sizeof(T));
    };
    dup(pos, &out->positions); out->num_positions = (int64_t)pos.size() / 3;
    dup(nrm, &out->normals); out->num_normals = (int64_t)nrm.size() / 3;
    dup(uv, &out->texcoords); out->num_texcoords = (int64_t)uv.size() / 2;
    dup(idx, &out->indices); out->num_indices = (int64_t)idx.size();
    return RT_OK;
}

void rt_ply_free(rt_ply_mesh* m) {
    if (!m) return;
    std::free(m->positions); std::free(m->normals); std::free(m->texcoords); std::free(m->indices);
    std::memset(m, 0, sizeof(*m));
}

// ---- debug / test hooks ---------------------------------------------------------------
// Host-only scene build (no device): BVH hashes per instance (+ TLAS at [n]) and info.
int32_t rt_debug_host_build(const rt_scene_desc* desc, uint64_t* hashes, int32_t max_hashes, int32_t* n_instances,
                            rt_scene_info* info) {
    if (!desc) return fail(RT_ERR_NO_SCENE, "No scene loaded.");
    try {
        HostScene S;
        std::string err;
        int32_t rc = build_host_scene(desc, S, err);
        if (rc != RT_OK) return fail(rc, err);
        const int32_t n = (int32_t)S.inst_bvh_hash.size();
        if (n_instances) *n_instances = n;
        if (hashes) {
            for (int32_t k = 0; k < n && k < max_hashes; ++k) hashes[k] = S.inst_bvh_hash[k];
            if (n < max_hashes) hashes[n] = S.tlas_hash;
        }
        if (info) {
            std::memset(info, 0, sizeof(*info));
            info->meshes = S.n_meshes; info->triangles = S.n_tris; info->instances = n;
            info->blas_nodes = S.blas_records; info->tlas_nodes = S.tlas_records; info->max_depth = S.max_stack;
            info->build_ms = S.build_ms;
            info->device_bytes = (int64_t)(S.recs.size() * sizeof(WRec) + S.tris.size() * sizeof(TriRec) +
                                           S.normals.size() * sizeof(double));
        }
        return RT_OK;
    } catch (const std::exception& e) {
        return fail(RT_ERR_INVALID_ARG, e.what());
    }
}

int32_t rt_debug_fit_build(const rt_scene_desc* desc, int64_t* out) {
    if (!desc) return fail(RT_ERR_NO_SCENE, "No scene loaded.");
    if (!out) return fail(RT_ERR_INVALID_ARG, "NULL argument");
    try {
        HostScene S;
        std::string err;
        const int32_t rc = build_host_scene(desc, S, err);
        if (rc != RT_OK) return fail(rc, err);
        for (int k = 0; k < 5; ++k) out[k] = 0;
        int64_t runs = 0;                       // leaf runs over all instances (the pairs the tree must hold)
        for (const DInstance& I : S.insts) {
            if (I.kind != kPrimTriangles) continue;
            if (I.root_ref < 0) { ++runs; continue; }
            std::vector<int32_t> st{I.root_ref};
            while (!st.empty()) {
                const WRec& r = S.recs[st.back()];
                st.pop_back();
                for (int c = 0; c < 2; ++c) {
                    if (r.ref[c] < 0) ++runs;
                    else st.push_back(r.ref[c]);
                }
            }
        }
        out[3] = runs;
        if (S.fit_root < 0) return RT_OK;
        uint64_t h = 1469598103934665603ull;
        auto mix = [&](const void* p, size_t n) {
            const unsigned char* b = static_cast<const unsigned char*>(p);
            for (size_t i = 0; i < n; ++i) { h ^= b[i]; h *= 1099511628211ull; }
        };
        mix(S.fpairs.data(), S.fpairs.size() * sizeof(DFitPair));
        mix(&S.wnodes[(size_t)S.fit_root], (size_t)S.fit_nodes * sizeof(W4Node));
        out[0] = (int64_t)S.fpairs.size();
        out[1] = S.fit_nodes;
        out[2] = S.fit_depth;
        out[4] = (int64_t)(h >> 1);
        return RT_OK;
    } catch (const std::exception& e) {
        return fail(RT_ERR_INVALID_ARG, e.what());
    }
}

// ---- debug: explicit rays through the render kernels' traversal
static int32_t debug_rays(rt_scene* s, int32_t slot, int32_t n, const double* o, const double* d, const double* tl,
                          const double* time, double* out_t, double* out_p, double* out_n, int32_t* out_mat,
                          uint8_t* out_occ) {
    if (!s) return fail(RT_ERR_NO_SCENE, "No scene loaded.");
    if (slot < 0 || slot >= (int32_t)s->devs.size()) return fail(RT_ERR_INVALID_ARG, "bad device slot");
    if (n < 0 || (n > 0 && (!o || !d || !tl || !time))) return fail(RT_ERR_INVALID_ARG, "bad ray arrays");
    if (n == 0) return RT_OK;
    std::lock_guard<std::mutex> lock(s->mu);
    DeviceReplica& r = s->devs[slot];
    HIP_TRY(hipSetDevice(r.device));
    RenderParams P = make_params(s, r, 0, 0, 1, nullptr, nullptr);
    {   // margin for these rays' own origins
        double od = 0.0;
        double dm = 0.0;
        for (int32_t k = 0; k < n; ++k) {
            od = std::max(od, dist_to_center(s->host, o + 3 * (size_t)k));
            const double* dk = d + 3 * (size_t)k;
            const double dn = std::sqrt(dk[0] * dk[0] + dk[1] * dk[1] + dk[2] * dk[2]);
            dm = std::isfinite(dn) ? std::max(dm, dn) : HUGE_VAL;
        }
        P.prune_abs = prune_abs_for(s->host, od);
        P.fast_rcp = fast_rcp_for(s->host, 2.0 * dm + 1.0);
        double oc = 0.0;                      // the wide walk's widening for these origins
        for (int32_t k = 0; k < 3 * n; ++k) oc = std::isfinite(o[k]) ? std::max(oc, std::fabs(o[k])) : HUGE_VAL;
        set_wide(s->host, r, P, oc, s->opt[kOptWide] != 0, s->opt[kOptWideDeltaScale], s->opt[kOptFit] != 0);
    }
    dev::RayBatch B{};
    B.n = n;
    const bool unified = P.has_tlas && s->opt[kOptUnified] != 0;
    B.uni = (unified && P.identity) ? 1 : (unified && P.ut) ? (P.fit ? 3 : 2) : 0;   // the render kernels' walk
    std::vector<void*> allocs;
    auto dalloc = [&](size_t bytes, void** p) -> int32_t {
        HIP_TRY(hipMalloc(p, std::max<size_t>(bytes, 8)));
        allocs.push_back(*p);
        return RT_OK;
    };
    int32_t rc = RT_OK;
    double *dO, *dD, *dL, *dT;
    if ((rc = dalloc((size_t)n * 24, (void**)&dO)) || (rc = dalloc((size_t)n * 24, (void**)&dD)) ||
        (rc = dalloc((size_t)n * 8, (void**)&dL)) || (rc = dalloc((size_t)n * 8, (void**)&dT))) {
        for (void* p : allocs) (void)hipFree(p);
        return rc;
    }
    HIP_TRY(hipMemcpy(dO, o, (size_t)n * 24, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(dD, d, (size_t)n * 24, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(dL, tl, (size_t)n * 8, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(dT, time, (size_t)n * 8, hipMemcpyHostToDevice));
    B.o = dO; B.d = dD; B.tlim = dL; B.time = dT;
    const dim3 grid((unsigned)((n + 255) / 256)), block(256);
    const size_t lds = (size_t)dev::kLds * 256 * sizeof(unsigned long long);
    if (out_occ) {
        if ((rc = dalloc((size_t)n, (void**)&B.out_occ)) != RT_OK) { for (void* p : allocs) (void)hipFree(p); return rc; }
        hipLaunchKernelGGL(dev::k_occluded_rays, grid, block, lds, r.stream, P, B);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipStreamSynchronize(r.stream));
        HIP_TRY(hipMemcpy(out_occ, B.out_occ, (size_t)n, hipMemcpyDeviceToHost));
    } else {
        if ((rc = dalloc((size_t)n * 8, (void**)&B.out_t)) || (rc = dalloc((size_t)n * 24, (void**)&B.out_p)) ||
            (rc = dalloc((size_t)n * 24, (void**)&B.out_n)) || (rc = dalloc((size_t)n * 4, (void**)&B.out_mat))) {
            for (void* p : allocs) (void)hipFree(p);
            return rc;
        }
        hipLaunchKernelGGL(dev::k_trace_rays, grid, block, lds, r.stream, P, B);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipStreamSynchronize(r.stream));
        HIP_TRY(hipMemcpy(out_t, B.out_t, (size_t)n * 8, hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(out_p, B.out_p, (size_t)n * 24, hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(out_n, B.out_n, (size_t)n * 24, hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(out_mat, B.out_mat, (size_t)n * 4, hipMemcpyDeviceToHost));
    }
    for (void* p : allocs) (void)hipFree(p);
    return RT_OK;
}

int32_t rt_debug_trace_rays(rt_scene* s, int32_t slot, int32_t n, const double* o, const double* d,
                            const double* tmin, const double* time, double* out_t, double* out_p, double* out_n,
                            int32_t* out_mat) {
    if (n > 0 && (!out_t || !out_p || !out_n || !out_mat)) return fail(RT_ERR_INVALID_ARG, "bad output arrays");
    return debug_rays(s, slot, n, o, d, tmin, time, out_t, out_p, out_n, out_mat, nullptr);
}
int32_t rt_debug_occluded_rays(rt_scene* s, int32_t slot, int32_t n, const double* o, const double* d,
                               const double* tmax, const double* time, uint8_t* out) {
    if (n > 0 && !out) return fail(RT_ERR_INVALID_ARG, "bad output array");
    return debug_rays(s, slot, n, o, d, tmax, time, nullptr, nullptr, nullptr, nullptr, out);
}

// ---- debug: canonical BVH hashes (tests compare them with the oracle's)
int32_t rt_debug_wave_times(rt_scene* s, int32_t slot, int32_t cam, int32_t first, int32_t step, double* d_out_rgb,
                            uint64_t* out, int64_t max_waves, int64_t* n_waves) {
    if (!MYRT_WAVE_TIMES)
        return fail(RT_ERR_UNSUPPORTED, "wave timeline not compiled in (build with -DMYRT_WAVE_TIMES=1, "
                                        "tools/build_variants.sh)");
    if (!s) return fail(RT_ERR_NO_SCENE, "No scene loaded. Can't render.");
    if (slot < 0 || slot >= (int32_t)s->devs.size()) return fail(RT_ERR_INVALID_ARG, "bad device slot");
    int32_t rc = check_renderable(s, cam);
    if (rc != RT_OK) return rc;
    std::lock_guard<std::mutex> lock(s->mu);
    DeviceReplica& r = s->devs[slot];
    HIP_TRY(hipSetDevice(r.device));
    RenderParams P = make_params(s, r, cam, first, step, d_out_rgb, nullptr);
    const int bt = kRenderBlock;
    const int64_t waves = (int64_t)render_grid(P, bt, dev::kTileW).x * (bt / 64);
    if (waves > r.wave_times_cap) {
        (void)hipFree(r.wave_times); r.wave_times = nullptr; r.wave_times_cap = 0;
        HIP_TRY(hipMalloc((void**)&r.wave_times, (size_t)waves * 3 * sizeof(unsigned long long)));
        r.wave_times_cap = waves;
    }
    HIP_TRY(hipMemsetAsync(r.wave_times, 0, (size_t)waves * 3 * sizeof(unsigned long long), r.stream));
    P.wave_times = r.wave_times;
    HIP_TRY(hipMemsetAsync(r.counters, 0, kCounterWords * sizeof(unsigned long long), r.stream));
    r.counters_zero = false;
    if ((rc = launch(s, r, P, r.stream, false, &r.arena)) != RT_OK) return rc;
    HIP_TRY(hipStreamSynchronize(r.stream));
    const int64_t n = std::min<int64_t>(waves, max_waves);
    if (out && n > 0) HIP_TRY(hipMemcpy(out, r.wave_times, (size_t)n * 3 * sizeof(uint64_t), hipMemcpyDeviceToHost));
    if (n_waves) *n_waves = waves;
    return RT_OK;
}

namespace myrt {
namespace dev {
__global__ void k_rcp(int32_t n, const double* x, double* f, double* q) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    f[i] = rcp_rn(x[i]);
    q[i] = 1.0 / x[i];
}
}  // namespace dev
}  // namespace myrt

int32_t rt_debug_rcp(int32_t n, const double* x, double* out_fast, double* out_div) {
    if (n < 0 || (n > 0 && (!x || !out_fast || !out_div))) return fail(RT_ERR_INVALID_ARG, "bad arrays");
    if (n == 0) return RT_OK;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        (void)hipGetLastError();
        return fail(RT_ERR_DEVICE, "no HIP device");
    }
    HIP_TRY(hipSetDevice(0));
    double* d = nullptr;
    HIP_TRY(hipMalloc((void**)&d, (size_t)n * 3 * sizeof(double)));
    hipError_t e = hipMemcpy(d, x, (size_t)n * sizeof(double), hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(dev::k_rcp, dim3((n + 255) / 256), dim3(256), 0, 0, n, d, d + n, d + 2 * (size_t)n);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpy(out_fast, d + n, (size_t)n * sizeof(double), hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(out_div, d + 2 * (size_t)n, (size_t)n * sizeof(double), hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (e != hipSuccess) return fail(RT_ERR_DEVICE, hipGetErrorString(e));
    return RT_OK;
}

uint64_t rt_debug_bvh_hash(const rt_scene* s, int32_t instance) {
    if (!s) return 0;
    if (instance < 0) return s->host.tlas_hash;
    if (instance >= (int32_t)s->host.inst_bvh_hash.size()) return 0;
    return s->host.inst_bvh_hash[instance];
}

}  // extern "C"
