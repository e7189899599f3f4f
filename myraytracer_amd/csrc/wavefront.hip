// wavefront.hip — the wavefront render pipeline (default path on MI355X).
//
// trace() (RT/Extensions/Object+Extension.swift:96-283) is split by ray type so that
// each kernel keeps only the registers its own phase needs (the megakernel holds the
// shading state live across the shadow traversal and runs at 2 waves/SIMD):
//
//   k_trace   closest hit (primary generation fused at level 0)  RTContext.swift:619-720
//   k_shade   hit reconstruction, material, Blinn-Phong terms, shadow-ray and bounce-ray
//             generation, appended to queues with wave ballot/prefix + one atomic per wave
//   k_shadow  any-hit occlusion of the shadow queue                RTContext.swift:724-848
//   k_gather  Lo = ambient + sum of unoccluded light terms, in light order (:116-143)
//   k_resolve recursion unwound backward per pixel with the per-level NaN guard (:277-280),
//             sample averaging (:354), FP64 + RGBA8 output (RayTracer.swift:186-195)
//
// Levels run bounce by bounce (mirror/conductor, depth < maxRecursionDepth); samples run
// one after another with each pixel's PCG32 state kept in HBM, so every draw happens in
// the reference's order.  Results are bit-identical to the recursive formulation.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "../../include/rtcore.h"
#include "device.h"
#include "layout.h"
#include "wavefront.h"

namespace myrt {
namespace dev {

struct TraceItem { double o[3], d[3]; double tlo, time; int32_t path, pad; };                 // 80 B
struct HitOut { double t, u, v; int32_t tri, inst; };                                          // 32 B
struct ShadowItem { double o[3], d[3]; double tmax, time; };                                   // 64 B
struct ShadowContrib { double c[3]; int32_t has, pad; };                                      // 32 B
struct ShadeOut { double lo[3]; int32_t first, n; };                                           // 32 B

constexpr int32_t kMissFlag = 1 << 30;
constexpr int kCounterSlots = 4096;   // traversal launches per frame (8 work counters each)

struct WaveParams {
    RenderParams R;
    TraceItem* items[2];
    HitOut* hits;
    ShadowItem* shadows;
    ShadowContrib* contrib;
    unsigned char* occluded;
    ShadeOut* shade;
    double* lod;
    double* md;
    int32_t* term;
    unsigned long long* rng;
    double* accum;
    unsigned* qcount;
    int64_t P;            // path slots
    int32_t tilesX;
    int32_t depth;        // current level
    int32_t sample;       // current sample index
    int32_t nsamples;     // n*n samples traced per pixel
};

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

struct PixelOf { int i, j, outRow; bool valid; };
__device__ __forceinline__ PixelOf pixel_of(const WaveParams& W, int64_t slot) {
    const int64_t tile = slot >> 6;
    const int lane = (int)(slot & 63);
    const int chunkSlot = (int)(tile / W.tilesX), tileX = (int)(tile % W.tilesX);
    PixelOf p;
    p.i = tileX * 8 + (lane & 7);
    const int r = lane >> 3;
    const int chunk = W.R.chunk_first + chunkSlot * W.R.chunk_step;
    p.j = chunk * 8 + r;
    p.outRow = (int)out_row_of(W.R, chunk, r);
    p.valid = p.i < W.R.cam.width && p.j < W.R.cam.height;
    return p;
}

__device__ __forceinline__ void flush_counts(const WaveParams& W, const Counts& c, bool count) {
    if (!count) return;
    const unsigned long long a = wave_sum(c.recs), b = wave_sum(c.tris), cc = wave_sum(c.normals),
                             dd = wave_sum(c.insts);
    if (lane_id() == 0) {
        if (a) atomicAdd(&W.R.counters[2], a);
        if (b) atomicAdd(&W.R.counters[3], b);
        if (cc) atomicAdd(&W.R.counters[4], cc);
        if (dd) atomicAdd(&W.R.counters[5], dd);
    }
}

// Queues are indexed by PATH (= primary pixel slot) at every level, not compacted: an
// empty entry is marked (TraceItem.path < 0, ShadowItem.tmax < 0).  Compaction by
// per-wave atomics on one counter serialises (~88 adds/us for one word,
// MI355X_MICROARCH "dequeue"); the persistent traversal kernels below skip empty
// entries at fetch time instead, so no short kernel issues same-address atomics.

// ------------------------------------------------------------------ ray generation
// Primary ray of (pixel, sample) exactly as Renderer.render (Object+Extension.swift:294-344).
__device__ __forceinline__ void gen_primary(const WaveParams& W, const PixelOf& px, int64_t slot, V3& o, V3& d,
                                            double& tlo, double& time) {
    const DCamera& C = W.R.cam;
    unsigned long long* rs = W.rng + 2 * slot;
    PCG32 rng(0ull);
    if (W.sample == 0) {
        rng = PCG32((((unsigned long long)px.j << 32) ^ (unsigned long long)px.i) + 0x9E3779B97F4A7C15ull);
    } else {
        rng.state = rs[0];
        rng.inc = rs[1];
    }
    const int sx = W.sample % C.n, sy = W.sample / C.n;
    const V3 eye = ld3(C.eye), u = ld3(C.u), v = ld3(C.v), w = ld3(C.w), q00 = ld3(C.q00);
    const double xi1 = rng.nextFloat();
    const double xi2 = rng.nextFloat();
    const double iOffset = ((double)sx + xi1) / (double)C.n;
    const double jOffset = ((double)sy + xi2) / (double)C.n;
    const double currentI = (double)px.i + iOffset;
    const double currentJ = (double)px.j + jOffset;
    const V3 s = (q00 - v * (currentJ * C.dv)) + u * (currentI * C.du);
    const V3 dir0 = normalize(s - eye);
    V3 dir = dir0, camEye = eye;
    if (C.aperture > 0 && C.focus > 0) {                       // DOF (:325-338)
        const double denom = dot(dir0, -w);
        const double tFocus = fabs(denom) < 1e-6 ? C.focus : (C.focus / denom);
        const V3 pFocus = eye + dir0 * tFocus;
        const double uRand = rng.nextFloat() - 0.5;
        const double vRand = rng.nextFloat() - 0.5;
        const V3 a = eye + ((uRand * u) + (vRand * v)) * C.aperture;
        dir = normalize(pFocus - a);
        camEye = a;
    }
    time = rng.nextFloat();
    const double denom = dot(dir, w);
    const double tImg = dot((eye - w * C.nd) - camEye, w) / (denom == 0.0 ? 4.9406564584124654e-324 : denom);
    tlo = smax(tImg, 0.0);
    rs[0] = rng.state;
    rs[1] = rng.inc;
    o = camEye;
    d = dir;
    TraceItem it;
    it.o[0] = o.x; it.o[1] = o.y; it.o[2] = o.z;
    it.d[0] = d.x; it.d[1] = d.y; it.d[2] = d.z;
    it.tlo = tlo; it.time = time; it.path = (int32_t)slot; it.pad = 0;
    W.items[0][slot] = it;
}

// Fetch item `slot` of the current level: returns false for an empty entry.
template <int MODE>   // 0 = primary, 1 = bounce queue, 2 = shadow queue
__device__ __forceinline__ bool fetch_item(const WaveParams& W, int64_t slot, V3& o, V3& d, double& tlo,
                                           double& tmax, double& time) {
    if (MODE == 0) {
        const PixelOf px = pixel_of(W, slot);
        if (!px.valid) return false;
        gen_primary(W, px, slot, o, d, tlo, time);
        tmax = DINF;
        return true;
    } else if (MODE == 1) {
        const TraceItem& it = W.items[W.depth & 1][slot];
        if (it.path < 0) return false;
        o = ld3(it.o); d = ld3(it.d); tlo = it.tlo; time = it.time; tmax = DINF;
        return true;
    } else {
        const ShadowItem& si = W.shadows[slot];
        if (!(si.tmax >= 0.0)) return false;
        o = ld3(si.o); d = ld3(si.d); tmax = si.tmax; time = si.time; tlo = 0.0;
        return true;
    }
}

// ------------------------------------------------------- persistent traversal (identity)
// Every wave keeps 64 rays in flight and refills lanes whose ray finished from a
// work pool (Aila & Laine's persistent threads with ray replacement): lane utilisation
// no longer decays with the longest ray of a tile.  Work is split into 8 home ranges,
// one per XCD (blocks are dealt round-robin to XCDs, so block b runs on XCD b % 8):
// a wave grabs 64-item tiles from its home range - neighbouring image tiles share an
// L2 - and steals from the other ranges once its own is exhausted.
constexpr int kGrab = 64;
constexpr int kRefillMin = 16;

struct WaveWork {
    int64_t next, end;
    int home, tries;
    bool done;
};

__device__ __forceinline__ bool grab_work(WaveWork& w, unsigned* ctr, int64_t N) {
    const int64_t R = ((N + 7) / 8 + kGrab - 1) / kGrab * kGrab;
    while (w.tries < 8) {
        const int h = (w.home + w.tries) & 7;
        const int64_t base = (int64_t)h * R, lim = min(N, base + R);
        unsigned got = 0;
        if (lane_id() == 0 && base < lim) got = atomicAdd(&ctr[h], (unsigned)kGrab);
        got = __shfl(got, 0, 64);
        if (base + (int64_t)got < lim) {
            w.next = base + got;
            w.end = min(lim, w.next + kGrab);
            return true;
        }
        w.tries++;
    }
    w.done = true;
    return false;
}

template <bool COUNT, int MODE>
__global__ __launch_bounds__(256) void k_persist(WaveParams W, int64_t N, unsigned* ctr) {
    extern __shared__ unsigned long long lds_stack[];
    const RenderParams& P = W.R;
    constexpr bool SHADOW = (MODE == 2);
    MYRT_STACK(st, lds_stack);
    Counts cnt{};
    const int lane = lane_id();
    const unsigned long long ltMask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    WaveWork w{0, 0, (int)(blockIdx.x & 7), 0, false};
    int64_t slot = -1;
    int ref = 0;
    V3 o{0, 0, 0}, d{0, 0, 0}, inv{0, 0, 0};
    double tlo = 0, tmax = DINF, time = 0;
    Hit h;
    h.t = DINF; h.u = 0; h.v = 0; h.tri = -1; h.inst = -1;
    unsigned rays = 0;
    for (;;) {
        // ---- refill idle lanes (wave-uniform decision)
        const unsigned long long idle = __ballot(slot < 0);
        const int nIdle = __popcll(idle);
        if (!w.done && (nIdle >= kRefillMin || nIdle == 64)) {
            const int rank = __popcll(idle & ltMask);
            int assigned = 0;
            int64_t mine = -1;
            while (assigned < nIdle) {
                if (w.next >= w.end && !grab_work(w, ctr, N)) break;
                const int take = (int)min((int64_t)(nIdle - assigned), w.end - w.next);
                if (slot < 0 && rank >= assigned && rank < assigned + take) mine = w.next + (rank - assigned);
                w.next += take;
                assigned += take;
            }
            if (mine >= 0) {
                slot = mine;
                bool live = fetch_item<MODE>(W, slot, o, d, tlo, tmax, time);
                if (live) {
                    rays++;
                    inv = rcp(d);
                    h.t = DINF; h.u = 0; h.v = 0; h.tri = -1; h.inst = -1;
                    st.reset(0);
                    live = unified_begin(P, o, inv, SHADOW ? tmax * P.prune_rel + P.prune_abs : DINF, ref);
                    if (!live) {                                   // missed the whole scene
                        if (SHADOW) W.occluded[slot] = 0;
                        else {
                            HitOut ho; ho.t = DINF; ho.u = 0; ho.v = 0; ho.tri = -1; ho.inst = -1;
                            W.hits[slot] = ho;
                        }
                    }
                }
                if (!live) slot = -1;
            }
        }
        if (__ballot(slot >= 0) == 0) {
            if (w.done) break;
            continue;
        }
        // ---- one traversal step per live lane (FAST slabs unless some live ray has a
        //      zero direction component, see slab_hit)
        const bool fast = __all(slot < 0 || finite3(inv));
        if (slot >= 0) {
            const int r = fast ? unified_step<COUNT, SHADOW, true>(P, ref, st, o, d, inv, tlo, tmax, h, cnt)
                               : unified_step<COUNT, SHADOW, false>(P, ref, st, o, d, inv, tlo, tmax, h, cnt);
            if (r != 0) {
                if (SHADOW) {
                    W.occluded[slot] = (r == 2) ? 1 : 0;
                } else {
                    HitOut ho; ho.t = h.t; ho.u = h.u; ho.v = h.v; ho.tri = h.tri; ho.inst = h.inst;
                    W.hits[slot] = ho;
                }
                slot = -1;
            }
        }
    }
    // ray counters: shadow rays (MODE 2) and secondary rays (MODE 1), one atomic per wave
    const unsigned long long nr = wave_sum((unsigned long long)rays);
    if (lane == 0 && nr) {
        if (MODE == 2) { atomicAdd(&P.counters[0], nr); atomicAdd(&P.counters[kCounterShadowTraced], nr); }
        if (MODE == 1) atomicAdd(&P.counters[1], nr);
    }
    flush_counts(W, cnt, COUNT);
}

// ------------------------------------------------------- general traversal (any instances)
template <bool COUNT, int MODE>
__global__ __launch_bounds__(256) void k_general(WaveParams W, int64_t N) {
    extern __shared__ unsigned long long lds_stack[];
    const RenderParams& P = W.R;
    const int64_t slot = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    Counts cnt{};
    unsigned rays = 0;
    V3 o, d;
    double tlo, tmax, time;
    if (slot < N && fetch_item<MODE>(W, slot, o, d, tlo, tmax, time)) {
        rays = 1;
        MYRT_STACK(st, lds_stack);
        if (MODE == 2) {
            W.occluded[slot] = occluded<COUNT>(P, o, d, tmax, time, st, cnt) ? 1 : 0;
        } else {
            Hit h;
            if (P.has_tlas) intersect_closest<COUNT>(P, o, d, rcp(d), tlo, time, h, st, cnt);
            else { h.t = DINF; h.inst = -1; h.tri = -1; h.u = 0; h.v = 0; }
            HitOut ho; ho.t = h.t; ho.u = h.u; ho.v = h.v; ho.tri = h.tri; ho.inst = h.inst;
            W.hits[slot] = ho;
        }
    }
    const unsigned long long nr = wave_sum((unsigned long long)rays);
    if (lane_id() == 0 && nr) {
        if (MODE == 2) { atomicAdd(&P.counters[0], nr); atomicAdd(&P.counters[kCounterShadowTraced], nr); }
        if (MODE == 1) atomicAdd(&P.counters[1], nr);
    }
    flush_counts(W, cnt, COUNT);
}

// ---------------------------------------------------------------------- k_shade
// One lane per path: hit reconstruction, material, direct-light terms, shadow rays
// (path*L + l) and the bounce ray (same path slot, next level).
template <bool COUNT, bool BOUNCE>
__global__ __launch_bounds__(256) void k_shade(WaveParams W) {
    const RenderParams& P = W.R;
    const int depth = W.depth;
    const int64_t path = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (path >= W.P) return;
    Counts cnt{};
    const int L = P.num_plights;
    bool active;
    TraceItem it;
    if (depth == 0) {
        active = pixel_of(W, path).valid;
        if (active) it = W.items[0][path];
    } else {
        it = W.items[depth & 1][path];
        active = it.path >= 0;
    }
    HitOut h;
    if (active) h = W.hits[path];
    const bool hit = active && h.inst >= 0 && P.has_tlas;
    bool bounce = false;
    if (active && !hit) {                         // miss -> backgroundColor (:101-103); no TLAS -> 0 (:98)
        W.term[path] = depth | kMissFlag;
        double* lo = W.lod + ((size_t)depth * W.P + path) * 3;
        if (P.has_tlas) { lo[0] = P.background[0]; lo[1] = P.background[1]; lo[2] = P.background[2]; }
        else { lo[0] = 0.0; lo[1] = 0.0; lo[2] = 0.0; }
    }
    unsigned nShadow = 0;
    if (hit) {
        const V3 d = ld3(it.d);
        const double time = it.time;
        const TriRec& T = P.tris[h.tri];
        const DInstance& I = P.insts[h.inst];
        const V3 e1 = ld3(T.e1), e2 = ld3(T.e2), v0 = ld3(T.v0);
        V3 nl;
        if (I.smooth) {
            if (COUNT) cnt.normals++;
            const double* nn = P.normals + (size_t)h.tri * 9;
            const double w = 1.0 - h.u - h.v;
            nl = normalize(((w * ld3(nn)) + (h.u * ld3(nn + 3))) + (h.v * ld3(nn + 6)));
        } else {
            nl = normalize(cross(e1, e2));
        }
        const V3 pl = (v0 + (h.u * e1)) + (h.v * e2);
        const V3 p = m4_point(I.l2w, pl, 1.0) + ld3(I.motion) * time;
        V3 Ngeo = normalize(m3_mul(I.nmat, nl));
        if (I.det_neg) Ngeo = -Ngeo;
        const int matIndex = max(0, min(P.num_mats - 1, I.material - 1));
        const DMaterial& M = P.mats[matIndex];
        const bool frontFacing = dot(d, Ngeo) < 0;
        const V3 N = frontFacing ? Ngeo : -Ngeo;
        const bool computeDirect = !(M.ior > 0) || frontFacing;
        const V3 Lo = computeDirect ? ld3(P.ambient) * ld3(M.ambient) : v3(0, 0, 0);
        nShadow = computeDirect ? (unsigned)L : 0u;
        ShadeOut so;
        so.lo[0] = Lo.x; so.lo[1] = Lo.y; so.lo[2] = Lo.z;
        so.first = (int32_t)(path * L);
        so.n = (int32_t)nShadow;
        W.shade[path] = so;
        for (int li = 0; li < (int)nShadow; ++li) {                 // :118-143
            const DPointLight& PL = P.plights[li];
            V3 wi = ld3(PL.position) - p;
            const double dist = length(wi);
            wi = normalize(wi);
            const V3 so3 = p + wi * P.shadow_eps;
            ShadowItem si;
            si.o[0] = so3.x; si.o[1] = so3.y; si.o[2] = so3.z;
            si.d[0] = wi.x; si.d[1] = wi.y; si.d[2] = wi.z;
            si.tmax = dist; si.time = time;
            W.shadows[path * L + li] = si;
            ShadowContrib sc;
            const double NdotL = smax(0.0, dot(N, wi));
            sc.has = NdotL > 0 ? 1 : 0;
            sc.pad = 0;
            if (sc.has) {
                const double shininess = smax(1.0, M.phong);
                const V3 Ld = ld3(M.diffuse) * NdotL;
                const V3 view = normalize(-d);
                const V3 hv = normalize(wi + view);
                const double NdotH = smax(0.0, dot(N, hv));
                const V3 Ls = ld3(M.specular) * pow(NdotH, shininess);
                const V3 atten = ld3(PL.intensity) / smax(dist * dist, 1e-12);
                const V3 c = (Ld + Ls) * atten;
                sc.c[0] = c.x; sc.c[1] = c.y; sc.c[2] = c.z;
            } else {
                sc.c[0] = 0.0; sc.c[1] = 0.0; sc.c[2] = 0.0;
            }
            W.contrib[path * L + li] = sc;
        }
        if (BOUNCE && (M.type == RT_MAT_MIRROR || M.type == RT_MAT_CONDUCTOR) && depth < P.max_depth &&
            depth < kMaxDepthGPU) {
            bounce = true;
            V3 mult;
            if (M.type == RT_MAT_MIRROR) {
                mult = ld3(M.mirror);
            } else {
                const double cosI = smax(0.0, -dot(d, N));
                mult = fresnel_conductor(M.ior, M.absorption_index, cosI) * ld3(M.mirror);
            }
            V3 rd = normalize(reflect(d, N));
            if (M.roughness != 0.0) {                    // glossy perturbation (:191-197)
                unsigned long long* rs = W.rng + 2 * path;
                PCG32 rng(0ull);
                rng.state = rs[0];
                rng.inc = rs[1];
                V3 t, b;
                onb(rd, t, b);
                const double r1 = rng.nextFloat() - 0.5;
                const double r2 = rng.nextFloat() - 0.5;
                rd = (rd + (M.roughness * r1) * b) + (M.roughness * r2) * t;
                rd = normalize(rd);
                rs[0] = rng.state;
                rs[1] = rng.inc;
            }
            TraceItem nx;
            const V3 no = p + N * P.shadow_eps;
            nx.o[0] = no.x; nx.o[1] = no.y; nx.o[2] = no.z;
            nx.d[0] = rd.x; nx.d[1] = rd.y; nx.d[2] = rd.z;
            nx.tlo = 0.0; nx.time = time; nx.path = (int32_t)path; nx.pad = 0;
            W.items[(depth + 1) & 1][path] = nx;
            double* m = W.md + ((size_t)depth * W.P + path) * 3;
            m[0] = mult.x; m[1] = mult.y; m[2] = mult.z;
        }
        if (!bounce) W.term[path] = depth;
    }
    // empty queue entries for the shadow and next-level queues
    for (int li = (int)nShadow; li < L; ++li) W.shadows[path * L + li].tmax = -1.0;
    if (BOUNCE && !bounce) W.items[(depth + 1) & 1][path].path = -1;
    flush_counts(W, cnt, COUNT);
}

// ---------------------------------------------------------------------- k_gather
__global__ __launch_bounds__(256) void k_gather(WaveParams W) {
    const int depth = W.depth;
    const int64_t path = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (path >= W.P) return;
    if (depth == 0 ? !pixel_of(W, path).valid : W.items[depth & 1][path].path < 0) return;
    if (W.hits[path].inst < 0 || !W.R.has_tlas) return;     // misses were written by k_shade
    const ShadeOut so = W.shade[path];
    V3 Lo = ld3(so.lo);
    for (int l = 0; l < so.n; ++l) {                          // light order, :118-143
        const ShadowContrib& c = W.contrib[so.first + l];
        if (c.has && !W.occluded[so.first + l]) Lo = Lo + ld3(c.c);
    }
    double* lo = W.lod + ((size_t)depth * W.P + path) * 3;
    lo[0] = Lo.x; lo[1] = Lo.y; lo[2] = Lo.z;
}

// ---------------------------------------------------------------------- k_resolve
template <bool COUNT>
__global__ __launch_bounds__(256) void k_resolve(WaveParams W) {
    const int64_t slot = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool valid = false;
    if (slot < W.P) {
        const PixelOf px = pixel_of(W, slot);
        valid = px.valid;
        if (valid) {
            const int32_t tm = W.term[slot];
            const int D = tm & ~kMissFlag;
            const double* lo = W.lod + ((size_t)D * W.P + slot) * 3;
            V3 L = ld3(lo);
            if (!(tm & kMissFlag)) L = isfin(L) ? L : v3(0, 0, 0);
            for (int q = D - 1; q >= 0; --q) {                 // Lo_q += M_q * trace(q+1); NaN guard
                const V3 Lq = ld3(W.lod + ((size_t)q * W.P + slot) * 3) +
                              ld3(W.md + ((size_t)q * W.P + slot) * 3) * L;
                L = isfin(Lq) ? Lq : v3(0, 0, 0);
            }
            double* acc = W.accum + slot * 3;
            V3 sum = (W.sample == 0) ? v3(0, 0, 0) : ld3(acc);
            sum = sum + L;
            if (W.sample + 1 < W.nsamples) {
                acc[0] = sum.x; acc[1] = sum.y; acc[2] = sum.z;
            } else {
                const V3 pxc = sum / (double)W.R.cam.samples;
                const size_t o = (size_t)px.outRow * W.R.cam.width + px.i;
                if (W.R.out_rgb) {
                    W.R.out_rgb[o * 3 + 0] = pxc.x;
                    W.R.out_rgb[o * 3 + 1] = pxc.y;
                    W.R.out_rgb[o * 3 + 2] = pxc.z;
                }
                if (W.R.out_rgba8) {
                    const double cx = fmin(fmax(pxc.x, 0.0), 255.0), cy = fmin(fmax(pxc.y, 0.0), 255.0),
                                 cz = fmin(fmax(pxc.z, 0.0), 255.0);
                    const unsigned packed = (unsigned)(unsigned char)cx | ((unsigned)(unsigned char)cy << 8) |
                                            ((unsigned)(unsigned char)cz << 16) | (255u << 24);
                    reinterpret_cast<unsigned*>(W.R.out_rgba8)[o] = packed;
                }
            }
        }
    }
    if (COUNT && W.sample + 1 == W.nsamples) {
        const unsigned long long n = wave_sum(valid ? 1ull : 0ull);
        if (lane_id() == 0 && n) atomicAdd(&W.R.counters[6], n);
    }
}

}  // namespace dev

// ================================================================== host side
template <class T>
static int32_t grow(void** p, int64_t n, int64_t& bytes) {
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    if (n <= 0) n = 1;
    if (hipMalloc(p, (size_t)n * sizeof(T)) != hipSuccess) return RT_ERR_OOM;
    bytes += n * (int64_t)sizeof(T);
    return RT_OK;
}

void wave_release(WaveBuffers& b) {
    void* ps[] = {b.items[0], b.items[1], b.hits, b.shadows, b.contrib, b.occluded, b.shade, b.lod, b.md,
                  b.term, b.rng, b.accum, b.qcount};
    for (void* p : ps) if (p) (void)hipFree(p);
    b = WaveBuffers();
}

int32_t wave_reserve(WaveBuffers& b, int64_t paths, int32_t lights, int32_t depth) {
    if (paths <= b.cap_paths && lights <= b.cap_lights && depth <= b.cap_depth && b.qcount) return RT_OK;
    const int64_t P = std::max<int64_t>(paths, b.cap_paths);
    const int32_t L = std::max<int32_t>(std::max(lights, 1), b.cap_lights);
    const int32_t D = std::max<int32_t>(depth, b.cap_depth);
    wave_release(b);
    int64_t by = 0;
    int32_t rc = RT_OK;
    using namespace dev;
    rc |= grow<TraceItem>(&b.items[0], P, by);
    rc |= grow<TraceItem>(&b.items[1], P, by);
    rc |= grow<HitOut>(&b.hits, P, by);
    rc |= grow<ShadowItem>(&b.shadows, P * L, by);
    rc |= grow<ShadowContrib>(&b.contrib, P * L, by);
    rc |= grow<unsigned char>((void**)&b.occluded, P * L, by);
    rc |= grow<ShadeOut>(&b.shade, P, by);
    rc |= grow<double>((void**)&b.lod, (int64_t)(D + 1) * P * 3, by);
    rc |= grow<double>((void**)&b.md, (int64_t)std::max(D, 1) * P * 3, by);
    rc |= grow<int32_t>((void**)&b.term, P, by);
    rc |= grow<unsigned long long>((void**)&b.rng, 2 * P, by);
    rc |= grow<double>((void**)&b.accum, 3 * P, by);
    rc |= grow<unsigned>((void**)&b.qcount, kCounterSlots * 8, by);
    if (rc != RT_OK) { wave_release(b); return RT_ERR_OOM; }
    b.cap_paths = P; b.cap_lights = L; b.cap_depth = D; b.bytes = by;
    return RT_OK;
}

int32_t wave_render(const RenderParams& R, WaveBuffers& b, bool bounce, bool count, hipStream_t stream) {
    using namespace dev;
    const int32_t tilesX = (R.cam.width + 7) / 8;
    const int64_t P = (int64_t)R.num_chunks * tilesX * 64;
    if (P == 0) return RT_OK;
    const int32_t L = R.num_plights;
    const int32_t maxd = bounce ? std::min(R.max_depth, kMaxDepthGPU) : 0;
    int32_t rc = wave_reserve(b, P, L, maxd);
    if (rc != RT_OK) return rc;
    WaveParams W{};
    W.R = R;
    W.items[0] = (TraceItem*)b.items[0]; W.items[1] = (TraceItem*)b.items[1];
    W.hits = (HitOut*)b.hits; W.shadows = (ShadowItem*)b.shadows; W.contrib = (ShadowContrib*)b.contrib;
    W.occluded = b.occluded; W.shade = (ShadeOut*)b.shade; W.lod = b.lod; W.md = b.md; W.term = b.term;
    W.rng = b.rng; W.accum = b.accum; W.qcount = b.qcount;
    W.P = P; W.tilesX = tilesX;
    W.nsamples = R.cam.n * R.cam.n;
    // Persistent refill traversal (k_persist) is opt-in (MYRT_PERSIST=1): replacing
    // finished rays mid-flight breaks the 8x8-tile coherence of a wave's node fetches and
    // measured 2.2x slower than one-ray-per-lane launches on C3 (profiles/r01_v3_*).
    const char* pe = std::getenv("MYRT_PERSIST");
    const bool persist = R.identity && R.has_tlas && (pe && pe[0] == '1');
    const dim3 block(256);
    const dim3 gP((unsigned)((P + 255) / 256));
    const int64_t NS = P * std::max(L, 1);
    const dim3 gS((unsigned)((NS + 255) / 256));
    const dim3 gPersist(256 * 8);                 // >= resident blocks; extra blocks find no work
    const size_t lds = (size_t)kLds * 256 * sizeof(unsigned long long);
    // qcount: 8 XCD-homed work counters per traversal launch, fresh block per launch
    const int launchesPerFrame = W.nsamples * (maxd + 1) * 2;
    if (launchesPerFrame > kCounterSlots) return RT_ERR_UNSUPPORTED;
    if (hipMemsetAsync(b.qcount, 0, (size_t)launchesPerFrame * 8 * sizeof(unsigned), stream) != hipSuccess)
        return RT_ERR_DEVICE;
    int ctrSlot = 0;
    auto trace = [&](int mode, int64_t N) {
        unsigned* ctr = b.qcount + 8 * (ctrSlot++);
        const dim3 g = mode == 2 ? gS : gP;
        if (persist) {
            if (mode == 0) { if (count) hipLaunchKernelGGL((k_persist<true, 0>), gPersist, block, lds, stream, W, N, ctr);
                             else hipLaunchKernelGGL((k_persist<false, 0>), gPersist, block, lds, stream, W, N, ctr); }
            if (mode == 1) { if (count) hipLaunchKernelGGL((k_persist<true, 1>), gPersist, block, lds, stream, W, N, ctr);
                             else hipLaunchKernelGGL((k_persist<false, 1>), gPersist, block, lds, stream, W, N, ctr); }
            if (mode == 2) { if (count) hipLaunchKernelGGL((k_persist<true, 2>), gPersist, block, lds, stream, W, N, ctr);
                             else hipLaunchKernelGGL((k_persist<false, 2>), gPersist, block, lds, stream, W, N, ctr); }
        } else {
            if (mode == 0) { if (count) hipLaunchKernelGGL((k_general<true, 0>), g, block, lds, stream, W, N);
                             else hipLaunchKernelGGL((k_general<false, 0>), g, block, lds, stream, W, N); }
            if (mode == 1) { if (count) hipLaunchKernelGGL((k_general<true, 1>), g, block, lds, stream, W, N);
                             else hipLaunchKernelGGL((k_general<false, 1>), g, block, lds, stream, W, N); }
            if (mode == 2) { if (count) hipLaunchKernelGGL((k_general<true, 2>), g, block, lds, stream, W, N);
                             else hipLaunchKernelGGL((k_general<false, 2>), g, block, lds, stream, W, N); }
        }
    };
    for (int s = 0; s < W.nsamples; ++s) {
        W.sample = s;
        for (int dl = 0; dl <= maxd; ++dl) {
            W.depth = dl;
            trace(dl == 0 ? 0 : 1, P);
            if (bounce) {
                if (count) hipLaunchKernelGGL((k_shade<true, true>), gP, block, 0, stream, W);
                else hipLaunchKernelGGL((k_shade<false, true>), gP, block, 0, stream, W);
            } else {
                if (count) hipLaunchKernelGGL((k_shade<true, false>), gP, block, 0, stream, W);
                else hipLaunchKernelGGL((k_shade<false, false>), gP, block, 0, stream, W);
            }
            if (L > 0) trace(2, NS);
            else ctrSlot++;
            hipLaunchKernelGGL(k_gather, gP, block, 0, stream, W);
        }
        if (count) hipLaunchKernelGGL((k_resolve<true>), gP, block, 0, stream, W);
        else hipLaunchKernelGGL((k_resolve<false>), gP, block, 0, stream, W);
    }
    if (hipGetLastError() != hipSuccess) return RT_ERR_DEVICE;
    return RT_OK;
}

}  // namespace myrt
