// render_full.h — the complete trace() for scenes the fast megakernel does not take:
// dielectric materials (two child rays per bounce) and area lights (the chunk-sequential
// jitterIndex).  Included by render.hip.
//
// trace() (Object+Extension.swift:96-283) recurses depth-first: reflection subtree, then
// transmission subtree.  Here the recursion is an explicit per-lane frame stack (private
// memory, <= maxRecursionDepth + 1 frames) visited in the same order, so the PCG32 draws
// (roughness, :193-198, :209-216, :258-263) and the area-light jitterIndex increments
// (:152-154) happen in the reference's sequence.
//
// jitterIndex is one counter per 8-row chunk that runs through the chunk's pixels in
// row-major order (:288, Renderer.renderChunk).  A lane cannot know how many area-light
// evaluations the pixels before it made, so area-light frames take three launches:
//   k_events   - the same paths without lighting, counting evaluations per pixel
//                (an evaluation = one area light at one hit with computeDirectLight), and
//                logging each path's closest hits (RenderParams::hits, the first hit_slots
//                walks of every pixel);
//   k_jscan    - per-chunk exclusive prefix sum in row-major pixel order;
//   render_full- the real render, each pixel starting at its prefix; logged hits are read
//                back instead of walked again (the walk is deterministic: same ray, same hit).
#pragma once

namespace myrt {
namespace dev {

enum : int { kFrameMirror = 1, kFrameDielR = 2, kFrameDielT = 3 };

// pow as an out-of-line call: inlined, OCML's pow (extended-precision log, all ranges) adds its
// working registers to the whole full-trace kernel (cf. device.h phong_pow, which the megakernel
// uses only where its domain is known)
__device__ __noinline__ double pow_call(double x, double y) { return pow(x, y); }

struct Frame {            // one suspended trace() level waiting for a child
    V3 Lo;                // radiance of this level so far
    V3 p;                 // hit point (transmission origin)
    V3 aux;               // mirror/conductor: multiplier; dielectric: LiR once known
    V3 td;                // dielectric: transmitted direction
    double R;             // dielectric: Fresnel reflectance
    double t;             // this level's hit distance (its parent's Beer test)
    int hitmat;           // hit.mat (materialOverride) of this level
    int mat;              // clamped material index
    int state;
    bool tir, entering;
};

struct LevelOut { V3 L; bool hit; int hitmat; double t; };

// fresnelDielectric (Object+Extension.swift:467-491)
__device__ __forceinline__ void fresnel_dielectric(double n1, double n2, double cosI, double& R, bool& hasCosT,
                                                   double& cosT, double& sin2T) {
    const double cosTheta = smax(0.0, smin(1.0, fabs(cosI)));
    const double eta = n1 / n2;
    sin2T = (eta * eta) * smax(0.0, 1.0 - cosTheta * cosTheta);
    if (sin2T > 1.0) { R = 1.0; hasCosT = false; cosT = 0; return; }
    const double cosPhi = dsqrt(smax(0.0, 1.0 - sin2T));
    const double Rs = (n2 * cosTheta - n1 * cosPhi) / (n2 * cosTheta + n1 * cosPhi);
    const double Rp = (n1 * cosTheta - n2 * cosPhi) / (n1 * cosTheta + n2 * cosPhi);
    R = 0.5 * (Rs * Rs + Rp * Rp);
    hasCosT = true;
    cosT = cosPhi;
}

// EVENTS: count area-light evaluations only (no light sampling, no shadow rays); the
// paths, PCG32 draws and jitterIndex increments are the same as the real render.
// DEEP: maxRecursionDepth > kMaxDepthGPU; levels beyond the private frames live in the
// launch's deep-frame buffer (RenderParams::deep, one Frame per level and lane of the launch).
template <bool DEEP>
struct FrameStack {
    Frame loc[kMaxDepthGPU + 1];
    Frame* deep;              // this lane's level kMaxDepthGPU + 1
    size_t stride;            // lanes of the launch
    __device__ __forceinline__ Frame& operator[](int d) {
        if (!DEEP || d <= kMaxDepthGPU) return loc[d];
        return deep[(size_t)(d - kMaxDepthGPU - 1) * stride];
    }
};

// Direct light at a hit (Object+Extension.swift:116-186): point lights (:118-143), then area
// lights (:145-186), through ONE shadow-walk call site (one inlined copy of the walk): each light's
// contribution is formed before its walk - the same expressions on the same values - and added to
// Lo in light order when the walk finds the light unblocked.  jitterIndex advances once per area
// light (:152-154).
template <bool COUNT, int WALK>
__device__ __forceinline__ void direct_light(const RenderParams& P, const DMaterial& M, const V3& N, const V3& p,
                                             const V3& d, double time, long long& jitterIndex, Stack& st, Counts& c,
                                             V3& Lo) {
    const int nl = P.num_plights + P.num_alights;
    for (int li = 0; li < nl; ++li) {
        V3 wi, contrib = v3(0, 0, 0);
        double tmax = 0.0;
        bool trace = false, use = false;
        if (li < P.num_plights) {
            const DPointLight& PL = P.plights[li];
            wi = ld3(PL.position) - p;
            const double dist = length(wi);
            wi = normalize(wi);
            c.shadow++;
            const double NdotL = smax(0.0, dot(N, wi));
            trace = NdotL > 0 || MYRT_REF(P);                  // else the result is discarded
            use = NdotL > 0;
            tmax = dist;
            if (use) {
                const double shininess = smax(1.0, M.phong);
                const V3 Ld = ld3(M.diffuse) * NdotL;
                const V3 view = normalize(-d);
                const V3 hv = normalize(wi + view);
                const double NdotH = smax(0.0, dot(N, hv));
                const V3 Ls = ld3(M.specular) * pow_call(NdotH, shininess);
                const V3 atten = ld3(PL.intensity) / smax(dist * dist, 1e-12);
                contrib = (Ld + Ls) * atten;
            }
        } else {
            const DAreaLight& AL = P.alights[li - P.num_plights];
            const V3 nL = normalize(ld3(AL.normal));
            V3 tg, bt;
            onb(nL, tg, bt);
            const double size = AL.size;
            const double area = size * size;
            const int cell = (int)(jitterIndex % kJitterCells);
            const double r1 = P.jitter[cell] / 10.0 - 0.5;
            const double r2 = P.jitter[kJitterCells + cell] / 10.0 - 0.5;
            jitterIndex += 1;
            const V3 samplePos = (ld3(AL.position) + tg * (r1 * size)) + bt * (r2 * size);
            wi = samplePos - p;
            const double dist2 = dot(wi, wi);
            const double dist = dsqrt(dist2);
            wi = wi / dist;
            const double NdotL = dot(N, wi);
            const double Ln = fabs(dot(nL, -wi));
            if (NdotL > 0 && Ln > 0) {
                c.shadow++;
                trace = use = true;
                tmax = dist - P.shadow_eps;
                const V3 view = normalize(-d);
                const V3 hv = normalize(wi + view);
                const V3 Ld = ld3(M.diffuse) * NdotL;
                const V3 Ls = ld3(M.specular) * pow_call(smax(0.0, dot(N, hv)), M.phong);
                const V3 brdf = Ld + Ls;
                contrib = ((brdf * ld3(AL.radiance)) * (Ln / dist2)) * area;
            }
        }
        if (trace) {
            c.shadow_traced++;
            const bool blocked = walk_occluded<COUNT, WALK>(P, p + wi * P.shadow_eps, wi, tmax, time, st, c);
            if (!blocked && use) Lo = Lo + contrib;
        }
    }
}

// This pixel's closest-hit log (k_events writes it, render_full reads it).  k counts the pixel's
// walks in trace order, which both passes share: the paths do not depend on the lighting.
// Tree-indexed logs (P.hit_tree != 0, the breadth-first events passes below): node h of traced
// sample s at entry s * tree_size + h instead of the k-th walk.
struct HitLog {
    DHitRec* p;           // walk 0 of this pixel
    size_t stride;
    int k, cap;
    int tree = 0, node = 0, sbase = 0;
};
enum : uint8_t { kNodeExists = 1, kNodeEval = 2, kNodeHit = 4 };
__device__ __forceinline__ int tree_child(int b, int h, int which) { return b == 2 ? 2 * h + 1 + which : h + 1; }
__device__ __forceinline__ int tree_parent(int b, int h) { return b == 2 ? (h - 1) >> 1 : h - 1; }
// Level L of a tree: its first node and its width; a wave runs up to P.tree_ppw of its node
// positions one after another (grid rows per level: tree_rows)
__device__ __host__ __forceinline__ int tree_first(int b, int L) { return b == 2 ? (1 << L) - 1 : L; }
__device__ __host__ __forceinline__ int tree_width(int b, int L) { return b == 2 ? (1 << L) : 1; }
__device__ __host__ __forceinline__ int tree_rows(int b, int L, int ppw) { return (tree_width(b, L) + ppw - 1) / ppw; }

template <bool COUNT, bool EVENTS, bool DEEP, int WALK>
__device__ V3 trace_full(const RenderParams& P, V3 o, V3 d, double tlo, double time, PCG32& rng,
                         long long& jitterIndex, Stack& st, Counts& c, HitLog& hl) {
    FrameStack<DEEP> F;
    if (DEEP) {
        F.stride = (size_t)gridDim.x * blockDim.x;
        F.deep = reinterpret_cast<Frame*>(P.deep) + ((size_t)blockIdx.x * blockDim.x + threadIdx.x);
    }
    int depth = 0;
    LevelOut out{};
    for (;;) {
        // ======================================================== enter level `depth`
        bool descend = false;
        if (depth > P.max_depth) {                                   // :97
            out = LevelOut{ld3(P.background), false, 0, DINF};
        } else if (!P.has_tlas) {                                    // :98
            out = LevelOut{v3(0, 0, 0), false, 0, DINF};
        } else {
            Hit h;
            const int kk = hl.tree ? hl.sbase + hl.node : hl.k;     // this walk's log entry
            const bool logged = kk < hl.cap;
            if (!COUNT && !EVENTS && logged) {
                const DHitRec r = hl.p[(size_t)kk * hl.stride];
                h.t = r.t; h.u = r.u; h.v = r.v; h.tri = r.tri; h.inst = r.inst;
            } else {
                walk_closest<COUNT, WALK>(P, o, d, rcp(d), tlo, time, h, st, c);
                if (EVENTS && logged) {
                    DHitRec r;
                    r.t = h.t; r.u = h.u; r.v = h.v; r.tri = h.tri; r.inst = h.inst;
                    hl.p[(size_t)hl.k * hl.stride] = r;
                    if (P.nodes) {                                   // the ray, for k_shade
                        DNodeRec n;
                        n.o[0] = o.x; n.o[1] = o.y; n.o[2] = o.z;
                        n.d[0] = d.x; n.d[1] = d.y; n.d[2] = d.z;
                        n.time = time;
                        n.jofs = (int32_t)jitterIndex;
                        n.hit = h.inst >= 0 ? 1 : 0;
                        P.nodes[(size_t)hl.k * hl.stride + (size_t)(hl.p - P.hits)] = n;
                        // node lists (render.hip k_clist): the walks k_shade_c shades
                        if (P.nflags && h.inst >= 0) P.nflags[(size_t)hl.k * hl.stride + (size_t)(hl.p - P.hits)] = kNodeHit;
                    }
                }
            }
            hl.k++;
            if (h.inst < 0) {                                        // :101-103
                out = LevelOut{ld3(P.background), false, 0, DINF};
            } else {
                V3 p, Ngeo;
                hit_geometry<COUNT>(P, o, d, time, h, p, Ngeo, c);
                const int hitmat = P.insts[h.inst].material;
                const int mi = max(0, min(P.num_mats - 1, hitmat - 1));
                const DMaterial& M = P.mats[mi];
                const bool frontFacing = dot(d, Ngeo) < 0;
                const V3 N = frontFacing ? Ngeo : -Ngeo;
                const bool computeDirect = !(M.ior > 0) || frontFacing;
                // EVENTS passes keep only what steers the path (directions, origins, the PCG32
                // draws, the dielectric's TIR test): no radiance, no Beer data in the frames
                V3 Lo = (!EVENTS && computeDirect) ? ld3(P.ambient) * ld3(M.ambient) : v3(0, 0, 0);
                if (computeDirect && EVENTS) jitterIndex += P.num_alights;   // one per area light (:152-154)
                if (computeDirect && !EVENTS) {
                    if (logged && P.node_lo) {                       // shaded by k_shade
                        const double* lo =
                            P.node_lo + 3 * ((size_t)kk * hl.stride + (size_t)(hl.p - P.hits));
                        Lo = v3(lo[0], lo[1], lo[2]);
                        jitterIndex += P.num_alights;
                    } else {
                        direct_light<COUNT, WALK>(P, M, N, p, d, time, jitterIndex, st, c, Lo);
                    }
                }
                Frame& f = F[depth];
                f.p = p;
                if (!EVENTS) { f.Lo = Lo; f.t = h.t; f.hitmat = hitmat; f.mat = mi; }
                if ((M.type == RT_MAT_MIRROR || M.type == RT_MAT_CONDUCTOR) && depth < P.max_depth) {   // :189-206, :252-275
                    if (EVENTS) {
                    } else if (M.type == RT_MAT_MIRROR) {
                        f.aux = ld3(M.mirror);
                    } else {
                        const double cosI = smax(0.0, -dot(d, N));
                        f.aux = fresnel_conductor(M.ior, M.absorption_index, cosI) * ld3(M.mirror);
                    }
                    V3 rd = normalize(reflect(d, N));
                    if (M.roughness != 0.0) {
                        V3 tg, bt;
                        onb(rd, tg, bt);
                        const double rand1 = rng.nextFloat() - 0.5;
                        const double rand2 = rng.nextFloat() - 0.5;
                        rd = (rd + (M.roughness * rand1) * bt) + (M.roughness * rand2) * tg;
                        rd = normalize(rd);
                    }
                    f.state = kFrameMirror;
                    if (hl.tree) hl.node = tree_child(hl.tree, hl.node, 0);
                    c.secondary++;
                    o = p + N * P.shadow_eps;
                    d = rd;
                    tlo = 0.0;
                    descend = true;
                } else if (M.type == RT_MAT_DIELECTRIC && depth < P.max_depth) {                    // :207-251
                    V3 mfN = N;
                    if (M.roughness != 0.0) {
                        V3 tg, bt;
                        onb(N, tg, bt);
                        const double r1 = (rng.nextFloat() * 2.0) - 1.0;
                        const double r2 = (rng.nextFloat() * 2.0) - 1.0;
                        mfN = normalize((N + ((tg * r1) * M.roughness)) + ((bt * r2) * M.roughness));
                    }
                    const bool entering = frontFacing;
                    const double n1 = entering ? 1.0 : M.ior;
                    const double n2 = entering ? M.ior : 1.0;
                    const double cosI = -dot(d, mfN);
                    double R, cosT, sin2T;
                    bool hasCosT;
                    fresnel_dielectric(n1, n2, cosI, R, hasCosT, cosT, sin2T);
                    const V3 rd = normalize(reflect(d, mfN));
                    f.tir = !hasCosT || sin2T > 1;
                    if (!f.tir) {
                        const double eta = n1 / n2;
                        f.td = normalize((d * eta) + (mfN * (eta * cosI - cosT)));
                    }
                    if (!EVENTS) { f.R = R; f.entering = entering; }
                    f.state = kFrameDielR;
                    if (hl.tree) hl.node = tree_child(hl.tree, hl.node, 0);
                    c.secondary++;
                    o = p + rd * P.shadow_eps;
                    d = rd;
                    tlo = 0.0;
                    descend = true;
                } else if (!EVENTS) {
                    out = LevelOut{isfin(Lo) ? Lo : v3(0, 0, 0), true, hitmat, h.t};   // :277-280
                }
            }
        }
        if (descend) { depth++; continue; }
        // ======================================================== return to parents
        for (;;) {
            if (depth == 0) return out.L;
            depth--;
            if (hl.tree) hl.node = tree_parent(hl.tree, hl.node);
            Frame& f = F[depth];
            if (f.state == kFrameMirror) {
                if (EVENTS) continue;
                const V3 Lo = f.Lo + f.aux * out.L;
                out = LevelOut{isfin(Lo) ? Lo : v3(0, 0, 0), true, f.hitmat, f.t};
                continue;
            }
            if (f.state == kFrameDielR) {
                if (f.tir) {
                    if (EVENTS) continue;
                    const V3 Lo = f.Lo + out.L;
                    out = LevelOut{isfin(Lo) ? Lo : v3(0, 0, 0), true, f.hitmat, f.t};
                    continue;
                }
                if (!EVENTS) f.aux = out.L;                          // LiR
                f.state = kFrameDielT;
                if (hl.tree) hl.node = tree_child(hl.tree, hl.node, 1);
                c.secondary++;
                o = f.p + f.td * P.shadow_eps;                       // Ray(origin:dir:time:), tMin 0
                d = f.td;
                tlo = 0.0;
                depth++;
                descend = true;
                break;
            }
            // kFrameDielT
            if (EVENTS) continue;
            V3 LiT = out.L;
            const DMaterial& M = P.mats[f.mat];
            const bool absNonZero = !(M.absorption[0] == 0 && M.absorption[1] == 0 && M.absorption[2] == 0);
            if (f.entering && absNonZero && out.hit && out.hitmat == f.hitmat) {   // beerAttenuate quirk
                const double dd = smax(out.t, 0.0);
                const V3 a = -ld3(M.absorption) * dd;
                const V3 att = (__builtin_isfinite(dd) && dd > 0) ? v3(exp(a.x), exp(a.y), exp(a.z)) : LiT;
                LiT = LiT * att;
            }
            const V3 Lo = f.Lo + ((f.aux * f.R) + (LiT * (1.0 - f.R)));
            out = LevelOut{isfin(Lo) ? Lo : v3(0, 0, 0), true, f.hitmat, f.t};
        }
        if (!descend) return out.L;
    }
}

// Pixel loop shared by k_events and render_full (Object+Extension.swift:292-356).
template <bool COUNT, bool EVENTS, bool DEEP, int WALK>
__device__ __forceinline__ V3 pixel_full(const RenderParams& P, int i, int j, long long& jitterIndex, Stack& st,
                                         Counts& c, HitLog& hl) {
    const DCamera& C = P.cam;
    PCG32 rng((((unsigned long long)j << 32) ^ (unsigned long long)i) + 0x9E3779B97F4A7C15ull);
    V3 pixel = v3(0, 0, 0);
    const V3 eye = ld3(C.eye), u = ld3(C.u), v = ld3(C.v), w = ld3(C.w), q00 = ld3(C.q00);
    const int n = C.n;
    int sampleIndex = 0;
    for (int sy = 0; sy < n && sampleIndex < C.samples; ++sy) {
        for (int sx = 0; sx < n; ++sx) {
            const double xi1 = rng.nextFloat();
            const double xi2 = rng.nextFloat();
            const double currentI = (double)i + ((double)sx + xi1) / (double)n;
            const double currentJ = (double)j + ((double)sy + xi2) / (double)n;
            const V3 s = (q00 - v * (currentJ * C.dv)) + u * (currentI * C.du);
            const V3 dir0 = normalize(s - eye);
            V3 dir = dir0, camEye = eye;
            if (C.aperture > 0 && C.focus > 0) {                      // :325-338
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
            const double tImg = dot((eye - w * C.nd) - camEye, w) / (denom == 0.0 ? 4.9406564584124654e-324 : denom);
            pixel = pixel + trace_full<COUNT, EVENTS, DEEP, WALK>(P, camEye, dir, smax(tImg, 0.0), time, rng, jitterIndex,
                                                                  st, c, hl);
            if (hl.tree) { hl.sbase += P.tree_size; hl.node = 0; }
            sampleIndex += 1;
            if (sampleIndex >= C.samples) break;
        }
    }
    return pixel;
}

__device__ __forceinline__ void full_pixel_of(const RenderParams& P, int& i, int& j, int& slot, int& row) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int wpb = (int)(blockDim.x >> 6);
    const int gx = (P.cam.width + 8 * wpb - 1) / (8 * wpb);
    const int tile = (int)blockIdx.x;
    i = (tile % gx) * (8 * wpb) + wave * 8 + (lane & 7);
    slot = P.slot_base + tile / gx;
    const int chunk = P.chunk_first + slot * P.chunk_step;
    row = lane >> 3;
    j = chunk * 8 + row;
}

// Pass 1: area-light evaluations per pixel of the selection (packed rows).
// waves/SIMD for the full trace() passes (k_events, k_level, k_shade, render_full; 0 = the compiler's
// choice, 3 for k_level / k_shade at 138-150 VGPRs).  4 since the four-wide walk: C3g 4.22 -> 3.92,
// C3d 2.97 -> 2.90, C3r 4.96 -> 4.57 ms per frame pipelined (profiles/r04k_*).
#ifndef MYRT_FULL_WPE
#define MYRT_FULL_WPE 4
#endif
#if MYRT_FULL_WPE > 0
#define MYRT_FULL_ATTR __attribute__((amdgpu_waves_per_eu(MYRT_FULL_WPE)))
#else
#define MYRT_FULL_ATTR
#endif
// k_events alone (the depth-first events pass of rough / deep frames)
#ifndef MYRT_EV_WPE
#define MYRT_EV_WPE MYRT_FULL_WPE
#endif
#if MYRT_EV_WPE > 0
#define MYRT_EV_ATTR __attribute__((amdgpu_waves_per_eu(MYRT_EV_WPE)))
#else
#define MYRT_EV_ATTR
#endif
// render_full alone (the combine pass over the logged hits, with its per-lane trace() frames): 2
// waves/SIMD - its 256 VGPRs hold what 4 waves spilled (112 spills, ~1 GB of writes per C3g
// frame): C3g 3.20 -> 3.12, C3r 3.80 -> 3.72 ms per frame (3 waves: 3.16 / 3.80;
// profiles/r06s_ab_c3g.txt, r06s_ab_c3r.txt)
#ifndef MYRT_RF_WPE
#define MYRT_RF_WPE 2
#endif
#if MYRT_RF_WPE > 0
#define MYRT_RF_ATTR __attribute__((amdgpu_waves_per_eu(MYRT_RF_WPE)))
#else
#define MYRT_RF_ATTR
#endif
// The closest-hit walks' equal-t re-walks (wide.h ties; rt_stats.rewalked) of one wave, counted
// where the walks run (every lane of the wave must reach this: wave_sum reads all 64 lanes).
__device__ __forceinline__ void flush_ties(const RenderParams& P, const Counts& c) {
    const unsigned long long t = wave_sum(c.ties);
    if ((threadIdx.x & 63) == 0 && t) atomicAdd(&P.counters[kCounterTies], t);
}

template <bool DEEP, int WALK>
__global__ __launch_bounds__(256) MYRT_EV_ATTR void k_events(RenderParams P) {
    extern __shared__ unsigned long long lds_stack[];
    int i, j, slot, row;
    full_pixel_of(P, i, j, slot, row);
    Counts cnt{};
    if (i < P.cam.width && j < P.cam.height) {
        MYRT_STACK(st, lds_stack);
        long long events = 0;
        const size_t q = ((size_t)slot * 8 + row) * (size_t)P.cam.width + i;
        HitLog hl{P.hits + q, (size_t)P.hit_stride, 0, P.hits ? P.hit_slots : 0};
        (void)pixel_full<false, true, DEEP, WALK>(P, i, j, events, st, cnt, hl);
        P.events[q] = events;
        if (P.walks) P.walks[q] = hl.k;
    }
    flush_ties(P, cnt);
}

// ---- breadth-first events passes (P.hit_tree != 0) -------------------------------------------
// Without rough materials no PCG32 draw happens inside trace() (:193-198, :209-216, :258-263), so
// a trace() tree's rays do not depend on the order its nodes are walked in.  Then k_events'
// depth-first walk of every pixel's tree (a wave runs as long as its deepest tree, lane by lane)
// becomes one pass per tree level: k_level(0) walks every pixel's primary rays (coherent), and
// k_level(L) the level-L nodes, one grid row per node position, so a wave holds the same node of
// 64 neighbouring pixels.  Node h of sample s sits at log entry s * tree_size + h: heap order with
// dielectrics (reflection child 2h + 1, transmission 2h + 2; hit_tree = 2), the chain h = depth
// without (hit_tree = 1); the log holds the whole tree.  A parent writes its children's rays
// (DNodeRec o, d, time) and existence flags; k_jofs then visits each pixel's nodes in trace()'s
// depth-first order (the node, its reflection subtree, its transmission subtree) to give every
// node the jitterIndex offset the depth-first render reaches there and the pixel its evaluation
// count (k_jscan's input).  render_full and k_shade index the log the same way.

// One node: walk its ray, log the hit, flag it, write its children (trace_full's EVENTS steps on
// the same values: the same expressions, so the same rays).
template <int WALK>
__device__ __forceinline__ void level_node(const RenderParams& P, size_t q, int s, int h, int level, const V3& o,
                                           const V3& d, double tlo, double time, Stack& st, Counts& c) {
    const size_t S = (size_t)P.hit_stride;
    const int b = P.hit_tree, per = P.tree_size;
    const size_t at = (size_t)(s * per + h) * S + q;
    Hit hh;
    walk_closest<false, WALK>(P, o, d, rcp(d), tlo, time, hh, st, c);
    DHitRec r;
    r.t = hh.t; r.u = hh.u; r.v = hh.v; r.tri = hh.tri; r.inst = hh.inst;
    P.hits[at] = r;
    uint8_t fl = kNodeExists;
    if (hh.inst >= 0) {
        fl |= kNodeHit;
        V3 p, Ngeo;
        hit_geometry<false>(P, o, d, time, hh, p, Ngeo, c);
        const DMaterial& M = P.mats[max(0, min(P.num_mats - 1, P.insts[hh.inst].material - 1))];
        const bool frontFacing = dot(d, Ngeo) < 0;
        const V3 N = frontFacing ? Ngeo : -Ngeo;
        if (!(M.ior > 0) || frontFacing) fl |= kNodeEval;                 // computeDirect
        auto spawn = [&](int which, const V3& co, const V3& cd) {
            const size_t ca = (size_t)(s * per + tree_child(b, h, which)) * S + q;
            DNodeRec& n = P.nodes[ca];
            n.o[0] = co.x; n.o[1] = co.y; n.o[2] = co.z;
            n.d[0] = cd.x; n.d[1] = cd.y; n.d[2] = cd.z;
            n.time = time;
            P.nflags[ca] = kNodeExists;
        };
        if (level < P.max_depth) {
            if (M.type == RT_MAT_MIRROR || M.type == RT_MAT_CONDUCTOR) {        // :189-206, :252-275
                spawn(0, p + N * P.shadow_eps, normalize(reflect(d, N)));
            } else if (M.type == RT_MAT_DIELECTRIC) {                          // :207-251
                const bool entering = frontFacing;
                const double n1 = entering ? 1.0 : M.ior;
                const double n2 = entering ? M.ior : 1.0;
                const double cosI = -dot(d, N);
                double R, cosT, sin2T;
                bool hasCosT;
                fresnel_dielectric(n1, n2, cosI, R, hasCosT, cosT, sin2T);
                const V3 rd = normalize(reflect(d, N));
                spawn(0, p + rd * P.shadow_eps, rd);
                if (!(!hasCosT || sin2T > 1)) {
                    const double eta = n1 / n2;
                    const V3 td = normalize((d * eta) + (N * (eta * cosI - cosT)));
                    spawn(1, p + td * P.shadow_eps, td);
                }
            }
        }
    }
    P.nflags[at] = fl;
    P.nodes[at].hit = hh.inst >= 0 ? 1 : 0;
}

template <int WALK>
__device__ __forceinline__ void level_pixel(const RenderParams& P, int level, int i, int j, int slot, int row,
                                            Counts& cnt);
template <int WALK>
__global__ __launch_bounds__(256) MYRT_FULL_ATTR void k_level(RenderParams P, int level) {
    int i, j, slot, row;
    full_pixel_of(P, i, j, slot, row);
    Counts cnt{};
    if (i < P.cam.width && j < P.cam.height) level_pixel<WALK>(P, level, i, j, slot, row, cnt);
    flush_ties(P, cnt);
}

template <int WALK>
__device__ __forceinline__ void level_pixel(const RenderParams& P, int level, int i, int j, int slot, int row,
                                            Counts& cnt) {
    extern __shared__ unsigned long long lds_stack[];
    const size_t q = ((size_t)slot * 8 + row) * (size_t)P.cam.width + i;
    if (level > 0) {
        // one wave per tile and traced sample runs the level's node positions one after another
        // (a position's lanes are the same node of neighbouring pixels); a position no lane of
        // the wave has is one flag load (launching one wave per position cost more in
        // dispatching the empty ones than the walks)
        const int rows = tree_rows(P.hit_tree, level, P.tree_ppw);
        const int s = (int)blockIdx.y / rows, g = (int)blockIdx.y % rows;
        const int width = min(P.tree_ppw, tree_width(P.hit_tree, level) - g * P.tree_ppw);
        const int h0 = tree_first(P.hit_tree, level) + g * P.tree_ppw;
        MYRT_STACK(st, lds_stack);
        for (int pos = 0; pos < width; ++pos) {
            const size_t at = (size_t)(s * P.tree_size + h0 + pos) * (size_t)P.hit_stride + q;
            const bool ex = (P.nflags[at] & kNodeExists) != 0;
            if (!__any(ex)) continue;
            if (ex) {
                const DNodeRec n = P.nodes[at];
                level_node<WALK>(P, q, s, h0 + pos, level, v3(n.o[0], n.o[1], n.o[2]), v3(n.d[0], n.d[1], n.d[2]),
                                 0.0, n.time, st, cnt);
            }
        }
        return;
    }
    // level 0: the pixel's primary rays, sample by sample, with pixel_full's draws
    MYRT_STACK(st, lds_stack);
    const DCamera& C = P.cam;
    PCG32 rng((((unsigned long long)j << 32) ^ (unsigned long long)i) + 0x9E3779B97F4A7C15ull);
    const V3 eye = ld3(C.eye), u = ld3(C.u), v = ld3(C.v), w = ld3(C.w), q00 = ld3(C.q00);
    const int n = C.n;
    int sampleIndex = 0;
    for (int sy = 0; sy < n && sampleIndex < C.samples; ++sy) {
        for (int sx = 0; sx < n; ++sx) {
            const double xi1 = rng.nextFloat();
            const double xi2 = rng.nextFloat();
            const double currentI = (double)i + ((double)sx + xi1) / (double)n;
            const double currentJ = (double)j + ((double)sy + xi2) / (double)n;
            const V3 s = (q00 - v * (currentJ * C.dv)) + u * (currentI * C.du);
            const V3 dir0 = normalize(s - eye);
            V3 dir = dir0, camEye = eye;
            if (C.aperture > 0 && C.focus > 0) {
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
            const double tImg = dot((eye - w * C.nd) - camEye, w) / (denom == 0.0 ? 4.9406564584124654e-324 : denom);
            const size_t at = (size_t)(sampleIndex * P.tree_size) * (size_t)P.hit_stride + q;
            DNodeRec& nr = P.nodes[at];
            nr.o[0] = camEye.x; nr.o[1] = camEye.y; nr.o[2] = camEye.z;
            nr.d[0] = dir.x; nr.d[1] = dir.y; nr.d[2] = dir.z;
            nr.time = time;
            level_node<WALK>(P, q, sampleIndex, 0, 0, camEye, dir, smax(tImg, 0.0), time, st, cnt);
            sampleIndex += 1;
            if (sampleIndex >= C.samples) break;
        }
    }
}

// After the last level: each node's jitterIndex offset in trace()'s depth-first order, and the
// pixel's area-light evaluations (k_events' outputs).  Flags only: no walks.
__global__ __launch_bounds__(256) void k_jofs(RenderParams P) {
    int i, j, slot, row;
    full_pixel_of(P, i, j, slot, row);
    if (i >= P.cam.width || j >= P.cam.height) return;
    const size_t q = ((size_t)slot * 8 + row) * (size_t)P.cam.width + i;
    const size_t S = (size_t)P.hit_stride;
    const int b = P.hit_tree, per = P.tree_size, traced = P.hit_slots / P.tree_size;
    const long long na = P.num_alights;
    long long ev = 0;
    for (int s = 0; s < traced; ++s) {
        auto at = [&](int h) { return (size_t)(s * per + h) * S + q; };
        auto exists = [&](int h) { return h < per && (P.nflags[at(h)] & kNodeExists); };
        int h = 0;                                            // the root always exists
        for (;;) {
            P.nodes[at(h)].jofs = (int32_t)ev;
            if (P.nflags[at(h)] & kNodeEval) ev += na;
            int nx = -1;                                      // next node in preorder
            if (exists(tree_child(b, h, 0))) nx = tree_child(b, h, 0);
            else if (b == 2 && exists(tree_child(b, h, 1))) nx = tree_child(b, h, 1);
            else if (b == 2) {
                for (int c = h; c != 0;) {
                    const int p = tree_parent(b, c);
                    if ((c & 1) && exists(tree_child(b, p, 1))) { nx = tree_child(b, p, 1); break; }
                    c = p;
                }
            }
            if (nx < 0) break;
            h = nx;
        }
    }
    P.events[q] = ev;
}

// Node-parallel shading (after k_jscan): the direct light of every logged walk k that hit,
// one lane per (pixel, k) - the same hit_geometry and direct_light as render_full on the same
// ray and hit, with the jitterIndex the render pass reaches at that node (the pixel's prefix +
// the node's offset, both counted by k_events).  Grid: (the selection's tiles, hit_slots).
// render_full then shades no logged hit itself: its waves no longer run the shadow walks of the
// longest path tree with the other lanes idle.
// One logged walk k of pixel q that hit: its direct light into node_lo.
template <int WALK>
__device__ __forceinline__ void shade_node(const RenderParams& P, size_t q, int k, Stack& st, Counts& cnt) {
    const size_t at = (size_t)k * (size_t)P.hit_stride + q;
    const DNodeRec n = P.nodes[at];
    if (!n.hit) return;
    const DHitRec r = P.hits[at];
    Hit h;
    h.t = r.t; h.u = r.u; h.v = r.v; h.tri = r.tri; h.inst = r.inst;
    const V3 o = v3(n.o[0], n.o[1], n.o[2]), d = v3(n.d[0], n.d[1], n.d[2]);
    V3 p, Ngeo;
    hit_geometry<false>(P, o, d, n.time, h, p, Ngeo, cnt);
    const int hitmat = P.insts[h.inst].material;
    const int mi = max(0, min(P.num_mats - 1, hitmat - 1));
    const DMaterial& M = P.mats[mi];
    const bool frontFacing = dot(d, Ngeo) < 0;
    const V3 N = frontFacing ? Ngeo : -Ngeo;
    const bool computeDirect = !(M.ior > 0) || frontFacing;
    V3 Lo = computeDirect ? ld3(P.ambient) * ld3(M.ambient) : v3(0, 0, 0);
    if (computeDirect) {
        long long jitterIndex = (P.num_alights > 0 ? P.jstart[q] : 0) + n.jofs;
        direct_light<false, WALK>(P, M, N, p, d, n.time, jitterIndex, st, cnt, Lo);
    }
    double* lo = P.node_lo + 3 * at;
    lo[0] = Lo.x; lo[1] = Lo.y; lo[2] = Lo.z;
}

// Grid (the selection's tiles, hit_slots) for the k-th walk log; with tree-indexed logs
// (hit_tree) grid (tiles, traced samples x tree levels), one wave running the level's node
// positions one after another (as k_level).
template <int WALK>
__global__ __launch_bounds__(256) MYRT_FULL_ATTR void k_shade(RenderParams P) {
    extern __shared__ unsigned long long lds_stack[];
    int i, j, slot, row;
    full_pixel_of(P, i, j, slot, row);
    const int lane = threadIdx.x & 63;
    Counts cnt{};
    const bool valid = (i < P.cam.width) && (j < P.cam.height);
    const size_t q = valid ? ((size_t)slot * 8 + row) * (size_t)P.cam.width + i : 0;
    MYRT_STACK(st, lds_stack);
    int k0 = (int)blockIdx.y, width = 1;                    // log entries k0 .. k0 + width - 1
    if (P.hit_tree) {                                       // row -> (sample, level, group)
        int per = 0;
        for (int L = 0; L <= P.max_depth; ++L) per += tree_rows(P.hit_tree, L, P.tree_ppw);
        const int s = (int)blockIdx.y / per;
        int r = (int)blockIdx.y % per, level = 0;
        while (r >= tree_rows(P.hit_tree, level, P.tree_ppw)) r -= tree_rows(P.hit_tree, level++, P.tree_ppw);
        width = min(P.tree_ppw, tree_width(P.hit_tree, level) - r * P.tree_ppw);
        k0 = s * P.tree_size + tree_first(P.hit_tree, level) + r * P.tree_ppw;
    }
    for (int k = k0; k < k0 + width; ++k) {                 // one call site of the shadow walk
        const bool ex = valid && (P.hit_tree ? (P.nflags[(size_t)k * (size_t)P.hit_stride + q] & kNodeExists) != 0
                                             : k < P.walks[q]);
        if (!__any(ex)) continue;
        if (ex) shade_node<WALK>(P, q, k, st, cnt);
    }
    const unsigned long long s0 = wave_sum(cnt.shadow), s2 = wave_sum(cnt.shadow_traced);
    if (lane == 0) {
        if (s0) atomicAdd(&P.counters[0], s0);
        if (s2) atomicAdd(&P.counters[kCounterShadowTraced], s2);
    }
}

// Pass 2: exclusive prefix of the events over each chunk, row-major (one block per chunk).
__global__ __launch_bounds__(256) void k_jscan(RenderParams P) {
    __shared__ long long part[256];
    const int slot = blockIdx.x;
    const int chunk = P.chunk_first + slot * P.chunk_step;
    const int rows = min(8, P.cam.height - chunk * 8);
    const long long n = (long long)rows * P.cam.width;
    const size_t base = (size_t)slot * 8 * (size_t)P.cam.width;
    const long long seg = (n + 255) / 256;
    const long long b = min(n, (long long)threadIdx.x * seg), e = min(n, b + seg);
    long long sum = 0;
    for (long long k = b; k < e; ++k) sum += P.events[base + k];
    part[threadIdx.x] = sum;
    __syncthreads();
    if (threadIdx.x == 0) {
        long long run = 0;
        for (int t = 0; t < 256; ++t) { const long long x = part[t]; part[t] = run; run += x; }
    }
    __syncthreads();
    long long run = part[threadIdx.x];
    long long* js = const_cast<long long*>(P.jstart);
    for (long long k = b; k < e; ++k) { js[base + k] = run; run += P.events[base + k]; }
}

// Pass 3 (or the only pass without area lights): the render.
template <bool COUNT, bool DEEP, int WALK>
__global__ __launch_bounds__(256) MYRT_RF_ATTR void render_full(RenderParams P) {
    extern __shared__ unsigned long long lds_stack[];
    int i, j, slot, row;
    full_pixel_of(P, i, j, slot, row);
    const bool valid = (i < P.cam.width) && (j < P.cam.height);
    const int lane = threadIdx.x & 63;
    Counts cnt{};
    if (valid) {
        MYRT_STACK(st, lds_stack);
        const size_t q = ((size_t)slot * 8 + row) * (size_t)P.cam.width + i;   // packed selection index
        long long jitterIndex = P.num_alights > 0 ? P.jstart[q] : 0;
        HitLog hl{P.hits + q, (size_t)P.hit_stride, 0, P.hits ? P.hit_slots : 0};
        hl.tree = P.hits ? P.hit_tree : 0;
        const V3 px = pixel_full<COUNT, false, DEEP, WALK>(P, i, j, jitterIndex, st, cnt, hl) / (double)P.cam.samples;
        const size_t o = out_row_of(P, j >> 3, row) * (size_t)P.cam.width + i;
        if (P.out_rgb) {
            P.out_rgb[o * 3 + 0] = px.x;
            P.out_rgb[o * 3 + 1] = px.y;
            P.out_rgb[o * 3 + 2] = px.z;
        }
        if (P.out_rgba8) {                                           // RayTracer.swift:186-195
            const double cx = fmin(fmax(px.x, 0.0), 255.0), cy = fmin(fmax(px.y, 0.0), 255.0),
                         cz = fmin(fmax(px.z, 0.0), 255.0);
            const unsigned packed = (unsigned)(unsigned char)cx | ((unsigned)(unsigned char)cy << 8) |
                                    ((unsigned)(unsigned char)cz << 16) | (255u << 24);
            reinterpret_cast<unsigned*>(P.out_rgba8)[o] = packed;
        }
    }
    const unsigned long long s0 = wave_sum(cnt.shadow), s1 = wave_sum(cnt.secondary),
                             s2 = wave_sum(cnt.shadow_traced);
    if (lane == 0) {
        if (s0) atomicAdd(&P.counters[0], s0);
        if (s1) atomicAdd(&P.counters[1], s1);
        if (s2) atomicAdd(&P.counters[kCounterShadowTraced], s2);
    }
    flush_ties(P, cnt);
    if (COUNT) {
        const unsigned long long a = wave_sum(cnt.recs), b = wave_sum(cnt.tris), cc = wave_sum(cnt.normals),
                                 dd = wave_sum(cnt.insts), ee = wave_sum(valid ? 1ull : 0ull);
        if (lane == 0) {
            atomicAdd(&P.counters[2], a); atomicAdd(&P.counters[3], b); atomicAdd(&P.counters[4], cc);
            atomicAdd(&P.counters[5], dd); atomicAdd(&P.counters[6], ee);
        }
        const unsigned long long ff = wave_sum(cnt.nodes), gg = wave_sum(cnt.smooth);
        if (lane == 0 && P.count_ref) { atomicAdd(&P.counters[7], ff); atomicAdd(&P.counters[8], gg); }
    }
}

}  // namespace dev
}  // namespace myrt
