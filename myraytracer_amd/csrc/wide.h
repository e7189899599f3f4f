// wide.h — the conservative FP32 four-wide walk of identity scenes, exact by construction.
//
// Why it returns the reference's hit (reference RTContext.swift:544-610,
// 722-829).  For a ray whose 1/d components are all finite:
//  * child boxes nest inside parent boxes (min/max over a subset of the parent's primitives,
//    BVH.swift:108-124, 184-185; a TLAS leaf box holds its identity instances' BLAS root boxes),
//    and the FP64 slab test of hitAABB (:557-565) is monotone in the bounds, so a leaf whose box
//    passes has ancestors that pass: intersectBLAS tests exactly the triangles of the leaves
//    whose box passes, whatever the inner boxes;
//  * the closest hit is therefore the minimum Moeller-Trumbore t over those triangles; the visit
//    order matters only between triangles of EQUAL t (strict t < hit.t, :494, keeps the first).
// The walk below tests inner boxes in FP32 against boxes widened so that the test passes
// whenever the reference's FP64 test of any leaf box below passes (a superset of leaves is
// reached), tests triangles with the reference's FP64 Moeller-Trumbore, and accepts a candidate
// only after the exact FP64 test of its own leaf box (lbox; rare: only candidates that would
// lower or equal the current hit).  A lane that met a second candidate at its final t is
// re-walked with the reference-order binary walk (device.h uni_closest_walk).  Any-hit walks
// are order-free: occluded iff some reached triangle passes triShadowHit and its leaf box
// passes.  Lanes whose direction has a component below 2^-100 (or zero) take the binary walk.
//
// Widening (RenderParams::wdelta, make_params): per axis the walk computes
//   t_lo = fma(lo, 1/d_f, -(o/d) - wdelta/d),  t_hi = fma(hi, 1/d_f, -(o/d) + wdelta/d)
// in FP32 with the offsets rounded from FP64.  Against the exact (lo - o)/d this carries an
// error below |1/d| * 2^-24 * (2|b| + 2|o| + 2 wdelta) (rounding of 1/d, of the offset and of
// the FMA), so with wdelta >= 8 * 2^-24 * max(|b|, |o|) the computed near-plane value lies below
// the exact one and the far-plane value above it, for either sign of d: the FP32 entry distance
// is <= the FP64 one and the FP32 exit distance >= it.  Box coordinates are rounded outward to
// float (layout.h W4Node), eps rounded down (weps), the pruning limit rounded up.
#pragma once

namespace myrt {
namespace dev {

// The ray in the walk's FP32 form.  The node array holds one copy of the tree per direction
// octant (layout.h W4Node): in the copy of the ray's octant every node's rows are already its
// near planes (the box minimum along a when d[a] >= 0, the maximum otherwise) and far planes, so a
// slot's entry distance is max3 of three FMAs on the near row and its exit min3 on the far row -
// the same values as min/max of both plane distances (FMA is monotone, and the lo-plane offset is
// below the hi-plane one) - and its slots are in front-to-back order for that octant.
typedef float wf2 __attribute__((ext_vector_type(2)));
typedef float wf4 __attribute__((ext_vector_type(4)));
typedef int wi4 __attribute__((ext_vector_type(4)));
struct WRay {
    float ix, iy, iz;     // 1/d in FP32
    float nox, noy, noz;  // offset of the near planes: -(o/d) - wdelta*|1/d|
    float fox, foy, foz;  // offset of the far planes:  -(o/d) + wdelta*|1/d|
    unsigned obase;       // byte offset of this octant's copy of the node array
    bool uoct;            // every lane of the wave has this direction octant (wave-uniform)
};

// every |1/d| within [2^-100, 2^100] (finite; FP32 products of scene coordinates stay finite)
__device__ __forceinline__ bool wide_ok(const V3& inv) {
    const double ax = fabs(inv.x), ay = fabs(inv.y), az = fabs(inv.z);
    return ax <= 0x1p100 && ax >= 0x1p-100 && ay <= 0x1p100 && ay >= 0x1p-100 && az <= 0x1p100 && az >= 0x1p-100;
}

__device__ __forceinline__ WRay wide_ray(const RenderParams& P, const V3& o, const V3& inv, double wdelta) {
    WRay r;
    r.ix = (float)inv.x; r.iy = (float)inv.y; r.iz = (float)inv.z;
    const double ox = o.x * inv.x, oy = o.y * inv.y, oz = o.z * inv.z;
    const double dx = wdelta * fabs(inv.x), dy = wdelta * fabs(inv.y), dz = wdelta * fabs(inv.z);
    r.nox = (float)(-ox - dx); r.noy = (float)(-oy - dy); r.noz = (float)(-oz - dz);
    r.fox = (float)(-ox + dx); r.foy = (float)(-oy + dy); r.foz = (float)(-oz + dz);
    const unsigned oct = (inv.x >= 0 ? 0u : 1u) | (inv.y >= 0 ? 0u : 2u) | (inv.z >= 0 ? 0u : 4u);
    r.obase = oct * P.wide_copy_bytes;
    r.uoct = __all(oct == (unsigned)__builtin_amdgcn_readfirstlane((int)oct));
    return r;
}

// FP32 pruning limit >= t * prune_rel + prune_abs (finite: empty slots compare against it)
__device__ __forceinline__ float wide_limit(const RenderParams& P, double t) {
    const double x = fmin(t * P.prune_rel + P.prune_abs, 3.0e38);
    return (float)x * (1.0f + 0x1p-20f);
}

__device__ __forceinline__ unsigned long long wide_entry(int ref, float t) {
    return (unsigned long long)(unsigned)ref | ((unsigned long long)__float_as_uint(t) << 32);
}

// One four-wide node: the slots whose widened box the ray enters within [weps, lim].  The walk
// continues with the first slot hit in the node's (octant) order and pushes the others last
// first, so they pop in that order; for any-hit walks the order is immaterial.  Returns false
// when no slot is hit (the caller pops).
template <class RowF4, class RowI4>
__device__ __forceinline__ bool wide_node(const RenderParams& P, int& ref, const WRay& R, float lim, Stack& st,
                                          RowF4 row, RowI4 refrow) {
    constexpr unsigned kFar = offsetof(W4Node, pfar), kRef = offsetof(W4Node, ref);
    const wf4 nx = row(0u), ny = row(16u), nz = row(32u);
    const wf4 fx = row(kFar), fy = row(kFar + 16u), fz = row(kFar + 32u);
    const wi4 refs = refrow(kRef);
    // the 24 plane distances (FP32 FMAs; packed v_pk_fma_f32 forms measured slower: their splat
    // register pairs spilled, and the op_sel inline-asm form lost the loads' latency overlap,
    // profiles/r05c_ab_c3.txt)
    auto fm = [](wf2 a, float b, float c) { return wf2{__builtin_fmaf(a.x, b, c), __builtin_fmaf(a.y, b, c)}; };
    const wf2 anx0 = fm(nx.xy, R.ix, R.nox), anx1 = fm(nx.zw, R.ix, R.nox);
    const wf2 any0 = fm(ny.xy, R.iy, R.noy), any1 = fm(ny.zw, R.iy, R.noy);
    const wf2 anz0 = fm(nz.xy, R.iz, R.noz), anz1 = fm(nz.zw, R.iz, R.noz);
    const wf2 afx0 = fm(fx.xy, R.ix, R.fox), afx1 = fm(fx.zw, R.ix, R.fox);
    const wf2 afy0 = fm(fy.xy, R.iy, R.foy), afy1 = fm(fy.zw, R.iy, R.foy);
    const wf2 afz0 = fm(fz.xy, R.iz, R.foz), afz1 = fm(fz.zw, R.iz, R.foz);
    const float tn[4] = {__builtin_fmaxf(__builtin_fmaxf(anx0.x, any0.x), anz0.x),
                         __builtin_fmaxf(__builtin_fmaxf(anx0.y, any0.y), anz0.y),
                         __builtin_fmaxf(__builtin_fmaxf(anx1.x, any1.x), anz1.x),
                         __builtin_fmaxf(__builtin_fmaxf(anx1.y, any1.y), anz1.y)};
    const float tf[4] = {__builtin_fminf(__builtin_fminf(afx0.x, afy0.x), afz0.x),
                         __builtin_fminf(__builtin_fminf(afx0.y, afy0.y), afz0.y),
                         __builtin_fminf(__builtin_fminf(afx1.x, afy1.x), afz1.x),
                         __builtin_fminf(__builtin_fminf(afx1.y, afy1.y), afz1.y)};
    const int nr[4] = {refs.x, refs.y, refs.z, refs.w};
    bool h[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) h[c] = __builtin_fmaxf(tn[c], P.weps) <= __builtin_fminf(tf[c], lim);
    // continue with the first slot hit; keep the later hits (they all come after it)
    const int nref = h[0] ? nr[0] : h[1] ? nr[1] : h[2] ? nr[2] : nr[3];
    const bool keep[4] = {false, h[1] && h[0], h[2] && (h[0] || h[1]), h[3] && (h[0] || h[1] || h[2])};
    if (!__any(st.sp > kLds - 3)) {
        // every lane's three candidate entries lie in LDS: unconditional stores at running
        // positions (a dropped entry is overwritten by the next kept one, or lies above the top)
        int p = st.sp;
#pragma unroll
        for (int c = 3; c >= 1; --c) {
            st.lds[p * Stack::stride] = wide_entry(nr[c], tn[c]);
            p += keep[c] ? 1 : 0;
        }
        st.sp = p;
    } else {
#pragma unroll
        for (int c = 3; c >= 1; --c) st.push_raw_if(keep[c], wide_entry(nr[c], tn[c]));
    }
    ref = nref;
    return h[0] || h[1] || h[2] || h[3];
}

// One node step: the rows of node `ref` in this ray's octant copy (base = P.wnodes).
__device__ __forceinline__ bool wide_inner(const RenderParams& P, const char* base, int& ref, const WRay& R, float lim,
                                           Stack& st) {
    if (R.uoct) {
        // Every lane at the same node with the same octant (the top of the tree for a tile's
        // coherent rays): the rows come through the scalar cache into SGPRs once for the wave,
        // instead of 64 copies through the vector-memory data path (TD, ~0.87 busy).
        // (uoct is a hint: a lane that set it may share the branch with lanes whose ray - another
        // instance's local ray, tw_walk - has another octant, so the copy is checked too)
        const int r0 = __builtin_amdgcn_readfirstlane(ref);
        const unsigned ob0 = __builtin_amdgcn_readfirstlane(R.obase);
        if (__all(ref == r0 && R.obase == ob0)) {
            const unsigned nb = ob0 + (unsigned)r0 * (unsigned)sizeof(W4Node);
            const unsigned long long av = (unsigned long long)(base + (size_t)nb);
            const unsigned alo = __builtin_amdgcn_readfirstlane((unsigned)av);
            const unsigned ahi = __builtin_amdgcn_readfirstlane((unsigned)(av >> 32));
            typedef const __attribute__((address_space(4))) char c4_char;
            c4_char* sb = (c4_char*)((unsigned long long)alo | ((unsigned long long)ahi << 32));
            typedef const __attribute__((address_space(4))) wf4 c4_f4;
            typedef const __attribute__((address_space(4))) wi4 c4_i4;
            return wide_node(P, ref, R, lim, st, [&](unsigned off) { return *(c4_f4*)(sb + off); },
                             [&](unsigned off) { return *(c4_i4*)(sb + off); });
        }
    }
    // 32-bit byte offsets from the array base (the host keeps the array below 4 GB): the loads
    // take the SGPR-base + VGPR-offset + immediate form, one address per node
    const unsigned nb = R.obase + (unsigned)ref * (unsigned)sizeof(W4Node);
    return wide_node(P, ref, R, lim, st, [&](unsigned off) { return *reinterpret_cast<const wf4*>(base + (size_t)nb + off); },
                     [&](unsigned off) { return *reinterpret_cast<const wi4*>(base + (size_t)nb + off); });
}

// next entry whose (FP32, <= FP64) entry distance does not exceed lim
__device__ __forceinline__ bool wide_pop(Stack& st, int base, float lim, int& ref) {
    while (st.sp > base) {
        const unsigned long long e = st.pop_raw();
        if (__uint_as_float((unsigned)(e >> 32)) > lim) continue;
        ref = (int)(unsigned)(e & 0xffffffffull);
        return true;
    }
    return false;
}

// hitAABB of the reference leaf run starting at TriRec t0, exactly (FP64, RTContext.swift:557-565;
// the FAST form: every 1/d is finite here)
__device__ __forceinline__ bool leaf_box_exact(const RenderParams& P, int t0, const V3& o, const V3& d) {
    const double* b = P.lbox + 6 * (size_t)t0;
    const V3 inv = rcp(d);
    double tm;
    return slab_hit<true>(b[0], b[1], b[2], b[3], b[4], b[5], o, inv, P.eps, tm);
}

// intersectTriangle's tests (RTContext.swift:479-510) against the current closest t: 0 = rejected,
// 1 = closer (strict t < hit.t: accepted by the reference when reached), 2 = equal to hit.t.
template <class Tri>
__device__ __forceinline__ int tri_candidate(const Tri& T, const V3& o, const V3& d, double tlo, double eps,
                                             double ht, double& t_out, double& u_out, double& v_out, bool frcp) {
    V3 v0, e1, e2;
    tri_geom(T, v0, e1, e2);
    const V3 pvec = cross(d, e2);
    const double det = dot(e1, pvec);
    if (fabs(det) < eps) return 0;
    const double invDet = inv_det(det, frcp);
    const V3 tvec = o - v0;
    const double u = dot(tvec, pvec) * invDet;
    if (u < 0.0 || u > 1.0) return 0;
    const V3 q = cross(tvec, e1);
    const double v = dot(d, q) * invDet;
    if (v < 0.0 || u + v > 1.0) return 0;
    const double t = dot(e2, q) * invDet;
    if (t <= smax(eps, tlo)) return 0;
    t_out = t; u_out = u; v_out = v;
    return t < ht ? 1 : (t == ht ? 2 : 0);
}

// The world ray of a transformed walk: kept by the caller (TwWorld) or parked in this lane's
// private memory (TwParked: read back only where the walk needs it - its start, an instance's
// marker, the return to the TLAS - so it is not live, spilled, across the BLAS walks; the empty
// asm with the array's address keeps the compiler from forwarding the stored values.  1/d is
// recomputed there: parking it too, or a volatile park, measured slower, profiles/r05h_ab_c3i.txt).
struct TwWorld {
    const V3& o_;
    const V3& d_;
    __device__ __forceinline__ V3 o() const { return o_; }
    __device__ __forceinline__ V3 d() const { return d_; }
    static constexpr bool kParked = false;
};
struct TwParked {
    double v[6];                                          // o, d
    __device__ __forceinline__ void store(const V3& o, const V3& d) {
        v[0] = o.x; v[1] = o.y; v[2] = o.z; v[3] = d.x; v[4] = d.y; v[5] = d.z;
        asm volatile("" :: "v"(&v[0]) : "memory");
    }
    __device__ __forceinline__ V3 o() const { asm volatile("" :: "v"(&v[0]) : "memory"); return v3(v[0], v[1], v[2]); }
    __device__ __forceinline__ V3 d() const { asm volatile("" :: "v"(&v[0]) : "memory"); return v3(v[3], v[4], v[5]); }
    static constexpr bool kParked = true;
};

// ---- flattened instance tree (transformed scenes; scene.cpp build_fit, option fit).  One
// world-space four-wide tree over every (instance, BLAS leaf run) pair: a pair's box is its local
// leaf box through localToWorld (AABB.transformed, AABB.swift:71-92).  Why the walk returns the
// reference's hit: the reference tests the triangles of leaf L of instance k iff hitAABB passes
// for k's TLAS leaf box (world ray), k's BLAS root box and L's box (local ray: w2l applied to the
// world ray in FP64, RTContext.swift:632-673, 567-571; ancestors pass by nesting, wide.h header),
// and compares local t, which is world t (the local direction is not renormalised).  If the local
// FP64 test of L passes, some t* >= eps puts the computed local ray within 2^-50 max(|box|, |o_l|)
// of L per axis; through localToWorld (l2w w2l = I within kappa 2^-50, kappa = |l2w||w2l| <=
// kFitKappa = 2^12, scene.cpp) the exact world ray at t* lies within ~2^-44 kappa R <= 2^-32 R
// of the pair's box, R = fit_coord (every world/local magnitude and translation, scene.cpp) or
// the ray origin's reach.  The render widens every box by wdelta = 2^-21 R (the FP32 bound of the
// header) plus 2^-27 R (set_wide, fit scenes), so the walk enters every pair whose triangles the
// reference tests, with the same pruning limits as the other walks (lim >= the current local t).
// A candidate is accepted only after the exact FP64 tests of the three boxes, with the reference's
// local ray (the same m4_point arithmetic as ut_walk); equal-t candidates raise `tie` and are
// re-walked in the reference's order (ut_walk).  No local FP32 walk: local rays need no range.
__device__ __forceinline__ bool fit_boxes_exact(const RenderParams& P, int k, int t0, const V3& o, const V3& d,
                                                const V3& ol, const V3& dl) {
    const DWideInst& WI = P.winst[k];
    const DInstance& I = P.insts[k];
    const double* b = P.lbox + 6 * (size_t)t0;
    const V3 il = rcp(dl);
    double tm;
    return slab_hit<false>(b[0], b[1], b[2], b[3], b[4], b[5], ol, il, P.eps, tm) &&
           slab_hit<false>(I.root_lo[0], I.root_lo[1], I.root_lo[2], I.root_hi[0], I.root_hi[1], I.root_hi[2], ol, il,
                           P.eps, tm) &&
           slab_hit<true>(WI.tbox[0], WI.tbox[1], WI.tbox[2], WI.tbox[3], WI.tbox[4], WI.tbox[5], o, rcp(d), P.eps, tm);
}
// instance k's local ray (ut_local's arithmetic for a static instance): worldToLocal through the
// scalar cache when every active lane is in the same instance
#ifndef MYRT_FIT_SCALAR
#define MYRT_FIT_SCALAR 1   // worldToLocal through the scalar cache when uniform: 6,315 vs 6,237 Mrays/s without
#endif
#ifndef MYRT_FIT_CACHE
#define MYRT_FIT_CACHE 1    // keep the last pair's local ray (its instance) across the walk: C3i 6,315 -> 6,567 Mrays/s (profiles/r06d_ab_c3i.txt)
#endif
__device__ __forceinline__ void fit_local(const RenderParams& P, int k, const V3& o, const V3& d, V3& ol, V3& dl) {
    const int k0 = __builtin_amdgcn_readfirstlane(k);
    if (MYRT_FIT_SCALAR && __all(k == k0)) {
        const unsigned long long av = (unsigned long long)P.insts[k0].w2l;
        const unsigned alo = __builtin_amdgcn_readfirstlane((unsigned)av);
        const unsigned ahi = __builtin_amdgcn_readfirstlane((unsigned)(av >> 32));
        typedef const __attribute__((address_space(4))) double c4_double;
        c4_double* M = (c4_double*)((unsigned long long)alo | ((unsigned long long)ahi << 32));
        double w[12];
#pragma unroll
        for (int i = 0; i < 12; ++i) w[i] = M[(i / 3) * 4 + i % 3];
        double m[16] = {w[0], w[1], w[2], 0.0, w[3], w[4], w[5], 0.0, w[6], w[7], w[8], 0.0, w[9], w[10], w[11], 1.0};
        ol = m4_point(m, o, 1.0);
        dl = m4_point(m, d, 0.0);
        return;
    }
    const double* M = P.insts[k].w2l;
    ol = m4_point(M, o, 1.0);
    dl = m4_point(M, d, 0.0);
}

// Closest hit (SHADOW = false: h, tie) or any hit (SHADOW: returns occluded) of one ray.
// COUNT: the work this walk executes (c.recs = four-wide nodes, c.tris = triangle tests) and its
// per-iteration divergence (inner step / leaf run), as the binary walk's counters.
// FIT: the flattened instance tree of a transformed scene (above): terminal slots are pairs.
//
// (Postponed leaf runs - Aila-Laine speculative traversal: a lane parks its leaf run and keeps
// stepping inner nodes until enough lanes hold one - measured 8,368 -> 6,631..6,941 Mrays/s on C3
// at thresholds of 16..64 lanes, profiles/r06a_ab_c3_postpone.txt: a closest-hit walk that defers
// its leaves keeps its pruning limit high.  Removed; git history keeps it.)
// W: the ray, kept by the caller (TwWorld) or parked (fit walks of the megakernels: the world ray
// is read back at a pair, where its local ray is formed, and not live across the walk).
template <bool COUNT, bool SHADOW, bool FIT = false, class World = TwWorld>
__device__ __forceinline__ bool wide_walk(const RenderParams& P, const World& W, const V3& inv, double tlo,
                                          double tmax, Hit& h, bool& tie, Stack& st, Counts& c) {
    const WRay R = wide_ray(P, W.o(), inv, P.wdelta);
    const double eps = P.eps;
    float lim = SHADOW ? wide_limit(P, tmax) : 3.0e38f;
    const int base = st.sp;
    int ref = FIT ? P.fit_root : P.wide_root;
    bool occ = false;
    const char* wbase = reinterpret_cast<const char*>(P.wnodes);
    const auto* ctris = P.ctris;
    const auto* tris = P.tris;
    // the terminal slot ~x: the leaf run starting at TriRec x, or (FIT) pair x; true = occluded
    // FIT: the instance of the local ray kept in cro/crd (MYRT_FIT_CACHE: 1 = every walk, 2 = closest hit)
    constexpr bool kCache = MYRT_FIT_CACHE == 1 || (MYRT_FIT_CACHE == 2 && !SHADOW);
    int ck = -1;
    V3 cro = v3(0, 0, 0), crd = v3(0, 0, 0);
    auto leaf = [&](const int x) -> bool {
        int t0 = x, k = 0;
        V3 ro, rd;                                         // the ray the triangles are tested with
        if (FIT) {
            const DFitPair pr = P.fpairs[x];
            t0 = pr.t0;
            k = pr.inst;
            if (kCache) {
                if (k != ck) {
                    fit_local(P, k, W.o(), W.d(), cro, crd);
                    ck = k;
                }
                ro = cro;
                rd = crd;
            } else {
                fit_local(P, k, W.o(), W.d(), ro, rd);
            }
        } else {
            ro = W.o();
            rd = W.d();
        }
        int box = 0;                                       // leaf box: 0 unchecked, 1 passes, 2 fails
        auto exact = [&]() {
            return FIT ? fit_boxes_exact(P, k, t0, W.o(), W.d(), ro, rd) : leaf_box_exact(P, t0, ro, rd);
        };
        auto run = [&](const auto* tris) {
            for (int t = t0;; ++t) {
                const auto T = tris[t];                    // by value: `last` arrives with the vertices
                if (COUNT) c.tris++;
                if (SHADOW) {
                    if (tri_shadow(T, ro, rd, 0.0, tmax, eps, P.fast_rcp)) {
                        if (box == 0) box = exact() ? 1 : 2;
                        if (box == 1) return true;
                    }
                } else {
                    double tt, uu, vv;
                    const int r = tri_candidate(T, ro, rd, tlo, eps, h.t, tt, uu, vv, P.fast_rcp);
                    if (r != 0) {
                        if (box == 0) box = exact() ? 1 : 2;
                        if (box == 1) {
                            if (r == 1) {
                                h.t = tt; h.u = uu; h.v = vv; h.tri = t; h.inst = FIT ? k : T.prim;
                                tie = false;
                                lim = wide_limit(P, tt);
                            } else {
                                tie = true;
                            }
                        }
                    }
                }
                if (T.last) break;
            }
            return false;
        };
        return ctris ? run(ctris) : run(tris);
    };
    for (;;) {
        if (COUNT) {
            const bool in = ref >= 0;
            const unsigned long long bi = __ballot(in), bl = __ballot(!in);
            const bool first = (int)(threadIdx.x & 63) == __builtin_ctzll(__ballot(1));
            c.it_wave_inner[SHADOW] += (first && bi) ? 1 : 0;
            c.it_wave_leaf[SHADOW] += (first && bl) ? 1 : 0;
            c.it_lane_inner[SHADOW] += in ? 1 : 0;
            c.it_lane_leaf[SHADOW] += in ? 0 : 1;
            if (SHADOW) c.it_shadow++; else c.it_closest++;
            if (in) c.recs++;
        }
        if (ref >= 0) {
            if (wide_inner(P, wbase, ref, R, lim, st)) continue;
        } else if (leaf(~ref)) {
            occ = true;
            break;
        }
        if (!wide_pop(st, base, lim, ref)) break;
    }
    st.reset(base);
    return occ;
}

// ---- transformed scenes (static instances with transforms, triangles only; scene.cpp
// build_wide_tw).  The reference walks the TLAS with the world ray and, at each TLAS leaf, every
// instance's BLAS with that instance's local ray (RTContext.swift:619-720; the local direction is
// not renormalised, so t is the same in both spaces).  A triangle is tested iff its TLAS leaf box
// passes hitAABB with the world ray and its BLAS leaf box with the local ray (box nesting within
// each tree, wide.h header).  This walk: the TLAS's four-wide nodes in world space (FP32,
// widened by P.wdelta); a marker slot (its TLAS leaf's box) enters the instance with the exact
// FP64 tests of the TLAS leaf box (world ray) and of the BLAS root box (local ray, :567-571) -
// only instances the reference visits are entered - and continues with the BLAS's nodes and the
// local ray, widened per ray by 2^-21 * max(|BLAS coordinate|, |local origin|) (the bound of the
// wide.h header for this ray); candidates are accepted after the exact FP64 test of their leaf
// box (local).  Stack entries above an instance's marker are its BLAS's, so popping a TLAS entry
// (node < tw_tlas_nodes, or a marker) brings the world ray back.  Equal-t candidates (tie) and
// lanes whose local 1/d leaves the FP32 range (redo) are re-walked in the reference's order
// (device.h ut_walk) by the caller.
__device__ __forceinline__ bool tw_is_tlas(const RenderParams& P, int ref) {
    return ref >= 0 ? ref < P.tw_tlas_nodes : ~ref >= P.ut_marker_base;
}
template <bool SHADOW, class World>
__device__ __forceinline__ bool tw_walk(const RenderParams& P, const World& W, double tlo, double tmax,
                                        Hit& h, bool& tie, bool& redo, Stack& st) {
    const double eps = P.eps;
    WRay R;
    {
        const V3 o = W.o(), d = W.d();
        R = wide_ray(P, o, rcp(d), P.wdelta);
    }
    float lim = SHADOW ? wide_limit(P, tmax) : 3.0e38f;
    const int base = st.sp;
    int ref = P.wide_root;
    int inst = -1;
    V3 ol = v3(0, 0, 0), dl = v3(0, 0, 0);             // the local ray (kept when the world ray is parked)
    bool occ = false;
    const char* wbase = reinterpret_cast<const char*>(P.wnodes);
    const auto* ctris = P.ctris;
    const auto* tris = P.tris;
    for (;;) {
        if (ref >= 0) {
            if (wide_inner(P, wbase, ref, R, lim, st)) continue;
        } else if (~ref >= P.ut_marker_base) {
            // enter instance k: the reference's TLAS leaf test (world) and BLAS root test (local)
            const int k = ~ref - P.ut_marker_base;
            const DWideInst& WI = P.winst[k];
            const double limd = (SHADOW ? tmax : h.t) * P.prune_rel + P.prune_abs;
            const V3 o = W.o(), d = W.d();
            const V3 inv = rcp(d);
            double dt;
            if (slab_hit<true>(WI.tbox[0], WI.tbox[1], WI.tbox[2], WI.tbox[3], WI.tbox[4], WI.tbox[5], o, inv, eps, dt) &&
                !(dt > limd)) {
                const DInstance& I = P.insts[k];
                const V3 ol2 = m4_point(I.w2l, o, 1.0), dl2 = m4_point(I.w2l, d, 0.0);
                const V3 il = rcp(dl2);
                if (!wide_ok(il)) { redo = true; break; }
                double dr;
                if (slab_hit<true>(I.root_lo[0], I.root_lo[1], I.root_lo[2], I.root_hi[0], I.root_hi[1], I.root_hi[2],
                                   ol2, il, eps, dr) && !(dr > limd)) {
                    inst = k;
                    if (World::kParked) { ol = ol2; dl = dl2; }
                    const double oc = fmax(fmax(fabs(ol2.x), fabs(ol2.y)), fabs(ol2.z));
                    R = wide_ray(P, ol2, il, 0x1p-21 * (double)P.tw_wscale * fmax(WI.bcoord, oc));
                    ref = WI.wroot;
                    continue;
                }
            }
        } else {
            const int t0 = ~ref;                          // a BLAS leaf run of instance `inst`
            int box = 0;                                   // leaf box: 0 unchecked, 1 passes, 2 fails
            // the local ray: kept (parked world ray), or recomputed with the marker's arithmetic
            // rather than kept live beside the world ray across the walk
            if (!World::kParked) {
                const DInstance& I = P.insts[inst];
                ol = m4_point(I.w2l, W.o(), 1.0);
                dl = m4_point(I.w2l, W.d(), 0.0);
            }
            auto leaf_ok = [&]() {
                const double* b = P.lbox + 6 * (size_t)t0;
                double tm;
                return slab_hit<true>(b[0], b[1], b[2], b[3], b[4], b[5], ol, rcp(dl), eps, tm);
            };
            auto run = [&](const auto* tris) {
                for (int t = t0;; ++t) {
                    const auto T = tris[t];
                    if (SHADOW) {
                        if (tri_shadow(T, ol, dl, 0.0, tmax, eps, P.fast_rcp)) {
                            if (box == 0) box = leaf_ok() ? 1 : 2;
                            if (box == 1) return true;
                        }
                    } else {
                        double tt, uu, vv;
                        const int r = tri_candidate(T, ol, dl, tlo, eps, h.t, tt, uu, vv, P.fast_rcp);
                        if (r != 0) {
                            if (box == 0) box = leaf_ok() ? 1 : 2;
                            if (box == 1) {
                                if (r == 1) {
                                    h.t = tt; h.u = uu; h.v = vv; h.tri = t; h.inst = inst;
                                    tie = false;
                                    lim = wide_limit(P, tt);
                                } else {
                                    tie = true;
                                }
                            }
                        }
                    }
                    if (T.last) break;
                }
                return false;
            };
            if (ctris ? run(ctris) : run(tris)) { occ = true; break; }
        }
        if (!wide_pop(st, base, lim, ref)) break;
        if (inst >= 0 && tw_is_tlas(P, ref)) {            // back to the world ray
            inst = -1;
            const V3 o = W.o(), d = W.d();
            R = wide_ray(P, o, rcp(d), P.wdelta);
        }
    }
    st.reset(base);
    return occ;
}

}  // namespace dev
}  // namespace myrt
