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

// The ray in the walk's FP32 form.  Per axis the near plane of every box is lo when 1/d >= 0 and
// hi otherwise: the walk reads each slot's near and far planes directly (a per-lane byte offset
// into the node, nx/ny/nz) instead of taking min/max of both plane distances - the same values
// (FMA is monotone, and the lo-plane offset is below the hi-plane one), 24 VALU fewer per node.
struct WRay {
    float ix, iy, iz;     // 1/d in FP32
    float nox, noy, noz;  // offset of the near planes: -(o/d) - wdelta*|1/d|
    float fox, foy, foz;  // offset of the far planes:  -(o/d) + wdelta*|1/d|
    unsigned nx, ny, nz;  // byte offset of the near-plane row of axis a in a W4Node (lo or hi)
    bool uoct;            // every lane of the wave has this direction octant (wave-uniform)
};

// every |1/d| within [2^-100, 2^100] (finite; FP32 products of scene coordinates stay finite)
__device__ __forceinline__ bool wide_ok(const V3& inv) {
    const double ax = fabs(inv.x), ay = fabs(inv.y), az = fabs(inv.z);
    return ax <= 0x1p100 && ax >= 0x1p-100 && ay <= 0x1p100 && ay >= 0x1p-100 && az <= 0x1p100 && az >= 0x1p-100;
}

__device__ __forceinline__ WRay wide_ray(const RenderParams& P, const V3& o, const V3& inv) {
    WRay r;
    r.ix = (float)inv.x; r.iy = (float)inv.y; r.iz = (float)inv.z;
    const double ox = o.x * inv.x, oy = o.y * inv.y, oz = o.z * inv.z;
    const double dx = P.wdelta * fabs(inv.x), dy = P.wdelta * fabs(inv.y), dz = P.wdelta * fabs(inv.z);
    r.nox = (float)(-ox - dx); r.noy = (float)(-oy - dy); r.noz = (float)(-oz - dz);
    r.fox = (float)(-ox + dx); r.foy = (float)(-oy + dy); r.foz = (float)(-oz + dz);
    constexpr unsigned kHi = offsetof(W4Node, hi);        // 64: hi row a = lo row a + 64 B
    r.nx = (inv.x >= 0 ? 0u : kHi) + 0u * 16u;
    r.ny = (inv.y >= 0 ? 0u : kHi) + 1u * 16u;
    r.nz = (inv.z >= 0 ? 0u : kHi) + 2u * 16u;
    const unsigned oct = r.nx | (r.ny << 8) | (r.nz << 16);
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

// One four-wide node: the slots whose widened box the ray enters within [weps, lim].  Closest
// hit: continue with the nearest entry, the others are pushed; any hit: continue with the first
// slot hit (the reference's occludedBLAS takes L first, RTContext.swift:823-825).  Returns false
// when no slot is hit (the caller pops).
#ifndef MYRT_MT_TWICE
#define MYRT_MT_TWICE 0
#endif
typedef float wf4 __attribute__((ext_vector_type(4)));
typedef int wi4 __attribute__((ext_vector_type(4)));
#ifndef MYRT_WIDE_SCALAR
#define MYRT_WIDE_SCALAR 1
#endif
template <bool SHADOW>
__device__ __forceinline__ bool wide_node(const RenderParams& P, int& ref, const WRay& R, float lim, Stack& st,
                                          const wf4& nx, const wf4& fx, const wf4& ny, const wf4& fy, const wf4& nz,
                                          const wf4& fz, const wi4& refs);
template <bool SHADOW>
__device__ __forceinline__ bool wide_inner(const RenderParams& P, const char* base, int& ref, const WRay& R, float lim,
                                           Stack& st) {
    // near / far plane rows of this lane's direction octant (the far row of axis a is the other of
    // lo[a] / hi[a], 64 B away: offset n ^ 64); base = P.wnodes
    constexpr unsigned kHi = offsetof(W4Node, hi);
    if (MYRT_WIDE_SCALAR && R.uoct) {
        // Every lane at the same node with the same octant (the top of the tree for a tile's
        // coherent rays): the rows come through the scalar cache into SGPRs once for the wave,
        // instead of 64 copies through the vector-memory data path (TD, ~0.87 busy).
        const int r0 = __builtin_amdgcn_readfirstlane(ref);
        if (__all(ref == r0)) {
            const unsigned long long av = (unsigned long long)(base + (size_t)r0 * sizeof(W4Node));
            const unsigned alo = __builtin_amdgcn_readfirstlane((unsigned)av);
            const unsigned ahi = __builtin_amdgcn_readfirstlane((unsigned)(av >> 32));
            typedef const __attribute__((address_space(4))) char c4_char;
            c4_char* sb = (c4_char*)((unsigned long long)alo | ((unsigned long long)ahi << 32));
            typedef const __attribute__((address_space(4))) wf4 c4_f4;
            typedef const __attribute__((address_space(4))) wi4 c4_i4;
            const unsigned ox = __builtin_amdgcn_readfirstlane(R.nx), oy = __builtin_amdgcn_readfirstlane(R.ny),
                           oz = __builtin_amdgcn_readfirstlane(R.nz);
            const wf4 nx = *(c4_f4*)(sb + ox), fx = *(c4_f4*)(sb + (ox ^ kHi));
            const wf4 ny = *(c4_f4*)(sb + oy), fy = *(c4_f4*)(sb + (oy ^ kHi));
            const wf4 nz = *(c4_f4*)(sb + oz), fz = *(c4_f4*)(sb + (oz ^ kHi));
            const wi4 refs = *(c4_i4*)(sb + offsetof(W4Node, ref));
            return wide_node<SHADOW>(P, ref, R, lim, st, nx, fx, ny, fy, nz, fz, refs);
        }
    }
    // 32-bit byte offsets from the array base (the host keeps the node array below 4 GB): the loads
    // take the SGPR-base + VGPR-offset form instead of a 64-bit address add per row
    const unsigned nb = (unsigned)ref * (unsigned)sizeof(W4Node);
    auto row = [&](unsigned off) { return *reinterpret_cast<const wf4*>(base + (size_t)(nb + off)); };
    const wf4 nx = row(R.nx), fx = row(R.nx ^ kHi);
    const wf4 ny = row(R.ny), fy = row(R.ny ^ kHi);
    const wf4 nz = row(R.nz), fz = row(R.nz ^ kHi);
    const wi4 refs = *reinterpret_cast<const wi4*>(base + (size_t)(nb + (unsigned)offsetof(W4Node, ref)));
    return wide_node<SHADOW>(P, ref, R, lim, st, nx, fx, ny, fy, nz, fz, refs);
}

// The slab tests of one node's four slots and the stack update (wide_inner).
template <bool SHADOW>
__device__ __forceinline__ bool wide_node(const RenderParams& P, int& ref, const WRay& R, float lim, Stack& st,
                                          const wf4& nx, const wf4& fx, const wf4& ny, const wf4& fy, const wf4& nz,
                                          const wf4& fz, const wi4& refs) {
    const int nr[4] = {refs.x, refs.y, refs.z, refs.w};
    float a[4];
    bool h[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const float tn = __builtin_fmaxf(__builtin_fmaxf(__builtin_fmaf(nx[c], R.ix, R.nox), __builtin_fmaf(ny[c], R.iy, R.noy)),
                                         __builtin_fmaf(nz[c], R.iz, R.noz));
        const float tf = __builtin_fminf(__builtin_fminf(__builtin_fmaf(fx[c], R.ix, R.fox), __builtin_fmaf(fy[c], R.iy, R.foy)),
                                         __builtin_fmaf(fz[c], R.iz, R.foz));
        a[c] = tn;
        h[c] = __builtin_fmaxf(tn, P.weps) <= __builtin_fminf(tf, lim);
    }
#ifndef MYRT_WIDE_SORT
#define MYRT_WIDE_SORT 1
#endif
    if ((!SHADOW && MYRT_WIDE_SORT) || (SHADOW && MYRT_WIDE_SORT >= 2)) {
        // closest hit (and, at MYRT_WIDE_SORT 2, any hit), full front-to-back order: sort the four
        // (entry, ref) pairs (5 compare-exchanges), continue with the nearest, push the others far
        // to near
        float k[4];
        int r[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) { k[c] = h[c] ? a[c] : __builtin_inff(); r[c] = nr[c]; }
        auto ce = [&](int i, int j) {
            const bool sw = k[j] < k[i];
            const float ki = sw ? k[j] : k[i], kj = sw ? k[i] : k[j];
            const int ri = sw ? r[j] : r[i], rj = sw ? r[i] : r[j];
            k[i] = ki; k[j] = kj; r[i] = ri; r[j] = rj;
        };
        ce(0, 1); ce(2, 3); ce(0, 2); ce(1, 3); ce(1, 2);
        if (!__any(st.sp > kLds - 4)) {
            int p = st.sp;
#pragma unroll
            for (int c = 3; c >= 1; --c) {
                st.lds[p * Stack::stride] = wide_entry(r[c], k[c]);
                p += k[c] < __builtin_inff() ? 1 : 0;
            }
            st.sp = p;
        } else {
#pragma unroll
            for (int c = 3; c >= 1; --c) st.push_raw_if(k[c] < __builtin_inff(), wide_entry(r[c], k[c]));
        }
        ref = r[0];
        return k[0] < __builtin_inff();
    }
    int n;          // the slot the walk continues with
    int nref;
    if (SHADOW) {
        n = h[0] ? 0 : h[1] ? 1 : h[2] ? 2 : 3;
        nref = h[0] ? nr[0] : h[1] ? nr[1] : h[2] ? nr[2] : nr[3];
    } else {
        const float k0 = h[0] ? a[0] : __builtin_inff(), k1 = h[1] ? a[1] : __builtin_inff();
        const float k2 = h[2] ? a[2] : __builtin_inff(), k3 = h[3] ? a[3] : __builtin_inff();
        const bool p = k1 < k0, q = k3 < k2;
        const float m01 = p ? k1 : k0, m23 = q ? k3 : k2;
        const int r01 = p ? nr[1] : nr[0], r23 = q ? nr[3] : nr[2];
        const bool z = m23 < m01;
        nref = z ? r23 : r01;
        n = z ? (q ? 3 : 2) : (p ? 1 : 0);
    }
    // the others, last slot first (they pop in slot order)
    bool keep[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) keep[c] = h[c] && c != n;
    if (!__any(st.sp > kLds - 4)) {
        // every lane's four candidate slots lie in LDS: unconditional stores at running positions
        // (a dropped entry is overwritten by the next kept one, or lies above the new top)
        int p = st.sp;
#pragma unroll
        for (int c = 3; c >= 0; --c) {
            st.lds[p * Stack::stride] = wide_entry(nr[c], a[c]);
            p += keep[c] ? 1 : 0;
        }
        st.sp = p;
    } else {
#pragma unroll
        for (int c = 3; c >= 0; --c) st.push_raw_if(keep[c], wide_entry(nr[c], a[c]));
    }
    ref = nref;
    return h[0] || h[1] || h[2] || h[3];
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

// Closest hit (SHADOW = false: h, tie) or any hit (SHADOW: returns occluded) of one ray.
// COUNT: the work this walk executes (c.recs = four-wide nodes, c.tris = triangle tests) and its
// per-iteration divergence (inner step / leaf run), as the binary walk's counters.
template <bool COUNT, bool SHADOW>
__device__ __forceinline__ bool wide_walk(const RenderParams& P, const V3& o, const V3& d, const V3& inv, double tlo,
                                          double tmax, Hit& h, bool& tie, Stack& st, Counts& c) {
    const WRay R = wide_ray(P, o, inv);
    const double eps = P.eps;
    float lim = SHADOW ? wide_limit(P, tmax) : 3.0e38f;
    const int base = st.sp;
    int ref = P.wide_root;
    bool occ = false;
    const char* wbase = reinterpret_cast<const char*>(P.wnodes);
    const auto* ctris = P.ctris;
    const auto* tris = P.tris;
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
            if (wide_inner<SHADOW>(P, wbase, ref, R, lim, st)) continue;
        } else {
            const int t0 = ~ref;
            int box = 0;                                   // leaf box: 0 unchecked, 1 passes, 2 fails
            auto run = [&](const auto* tris) {
                for (int t = t0;; ++t) {
                    const auto T = tris[t];                // by value: `last` arrives with the vertices
                    if (COUNT) c.tris++;
                    if (SHADOW) {
#if MYRT_MT_TWICE   // measurement variant: every triangle test runs twice (the difference prices the tests)
                        {
                            V3 o2 = o;
                            asm volatile("" : "+v"(o2.x));
                            if (tri_shadow(T, o2, d, 0.0, tmax, eps, P.fast_rcp)) asm volatile("" ::: "memory");
                        }
#endif
                        if (tri_shadow(T, o, d, 0.0, tmax, eps, P.fast_rcp)) {
                            if (box == 0) box = leaf_box_exact(P, t0, o, d) ? 1 : 2;
                            if (box == 1) return true;
                        }
                    } else {
                        double tt, uu, vv;
#if MYRT_MT_TWICE
                        {
                            V3 o2 = o;
                            asm volatile("" : "+v"(o2.x));
                            double t2, u2, v2;
                            if (tri_candidate(T, o2, d, tlo, eps, h.t, t2, u2, v2, P.fast_rcp)) asm volatile("" ::: "memory");
                        }
#endif
                        const int r = tri_candidate(T, o, d, tlo, eps, h.t, tt, uu, vv, P.fast_rcp);
                        if (r != 0) {
                            if (box == 0) box = leaf_box_exact(P, t0, o, d) ? 1 : 2;
                            if (box == 1) {
                                if (r == 1) {
                                    h.t = tt; h.u = uu; h.v = vv; h.tri = t; h.inst = T.prim;
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
    }
    st.reset(base);
    return occ;
}

}  // namespace dev
}  // namespace myrt
