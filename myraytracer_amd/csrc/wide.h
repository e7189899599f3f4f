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

struct WRay {
    float ix, iy, iz;     // 1/d in FP32
    float lx, ly, lz;     // -(o/d) - wdelta/d: offset of the lo planes
    float hx, hy, hz;     // -(o/d) + wdelta/d: offset of the hi planes
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
    const double dx = P.wdelta * inv.x, dy = P.wdelta * inv.y, dz = P.wdelta * inv.z;
    r.lx = (float)(-ox - dx); r.ly = (float)(-oy - dy); r.lz = (float)(-oz - dz);
    r.hx = (float)(-ox + dx); r.hy = (float)(-oy + dy); r.hz = (float)(-oz + dz);
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
template <bool SHADOW>
__device__ __forceinline__ bool wide_inner(const RenderParams& P, int& ref, const WRay& R, float lim, Stack& st) {
    const W4Node N = P.wnodes[ref];
    float a[4];
    bool h[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const float tlx = __builtin_fmaf(N.lo[0][c], R.ix, R.lx), thx = __builtin_fmaf(N.hi[0][c], R.ix, R.hx);
        const float tly = __builtin_fmaf(N.lo[1][c], R.iy, R.ly), thy = __builtin_fmaf(N.hi[1][c], R.iy, R.hy);
        const float tlz = __builtin_fmaf(N.lo[2][c], R.iz, R.lz), thz = __builtin_fmaf(N.hi[2][c], R.iz, R.hz);
        const float tn = __builtin_fmaxf(__builtin_fmaxf(__builtin_fminf(tlx, thx), __builtin_fminf(tly, thy)),
                                         __builtin_fminf(tlz, thz));
        const float tf = __builtin_fminf(__builtin_fminf(__builtin_fmaxf(tlx, thx), __builtin_fmaxf(tly, thy)),
                                         __builtin_fmaxf(tlz, thz));
        a[c] = tn;
        h[c] = __builtin_fmaxf(tn, P.weps) <= __builtin_fminf(tf, lim);
    }
    int n;          // the slot the walk continues with
    int nref;
    if (SHADOW) {
        n = h[0] ? 0 : h[1] ? 1 : h[2] ? 2 : 3;
        nref = h[0] ? N.ref[0] : h[1] ? N.ref[1] : h[2] ? N.ref[2] : N.ref[3];
    } else {
        const float k0 = h[0] ? a[0] : __builtin_inff(), k1 = h[1] ? a[1] : __builtin_inff();
        const float k2 = h[2] ? a[2] : __builtin_inff(), k3 = h[3] ? a[3] : __builtin_inff();
        const bool p = k1 < k0, q = k3 < k2;
        const float m01 = p ? k1 : k0, m23 = q ? k3 : k2;
        const int r01 = p ? N.ref[1] : N.ref[0], r23 = q ? N.ref[3] : N.ref[2];
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
            st.lds[p * Stack::stride] = wide_entry(N.ref[c], a[c]);
            p += keep[c] ? 1 : 0;
        }
        st.sp = p;
    } else {
#pragma unroll
        for (int c = 3; c >= 0; --c) st.push_raw_if(keep[c], wide_entry(N.ref[c], a[c]));
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
template <bool SHADOW>
__device__ __forceinline__ bool wide_walk(const RenderParams& P, const V3& o, const V3& d, const V3& inv, double tlo,
                                          double tmax, Hit& h, bool& tie, Stack& st) {
    const WRay R = wide_ray(P, o, inv);
    const double eps = P.eps;
    float lim = SHADOW ? wide_limit(P, tmax) : 3.0e38f;
    const int base = st.sp;
    int ref = P.wide_root;
    bool occ = false;
    for (;;) {
        if (ref >= 0) {
            if (wide_inner<SHADOW>(P, ref, R, lim, st)) continue;
        } else {
            const int t0 = ~ref;
            int box = 0;                                   // leaf box: 0 unchecked, 1 passes, 2 fails
            auto run = [&](const auto* tris) {
                for (int t = t0;; ++t) {
                    const auto T = tris[t];                // by value: `last` arrives with the vertices
                    if (SHADOW) {
                        if (tri_shadow(T, o, d, 0.0, tmax, eps, P.fast_rcp)) {
                            if (box == 0) box = leaf_box_exact(P, t0, o, d) ? 1 : 2;
                            if (box == 1) return true;
                        }
                    } else {
                        double tt, uu, vv;
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
            if (P.ctris ? run(P.ctris) : run(P.tris)) { occ = true; break; }
        }
        if (!wide_pop(st, base, lim, ref)) break;
    }
    st.reset(base);
    return occ;
}

}  // namespace dev
}  // namespace myrt
