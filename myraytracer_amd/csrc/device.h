// device.h — device-side building blocks of the render kernels (render.hip, render_full.h).
// IEEE binary64 throughout; every function
// restates a reference routine (file:line cited) in the same operation order.
#pragma once
#include <hip/hip_runtime.h>

#include "layout.h"

namespace myrt {
namespace dev {


#define DINF __builtin_huge_val()

struct V3 { double x, y, z; };
__device__ __forceinline__ V3 v3(double x, double y, double z) { return V3{x, y, z}; }
__device__ __forceinline__ V3 ld3(const double* p) { return V3{p[0], p[1], p[2]}; }
__device__ __forceinline__ V3 operator+(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ V3 operator-(V3 a) { return {-a.x, -a.y, -a.z}; }
__device__ __forceinline__ V3 operator*(V3 a, V3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
__device__ __forceinline__ V3 operator/(V3 a, V3 b) { return {a.x / b.x, a.y / b.y, a.z / b.z}; }
__device__ __forceinline__ V3 operator*(V3 a, double s) { return {a.x * s, a.y * s, a.z * s}; }
__device__ __forceinline__ V3 operator*(double s, V3 a) { return {s * a.x, s * a.y, s * a.z}; }
__device__ __forceinline__ V3 operator/(V3 a, double s) { return {a.x / s, a.y / s, a.z / s}; }
__device__ __forceinline__ V3 operator+(double s, V3 a) { return {s + a.x, s + a.y, s + a.z}; }
__device__ __forceinline__ V3 operator-(V3 a, double s) { return {a.x - s, a.y - s, a.z - s}; }
__device__ __forceinline__ V3 operator+(V3 a, double s) { return {a.x + s, a.y + s, a.z + s}; }
__device__ __forceinline__ V3 rcp(V3 a) { return {1.0 / a.x, 1.0 / a.y, 1.0 / a.z}; }
__device__ __forceinline__ double dot(V3 a, V3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
__device__ __forceinline__ V3 cross(V3 a, V3 b) {
    return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
__device__ __forceinline__ double dsqrt(double x) { return __builtin_sqrt(x); }
__device__ __forceinline__ V3 normalize(V3 v) { double r = 1.0 / dsqrt(dot(v, v)); return v * r; }
__device__ __forceinline__ double length(V3 v) { return dsqrt(dot(v, v)); }
__device__ __forceinline__ double smax(double x, double y) { return (y >= x) ? y : x; }   // Swift.max
__device__ __forceinline__ double smin(double x, double y) { return (y < x) ? y : x; }    // Swift.min
__device__ __forceinline__ bool isfin(V3 v) {
    return __builtin_isfinite(v.x) && __builtin_isfinite(v.y) && __builtin_isfinite(v.z);
}
// simd_mul(double4x4, double4) without FMA: ((c0*x + c1*y) + c2*z) + c3*w
__device__ __forceinline__ V3 m4_point(const double* M, V3 v, double w) {
    double o[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        double acc = M[0 * 4 + r] * v.x;
        acc = M[1 * 4 + r] * v.y + acc;
        acc = M[2 * 4 + r] * v.z + acc;
        acc = M[3 * 4 + r] * w + acc;
        o[r] = acc;
    }
    return {o[0], o[1], o[2]};
}
__device__ __forceinline__ V3 m3_mul(const double* M, V3 v) {
    double o[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        double acc = M[0 * 3 + r] * v.x;
        acc = M[1 * 3 + r] * v.y + acc;
        acc = M[2 * 3 + r] * v.z + acc;
        o[r] = acc;
    }
    return {o[0], o[1], o[2]};
}

// hitAABB (RTContext.swift:557-565): simd.min/max = fmin/fmax, scalar max/min = Swift's
__device__ __forceinline__ double slab(double lx, double ly, double lz, double hx, double hy, double hz,
                                       const V3& o, const V3& inv, double eps) {
    const double t1x = (lx - o.x) * inv.x, t1y = (ly - o.y) * inv.y, t1z = (lz - o.z) * inv.z;
    const double t2x = (hx - o.x) * inv.x, t2y = (hy - o.y) * inv.y, t2z = (hz - o.z) * inv.z;
    const double mnx = fmin(t1x, t2x), mny = fmin(t1y, t2y), mnz = fmin(t1z, t2z);
    const double mxx = fmax(t1x, t2x), mxy = fmax(t1y, t2y), mxz = fmax(t1z, t2z);
    const double tmin = smax(smax(mnx, mny), mnz);
    const double tmax = smin(mxx, smin(mxy, mxz));
    return (tmax >= smax(tmin, eps)) ? tmin : DINF;
}

// PCG32 (Object+Extension.swift:556-589)
struct PCG32 {
    unsigned long long state, inc;
    PCG32() = default;
    // a stream resumed at `state` (PCG32(seed) sets inc = seed << 1 | 1)
    __device__ static PCG32 resume(unsigned long long state, unsigned long long seed) {
        PCG32 r;
        r.state = state;
        r.inc = (seed << 1) | 1ull;
        return r;
    }
    __device__ explicit PCG32(unsigned long long seed) {
        state = 0ull; inc = (seed << 1) | 1ull;
        (void)next();
        state += 0x9E3779B97F4A7C15ull;
        (void)next();
    }
    __device__ __forceinline__ unsigned next() {
        const unsigned long long old = state;
        state = old * 6364136223846793005ull + inc;
        const unsigned xs = (unsigned)(((old >> 18) ^ old) >> 27);
        const unsigned rot = (unsigned)(old >> 59);
        return (xs >> rot) | (xs << ((~rot + 1u) & 31u));
    }
    __device__ __forceinline__ double nextFloat() { return (double)next() * 2.3283064365386963e-10; }
};

// XCD-aware tile order.  Workgroups are dealt to the 8 XCDs round-robin by linear id
// and each XCD has its own 4 MB L2.  Identity order gives XCD x every 8th tile; with
// group size G > 1 XCD x gets runs of G consecutive tiles instead (tile groups dealt
// round-robin), so neighbouring tiles - which walk the same BVH nodes - share one L2,
// while every XCD still samples the whole image (whole-band splits are badly
// imbalanced: sky rows cost a fraction of terrain rows).  Bijective on [0, nb): the
// tail beyond the last full 8*G round keeps identity order.
// Output row of chunk `chunk`, row `r` (RenderParams::out_first / out_step).
__device__ __forceinline__ size_t out_row_of(const RenderParams& P, int chunk, int r) {
    return (size_t)((chunk - P.out_first) / P.out_step) * 8 + (size_t)r;
}

__device__ __forceinline__ int xcd_tile(int b, int nb, int G) {
    if (G <= 1) return b;
    const int round = 8 * G, full = nb / round * round;
    if (b >= full) return b;
    const int x = b & 7, k = b >> 3;
    return ((k / G) * 8 + x) * G + (k % G);
}

// ----------------------------------------------------------------- traversal stack
// Per-lane stack: the first kLds entries live in LDS ([slot][lane], so each lane hits its
// own bank), deeper entries spill to a private (scratch) array that lives OUTSIDE the
// struct: with a dynamically indexed array inside, the whole struct - `sp` included -
// was demoted to scratch and every push stored `sp` to memory.
// Pointers carry their address space explicitly: a plain pointer is generic and every
// push/pop compiled to flat_* on the vector-memory path instead of ds_* / scratch_*.
// An entry packs {ref (low 32), high 32 bits of the entry distance (high 32)}: dropping
// the low mantissa word truncates toward zero, i.e. rounds a positive distance DOWN, so
// pop-time culling stays conservative (negative distances are never culled).
// LDS entries per lane: 16 in round 4 (the sorted four-wide walk pushed up to three entries per
// node; C3 +1.2 %, C5 +1.6 % over 8, profiles/r04g_*); 10 since round 5 - with the octant-ordered
// walk C3 is the same at 10, 12 and 16 (8,605 / 8,604 / 8,611 Mrays/s, profiles/r05l_ab_c3.txt,
// r05m_ab_c3.txt) - so the megakernel's 10 stack entries + 4 pixel slots + 6 world-ray park slots
// (render.hip TwParkedLds) are 10 KB per wave: the 16 waves of a CU at 4 waves/SIMD fill its 160 KB.
#ifndef MYRT_KLDS
#define MYRT_KLDS 10
#endif
constexpr int kLds = MYRT_KLDS;
constexpr int kSpill = kStackCap - kLds;   // the host refuses deeper scenes (scene.cpp, RT_ERR_STACK)
static_assert(kSpill > 0, "LDS part larger than the stack");
typedef __attribute__((address_space(3))) unsigned long long lds_u64;
typedef __attribute__((address_space(5))) unsigned long long priv_u64;
struct Stack {
    lds_u64* lds;        // this lane's column of the wave's [kLds][64] LDS slab
    priv_u64* spill;     // kSpill private entries
    // per-wave slab with a constant stride of 64: a slot address is a shift, not a multiply
    // by blockDim.x (C3/C5 -1 %)
    static constexpr int stride = 64;
    int sp;
    // uni_spill (MYRT_UNIFORM_SPILL): test once per wave whether any lane is past the LDS
    // part; when none is (nearly always), the push/pop is a plain LDS access with no per-lane
    // exec masking around the private-memory branch.  A compile-time constant per kernel
    // (everything here is inlined): on in the primary-ray megakernel (C3 -0.9 %), off where
    // it raised register spills (bounce megakernel: C5 +2 %)
#ifndef MYRT_UNIFORM_SPILL
#define MYRT_UNIFORM_SPILL 1
#endif
    bool uni_spill;
    __device__ __forceinline__ bool lds_only() const { return MYRT_UNIFORM_SPILL && uni_spill && !__any(sp >= kLds); }
    __device__ __forceinline__ static unsigned long long pack(int ref, double t) {
        return (unsigned long long)(unsigned)ref | ((unsigned long long)(unsigned)__double2hiint(t) << 32);
    }
    __device__ __forceinline__ void push(int ref, double t) {
        const unsigned long long e = pack(ref, t);
        if (lds_only()) {
            lds[sp * stride] = e;
        } else if (sp < kLds) {
            lds[sp * stride] = e;
        } else {
            asm volatile("" ::: "memory");   // keep the two stores apart (no select-of-pointers)
            spill[sp - kLds] = e;
        }
        ++sp;
    }
    // push when `keep`; the LDS store is issued regardless (slot sp is free), only the
    // rare spill store is conditional
    __device__ __forceinline__ void push_if(bool keep, int ref, double t) {
        const unsigned long long e = pack(ref, t);
        if (lds_only()) {
            lds[sp * stride] = e;
        } else if (sp < kLds) {
            lds[sp * stride] = e;
        } else if (keep) {
            asm volatile("" ::: "memory");
            spill[sp - kLds] = e;
        }
        sp += keep ? 1 : 0;
    }
    // returns the ref; `tlo` = lower bound of the entry distance
    __device__ __forceinline__ int pop(double& tlo) {
        --sp;
        unsigned long long e;
        if (lds_only()) {
            e = lds[sp * stride];
        } else {
            e = lds[min(sp, kLds - 1) * stride];   // unconditional ds_read
            if (sp >= kLds) {
                asm volatile("" ::: "memory");
                e = spill[sp - kLds];
            }
        }
        tlo = __hiloint2double((int)(unsigned)(e >> 32), 0);
        return (int)(unsigned)(e & 0xffffffffull);
    }
    // raw 64-bit entries (wide.h packs {ref, float entry distance})
    __device__ __forceinline__ void push_raw_if(bool keep, unsigned long long e) {
        if (lds_only()) {
            lds[sp * stride] = e;
        } else if (sp < kLds) {
            lds[sp * stride] = e;
        } else if (keep) {
            asm volatile("" ::: "memory");
            spill[sp - kLds] = e;
        }
        sp += keep ? 1 : 0;
    }
    __device__ __forceinline__ unsigned long long pop_raw() {
        --sp;
        unsigned long long e;
        if (lds_only()) {
            e = lds[sp * stride];
        } else {
            e = lds[min(sp, kLds - 1) * stride];
            if (sp >= kLds) {
                asm volatile("" ::: "memory");
                e = spill[sp - kLds];
            }
        }
        return e;
    }
    // drop every entry above `base`
    __device__ __forceinline__ void reset(int base) { sp = base; }
};
#define MYRT_STACK(name, lds_base)                                   \
    unsigned long long name##_spill_mem[kSpill];                     \
    Stack name;                                                      \
    name.lds = (lds_u64*)((lds_base) + (threadIdx.x >> 6) * (kLds * 64) + (threadIdx.x & 63)); \
    name.spill = (priv_u64*)(name##_spill_mem);                      \
    name.uni_spill = false;                                          \
    name.sp = 0

// Work counters (COUNT instantiations only).  recs/tris/normals/insts = work this kernel
// executed.  With RenderParams::count_ref set, the COUNT walk instead follows the
// reference's traversal exactly - no t-pruning, any-hit walks L before R - and `nodes` /
// `smooth` tally its N_nodeFetch / N_smoothHit as SURVEY.md §8(d) defines them (the
// oracle's Counters, oracle/rt_oracle.cpp intersectBLAS/occludedBLAS).
struct Counts {
    unsigned shadow, secondary;
    unsigned long long recs, tris, normals, insts, nodes, smooth;
    unsigned long long it_closest, it_shadow;   // loop iterations of this lane (divergence study)
    unsigned shadow_traced;                     // shadow rays whose any-hit walk ran (<= shadow)
    unsigned long long div_lanes, div_distinct; // per-lane inner steps / of them, first lane of its record
    // per walk iteration ([0] closest, [1] any-hit): waves whose lanes took an inner step /
    // a leaf run / the scalar-cache inner step, and lanes that took an inner step / a leaf
    unsigned long long it_wave_inner[2], it_wave_leaf[2], it_wave_scalar[2], it_lane_inner[2], it_lane_leaf[2];
    unsigned ties;                              // wide walks re-walked in reference order (equal-t hits)
};
constexpr int kMissRef = 0x7fffffff;   // count_ref any-hit: a pushed child whose slab test missed

// reference-order counting requested (a runtime flag read only by COUNT instantiations)
#define MYRT_REF(P) (COUNT && (P).count_ref)
#ifndef MYRT_WAVE_TIMES
#define MYRT_WAVE_TIMES 0    // per-wave timeline for rt_debug_wave_times (debug builds only: costs SGPRs)
#endif

struct Hit { double t, u, v; int tri, inst; };

// Slab test with an explicit hit flag.  FAST = the ray has no zero direction component
// (every 1/d finite), so no slab value can be NaN: then simd.min/max (minNum/maxNum)
// and Swift.max/min agree on every comparison the caller makes (they can differ only in
// the sign of a zero, which no comparison sees), and the scalar reductions become
// v_max_f64 / v_min_f64 instead of compare+select pairs.  Otherwise the literal
// NaN-asymmetric forms of hitAABB (RTContext.swift:557-565) are used.
template <bool FAST>
__device__ __forceinline__ bool slab_hit(double lx, double ly, double lz, double hx, double hy, double hz,
                                         const V3& o, const V3& inv, double eps, double& tmin_out) {
    const double t1x = (lx - o.x) * inv.x, t1y = (ly - o.y) * inv.y, t1z = (lz - o.z) * inv.z;
    const double t2x = (hx - o.x) * inv.x, t2y = (hy - o.y) * inv.y, t2z = (hz - o.z) * inv.z;
    const double mnx = fmin(t1x, t2x), mny = fmin(t1y, t2y), mnz = fmin(t1z, t2z);
    const double mxx = fmax(t1x, t2x), mxy = fmax(t1y, t2y), mxz = fmax(t1z, t2z);
    double tmin, tmax;
    bool hit;
    if (FAST) {
        tmin = fmax(fmax(mnx, mny), mnz);
        tmax = fmin(mxx, fmin(mxy, mxz));
        // no NaN here, so tmax >= max(tmin, eps) <=> tmax >= tmin && tmax >= eps (two compares)
        hit = tmax >= tmin && tmax >= eps;
    } else {
        tmin = smax(smax(mnx, mny), mnz);
        tmax = smin(mxx, smin(mxy, mxz));
        hit = tmax >= smax(tmin, eps);
    }
    tmin_out = tmin;
    return hit;
}
__device__ __forceinline__ bool finite3(const V3& a) {
    return __builtin_isfinite(a.x) && __builtin_isfinite(a.y) && __builtin_isfinite(a.z);
}

// Triangle geometry from either record format (layout.h TriRec / CTri).
__device__ __forceinline__ void tri_geom(const TriRec& T, V3& v0, V3& e1, V3& e2) {
    v0 = ld3(T.v0); e1 = ld3(T.e1); e2 = ld3(T.e2);
}
__device__ __forceinline__ void tri_geom(const CTri& T, V3& v0, V3& e1, V3& e2) {
    v0 = v3((double)T.v0[0], (double)T.v0[1], (double)T.v0[2]);
    e1 = v3((double)T.v1[0], (double)T.v1[1], (double)T.v1[2]) - v0;   // = host e1 = v1 - v0
    e2 = v3((double)T.v2[0], (double)T.v2[1], (double)T.v2[2]) - v0;
}

// 1/x correctly rounded, for x with 2^-700 <= |x| <= 2^1000 (RenderParams::fast_rcp: the host
// proves every Moeller-Trumbore determinant of the scene lies there, scene.cpp det bound).
// This is the compiler's IEEE division sequence for 1.0/x without its range steps: in that
// range v_div_scale leaves both operands unscaled (and clears VCC, so v_div_fmas is a plain
// FMA), 1.0*r is exact, and v_div_fixup only re-applies the sign the FMA result already has.
// Bit-identical to 1.0/x there, in 7 instead of 11 instructions.
__device__ __forceinline__ double rcp_rn(double x) {
    double r = __builtin_amdgcn_rcp(x);
    double e = __builtin_fma(-x, r, 1.0);
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-x, r, 1.0);
    r = __builtin_fma(r, e, r);
    const double rem = __builtin_fma(-x, r, 1.0);
    return __builtin_fma(rem, r, r);
}
#ifndef MYRT_FAST_RCP
#define MYRT_FAST_RCP 1
#endif
__device__ __forceinline__ double inv_det(double det, bool frcp) {
    return (MYRT_FAST_RCP && frcp) ? rcp_rn(det) : 1.0 / det;
}

// Closest-hit triangle test, intersectTriangle (RTContext.swift:479-510) minus the
// hit-point/normal writes, which are recomputed once for the final hit (same values).
template <class Tri>
__device__ __forceinline__ bool tri_closest(const Tri& T, const V3& o_mb, const V3& d, double tlo, double eps,
                                           Hit& h, int triIdx, int instIdx, bool frcp = false) {
    V3 v0, e1, e2;
    tri_geom(T, v0, e1, e2);
    const V3 pvec = cross(d, e2);
    const double det = dot(e1, pvec);
    if (fabs(det) < eps) return false;
    const double invDet = inv_det(det, frcp);
    const V3 tvec = o_mb - v0;
    const double u = dot(tvec, pvec) * invDet;
    if (u < 0.0 || u > 1.0) return false;
    const V3 q = cross(tvec, e1);
    const double v = dot(d, q) * invDet;
    if (v < 0.0 || u + v > 1.0) return false;
    const double t = dot(e2, q) * invDet;
    if (t <= smax(eps, tlo) || t >= h.t) return false;
    h.t = t; h.u = u; h.v = v; h.tri = triIdx; h.inst = instIdx;
    return true;
}
// triShadowHit (RTContext.swift:832-848)
template <class Tri>
__device__ __forceinline__ bool tri_shadow(const Tri& T, const V3& o_mb, const V3& d, double tlo, double thi,
                                           double eps, bool frcp = false) {
    V3 v0, e1, e2;
    tri_geom(T, v0, e1, e2);
    const V3 pvec = cross(d, e2);
    const double det = dot(e1, pvec);
    if (fabs(det) < eps) return false;
    const double invDet = inv_det(det, frcp);
    const V3 tvec = o_mb - v0;
    const double u = dot(tvec, pvec) * invDet;
    if (u < 0.0 || u > 1.0) return false;
    const V3 q = cross(tvec, e1);
    const double v = dot(d, q) * invDet;
    if (v < 0.0 || u + v > 1.0) return false;
    const double t = dot(e2, q) * invDet;
    return (t > smax(eps, tlo) && t < thi);
}

// intersectSphere / intersectPlane (RTContext.swift:513-538) and sphereShadowHit /
// planeShadowHit (:851-870) on the instance-local ray.  T encodes the primitive
// (layout.h kPrimSphere / kPrimPlane).
__device__ __forceinline__ bool prim_closest(int kind, const TriRec& T, const V3& o, const V3& d, double tlo,
                                             double eps, double& ht) {
    double t;
    if (kind == kPrimSphere) {
        const V3 oc = o - ld3(T.v0);
        const double rad = T.e1[0];
        const double a = dot(d, d);
        const double b = 2.0 * dot(oc, d);
        const double c = dot(oc, oc) - rad * rad;
        const double disc = b * b - (4.0 * a) * c;
        if (disc < 0) return false;
        const double sd = dsqrt(disc);
        t = (-b - sd) / (2.0 * a);
        if (t < eps) t = (-b + sd) / (2.0 * a);
    } else {
        const V3 nrm = ld3(T.e1);
        const double denom = dot(nrm, d);
        if (fabs(denom) < eps) return false;
        t = dot(ld3(T.v0) - o, nrm) / denom;
    }
    if (t <= smax(eps, tlo) || t >= ht) return false;
    ht = t;
    return true;
}
__device__ __forceinline__ bool prim_shadow(int kind, const TriRec& T, const V3& o, const V3& d, double thi,
                                            double eps) {
    const double tmin = smax(eps, 0.0);                       // shadow rays keep the Ray default tMin = 0
    double t;
    if (kind == kPrimSphere) {
        const V3 oc = o - ld3(T.v0);
        const double rad = T.e1[0];
        const double a = dot(d, d);
        const double b = 2.0 * dot(oc, d);
        const double c = dot(oc, oc) - rad * rad;
        const double disc = b * b - (4.0 * a) * c;
        if (disc < 0) return false;
        const double sd = dsqrt(disc);
        t = (-b - sd) / (2.0 * a);
        if (t < tmin) t = (-b + sd) / (2.0 * a);
    } else {
        const V3 nrm = ld3(T.e1);
        const double denom = dot(nrm, d);
        if (fabs(denom) < eps) return false;
        t = dot(ld3(T.v0) - o, nrm) / denom;
    }
    return t > tmin && t < thi;
}

// Test both children of inner record `ref`.  On return `ref` is the next node to visit
// (true), or the caller must pop (false).  Order = near first, ties to L (the reference
// pushes R then L after `if d1 > d2 swap`, RTContext.swift:600-606); the far child is
// pushed.  Children beyond `lim` (conservative t-pruning) count as misses.
template <bool COUNT, bool FAST, bool SHADOW, class Rec>
__device__ __forceinline__ bool inner_step_rec(const RenderParams& P, const Rec& R, int& ref, const V3& o,
                                               const V3& inv, double lim, Stack& st, Counts& c) {
    if (COUNT) c.recs++;
    double t0, t1;
    bool h0 = slab_hit<FAST>((double)R.lo[0][0], (double)R.lo[0][1], (double)R.lo[0][2], (double)R.hi[0][0],
                             (double)R.hi[0][1], (double)R.hi[0][2], o, inv, P.eps, t0);
    bool h1 = slab_hit<FAST>((double)R.lo[1][0], (double)R.lo[1][1], (double)R.lo[1][2], (double)R.hi[1][0],
                             (double)R.hi[1][1], (double)R.hi[1][2], o, inv, P.eps, t1);
    h0 = h0 && !(t0 > lim);
    h1 = h1 && !(t1 > lim);
    const int a = R.ref[0], b = R.ref[1];
    if (MYRT_REF(P)) {
        if (!SHADOW) {
            c.nodes += 2;                    // intersectBLAS loads both children (RTContext.swift:600-606)
        } else {
            // occludedBLAS pushes R then L unconditionally and tests each on pop
            // (RTContext.swift:818-826): L is popped next (+1); R - or a miss marker - waits.
            c.nodes += 1;
            st.push(h1 ? b : kMissRef, t1);
            if (h0) { ref = a; return true; }
            return false;
        }
    }
    // selects instead of branches: the far child's entry is written to the next LDS slot
    // unconditionally and kept only when both children are hit
    const bool both = h0 && h1;
#ifndef MYRT_SHADOW_ORDER
#define MYRT_SHADOW_ORDER 1
#endif
    // Closest hit: near child first (the reference's order).  Any-hit walks return a
    // boolean, so their order is free (the reference's occludedBLAS is unordered too,
    // RTContext.swift:818-826): MYRT_SHADOW_ORDER 1 = L first (default, measured best:
    // C3 -1%, C5 -4.5% vs near-first), 0 = near first, 2 = far first.
    const bool sw = !SHADOW ? (t0 > t1)
                  : MYRT_SHADOW_ORDER == 1 ? false
                  : MYRT_SHADOW_ORDER == 2 ? !(t0 > t1) : (t0 > t1);
    st.push_if(both, sw ? a : b, sw ? t0 : t1);
    ref = both ? (sw ? b : a) : (h0 ? a : b);
    return h0 || h1;
}

// A record held in SGPRs: loaded with scalar loads when every active lane of the wave is
// at the same node.  Vector loads of one node by 64 lanes return 64 copies through the
// texture-data path (7 instructions x 1 KB per wave step), which profiling showed ~90%
// busy (TD_TD_BUSY); the scalar path moves the 104 B once, through the scalar cache.
#ifndef MYRT_SCALAR_COMPACT
#define MYRT_SCALAR_COMPACT 1   // wave-uniform steps on compact BLAS records read them (16 SGPRs, not 26)
#endif
struct SRec {
    double lo[2][3], hi[2][3];
    int ref[2];
};
// The record is read through the constant address space (4) at a wave-uniform address, so
// the compiler emits the scalar loads itself and schedules them: measured against a hand-written
// s_load_dwordx16/x8/x2 + s_waitcnt block it has fewer SGPR spill reloads in the walk
// (C3 -0.8 %, C5 -1 %, identical frames; profiles/r03i_ab_sload_c4.txt).
typedef const __attribute__((address_space(4))) WRec c4_wrec;
__device__ __forceinline__ SRec load_rec_scalar(const WRec* pv) {
    // the address is wave-uniform; make that explicit so it lives in SGPRs
    const unsigned long long av = (unsigned long long)pv;
    const unsigned alo = __builtin_amdgcn_readfirstlane((unsigned)av);
    const unsigned ahi = __builtin_amdgcn_readfirstlane((unsigned)(av >> 32));
    c4_wrec* p = (c4_wrec*)((unsigned long long)alo | ((unsigned long long)ahi << 32));
    SRec R;
    for (int c = 0; c < 2; ++c)
        for (int a = 0; a < 3; ++a) {
            R.lo[c][a] = p->lo[c][a];
            R.hi[c][a] = p->hi[c][a];
        }
    R.ref[0] = p->ref[0];
    R.ref[1] = p->ref[1];
    return R;
}

// One inner record: compact (float32 bounds, exact) below P.compact_limit, else full;
// through the scalar cache when the whole wave is at this node.
template <bool COUNT, bool FAST, bool SHADOW>
__device__ __forceinline__ bool inner_step(const RenderParams& P, int& ref, const V3& o, const V3& inv, double lim,
                                           Stack& st, Counts& c) {
    const int r0 = __builtin_amdgcn_readfirstlane(ref);
    if (__all(ref == r0)) {
        if (COUNT && !P.count_ref)
            c.it_wave_scalar[SHADOW] += ((int)(threadIdx.x & 63) == __builtin_ctzll(__ballot(1))) ? 1 : 0;
        // The wave-uniform step reads the compact record when there is one: 16 SGPRs instead of
        // the FP64 record's 26 leave the walk loop fewer spilled SGPRs to restore at its back
        // edge (C3 -0.3 %, pipelined -0.46 %, C5 -0.6 %; profiles/r03t_ab_scalar_compact.txt),
        // though each step then converts 12 bounds (in round 2, before the register-allocation
        // changes since, the FP64 record had measured 0.5 % faster).
#if MYRT_SCALAR_COMPACT
        if (r0 < P.compact_limit) {          // the compact record: 16 SGPRs instead of 26
            const unsigned long long av = (unsigned long long)(P.crecs + r0);
            const unsigned alo = __builtin_amdgcn_readfirstlane((unsigned)av);
            const unsigned ahi = __builtin_amdgcn_readfirstlane((unsigned)(av >> 32));
            typedef const __attribute__((address_space(4))) CRec c4_crec;
            c4_crec* p = (c4_crec*)((unsigned long long)alo | ((unsigned long long)ahi << 32));
            CRec R;
            for (int k = 0; k < 2; ++k)
                for (int a = 0; a < 3; ++a) { R.lo[k][a] = p->lo[k][a]; R.hi[k][a] = p->hi[k][a]; }
            R.ref[0] = p->ref[0];
            R.ref[1] = p->ref[1];
            return inner_step_rec<COUNT, FAST, SHADOW>(P, R, ref, o, inv, lim, st, c);
        }
#endif
        const SRec R = load_rec_scalar(P.recs + r0);
        return inner_step_rec<COUNT, FAST, SHADOW>(P, R, ref, o, inv, lim, st, c);
    }
    if (COUNT && !P.count_ref) {             // redundancy of the per-lane loads below
        unsigned long long left = __ballot(1);
        int my_leader = -1;
        while (left) {                       // one group of equal refs per iteration
            const int leader = __builtin_ctzll(left);
            const int r = __shfl(ref, leader, 64);
            if (ref == r) my_leader = leader;
            left &= ~__ballot(ref == r);
        }
        c.div_lanes += 1;
        c.div_distinct += ((int)(threadIdx.x & 63) == my_leader) ? 1 : 0;
    }
    if (ref < P.compact_limit) return inner_step_rec<COUNT, FAST, SHADOW>(P, P.crecs[ref], ref, o, inv, lim, st, c);
    return inner_step_rec<COUNT, FAST, SHADOW>(P, P.recs[ref], ref, o, inv, lim, st, c);
}

// Pop the next node whose entry distance does not exceed `lim`; false when the stack
// (down to `base`) is exhausted.
template <bool COUNT, bool SHADOW>
__device__ __forceinline__ bool pop_next(const RenderParams& P, Stack& st, int base, double lim, int& ref, Counts& c) {
    while (st.sp > base) {
        double tlo;
        const int r = st.pop(tlo);
        if (SHADOW && MYRT_REF(P)) {         // every pop is a node fetch of occludedBLAS
            c.nodes += 1;
            if (r == kMissRef) continue;
        }
        if (tlo > lim) continue;
        ref = r;
        return true;
    }
    return false;
}

// One ordered BVH walk shared by the closest-hit and any-hit queries.  `ref` is a
// node the caller has already tested (the root); children are tested at the parent
// (one 128-B record holds both).  LEAF(ref) handles a leaf run and returns true to
// terminate the walk (any-hit).  LIMIT() gives the current pruning distance.
template <bool COUNT, bool FAST, bool SHADOW, class Leaf, class Limit>
__device__ __forceinline__ bool walk(const RenderParams& P, int ref, const V3& o, const V3& inv, Stack& st, int base,
                                     Counts& c, Leaf leaf, Limit limit) {
    for (;;) {
        if (ref >= 0) {
            if (inner_step<COUNT, FAST, SHADOW>(P, ref, o, inv, limit(), st, c)) continue;
        } else {
            if (leaf(ref)) return true;
        }
        if (!pop_next<COUNT, SHADOW>(P, st, base, limit(), ref, c)) return false;
    }
}
template <bool COUNT, bool SHADOW, class Leaf, class Limit>
__device__ __forceinline__ bool walk_any(const RenderParams& P, int ref, const V3& o, const V3& inv, Stack& st,
                                         int base, Counts& c, Leaf leaf, Limit limit) {
    if (__all(finite3(inv))) return walk<COUNT, true, SHADOW>(P, ref, o, inv, st, base, c, leaf, limit);
    return walk<COUNT, false, SHADOW>(P, ref, o, inv, st, base, c, leaf, limit);
}

template <bool COUNT>
__device__ void intersect_closest(const RenderParams& P, const V3& o, const V3& d, const V3& inv, double tlo,
                                  double time, Hit& h, Stack& st, Counts& c) {
    const double eps = P.eps;
    h.t = DINF; h.inst = -1; h.tri = -1; h.u = 0; h.v = 0;
    // prune_rel = 1 + delta; reference-order counting walks without pruning
    auto limit = [&]() { return MYRT_REF(P) ? DINF : h.t * P.prune_rel + P.prune_abs; };
    if (MYRT_REF(P)) c.nodes += 1;           // the TLAS root's bounds (RTContext.swift:642)
    double d0;
    if (!slab_hit<false>(P.tlas_root_lo[0], P.tlas_root_lo[1], P.tlas_root_lo[2], P.tlas_root_hi[0],
                         P.tlas_root_hi[1], P.tlas_root_hi[2], o, inv, eps, d0))
        return;
    auto tlas_leaf = [&](int ref) -> bool {
        for (int e = ~ref - P.tlas_leaf_base;; ++e) {
            const DTlasLeafEntry le = P.tlas_leaf[e];
            const DInstance& I = P.insts[le.inst];
            if (COUNT) c.insts++;
            if (MYRT_REF(P)) c.nodes += 1;   // the BLAS root's bounds (RTContext.swift:550-552)
            // world -> local (RTContext.swift:657-673)
            const V3 instOffset = ld3(I.motion) * time;
            const V3 ow = o - instOffset;
            const V3 ol = m4_point(I.w2l, ow, 1.0);
            const V3 dl = m4_point(I.w2l, d, 0.0);
            const V3 il = rcp(dl);
            double dr;
            if (slab_hit<false>(I.root_lo[0], I.root_lo[1], I.root_lo[2], I.root_hi[0], I.root_hi[1], I.root_hi[2],
                                ol, il, eps, dr) && !(dr > limit())) {
                const V3 omb = ol - ld3(I.tri_motion) * time;   // Triangle.motionBlur offset (:480-481)
                const int inst = le.inst;
                auto blas_leaf = [&](int r) -> bool {
                    auto run = [&](const auto* tris) {
                        for (int t = ~r;; ++t) {
                            const auto T = tris[t];          // by value: `last` arrives with the vertices
                            if (COUNT) c.tris++;
                            const bool closer = tri_closest(T, omb, dl, tlo, eps, h, t, inst, P.fast_rcp);
                            if (MYRT_REF(P) && closer && I.smooth) c.smooth++;
                            if (T.last) break;
                        }
                    };
                    if (P.ctris) run(P.ctris); else run(P.tris);
                    return false;
                };
                const int sbase = st.sp;
                if (I.kind != kPrimTriangles) {                           // sphere / plane instance
                    double ht = h.t;
                    if (prim_closest(I.kind, P.tris[~I.root_ref], ol, dl, tlo, eps, ht)) {
                        h.t = ht; h.tri = ~I.root_ref; h.inst = inst;
                    }
                } else if (I.root_ref < 0) blas_leaf(I.root_ref);
                else walk_any<COUNT, false>(P, I.root_ref, ol, il, st, sbase, c, blas_leaf, limit);
            }
            if (le.last) break;
        }
        return false;
    };
    const int base = st.sp;
    if (P.tlas_root_ref < 0) tlas_leaf(P.tlas_root_ref);
    else walk_any<COUNT, false>(P, P.tlas_root_ref, o, inv, st, base, c, tlas_leaf, limit);
}

template <bool COUNT>
__device__ bool occluded(const RenderParams& P, const V3& o, const V3& d, double tmax, double time, Stack& st,
                         Counts& c) {
    if (!P.has_tlas) return false;
    const double eps = P.eps;
    const V3 inv = rcp(d);
    const double lim = MYRT_REF(P) ? DINF : tmax * P.prune_rel + P.prune_abs;
    auto limit = [&]() { return lim; };
    if (MYRT_REF(P)) c.nodes += 1;           // occludedTLAS pops the root (RTContext.swift:727-731)
    double d0;
    if (!slab_hit<false>(P.tlas_root_lo[0], P.tlas_root_lo[1], P.tlas_root_lo[2], P.tlas_root_hi[0],
                         P.tlas_root_hi[1], P.tlas_root_hi[2], o, inv, eps, d0) || d0 > lim)
        return false;
    auto tlas_leaf = [&](int ref) -> bool {
        for (int e = ~ref - P.tlas_leaf_base;; ++e) {
            const DTlasLeafEntry le = P.tlas_leaf[e];
            const DInstance& I = P.insts[le.inst];
            if (COUNT) c.insts++;
            if (MYRT_REF(P)) c.nodes += 1;   // occludedBLAS pops its root (RTContext.swift:789-793)
            const V3 instOffset = ld3(I.motion) * time;
            const V3 ol = m4_point(I.w2l, o - instOffset, 1.0);
            const V3 dl = m4_point(I.w2l, d, 0.0);
            const V3 il = rcp(dl);
            double dr;
            if (slab_hit<false>(I.root_lo[0], I.root_lo[1], I.root_lo[2], I.root_hi[0], I.root_hi[1], I.root_hi[2],
                                ol, il, eps, dr) && !(dr > lim)) {
                const V3 omb = ol - ld3(I.tri_motion) * time;
                auto blas_leaf = [&](int r) -> bool {
                    auto run = [&](const auto* tris) -> bool {
                        for (int t = ~r;; ++t) {
                            const auto T = tris[t];          // by value: `last` arrives with the vertices
                            if (COUNT) c.tris++;
                            if (tri_shadow(T, omb, dl, 0.0, tmax, eps, P.fast_rcp)) return true;
                            if (T.last) break;
                        }
                        return false;
                    };
                    return P.ctris ? run(P.ctris) : run(P.tris);
                };
                const int sbase = st.sp;
                bool hit;
                if (I.kind != kPrimTriangles) hit = prim_shadow(I.kind, P.tris[~I.root_ref], ol, dl, tmax, eps);
                else if (I.root_ref < 0) hit = blas_leaf(I.root_ref);
                else hit = walk_any<COUNT, true>(P, I.root_ref, ol, il, st, sbase, c, blas_leaf, limit);
                if (hit) { st.reset(sbase); return true; }
            }
            if (le.last) break;
        }
        return false;
    };
    const int base = st.sp;
    bool hit;
    if (P.tlas_root_ref < 0) hit = tlas_leaf(P.tlas_root_ref);
    else hit = walk_any<COUNT, true>(P, P.tlas_root_ref, o, inv, st, base, c, tlas_leaf, limit);
    st.reset(base);
    return hit;
}

// ---------------------------------------------------------- unified identity walk
// When every instance is the identity and static (HostScene::identity), the local ray
// equals the world ray, so TLAS and BLAS records are walked as ONE tree with one stack:
// a TLAS leaf pushes its instances' BLAS roots (tested with the world ray) in reverse
// order, so they pop - and are traversed fully - in leaf order, as intersectTLAS does
// (RTContext.swift:648-706).  One call = one step: one inner record or one leaf run,
// followed by the pop of the next node.  Returns 0 = continue, 1 = stack exhausted,
// 2 = shadow ray occluded.
// Leaf of the unified walk: a BLAS leaf run (closest: record hits in h; any-hit: true when
// occluded) or a TLAS leaf (pushes its instances' BLAS roots in reverse order).
template <bool COUNT, bool SHADOW, bool FAST>
__device__ __forceinline__ bool unified_leaf(const RenderParams& P, int ref, Stack& st, const V3& o, const V3& d,
                                             const V3& inv, double tlo, double tmax, Hit& h, Counts& c) {
    const double eps = P.eps;
    const int e = ~ref;
    if (e < P.tlas_leaf_base) {                                  // BLAS leaf run
        auto test = [&](const auto& T, int t) -> bool {
            if (COUNT) c.tris++;
            if (SHADOW) return tri_shadow(T, o, d, 0.0, tmax, eps, P.fast_rcp);
            tri_closest(T, o, d, tlo, eps, h, t, T.prim, P.fast_rcp);   // prim = owning instance
            return false;
        };
        auto run = [&](const auto* tris) -> bool {
            for (int t = e;; ++t) {
                const auto T = tris[t];          // by value: `last` arrives with the vertices
                if (test(T, t)) return true;
                if (T.last) break;
            }
            return false;
        };
        return P.ctris ? run(P.ctris) : run(P.tris);
    }
    // TLAS leaf: instance list
    const int k0 = e - P.tlas_leaf_base;
    int k1 = k0;
    while (!P.tlas_leaf[k1].last) ++k1;
    const double lim = (SHADOW ? tmax : h.t) * P.prune_rel + P.prune_abs;
    for (int k = k1; k >= k0; --k) {
        const DInstance& I = P.insts[P.tlas_leaf[k].inst];
        if (COUNT) c.insts++;
        double dr;
        if (slab_hit<FAST>(I.root_lo[0], I.root_lo[1], I.root_lo[2], I.root_hi[0], I.root_hi[1],
                           I.root_hi[2], o, inv, eps, dr) && !(dr > lim))
            st.push(I.root_ref, dr);
    }
    return false;
}

template <bool COUNT, bool SHADOW, bool FAST>
__device__ __forceinline__ int unified_step(const RenderParams& P, int& ref, Stack& st, const V3& o, const V3& d,
                                            const V3& inv, double tlo, double tmax, Hit& h, Counts& c) {
    if (COUNT && !P.count_ref) {             // divergence breakdown of this iteration
        const bool in = ref >= 0;
        const unsigned long long bi = __ballot(in), bl = __ballot(!in);
        const bool first = (int)(threadIdx.x & 63) == __builtin_ctzll(__ballot(1));
        c.it_wave_inner[SHADOW] += (first && bi) ? 1 : 0;
        c.it_wave_leaf[SHADOW] += (first && bl) ? 1 : 0;
        c.it_lane_inner[SHADOW] += in ? 1 : 0;
        c.it_lane_leaf[SHADOW] += in ? 0 : 1;
    }
    if (ref >= 0) {
        if (inner_step<COUNT, FAST, SHADOW>(P, ref, o, inv, (SHADOW ? tmax : h.t) * P.prune_rel + P.prune_abs, st, c))
            return 0;
    } else if (unified_leaf<COUNT, SHADOW, FAST>(P, ref, st, o, d, inv, tlo, tmax, h, c)) {
        return 2;
    }
    return pop_next<COUNT, SHADOW>(P, st, 0, (SHADOW ? tmax : h.t) * P.prune_rel + P.prune_abs, ref, c) ? 0 : 1;
}

// Root test of the unified walk (the TLAS root is popped and tested first,
// RTContext.swift:642-646).  Returns false when the ray misses the whole scene.
__device__ __forceinline__ bool unified_begin(const RenderParams& P, const V3& o, const V3& inv, double lim, int& ref) {
    double d0;
    if (!slab_hit<false>(P.tlas_root_lo[0], P.tlas_root_lo[1], P.tlas_root_lo[2], P.tlas_root_hi[0],
                         P.tlas_root_hi[1], P.tlas_root_hi[2], o, inv, P.eps, d0) || d0 > lim)
        return false;
    ref = P.tlas_root_ref;
    return true;
}

}  // namespace dev
}  // namespace myrt
#include "wide.h"
namespace myrt {
namespace dev {

// Whole-ray unified walks (identity scenes): closest hit and any hit with one stack.  With a
// wide tree (RenderParams::wide) and every 1/d in range, the conservative FP32 four-wide walk
// (wide.h) runs instead; a lane that met two candidates at its final t is re-walked here in
// the reference's order.  Reference-order counting launches (count_ref) keep the binary walk.
template <bool COUNT, bool FAST>
__device__ __forceinline__ void uni_closest_walk(const RenderParams& P, const V3& o, const V3& d, const V3& inv,
                                                 double tlo, Hit& h, Stack& st, Counts& c) {
    int ref;
    if (!unified_begin(P, o, inv, DINF, ref)) return;   // the stack is empty here (base 0)
    do {
        if (COUNT || MYRT_WAVE_TIMES) c.it_closest++;
    } while (unified_step<COUNT, false, FAST>(P, ref, st, o, d, inv, tlo, DINF, h, c) == 0);
}
template <bool COUNT, bool WIDE = true>
__device__ __forceinline__ void uni_closest(const RenderParams& P, const V3& o, const V3& d, const V3& inv,
                                            double tlo, Hit& h, Stack& st, Counts& c) {
    h.t = DINF; h.inst = -1; h.tri = -1; h.u = 0; h.v = 0;
    if (WIDE && !MYRT_REF(P) && P.wide && __all(wide_ok(inv))) {
        bool tie = false;
        (void)wide_walk<COUNT, false>(P, TwWorld{o, d}, inv, tlo, DINF, h, tie, st, c);
#ifndef MYRT_REWALK
#define MYRT_REWALK 1
#endif
        if (MYRT_REWALK && __any(tie) && tie) {  // equal-t candidates: the reference's order decides
            c.ties++;
            h.t = DINF; h.inst = -1; h.tri = -1; h.u = 0; h.v = 0;
            uni_closest_walk<COUNT, true>(P, o, d, inv, tlo, h, st, c);
        }
        return;
    }
    if (__all(finite3(inv))) uni_closest_walk<COUNT, true>(P, o, d, inv, tlo, h, st, c);
    else uni_closest_walk<COUNT, false>(P, o, d, inv, tlo, h, st, c);
}
template <bool COUNT, bool FAST>
__device__ __forceinline__ bool uni_occluded_walk(const RenderParams& P, const V3& o, const V3& d, const V3& inv,
                                                  double tmax, Stack& st, Counts& c) {
    int ref;
    if (!unified_begin(P, o, inv, tmax * P.prune_rel + P.prune_abs, ref)) return false;
    Hit h;   // unused by any-hit steps
    h.t = DINF; h.inst = -1; h.tri = -1; h.u = 0; h.v = 0;
    const int base = st.sp;
    int r;
    do {
        if (COUNT || MYRT_WAVE_TIMES) c.it_shadow++;
    } while ((r = unified_step<COUNT, true, FAST>(P, ref, st, o, d, inv, 0.0, tmax, h, c)) == 0);
    st.reset(base);
    return r == 2;
}
template <bool COUNT, bool WIDE = true>
__device__ __forceinline__ bool uni_occluded(const RenderParams& P, const V3& o, const V3& d, double tmax,
                                             Stack& st, Counts& c) {
    if (!P.has_tlas) return false;
    const V3 inv = rcp(d);
    if (WIDE && !MYRT_REF(P) && P.wide && __all(wide_ok(inv))) {
        Hit hu;
        bool tie = false;
        return wide_walk<COUNT, true>(P, TwWorld{o, d}, inv, 0.0, tmax, hu, tie, st, c);
    }
    if (__all(finite3(inv))) return uni_occluded_walk<COUNT, true>(P, o, d, inv, tmax, st, c);
    return uni_occluded_walk<COUNT, false>(P, o, d, inv, tmax, st, c);
}

// Walks of the render kernels (render.hip WALK template argument)
// kWalkFit = transformed scenes through their flattened instance tree (wide.h fit_walk, option fit)
constexpr int kWalkGeneral = 0, kWalkIdentity = 1, kWalkTransformed = 2, kWalkFit = 3;

// ------------------------------------------------------- unified transformed walk (UT)
// Scenes whose instances carry transforms or motion (every object of a reference scene is an
// instance, RTContext.swift:122-241, 384-401).  intersect_closest/occluded nest a BLAS walk
// inside the TLAS walk, so the lanes of a wave sit in different loop nests and run them one
// after the other.  Here TLAS and BLAS records are walked in ONE loop with one stack: a TLAS
// leaf pushes a marker per instance (in reverse, so they pop in leaf order); popping a marker
// switches the lane's ray to that instance's local ray - the same world->local arithmetic as
// intersectTLAS (:655-673) - and tests the instance's BLAS root (intersectBLAS's first pop,
// :567-571); a popped TLAS entry switches back to the world ray.  Each BLAS is finished before
// the next marker pops, so instances and their nodes are visited in intersectTLAS's order
// (near child first, ties to L, :641-706): hits - including equal-t ties - are the reference's.
// Stack bound: TLAS path + the largest TLAS leaf + BLAS path (HostScene::max_stack_unified).
struct UtRay {
    V3 o, d, inv;      // the current ray (world, or instance `inst`'s local ray)
    int inst;          // -1 = world
    bool fast;         // every 1/d component finite (slab_hit<true> allowed)
};
// back to the world ray; 1/d is recomputed (the same IEEE divisions as the caller's) rather than
// kept live across the walk
__device__ __forceinline__ void ut_world(UtRay& R, const V3& o, const V3& d) {
    R.o = o; R.d = d; R.inv = rcp(d); R.inst = -1; R.fast = finite3(R.inv);
}
__device__ __forceinline__ void ut_local(const RenderParams& P, UtRay& R, int k, const V3& o, const V3& d,
                                         double time) {
    const DInstance& I = P.insts[k];
    const V3 instOffset = ld3(I.motion) * time;
    R.o = m4_point(I.w2l, o - instOffset, 1.0);
    R.d = m4_point(I.w2l, d, 0.0);
    R.inv = rcp(R.d);
    R.inst = k;
    R.fast = finite3(R.inv);
}
__device__ __forceinline__ bool ut_is_marker(const RenderParams& P, int ref) { return ref < 0 && ~ref >= P.ut_marker_base; }
__device__ __forceinline__ bool ut_is_tlas(const RenderParams& P, int ref) {
    return ref >= 0 ? ref >= P.tlas_rec_base : (~ref >= P.tlas_leaf_base);
}

// Pop the next node to visit.  Markers switch the ray to their instance and test its BLAS root
// (a sphere/plane instance's primitive is tested right there, `prim`); TLAS entries bring the
// world ray back.  Returns 0 = `ref` holds the next node, 1 = stack exhausted, 2 = occluded
// (SHADOW: a sphere/plane instance's primitive blocks the ray).
template <bool SHADOW, class Prim>
__device__ __forceinline__ int ut_pop(const RenderParams& P, Stack& st, int base, double lim, int& ref, UtRay& R,
                                      const V3& o, const V3& d, double time, Prim prim) {
    while (st.sp > base) {
        double tlo;
        const int r = st.pop(tlo);
        if (ut_is_marker(P, r)) {
            const int k = ~r - P.ut_marker_base;
            ut_local(P, R, k, o, d, time);
            const DInstance& I = P.insts[k];
            double dr;
            if (!slab_hit<false>(I.root_lo[0], I.root_lo[1], I.root_lo[2], I.root_hi[0], I.root_hi[1], I.root_hi[2],
                                 R.o, R.inv, P.eps, dr) || dr > lim)
                continue;
            if (I.kind != kPrimTriangles) {            // single-primitive BLAS (RTContext.swift:122-192)
                if (prim(I, k)) return 2;
                continue;
            }
            ref = I.root_ref;
            return 0;
        }
        if (tlo > lim) continue;
        if (R.inst >= 0 && ut_is_tlas(P, r)) ut_world(R, o, d);
        ref = r;
        return 0;
    }
    return 1;
}

// Closest hit (intersectTLAS) or any hit (occludedTLAS, order-free) of one world ray.
// Returns the occlusion for SHADOW.
template <bool SHADOW>
__device__ __forceinline__ bool ut_walk(const RenderParams& P, const V3& o, const V3& d, const V3& inv, double tlo,
                                        double tmax, double time, Hit& h, Stack& st) {
    Counts c{};
    const double eps = P.eps;
    const int base = st.sp;
    UtRay R;
    R.o = o; R.d = d; R.inv = inv; R.inst = -1; R.fast = finite3(inv);
    int ref;
    if (!unified_begin(P, o, inv, SHADOW ? tmax * P.prune_rel + P.prune_abs : DINF, ref)) return false;
    bool occ = false;
    auto prim = [&](const DInstance& I, int k) -> bool {
        const TriRec& T = P.tris[~I.root_ref];
        if (SHADOW) return prim_shadow(I.kind, T, R.o, R.d, tmax, eps);
        double ht = h.t;
        if (prim_closest(I.kind, T, R.o, R.d, tlo, eps, ht)) { h.t = ht; h.tri = ~I.root_ref; h.inst = k; }
        return false;
    };
    for (;;) {
        const double lim = (SHADOW ? tmax : h.t) * P.prune_rel + P.prune_abs;
        bool stepped = false;
        if (ref >= 0) {                                       // TLAS or BLAS inner record
            stepped = __all(R.fast) ? inner_step<false, true, SHADOW>(P, ref, R.o, R.inv, lim, st, c)
                                    : inner_step<false, false, SHADOW>(P, ref, R.o, R.inv, lim, st, c);
        } else if (~ref < P.tlas_leaf_base) {                 // BLAS leaf run, instance R.inst
            // local origin minus the mesh's triangle motion (intersectTriangle :480-481)
            const V3 omb = R.o - ld3(P.insts[R.inst].tri_motion) * time;
            auto run = [&](const auto* tris) -> bool {
                for (int t = ~ref;; ++t) {
                    const auto T = tris[t];
                    if (SHADOW) {
                        if (tri_shadow(T, omb, R.d, 0.0, tmax, eps, P.fast_rcp)) return true;
                    } else {
                        tri_closest(T, omb, R.d, tlo, eps, h, t, R.inst, P.fast_rcp);
                    }
                    if (T.last) break;
                }
                return false;
            };
            if (P.ctris ? run(P.ctris) : run(P.tris)) { occ = true; break; }
        } else {                                              // TLAS leaf: one marker per instance
            const int k0 = ~ref - P.tlas_leaf_base;
            int k1 = k0;
            while (!P.tlas_leaf[k1].last) ++k1;
            for (int k = k1; k >= k0; --k) st.push(~(P.ut_marker_base + P.tlas_leaf[k].inst), 0.0);
        }
        if (stepped) continue;
        const double lim2 = (SHADOW ? tmax : h.t) * P.prune_rel + P.prune_abs;
        const int pr = ut_pop<SHADOW>(P, st, base, lim2, ref, R, o, d, time, prim);
        if (pr == 2) { occ = true; break; }
        if (pr == 1) break;
    }
    st.reset(base);
    return occ;
}

// The hit record intersectTriangle/Sphere/Plane + intersectTLAS leave behind
// (RTContext.swift:479-538, 674-705), rebuilt once for the final (t, tri, u, v, inst):
// world hit point and the normalized, det-signed world geometric normal.
template <bool COUNT>
__device__ __forceinline__ void hit_geometry(const RenderParams& P, const V3& o, const V3& d, double time,
                                             const Hit& h, V3& p, V3& Ngeo, Counts& c) {
    const TriRec& T = P.tris[h.tri];
    const DInstance& I = P.insts[h.inst];
    V3 nl, pl;
    if (I.kind == kPrimTriangles) {
        const V3 e1 = ld3(T.e1), e2 = ld3(T.e2), v0 = ld3(T.v0);
        if (I.smooth) {
            if (COUNT) c.normals++;
            const double* nn = P.normals + (size_t)h.tri * 9;
            const double w = 1.0 - h.u - h.v;
            nl = normalize(((w * ld3(nn)) + (h.u * ld3(nn + 3))) + (h.v * ld3(nn + 6)));
        } else {
            nl = normalize(cross(e1, e2));
        }
        pl = (v0 + (h.u * e1)) + (h.v * e2);
    } else {                                                    // p = origin + dir * t, local ray
        const V3 ol = m4_point(I.w2l, o - ld3(I.motion) * time, 1.0);
        const V3 dl = m4_point(I.w2l, d, 0.0);
        pl = ol + dl * h.t;
        nl = (I.kind == kPrimSphere) ? normalize(pl - ld3(T.v0)) : normalize(ld3(T.e1));
    }
    p = m4_point(I.l2w, pl, 1.0) + ld3(I.motion) * time;
    Ngeo = normalize(m3_mul(I.nmat, nl));
    if (I.det_neg) Ngeo = -Ngeo;
}

// Blinn-Phong lobe pow(NdotH, shininess) for 0 <= NdotH <= 1 and shininess >= 1 (the
// point-light term, Object+Extension.swift:134-137): exp2(shininess * log2(NdotH)).  OCML
// pow carries an extended-precision log for correct rounding in every range and needs far
// more registers; here the result differs from pow by a few ulps (relative ~1e-14, vs
// the 1e-5 parity bar) and NdotH = 0 / 1 give exactly 0 / 1.
// Not inlined on purpose: inlined, the polynomial constants of log2/exp2 were hoisted
// to the kernel prologue and spilled to scratch once per lane (~0.3 GB of scratch
// writes per C3 frame); as a call they are materialized where they are used.
__device__ __noinline__ double phong_pow(double x, double y) {
    return exp2(y * log2(x));
}

// orthonormalBasis (Object+Extension.swift:531-552)
__device__ __forceinline__ void onb(V3 n, V3& tangent, V3& bitangent) {
    const double sign = n.z >= 0 ? 1.0 : -1.0;
    const double a = -1.0 / (sign + n.z);
    const double b = (n.x * n.y) * a;
    tangent = normalize(v3(1.0 + ((sign * n.x) * n.x) * a, sign * b, (-sign) * n.x));
    bitangent = normalize(v3(b, sign + (n.y * n.y) * a, -n.y));
}
__device__ __forceinline__ V3 reflect(V3 d, V3 n) { return d - (2.0 * dot(d, n)) * n; }
// fresnelConductorRGB (Object+Extension.swift:493-505)
__device__ __forceinline__ V3 fresnel_conductor(double eta, double k, double cosI_) {
    const double cosI = smax(0.0, smin(1.0, fabs(cosI_)));
    const double cos2 = cosI * cosI;
    const double eta2k2 = eta * eta + k * k;
    const double twoEtaCos = (2.0 * eta) * cosI;
    const V3 cos2v = v3(cos2, cos2, cos2), one = v3(1, 1, 1);
    const V3 Rs = ((eta2k2 - twoEtaCos) + cos2v) / ((eta2k2 + twoEtaCos) + cos2v);
    const V3 Rp = (((eta2k2 * cos2v) - twoEtaCos) + one) / (((eta2k2 * cos2v) + twoEtaCos) + one);
    return 0.5 * (Rs + Rp);
}

__device__ __forceinline__ unsigned long long wave_max(unsigned long long x) {   // all 64 lanes active
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) { const unsigned long long y = __shfl_xor(x, off, 64); x = y > x ? y : x; }
    return x;
}
__device__ __forceinline__ unsigned long long wave_sum(unsigned long long x) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
    return x;
}

}  // namespace dev
}  // namespace myrt
