// slab32.h — FP32-enclosed slab test (DESIGN.md "FP32-enclosed slabs").  Host + device:
// the megakernel's unified walks use it (device.h, MYRT_F32) and tests/cpp/slab32_test.cpp
// checks it on the CPU against the reference's FP64 slab (hitAABB, RTContext.swift:557-565).
//
// A slab value of a float bound b is t64 = (b - o) * (1/d) in FP64.  Here it is
//   t32 = fma(b, i32, -oi32)        i32 = (float)(1/d),  oi32 = (float)o * i32
// and |t32 - t64| <= E(t32) = |t32| 2^-20 + max_a|oi_a| 2^-21 + max_a|i_a| 2^-120.
// The rounding of the two forms is below |t| 2^-22.9 + max|oi| 2^-23 (+ 2^-126-sized
// underflow terms), so E has >= 4x slack, which also covers the roundings of E and t +- E;
// min/max propagate the bound to tmin and tmax.  A ray whose values could reach 2^100 for
// some box inside the scene bounds (bmax) gets c2 = NaN: every test of it is uncertain.
#pragma once
#include <cmath>

#if defined(__HIPCC__)
#define MYRT_HD __host__ __device__ __forceinline__
#else
#define MYRT_HD inline
#endif

namespace myrt {
namespace f32slab {

constexpr float kRel = 0x1p-20f;
constexpr float kAbs = 0x1p-21f;

struct RayF { float ix, iy, iz, oix, oiy, oiz, c2; };

// smallest float >= x / largest float <= x
MYRT_HD float up(double x) {
    const float f = (float)x;
    return ((double)f < x) ? nextafterf(f, __builtin_inff()) : f;
}
MYRT_HD float dn(double x) {
    const float f = (float)x;
    return ((double)f > x) ? nextafterf(f, -__builtin_inff()) : f;
}

// o and 1/d in FP64; bmax >= every |coordinate| of every box the ray is tested against
MYRT_HD RayF make(double ox, double oy, double oz, double ix, double iy, double iz, float bmax) {
    RayF r;
    const float fx = (float)ox, fy = (float)oy, fz = (float)oz;
    r.ix = (float)ix; r.iy = (float)iy; r.iz = (float)iz;
    r.oix = fx * r.ix; r.oiy = fy * r.iy; r.oiz = fz * r.iz;
    const float m = fmaxf(fmaxf(fabsf(r.oix), fabsf(r.oiy)), fabsf(r.oiz));
    const float mi = fmaxf(fmaxf(fabsf(r.ix), fabsf(r.iy)), fabsf(r.iz));
    const bool ok = __builtin_isfinite(r.oix) && __builtin_isfinite(r.oiy) && __builtin_isfinite(r.oiz) &&
                    __builtin_isfinite(r.ix) && __builtin_isfinite(r.iy) && __builtin_isfinite(r.iz) &&
                    bmax * mi + m < 0x1p100f;
    r.c2 = ok ? fmaf(m, kAbs, (mi * 0x1p-60f) * 0x1p-60f) : __builtin_nanf("");
    return r;
}

// 1 = certain hit, 0 = certain miss, -1 = uncertain.  [lo, hi] encloses the FP64 tmin and m
// is the FP32 tmin inside it (NaN bounds when c2 is NaN).
MYRT_HD int test(float lx, float ly, float lz, float hx, float hy, float hz, const RayF& F, float eps_up,
                 float eps_dn, float& m, float& lo, float& hi) {
    const float t1x = fmaf(lx, F.ix, -F.oix), t1y = fmaf(ly, F.iy, -F.oiy), t1z = fmaf(lz, F.iz, -F.oiz);
    const float t2x = fmaf(hx, F.ix, -F.oix), t2y = fmaf(hy, F.iy, -F.oiy), t2z = fmaf(hz, F.iz, -F.oiz);
    const float tmin = fmaxf(fmaxf(fminf(t1x, t2x), fminf(t1y, t2y)), fminf(t1z, t2z));
    const float tmax = fminf(fminf(fmaxf(t1x, t2x), fmaxf(t1y, t2y)), fmaxf(t1z, t2z));
    const float emin = fmaf(fabsf(tmin), kRel, F.c2), emax = fmaf(fabsf(tmax), kRel, F.c2);
    m = tmin;
    lo = tmin - emin;
    hi = tmin + emin;
    const float xlo = tmax - emax, xhi = tmax + emax;
    if (xlo >= fmaxf(hi, eps_up)) return 1;          // NaN (c2) makes both tests false
    if (xhi < fmaxf(lo, eps_dn)) return 0;
    return -1;
}

// the enclosure of an exact FP64 value
MYRT_HD void enclose(double t, float& m, float& lo, float& hi) {
    m = (float)t;
    lo = dn(t);
    hi = up(t);
}

}  // namespace f32slab
}  // namespace myrt
