// slab32_test.cpp — CPU check of the FP32-enclosed slab test (myraytracer_amd/csrc/slab32.h)
// against the reference's FP64 slab (hitAABB, RTContext.swift:557-565; FAST form, no zero
// direction component).  A decision slab32 calls certain must be the FP64 decision, its
// interval must enclose the FP64 entry distance, and for two boxes a certain near/far order
// must be the FP64 order.  Random and adversarial cases: rays through box faces, edges and
// corners perturbed by a few ulps, boxes sharing a face plane, near-axis directions, tiny
// and huge scales.  Test infrastructure (run by tests/test_slab32.py).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <random>
#include <utility>

#include "../../myraytracer_amd/csrc/slab32.h"

namespace S = myrt::f32slab;

namespace {

bool slab64(const float* lo, const float* hi, const double* o, const double* inv, double eps, double& tmin) {
    double mn[3], mx[3];
    for (int a = 0; a < 3; ++a) {
        const double t1 = ((double)lo[a] - o[a]) * inv[a];
        const double t2 = ((double)hi[a] - o[a]) * inv[a];
        mn[a] = std::fmin(t1, t2);
        mx[a] = std::fmax(t1, t2);
    }
    tmin = std::fmax(std::fmax(mn[0], mn[1]), mn[2]);
    const double tmax = std::fmin(mx[0], std::fmin(mx[1], mx[2]));
    return tmax >= std::fmax(tmin, eps);
}

struct Ctx {
    std::mt19937_64 g{20251016};
    const double eps = 1e-6;
    const float eps_up = S::up(1e-6), eps_dn = S::dn(1e-6);
    long long cases = 0, certain = 0, bad = 0, pairs = 0, order_certain = 0;

    double U(double a, double b) { return std::uniform_real_distribution<double>(a, b)(g); }
    int I(int n) { return (int)(g() % (uint64_t)n); }
    void dir(double* d, double tiny) {
        std::normal_distribution<double> N;
        for (;;) {
            for (int a = 0; a < 3; ++a) d[a] = N(g);
            if (tiny > 0) d[I(3)] = tiny * (I(2) ? 1 : -1);
            const double r = 1.0 / std::sqrt((d[0] * d[0] + d[1] * d[1]) + d[2] * d[2]);   // normalize (H5)
            for (int a = 0; a < 3; ++a) d[a] = d[a] * r;
            if (d[0] != 0 && d[1] != 0 && d[2] != 0) return;
        }
    }
    void box(float* lo, float* hi, double s) {
        for (int a = 0; a < 3; ++a) {
            float x = (float)U(-s, s), y = (float)U(-s, s);
            if (x > y) std::swap(x, y);
            if (I(8) == 0) y = x;                                     // flat in one axis
            lo[a] = x;
            hi[a] = y;
        }
    }
    void fail(const char* what, const float* lo, const float* hi, const double* o, const double* d) {
        if (bad++ < 12)
            std::printf("FAIL %s: lo %a %a %a hi %a %a %a o %a %a %a d %a %a %a\n", what, lo[0], lo[1], lo[2], hi[0],
                        hi[1], hi[2], o[0], o[1], o[2], d[0], d[1], d[2]);
    }
    // one (ray, box): FP32 decision c, FP64 hit/tmin; checks certainty and enclosure
    int one(const float* lo, const float* hi, const double* o, const double* d, float bmax, bool& h64, double& t64,
            float& m, float& l, float& h) {
        const double inv[3] = {1.0 / d[0], 1.0 / d[1], 1.0 / d[2]};
        const S::RayF F = S::make(o[0], o[1], o[2], inv[0], inv[1], inv[2], bmax);
        h64 = slab64(lo, hi, o, inv, eps, t64);
        const int c = S::test(lo[0], lo[1], lo[2], hi[0], hi[1], hi[2], F, eps_up, eps_dn, m, l, h);
        cases++;
        if (c >= 0) {
            certain++;
            if ((c == 1) != h64) fail("decision", lo, hi, o, d);
        }
        if (std::isfinite(l) && std::isfinite(h) && !((double)l <= t64 && t64 <= (double)h))
            fail("enclosure", lo, hi, o, d);
        return c;
    }
    static float bound(const float* lo, const float* hi) {
        double b = 0;
        for (int a = 0; a < 3; ++a) b = std::fmax(b, std::fmax(std::fabs(lo[a]), std::fabs(hi[a])));
        return S::up(b);
    }
    void nudge(double* o) {
        for (int a = 0; a < 3; ++a)
            for (int j = I(7) - 3; j != 0; j += (j > 0 ? -1 : 1)) o[a] = std::nextafter(o[a], j > 0 ? INFINITY : -INFINITY);
    }
};

}  // namespace

int main() {
    Ctx x;
    const double scales[] = {1.0, 100.0, 1e4, 1e-3, 1e-20, 1e20};
    bool h64;
    double t64;
    float m, l, h;
    for (double s : scales) {
        // random rays and boxes
        for (int k = 0; k < 200000; ++k) {
            float lo[3], hi[3];
            x.box(lo, hi, s);
            double o[3], d[3];
            for (auto& v : o) v = x.U(-2 * s, 2 * s);
            x.dir(d, x.I(4) == 0 ? std::pow(10.0, -x.U(2, 12)) : 0.0);
            x.one(lo, hi, o, d, Ctx::bound(lo, hi), h64, t64, m, l, h);
        }
        // grazing: through a face / edge / corner point, origin moved by a few ulps
        for (int k = 0; k < 300000; ++k) {
            float lo[3], hi[3];
            x.box(lo, hi, s);
            double p[3], d[3], o[3];
            for (int a = 0; a < 3; ++a) {
                const int w = x.I(3);
                p[a] = w == 0 ? lo[a] : w == 1 ? hi[a] : x.U(lo[a], hi[a]);
            }
            x.dir(d, x.I(4) == 0 ? std::pow(10.0, -x.U(2, 12)) : 0.0);
            const double t0 = x.U(0.01, 3.0) * s;
            for (int a = 0; a < 3; ++a) o[a] = p[a] - d[a] * t0;
            x.nudge(o);
            x.one(lo, hi, o, d, Ctx::bound(lo, hi), h64, t64, m, l, h);
        }
        // two boxes sharing face planes, rays through a shared plane: the order decision
        for (int k = 0; k < 200000; ++k) {
            float A[2][3], B[2][3];
            x.box(A[0], A[1], s);
            x.box(B[0], B[1], s);
            for (int q = 0, n = 1 + x.I(3); q < n; ++q) {
                const int a = x.I(3), side = x.I(2);
                B[side][a] = A[side][a];
                if (B[0][a] > B[1][a]) std::swap(B[0][a], B[1][a]);
            }
            double p[3], d[3], o[3];
            const int ax = x.I(3);
            for (int a = 0; a < 3; ++a) p[a] = x.U(std::fmin(A[0][a], B[0][a]), std::fmax(A[1][a], B[1][a]));
            p[ax] = A[x.I(2)][ax];
            x.dir(d, 0.0);
            const double t0 = x.U(0.01, 3.0) * s;
            for (int a = 0; a < 3; ++a) o[a] = p[a] - d[a] * t0;
            x.nudge(o);
            const float bm = std::fmax(Ctx::bound(A[0], A[1]), Ctx::bound(B[0], B[1]));
            bool hA, hB;
            double tA, tB;
            float mA, lA, uA, mB, lB, uB;
            const int cA = x.one(A[0], A[1], o, d, bm, hA, tA, mA, lA, uA);
            const int cB = x.one(B[0], B[1], o, d, bm, hB, tB, mB, lB, uB);
            if (cA == 1 && cB == 1) {
                x.pairs++;
                const bool yes = lA > uB, no = uA <= lB;
                if (yes || no) x.order_certain++;
                if (yes && !(tA > tB)) x.fail("order (yes)", A[0], A[1], o, d);
                if (no && (tA > tB)) x.fail("order (no)", A[0], A[1], o, d);
            }
        }
    }
    // the rounding helpers
    for (int k = 0; k < 100000; ++k) {
        const double v = x.U(-1e6, 1e6) * std::pow(10.0, -x.U(0, 30));
        if (!((double)S::dn(v) <= v && v <= (double)S::up(v))) {
            std::printf("FAIL up/dn %a\n", v);
            x.bad++;
        }
    }
    std::printf("slab32: %lld cases, %.4f%% certain, %lld sibling pairs with %.2f%% certain order, %lld failures\n",
                x.cases, 100.0 * (double)x.certain / (double)x.cases, x.pairs,
                x.pairs ? 100.0 * (double)x.order_certain / (double)x.pairs : 0.0, x.bad);
    std::printf("slab32: %s\n", x.bad ? "FAILED" : "ok");
    return x.bad ? 1 : 0;
}
