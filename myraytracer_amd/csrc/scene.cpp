// scene.cpp — host scene construction (product code; see scene.h).
//
// Arithmetic that feeds the kernels (edges, centroids, SAH costs, transformed
// bounds) follows the Swift expression order literally so the BVH is the
// reference's BVH bit for bit; compile with -ffp-contract=off.
#include "scene.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <thread>
#include <atomic>
#include <limits>
#include <map>
#include <memory>

namespace myrt {

static const double kInf = std::numeric_limits<double>::infinity();

// ------------------------------------------------------------------ small math
struct D3 { double x, y, z; };
static inline D3 d3(double x, double y, double z) { return D3{x, y, z}; }
static inline D3 operator+(D3 a, D3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
static inline D3 operator-(D3 a, D3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
static inline D3 operator*(D3 a, double s) { return {a.x * s, a.y * s, a.z * s}; }
static inline D3 operator-(D3 a, double s) { return {a.x - s, a.y - s, a.z - s}; }
static inline D3 operator+(D3 a, double s) { return {a.x + s, a.y + s, a.z + s}; }
static inline D3 operator*(double s, D3 a) { return {s * a.x, s * a.y, s * a.z}; }
static inline D3 operator/(D3 a, double s) { return {a.x / s, a.y / s, a.z / s}; }
static inline double dot(D3 a, D3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
static inline D3 cross(D3 a, D3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
static inline D3 normalize(D3 v) { double r = 1.0 / std::sqrt(dot(v, v)); return v * r; }
static inline D3 vmin(D3 a, D3 b) { return {std::fmin(a.x, b.x), std::fmin(a.y, b.y), std::fmin(a.z, b.z)}; }
static inline D3 vmax(D3 a, D3 b) { return {std::fmax(a.x, b.x), std::fmax(a.y, b.y), std::fmax(a.z, b.z)}; }
static inline D3 of(rt_vec3 v) { return {v.x, v.y, v.z}; }
static inline double smin(double x, double y) { return (y < x) ? y : x; }   // Swift.min
static inline double smax(double x, double y) { return (y >= x) ? y : x; }  // Swift.max

// ------------------------------------------------------- reference-exact BVH build
// BVHBuilder.init/subdivide/findBestSplitPlane (BVH.swift:78-250).
namespace {
int build_threads() {                  // MYRT_BUILD_THREADS, default: hardware threads (<= 64)
    static const int n = [] {
        const char* e = std::getenv("MYRT_BUILD_THREADS");
        const int v = e ? std::atoi(e) : (int)std::thread::hardware_concurrency();
        return std::max(1, std::min(v, 64));
    }();
    return n;
}
constexpr int64_t kParallelFold = 1 << 19;   // nodes this large fold their prims on several threads
int par_chunks(int64_t count) {
    if (count < kParallelFold) return 1;
    return (int)std::max<int64_t>(1, std::min<int64_t>(build_threads(), count / (kParallelFold / 8)));
}
template <class F>
void run_chunks(int T, F&& f) {
    if (T <= 1) { f(0); return; }
    std::vector<std::thread> th;
    for (int k = 1; k < T; ++k) th.emplace_back([&f, k] { f(k); });
    f(0);
    for (auto& t : th) t.join();
}
struct Builder {
    const PrimSet& P;
    RefBVH& B;
    int maxLeaf, N;
    // scratch reused across nodes
    std::vector<double> binLo, binHi;   // [axis][bin][3]
    std::vector<int64_t> binCnt;        // [axis][bin]

    Builder(const PrimSet& p, RefBVH& b, int ml, int bins) : P(p), B(b), maxLeaf(ml), N(std::max(2, bins)) {
        binLo.resize(3 * N * 3); binHi.resize(3 * N * 3); binCnt.resize(3 * N);
    }
    // updateNodeBounds (:108-124).  Large nodes fold chunks concurrently and merge the
    // chunk results in order: min/max folds are associative (for equal values the same
    // element wins whatever the grouping), so the bounds are bit-identical.
    void updateNodeBounds(int64_t idx) {
        const int64_t first = B.leftFirst[idx], cnt = B.count[idx];
        const int T = par_chunks(cnt);
        std::vector<D3> mnv(T, d3(kInf, kInf, kInf)), mxv(T, d3(-kInf, -kInf, -kInf));
        run_chunks(T, [&](int k) {
            D3 mn = d3(kInf, kInf, kInf), mx = d3(-kInf, -kInf, -kInf);
            for (int64_t i = cnt * k / T, e = cnt * (k + 1) / T; i < e; ++i) {
                const int64_t p = B.primIdx[first + i];
                mn = vmin(mn, d3(P.bmin[3 * p], P.bmin[3 * p + 1], P.bmin[3 * p + 2]));
                mx = vmax(mx, d3(P.bmax[3 * p], P.bmax[3 * p + 1], P.bmax[3 * p + 2]));
            }
            mnv[k] = mn; mxv[k] = mx;
        });
        D3 mn = d3(kInf, kInf, kInf), mx = d3(-kInf, -kInf, -kInf);
        for (int k = 0; k < T; ++k) { mn = vmin(mn, mnv[k]); mx = vmax(mx, mxv[k]); }
        B.lo[3 * idx] = mn.x; B.lo[3 * idx + 1] = mn.y; B.lo[3 * idx + 2] = mn.z;
        B.hi[3 * idx] = mx.x; B.hi[3 * idx + 1] = mx.y; B.hi[3 * idx + 2] = mx.z;
    }
    static inline double area(const double* lo, const double* hi) {      // AABB.swift:29-33
        const double ex = hi[0] - lo[0], ey = hi[1] - lo[1], ez = hi[2] - lo[2];
        return 2.0 * ((ex * ey + ey * ez) + ez * ex);
    }
    // returns bestAxis/bestPos exactly as findBestSplitPlane (BVH.swift:192-250)
    void findBestSplitPlane(int64_t first, int64_t count, int& axis, double& splitPos) {
        double bestCost = kInf;
        const int T = par_chunks(count);
        // centroid bounds (Swift.min/max folds), per chunk then in order
        std::vector<double> cpart(6 * T);
        run_chunks(T, [&](int k) {
            double mn[3] = {kInf, kInf, kInf}, mx[3] = {-kInf, -kInf, -kInf};
            for (int64_t i = count * k / T, e = count * (k + 1) / T; i < e; ++i) {
                const double* c = &P.cen[3 * B.primIdx[first + i]];
                for (int a = 0; a < 3; ++a) { mn[a] = smin(mn[a], c[a]); mx[a] = smax(mx[a], c[a]); }
            }
            for (int a = 0; a < 3; ++a) { cpart[6 * k + a] = mn[a]; cpart[6 * k + 3 + a] = mx[a]; }
        });
        double cmin[3] = {kInf, kInf, kInf}, cmax[3] = {-kInf, -kInf, -kInf};
        for (int k = 0; k < T; ++k)
            for (int a = 0; a < 3; ++a) { cmin[a] = smin(cmin[a], cpart[6 * k + a]); cmax[a] = smax(cmax[a], cpart[6 * k + 3 + a]); }
        bool valid[3];
        double scale[3];
        for (int a = 0; a < 3; ++a) {
            valid[a] = !(cmax[a] <= cmin[a]);
            scale[a] = valid[a] ? double(N) / (cmax[a] - cmin[a]) : 0.0;
        }
        // binning, per chunk into private bins, merged in chunk order
        const int NB = 3 * N;
        std::vector<int64_t> cntP((size_t)T * NB, 0);
        std::vector<double> loP((size_t)T * NB * 3, kInf), hiP((size_t)T * NB * 3, -kInf);
        run_chunks(T, [&](int k) {
            int64_t* bc = &cntP[(size_t)k * NB];
            double* blo = &loP[(size_t)k * NB * 3];
            double* bhi = &hiP[(size_t)k * NB * 3];
            for (int64_t i = count * k / T, e = count * (k + 1) / T; i < e; ++i) {
                const int64_t p = B.primIdx[first + i];
                const double* c = &P.cen[3 * p];
                const double* pl = &P.bmin[3 * p];
                const double* ph = &P.bmax[3 * p];
                for (int a = 0; a < 3; ++a) {
                    if (!valid[a]) continue;
                    int64_t q = (int64_t)((c[a] - cmin[a]) * scale[a]);
                    int64_t idx = (q < (int64_t)(N - 1)) ? q : (int64_t)(N - 1);
                    bc[a * N + idx] += 1;
                    double* bl = &blo[(a * N + idx) * 3];
                    double* bh = &bhi[(a * N + idx) * 3];
                    for (int kk = 0; kk < 3; ++kk) { bl[kk] = std::fmin(bl[kk], pl[kk]); bh[kk] = std::fmax(bh[kk], ph[kk]); }
                }
            }
        });
        for (int b = 0; b < NB; ++b) {
            binCnt[b] = 0;
            for (int kk = 0; kk < 3; ++kk) { binLo[b * 3 + kk] = kInf; binHi[b * 3 + kk] = -kInf; }
            for (int k = 0; k < T; ++k) {
                binCnt[b] += cntP[(size_t)k * NB + b];
                for (int kk = 0; kk < 3; ++kk) {
                    binLo[b * 3 + kk] = std::fmin(binLo[b * 3 + kk], loP[((size_t)k * NB + b) * 3 + kk]);
                    binHi[b * 3 + kk] = std::fmax(binHi[b * 3 + kk], hiP[((size_t)k * NB + b) * 3 + kk]);
                }
            }
        }
        double leftArea[64], rightArea[64];
        int64_t leftCnt[64], rightCnt[64];
        for (int a = 0; a < 3; ++a) {
            if (!valid[a]) continue;
            double Llo[3] = {kInf, kInf, kInf}, Lhi[3] = {-kInf, -kInf, -kInf};
            double Rlo[3] = {kInf, kInf, kInf}, Rhi[3] = {-kInf, -kInf, -kInf};
            int64_t sL = 0, sR = 0;
            for (int i = 0; i < N - 1; ++i) {
                sL += binCnt[a * N + i]; leftCnt[i] = sL;
                for (int k = 0; k < 3; ++k) {
                    Llo[k] = std::fmin(Llo[k], binLo[(a * N + i) * 3 + k]);
                    Lhi[k] = std::fmax(Lhi[k], binHi[(a * N + i) * 3 + k]);
                }
                leftArea[i] = area(Llo, Lhi);
                const int rb = N - 1 - i;
                sR += binCnt[a * N + rb]; rightCnt[N - 2 - i] = sR;
                for (int k = 0; k < 3; ++k) {
                    Rlo[k] = std::fmin(Rlo[k], binLo[(a * N + rb) * 3 + k]);
                    Rhi[k] = std::fmax(Rhi[k], binHi[(a * N + rb) * 3 + k]);
                }
                rightArea[N - 2 - i] = area(Rlo, Rhi);
            }
            const double step = (cmax[a] - cmin[a]) / double(N);
            for (int i = 0; i < N - 1; ++i) {
                if (leftCnt[i] == 0 || rightCnt[i] == 0) continue;
                const double cost = double(leftCnt[i]) * leftArea[i] + double(rightCnt[i]) * rightArea[i];
                if (cost < bestCost) { bestCost = cost; axis = a; splitPos = cmin[a] + step * double(i + 1); }
            }
        }
    }
    // subdivide (BVH.swift:128-188).  Node numbering differs from the reference's
    // depth-first `nodesUsed` counter - nothing downstream sees it (layout and hash walk
    // the structure) - so that subtrees can be built concurrently: the node covering prim
    // range [f, f+c) places its two children at slots D, D+1 and hands its left child the
    // descendant slots [D+2, D+2cl) and its right child [D+2cl, D+2c-2) (a subtree over c
    // prims has at most 2c-2 descendants).  Slot assignment depends only on the ranges,
    // so the result is independent of scheduling.
    void subdivide(int64_t nodeIdx, int64_t D);
};

// Concurrency budget for subtree builds (MYRT_BUILD_THREADS, default: hardware threads).
static std::atomic<int> g_build_slots{-1};
static bool take_build_slot() {
    int cur = g_build_slots.load();
    if (cur < 0) {
        const int n = build_threads() - 1;                            // the calling thread is one
        g_build_slots.compare_exchange_strong(cur, n);
        cur = g_build_slots.load();
    }
    while (cur > 0)
        if (g_build_slots.compare_exchange_weak(cur, cur - 1)) return true;
    return false;
}
static void give_build_slot() { g_build_slots.fetch_add(1); }
constexpr int64_t kParallelSubtree = 16384;   // prims below which a subtree stays on its thread

void Builder::subdivide(int64_t nodeIdx, int64_t D) {
    const int64_t primCount = B.count[nodeIdx];
    if (primCount <= maxLeaf && nodeIdx != 0) return;
    int bestAxis = 0; double bestPos = 0;
    const int64_t first = B.leftFirst[nodeIdx];
    findBestSplitPlane(first, primCount, bestAxis, bestPos);
    int64_t i = first, j = i + primCount - 1;
    while (i <= j) {
        if (P.cen[3 * B.primIdx[i] + bestAxis] < bestPos) i += 1;
        else { std::swap(B.primIdx[i], B.primIdx[j]); j -= 1; }
    }
    const int64_t leftCount = i - first;
    if (leftCount == 0 || leftCount == primCount) return;
    const int64_t leftChild = D;
    const int64_t rightChild = D + 1;
    B.leftFirst[leftChild] = first; B.count[leftChild] = leftCount;
    B.leftFirst[rightChild] = i; B.count[rightChild] = primCount - leftCount;
    B.leftFirst[nodeIdx] = leftChild; B.count[nodeIdx] = 0;
    updateNodeBounds(leftChild);
    updateNodeBounds(rightChild);
    const int64_t dLeft = D + 2, dRight = D + 2 * leftCount;
    if (primCount - leftCount >= kParallelSubtree && take_build_slot()) {
        std::thread t([this, rightChild, dRight] {
            Builder sub(P, B, maxLeaf, N);
            sub.subdivide(rightChild, dRight);
            give_build_slot();
        });
        subdivide(leftChild, dLeft);
        t.join();
    } else {
        subdivide(leftChild, dLeft);
        subdivide(rightChild, dRight);
    }
}
}  // namespace

RefBVH build_ref_bvh(const PrimSet& prims, int maxLeaf, int binCount) {
    RefBVH B;
    const int64_t n = prims.n;
    const int64_t nodeCount = std::max<int64_t>(1, n * 2 - 1);
    B.lo.assign(3 * nodeCount, 0.0); B.hi.assign(3 * nodeCount, 0.0);
    B.leftFirst.assign(nodeCount, 0); B.count.assign(nodeCount, 0);
    B.primIdx.resize(n);
    for (int64_t i = 0; i < n; ++i) B.primIdx[i] = i;
    B.leftFirst[0] = 0; B.count[0] = n; B.nodesUsed = 0;
    Builder bld(prims, B, maxLeaf, binCount);
    bld.updateNodeBounds(0);
    bld.subdivide(0, 1);
    B.nodesUsed = B.count[0] == 0 && n > 0 ? 2 * n - 2 : 0;   // > 0 iff the root was split
    return B;
}

uint64_t ref_bvh_hash(const RefBVH& b, const std::vector<int64_t>& primIndexOf) {
    // Same canonical walk as oracle_bvh_hash (tests compare the two).
    uint64_t h = 1469598103934665603ull;
    auto mix = [&](uint64_t x) { for (int i = 0; i < 8; ++i) { h ^= (x >> (8 * i)) & 0xff; h *= 1099511628211ull; } };
    auto mixd = [&](double d) { uint64_t u; std::memcpy(&u, &d, 8); mix(u); };
    std::vector<int64_t> st{0};
    while (!st.empty()) {
        int64_t i = st.back(); st.pop_back();
        for (int k = 0; k < 3; ++k) mixd(b.lo[3 * i + k]);
        for (int k = 0; k < 3; ++k) mixd(b.hi[3 * i + k]);
        if (b.isLeaf(i)) {
            mix(0xABCDull); mix((uint64_t)b.count[i]);
            for (int64_t q = 0; q < b.count[i]; ++q) mix((uint64_t)primIndexOf[b.primIdx[b.leftFirst[i] + q]]);
        } else {
            mix(0x1234ull);
            st.push_back(b.leftFirst[i] + 1);
            st.push_back(b.leftFirst[i]);
        }
    }
    return h;
}

int64_t ref_bvh_depth(const RefBVH& b) {
    int64_t best = 0;
    std::vector<std::pair<int64_t, int64_t>> st{{0, 0}};
    while (!st.empty()) {
        auto [i, d] = st.back(); st.pop_back();
        if (b.isLeaf(i) || b.count[i] == 0 && b.leftFirst[i] == 0) { best = std::max(best, d); continue; }
        st.push_back({b.leftFirst[i], d + 1});
        st.push_back({b.leftFirst[i] + 1, d + 1});
    }
    return best;
}

// -------------------------------------------------------------- matrices
static void m4_inverse(const double* m, double* out) {   // cofactor inverse (see oracle note)
    double inv[16];
    inv[0] = m[5] * m[10] * m[15] - m[5] * m[11] * m[14] - m[9] * m[6] * m[15] + m[9] * m[7] * m[14] + m[13] * m[6] * m[11] - m[13] * m[7] * m[10];
    inv[4] = -m[4] * m[10] * m[15] + m[4] * m[11] * m[14] + m[8] * m[6] * m[15] - m[8] * m[7] * m[14] - m[12] * m[6] * m[11] + m[12] * m[7] * m[10];
    inv[8] = m[4] * m[9] * m[15] - m[4] * m[11] * m[13] - m[8] * m[5] * m[15] + m[8] * m[7] * m[13] + m[12] * m[5] * m[11] - m[12] * m[7] * m[9];
    inv[12] = -m[4] * m[9] * m[14] + m[4] * m[10] * m[13] + m[8] * m[5] * m[14] - m[8] * m[6] * m[13] - m[12] * m[5] * m[10] + m[12] * m[6] * m[9];
    inv[1] = -m[1] * m[10] * m[15] + m[1] * m[11] * m[14] + m[9] * m[2] * m[15] - m[9] * m[3] * m[14] - m[13] * m[2] * m[11] + m[13] * m[3] * m[10];
    inv[5] = m[0] * m[10] * m[15] - m[0] * m[11] * m[14] - m[8] * m[2] * m[15] + m[8] * m[3] * m[14] + m[12] * m[2] * m[11] - m[12] * m[3] * m[10];
    inv[9] = -m[0] * m[9] * m[15] + m[0] * m[11] * m[13] + m[8] * m[1] * m[15] - m[8] * m[3] * m[13] - m[12] * m[1] * m[11] + m[12] * m[3] * m[9];
    inv[13] = m[0] * m[9] * m[14] - m[0] * m[10] * m[13] - m[8] * m[1] * m[14] + m[8] * m[2] * m[13] + m[12] * m[1] * m[10] - m[12] * m[2] * m[9];
    inv[2] = m[1] * m[6] * m[15] - m[1] * m[7] * m[14] - m[5] * m[2] * m[15] + m[5] * m[3] * m[14] + m[13] * m[2] * m[7] - m[13] * m[3] * m[6];
    inv[6] = -m[0] * m[6] * m[15] + m[0] * m[7] * m[14] + m[4] * m[2] * m[15] - m[4] * m[3] * m[14] - m[12] * m[2] * m[7] + m[12] * m[3] * m[6];
    inv[10] = m[0] * m[5] * m[15] - m[0] * m[7] * m[13] - m[4] * m[1] * m[15] + m[4] * m[3] * m[13] + m[12] * m[1] * m[7] - m[12] * m[3] * m[5];
    inv[14] = -m[0] * m[5] * m[14] + m[0] * m[6] * m[13] + m[4] * m[1] * m[14] - m[4] * m[2] * m[13] - m[12] * m[1] * m[6] + m[12] * m[2] * m[5];
    inv[3] = -m[1] * m[6] * m[11] + m[1] * m[7] * m[10] + m[5] * m[2] * m[11] - m[5] * m[3] * m[10] - m[9] * m[2] * m[7] + m[9] * m[3] * m[6];
    inv[7] = m[0] * m[6] * m[11] - m[0] * m[7] * m[10] - m[4] * m[2] * m[11] + m[4] * m[3] * m[10] + m[8] * m[2] * m[7] - m[8] * m[3] * m[6];
    inv[11] = -m[0] * m[5] * m[11] + m[0] * m[7] * m[9] + m[4] * m[1] * m[11] - m[4] * m[3] * m[9] - m[8] * m[1] * m[7] + m[8] * m[3] * m[5];
    inv[15] = m[0] * m[5] * m[10] - m[0] * m[6] * m[9] - m[4] * m[1] * m[10] + m[4] * m[2] * m[9] + m[8] * m[1] * m[6] - m[8] * m[2] * m[5];
    const double det = m[0] * inv[0] + m[1] * inv[4] + m[2] * inv[8] + m[3] * inv[12];
    for (int i = 0; i < 16; ++i) out[i] = inv[i] / det;
}
static double m3_det_of4(const double* M) {   // simd_determinant of the upper 3x3 (col-major a[c*3+r])
    double a[9];
    for (int c = 0; c < 3; ++c) for (int r = 0; r < 3; ++r) a[c * 3 + r] = M[c * 4 + r];
    return a[0] * (a[4] * a[8] - a[7] * a[5]) - a[3] * (a[1] * a[8] - a[7] * a[2]) + a[6] * (a[1] * a[5] - a[4] * a[2]);
}
static void normal_matrix(const double* M, double* out) {   // normalTransformMatrix (RTContext.swift:23-31)
    auto e = [&](int r, int c) { return M[c * 4 + r]; };
    const double det = m3_det_of4(M);
    double cof[3][3];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) {
            int r1 = (r + 1) % 3, r2 = (r + 2) % 3, c1 = (c + 1) % 3, c2 = (c + 2) % 3;
            cof[r][c] = e(r1, c1) * e(r2, c2) - e(r1, c2) * e(r2, c1);
        }
    double inv[9];   // inv (r,c) col-major
    for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) inv[c * 3 + r] = cof[c][r] / det;
    for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) out[c * 3 + r] = inv[r * 3 + c];   // transpose
}
// AABB.transformed(by:) (AABB.swift:71-92)
static void aabb_transformed(const double* lo, const double* hi, const double* M, double* olo, double* ohi) {
    const D3 mn = d3(lo[0], lo[1], lo[2]), mx = d3(hi[0], hi[1], hi[2]);
    const D3 cOld = 0.5 * (mn + mx);
    const D3 eOld = 0.5 * (mx - mn);
    D3 rc;
    {
        double o[3];
        for (int r = 0; r < 3; ++r) {
            double acc = M[0 * 4 + r] * cOld.x;
            acc = M[1 * 4 + r] * cOld.y + acc;
            acc = M[2 * 4 + r] * cOld.z + acc;
            o[r] = acc;
        }
        rc = d3(o[0], o[1], o[2]);
    }
    const D3 cNew = rc + d3(M[12], M[13], M[14]);
    double ar[9];
    for (int c = 0; c < 3; ++c) for (int r = 0; r < 3; ++r) ar[c * 3 + r] = std::fabs(M[c * 4 + r]);
    const D3 eNew = d3(ar[0] * eOld.x + ar[3] * eOld.y + ar[6] * eOld.z,
                       ar[1] * eOld.x + ar[4] * eOld.y + ar[7] * eOld.z,
                       ar[2] * eOld.x + ar[5] * eOld.y + ar[8] * eOld.z);
    const D3 a = cNew - eNew, b = cNew + eNew;
    olo[0] = a.x; olo[1] = a.y; olo[2] = a.z;
    ohi[0] = b.x; ohi[1] = b.y; ohi[2] = b.z;
}

// ------------------------------------------------------------ scene flattening
namespace {
struct Tri { D3 v0, v1, v2, e1, e2, n0, n1, n2; };
struct BlasBuild {
    std::vector<int64_t> triIndex;   // subset prims -> global triangle index
    PrimSet prims;
    RefBVH bvh;
    bool smooth = false;
    int32_t kind = kPrimTriangles;   // kPrimSphere / kPrimPlane: one primitive, bounds pmin/pmax
    D3 pmin{0, 0, 0}, pmax{0, 0, 0};
    D3 motion{0, 0, 0};
    uint64_t hash = 0;
    int64_t depth = 0;
    // filled by layout
    int32_t root_ref = 0;
    int64_t tri_first = 0, tri_end = 0;   // run of this BLAS's TriRecs in HostScene::tris
    double root_lo[3], root_hi[3];
};
struct InstBuild { int blas; double M[16]; int material; D3 motion; double wlo[3], whi[3]; };
}  // namespace

// Lay one reference-form BVH out as WRec records.  Inner nodes get records in DFS
// preorder (near-left first); each leaf's primitives become a contiguous run of
// entries produced by `emit_leaf(first_prim_slot, count)` which returns the index of
// the run's first entry.  Returns the root ref.
// With topRecords > 0 the first min(topRecords, inner nodes) records are the inner nodes
// nearest the root in breadth-first order (the near-root records every ray reads sit in a
// few adjacent lines); the rest follow in preorder.  Record numbering is free: traversal
// order depends only on the tree.
template <class EmitLeaf>
static int32_t layout_bvh(const RefBVH& b, std::vector<WRec>& recs, EmitLeaf emit_leaf, int64_t topRecords = 0) {
    if (b.isLeaf(0) || (b.count[0] == 0 && b.nodesUsed == 0)) {
        const int64_t first = emit_leaf(b.leftFirst[0], b.count[0]);
        return ~(int32_t)first;
    }
    std::vector<int64_t> recOf(b.leftFirst.size(), -1);
    std::vector<int64_t> order;
    if (topRecords > 0) {                                  // breadth-first prefix
        recOf[0] = (int64_t)recs.size();
        order.push_back(0);
        for (size_t q = 0; q < order.size() && (int64_t)order.size() < topRecords; ++q) {
            const int64_t i = order[q];
            for (int64_t c : {b.leftFirst[i], b.leftFirst[i] + 1}) {
                if (b.isLeaf(c) || (int64_t)order.size() >= topRecords) continue;
                recOf[c] = (int64_t)recs.size() + (int64_t)order.size();
                order.push_back(c);
            }
        }
    }
    // the rest in preorder
    std::vector<int64_t> st{0};
    while (!st.empty()) {
        int64_t i = st.back(); st.pop_back();
        if (recOf[i] < 0) {
            recOf[i] = (int64_t)recs.size() + (int64_t)order.size();
            order.push_back(i);
        }
        const int64_t L = b.leftFirst[i], R = L + 1;
        if (!b.isLeaf(R)) st.push_back(R);
        if (!b.isLeaf(L)) st.push_back(L);
    }
    const int64_t base = (int64_t)recs.size();
    recs.resize(base + order.size());
    // leaves are emitted in DFS order of the traversal (left before right)
    for (size_t q = 0; q < order.size(); ++q) {
        const int64_t i = order[q];
        WRec& r = recs[base + q];
        std::memset(&r, 0, sizeof(WRec));
        const int64_t ch[2] = {b.leftFirst[i], b.leftFirst[i] + 1};
        for (int c = 0; c < 2; ++c) {
            for (int k = 0; k < 3; ++k) { r.lo[c][k] = b.lo[3 * ch[c] + k]; r.hi[c][k] = b.hi[3 * ch[c] + k]; }
        }
    }
    // leaf runs: walk preorder so runs are laid out in traversal order
    std::vector<int64_t> st2{0};
    while (!st2.empty()) {
        int64_t i = st2.back(); st2.pop_back();
        WRec& r = recs[recOf[i]];
        const int64_t ch[2] = {b.leftFirst[i], b.leftFirst[i] + 1};
        for (int c = 0; c < 2; ++c) {
            if (b.isLeaf(ch[c])) {
                const int64_t first = emit_leaf(b.leftFirst[ch[c]], b.count[ch[c]]);
                r.ref[c] = ~(int32_t)first;
            } else {
                r.ref[c] = (int32_t)recOf[ch[c]];
            }
        }
        if (!b.isLeaf(ch[1])) st2.push_back(ch[1]);
        if (!b.isLeaf(ch[0])) st2.push_back(ch[0]);
    }
    return (int32_t)recOf[0];
}

// ------------------------------------------------------------ conservative four-wide tree
// Identity scenes: the unified TLAS + BLAS tree (TLAS inner records, TLAS leaves = their
// instances' BLAS roots, BLAS inner records, BLAS leaf runs) collapsed into W4Nodes (layout.h).
// A node starts from one tree node's children and repeatedly opens the child with the largest
// surface area while the children fit four slots (the usual BVH2 -> BVH4 collapse); a TLAS leaf
// with more than four instances is grouped.  Every reference leaf run becomes exactly one slot,
// and its exact FP64 box is kept in lbox for the walk's exact check (wide.h).  Slot order keeps
// the tree's left-to-right order.
namespace {
struct WItem {
    double lo[3], hi[3];
    int32_t ref;        // a tree ref (records / TLAS leaf / BLAS leaf run), unless group >= 0
    int32_t group;      // >= 0: a synthetic group of items (wide groups)
};
struct WideBuilder {
    HostScene& S;
    std::vector<std::vector<WItem>> groups;
    int depth = 0, max_depth = 0;        // wide levels on the current path / deepest
    // transformed scenes (build_wide_tw): a TLAS leaf expands to one marker per instance, carrying
    // the leaf's box, instead of its instances' BLAS roots; BLASes are built on their own
    bool tw = false;
    int64_t marker_base = 0;             // markers are ~(marker_base + instance) (render.hip ut_marker_base)
    double coord = 0.0;                  // largest |coordinate| of the boxes of the current build
    explicit WideBuilder(HostScene& s) : S(s), marker_base(s.tlas_leaf_base + (int64_t)s.tlas_leaf.size()) {}
    bool terminal(const WItem& x) const {
        if (x.group >= 0 || x.ref >= 0) return false;
        const int64_t e = ~(int64_t)x.ref;
        return e < S.tlas_leaf_base || (tw && e >= marker_base);
    }
    static double area(const WItem& x) {
        const double dx = x.hi[0] - x.lo[0], dy = x.hi[1] - x.lo[1], dz = x.hi[2] - x.lo[2];
        return dx * dy + dy * dz + dz * dx;
    }
    std::vector<WItem> expand(const WItem& x) const {
        std::vector<WItem> out;
        if (x.group >= 0) return groups[x.group];
        if (x.ref >= 0) {
            const WRec& r = S.recs[x.ref];
            for (int c = 0; c < 2; ++c) {
                WItem w{};
                for (int k = 0; k < 3; ++k) { w.lo[k] = r.lo[c][k]; w.hi[k] = r.hi[c][k]; }
                w.ref = r.ref[c];
                w.group = -1;
                out.push_back(w);
            }
            return out;
        }
        for (int64_t e = (int64_t)~x.ref - S.tlas_leaf_base;; ++e) {      // TLAS leaf: instance roots
            const DInstance& I = S.insts[S.tlas_leaf[e].inst];
            WItem w{};
            if (tw) {                                    // transformed: a marker with the leaf's box
                for (int k = 0; k < 3; ++k) { w.lo[k] = x.lo[k]; w.hi[k] = x.hi[k]; }
                w.ref = (int32_t)~(marker_base + S.tlas_leaf[e].inst);
            } else {
                for (int k = 0; k < 3; ++k) { w.lo[k] = I.root_lo[k]; w.hi[k] = I.root_hi[k]; }
                w.ref = I.root_ref;
            }
            w.group = -1;
            out.push_back(w);
            if (S.tlas_leaf[e].last) break;
        }
        return out;
    }
    size_t expand_count(const WItem& x) const {
        if (x.group >= 0) return groups[x.group].size();
        if (x.ref >= 0) return 2;
        size_t n = 0;
        for (int64_t e = (int64_t)~x.ref - S.tlas_leaf_base;; ++e) { ++n; if (S.tlas_leaf[e].last) break; }
        return n;
    }
    // more than four items: four consecutive groups
    std::vector<WItem> regroup(const std::vector<WItem>& c) {
        if (c.size() <= 4) return c;
        std::vector<WItem> out;
        const size_t n = c.size();
        for (size_t g = 0; g < 4; ++g) {
            const size_t a = n * g / 4, b = n * (g + 1) / 4;
            if (a == b) continue;
            if (b - a == 1) { out.push_back(c[a]); continue; }
            WItem w{};
            for (int k = 0; k < 3; ++k) { w.lo[k] = kInf; w.hi[k] = -kInf; }
            std::vector<WItem> part(c.begin() + a, c.begin() + b);
            for (const WItem& x : part)
                for (int k = 0; k < 3; ++k) { w.lo[k] = std::fmin(w.lo[k], x.lo[k]); w.hi[k] = std::fmax(w.hi[k], x.hi[k]); }
            w.ref = 0;
            w.group = (int32_t)groups.size();
            groups.push_back(std::move(part));
            out.push_back(w);
        }
        return out;
    }
    static float down(double x) {
        float f = (float)x;
        if ((double)f > x) f = std::nextafter(f, -HUGE_VALF);
        return f;
    }
    static float up(double x) {
        float f = (float)x;
        if ((double)f < x) f = std::nextafter(f, HUGE_VALF);
        return f;
    }
    int32_t build(const WItem& x) {
        std::vector<WItem> c = regroup(expand(x));
        for (;;) {                                       // open the largest child that still fits
            int best = -1;
            double bestA = -1.0;
            for (size_t i = 0; i < c.size(); ++i) {
                if (terminal(c[i])) continue;
                if (c.size() - 1 + expand_count(c[i]) > 4) continue;
                const double a = area(c[i]);
                if (a > bestA) { bestA = a; best = (int)i; }
            }
            if (best < 0) break;
            const std::vector<WItem> e = expand(c[best]);
            c.erase(c.begin() + best);
            c.insert(c.begin() + best, e.begin(), e.end());
        }
        const int32_t idx = (int32_t)S.wnodes.size();
        S.wnodes.emplace_back();
        max_depth = std::max(max_depth, ++depth);
        int32_t refs[4] = {0, 0, 0, 0};
        for (size_t i = 0; i < c.size(); ++i) {
            if (terminal(c[i])) {
                refs[i] = c[i].ref;
                const int64_t e = ~(int64_t)c[i].ref;
                double* b = e < S.tlas_leaf_base ? &S.lbox[6 * (size_t)e]                 // leaf run
                                                 : S.winst[(size_t)(e - marker_base)].tbox;   // marker
                for (int k = 0; k < 3; ++k) { b[k] = c[i].lo[k]; b[3 + k] = c[i].hi[k]; }
                if (e < S.tlas_leaf_base) S.wide_leaves++;
            } else {
                refs[i] = build(c[i]);                   // preorder: children follow their parent
            }
        }
        W4Node& n = S.wnodes[idx];                       // octant 0's copy: near = lo, far = hi
        std::memset(&n, 0, sizeof(n));
        for (int s = 0; s < 4; ++s) {
            for (int k = 0; k < 3; ++k) {
                if (s < (int)c.size()) {
                    n.pnear[k][s] = down(c[s].lo[k]);
                    n.pfar[k][s] = up(c[s].hi[k]);
                    coord = std::fmax(coord, std::fmax(std::fabs(c[s].lo[k]), std::fabs(c[s].hi[k])));
                } else {
                    n.pnear[k][s] = HUGE_VALF;           // empty slot: never hit (wide.h)
                    n.pfar[k][s] = HUGE_VALF;
                }
            }
            n.ref[s] = refs[s];
        }
        --depth;
        return idx;
    }
};
}  // namespace

// The eight octant copies of the four-wide tree (layout.h W4Node).  Copy o (bit a set: rays with
// d[a] < 0) holds each node with the rows of that octant's near planes first (the box maximum
// along a when d[a] < 0) and its slots sorted front to back for such rays: by the projection of
// each slot box's centre on the octant's diagonal (+-1, +-1, +-1), empty slots last, ties in
// slot order (measured on C3: centres 8,700 Mrays/s, near corners 8,567, slot order 6,105;
// profiles/r05b_ab_c3.txt).  The walk then continues with the first slot hit and pushes the others in reverse
// (wide.h), which replaces the per-node distance sort.  Exactness does not depend on the order
// (wide.h header: only equal-t candidates depend on it, and those are re-walked in the
// reference's order).  -DMYRT_WIDE_ORDER (compile-time measurement switch, like the other MYRT_*
// build switches; the product reads no environment variable here): 1 = near corners instead of
// centres, 2 = slot order kept.
#ifndef MYRT_WIDE_ORDER
#define MYRT_WIDE_ORDER 0
#endif
static void wide_octant_copies(HostScene& S) {
    const size_t N = S.wnodes.size();
    constexpr int mode = MYRT_WIDE_ORDER;
    std::vector<W4Node> out(8 * N);
    const std::vector<W4Node>& in = S.wnodes;
    run_chunks(std::min(8, build_threads()), [&](int k) {
        const int T = std::min(8, build_threads());
        for (size_t x = (size_t)k; x < 8 * N; x += (size_t)T) {
            const int o = (int)(x / N);
            const W4Node& a = in[x % N];
            W4Node& w = out[x];
            std::memset(&w, 0, sizeof(w));
            double key[4];
            int perm[4] = {0, 1, 2, 3};
            for (int c = 0; c < 4; ++c) {
                if (!(a.pnear[0][c] < HUGE_VALF)) { key[c] = HUGE_VAL; continue; }
                double proj = 0.0;
                for (int ax = 0; ax < 3; ++ax) {
                    const bool neg = (o >> ax) & 1;
                    const double lo = a.pnear[ax][c], hi = a.pfar[ax][c];
                    proj += mode == 1 ? (neg ? -hi : lo) : (neg ? -0.5 : 0.5) * (lo + hi);
                }
                key[c] = mode == 2 ? (double)c : proj;
            }
            std::stable_sort(perm, perm + 4, [&](int p, int q) { return key[p] < key[q]; });
            for (int i = 0; i < 4; ++i) {
                const int c = perm[i];
                for (int ax = 0; ax < 3; ++ax) {
                    const bool neg = (o >> ax) & 1;
                    w.pnear[ax][i] = neg ? a.pfar[ax][c] : a.pnear[ax][c];
                    w.pfar[ax][i] = neg ? a.pnear[ax][c] : a.pfar[ax][c];
                }
                w.ref[i] = a.ref[c];
            }
        }
    });
    S.wnodes.swap(out);
    S.wide_copy = (int64_t)N;
}

static void build_wide(HostScene& S) {
    S.wnodes.clear();
    S.lbox.clear();
    S.wide_root = -1;
    S.wide_leaves = 0;
    S.wide_coord = 0.0;
    // The widening bound (render.hip set_wide, wide.h header) needs every ray origin of a render
    // to lie within wide_coord (the boxes' largest coordinate) or the camera's reach: hit points
    // on triangles do, hit points on an unbounded plane or a sphere outside the triangle boxes
    // would not.  So the four-wide tree exists only for triangle-only scenes.
    if (S.has_special) return;
    S.lbox.assign(6 * S.tris.size(), 0.0);
    WideBuilder B(S);
    WItem root{};
    for (int k = 0; k < 3; ++k) { root.lo[k] = S.tlas_root_lo[k]; root.hi[k] = S.tlas_root_hi[k]; }
    root.ref = S.tlas_root_ref;
    root.group = -1;
    if (B.terminal(root)) { S.wnodes.clear(); S.lbox.clear(); S.wide_root = -1; return; }
    S.wnodes.reserve(S.recs.size() / 2 + 16);
    S.wide_root = B.build(root);
    S.wide_coord = B.coord;
    // a walk holds at most three deferred slots per wide level on its path (plus slack): it must
    // fit the device stack (device.h Stack, kStackCap), else the binary walk
    // (and the walk addresses nodes by 32-bit byte offsets: the array must stay below 4 GB)
    // (the eight octant copies included)
    if (!std::isfinite(S.wide_coord) || 3 * (int64_t)B.max_depth + 2 > kStackCap ||
        8 * S.wnodes.size() * sizeof(W4Node) >= (size_t(1) << 32)) {
        S.wnodes.clear(); S.lbox.clear(); S.wide_root = -1;
        return;
    }
    wide_octant_copies(S);
}

// Flattened instance tree (transformed scenes; wide.h fit_walk).  One four-wide tree in WORLD
// space over every (instance, BLAS leaf run) pair - the reference's binned SAH builder over the
// pairs' world boxes, collapsed to four-wide nodes like C3's tree - so that the terrain's leaves
// and the sphere instances' leaves interleave in one walk as an identity scene's do.  A pair's
// box is AABB.transformed (AABB.swift:71-92) of its local leaf box: the eight corners through
// localToWorld, min/max.  The walk tests the reference's boxes exactly (FP64) before it accepts a
// candidate: the instance's TLAS leaf box with the world ray, its BLAS root box and the leaf box
// with the local ray (RTContext.swift:632-673, 567-571), so the tree only has to be a superset
// filter: a triangle the reference tests lies in a pair whose world box the walk enters (wide.h
// fit_walk header: the widening covers the world <-> local rounding while the transforms'
// condition number stays below kFitKappa; above it the scene keeps tw_walk only).
constexpr double kFitKappa = 4096.0;
static double m3_inf_norm(const double* M) {      // column-major 4x4: the 3x3 part's max row sum
    double n = 0.0;
    for (int r = 0; r < 3; ++r) n = std::fmax(n, std::fabs(M[r]) + std::fabs(M[4 + r]) + std::fabs(M[8 + r]));
    return n;
}
// min / max of the builder's finite values: plain compares (std::fmin/fmax are libm calls here)
static inline double fmn(double a, double b) { return b < a ? b : a; }
static inline double fmx(double a, double b) { return b > a ? b : a; }
static void build_fit(HostScene& S) {
    const auto t_start = std::chrono::steady_clock::now();
    S.fpairs.clear(); S.fit_root = -1; S.fit_nodes = 0; S.fit_depth = 0; S.fit_coord = 0.0;
    struct Item { double lo[3], hi[3], c[3]; int32_t t0, inst; };
    std::vector<Item> items;
    double coord = 0.0;
    // leaf runs of each BLAS (local boxes), by BLAS root ref
    std::vector<std::pair<int32_t, std::vector<Item>>> leaves;
    for (size_t k = 0; k < S.insts.size(); ++k) {
        const DInstance& I = S.insts[k];
        const double ka = m3_inf_norm(I.l2w) * m3_inf_norm(I.w2l);
        if (!(ka <= kFitKappa)) return;
        const std::vector<Item>* L = nullptr;
        for (const auto& x : leaves) if (x.first == I.root_ref) { L = &x.second; break; }
        if (!L) {
            std::vector<Item> out;
            auto leaf = [&](int32_t ref, const double* lo, const double* hi) {
                Item it{};
                for (int a = 0; a < 3; ++a) { it.lo[a] = lo[a]; it.hi[a] = hi[a]; }
                it.t0 = ~ref;
                out.push_back(it);
            };
            if (I.root_ref < 0) {
                leaf(I.root_ref, I.root_lo, I.root_hi);
            } else {
                std::vector<int32_t> st{I.root_ref};
                while (!st.empty()) {
                    const WRec& r = S.recs[st.back()];
                    st.pop_back();
                    for (int c = 0; c < 2; ++c) {
                        if (r.ref[c] < 0) leaf(r.ref[c], r.lo[c], r.hi[c]);
                        else st.push_back(r.ref[c]);
                    }
                }
            }
            leaves.push_back({I.root_ref, std::move(out)});
            L = &leaves.back().second;
        }
        const double nl = m3_inf_norm(I.l2w);
        for (int a = 0; a < 3; ++a) coord = fmx(coord, std::fabs(I.l2w[12 + a]));
        for (const Item& x : *L) {
            Item w{};
            w.t0 = x.t0;
            w.inst = (int32_t)k;
            for (int a = 0; a < 3; ++a) { w.lo[a] = kInf; w.hi[a] = -kInf; }
            double lc = 0.0;
            for (int q = 0; q < 8; ++q) {
                const double p[3] = {(q & 1) ? x.hi[0] : x.lo[0], (q & 2) ? x.hi[1] : x.lo[1], (q & 4) ? x.hi[2] : x.lo[2]};
                for (int a = 0; a < 3; ++a) {
                    lc = fmx(lc, std::fabs(p[a]));
                    const double v = I.l2w[a] * p[0] + I.l2w[4 + a] * p[1] + I.l2w[8 + a] * p[2] + I.l2w[12 + a];
                    w.lo[a] = fmn(w.lo[a], v);
                    w.hi[a] = fmx(w.hi[a], v);
                }
            }
            coord = fmx(coord, nl * lc);
            for (int a = 0; a < 3; ++a) {
                coord = fmx(coord, fmx(std::fabs(w.lo[a]), std::fabs(w.hi[a])));
                w.c[a] = 0.5 * w.lo[a] + 0.5 * w.hi[a];
            }
            items.push_back(w);
        }
    }
    if (items.empty() || !std::isfinite(coord) || items.size() >= (size_t(1) << 30)) return;
    // A subtree: its nodes in preorder (node refs local to `nodes`, terminal slots ~index into `pairs`)
    struct FitOut {
        std::vector<W4Node> nodes;
        std::vector<DFitPair> pairs;
        int64_t depth = 0;
    };
    if (items.size() < 2) return;                        // one pair alone: tw_walk
    FitOut out;
    {
        // The reference's binned SAH builder (build_ref_bvh, BVH.swift:128-250) over the pairs'
        // world boxes, collapsed to four-wide nodes as build_wide collapses C3's tree: a node opens
        // its largest child while the children fit four slots; every pair is one terminal slot.
        // (A direct four-way binned SAH - split in two, each half in two - ran C3i 1 % slower:
        // profiles/r06o_ab_c3i_fit_builder.txt.)
        PrimSet ps;
        ps.n = (int64_t)items.size();
        ps.bmin.resize(3 * items.size()); ps.bmax.resize(3 * items.size()); ps.cen.resize(3 * items.size());
        for (size_t i = 0; i < items.size(); ++i)
            for (int y = 0; y < 3; ++y) {
                ps.bmin[3 * i + y] = items[i].lo[y];
                ps.bmax[3 * i + y] = items[i].hi[y];
                ps.cen[3 * i + y] = items[i].c[y];
            }
        const RefBVH B = build_ref_bvh(ps, 2, 12);
        // a slot: a BVH node (>= 0) or a pair (~index into items)
        auto area = [&](int64_t r) {
            const double* lo = r >= 0 ? &B.lo[3 * r] : items[~r].lo;
            const double* hi = r >= 0 ? &B.hi[3 * r] : items[~r].hi;
            const double dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
            return dx * dy + dy * dz + dz * dx;
        };
        auto expand = [&](int64_t r, std::vector<int64_t>& o) {
            if (B.isLeaf(r)) {
                for (int64_t q = 0; q < B.count[r]; ++q) o.push_back(~B.primIdx[B.leftFirst[r] + q]);
            } else {
                o.push_back(B.leftFirst[r]);
                o.push_back(B.leftFirst[r] + 1);
            }
        };
        auto size_of = [&](int64_t r) { return B.isLeaf(r) ? B.count[r] : 2; };
        auto term = [&](int64_t r) { return r < 0 || (B.isLeaf(r) && B.count[r] == 1); };
        std::function<void(int64_t, int64_t)> coll = [&](int64_t r, int64_t depth) {
            out.depth = std::max(out.depth, depth);
            std::vector<int64_t> c;
            expand(r, c);
            for (;;) {
                int best = -1;
                double bestA = -1.0;
                for (size_t i = 0; i < c.size(); ++i) {
                    if (term(c[i]) || c.size() - 1 + (size_t)size_of(c[i]) > 4) continue;
                    const double ar = area(c[i]);
                    if (ar > bestA) { bestA = ar; best = (int)i; }
                }
                if (best < 0) break;
                std::vector<int64_t> e;
                expand(c[best], e);
                c.erase(c.begin() + best);
                c.insert(c.begin() + best, e.begin(), e.end());
            }
            const size_t idx = out.nodes.size();
            out.nodes.emplace_back();
            int32_t refs[4] = {0, 0, 0, 0};
            for (size_t i = 0; i < c.size(); ++i) {
                if (term(c[i])) {
                    const int64_t pi = c[i] < 0 ? ~c[i] : B.primIdx[B.leftFirst[c[i]]];
                    refs[i] = ~(int32_t)out.pairs.size();
                    out.pairs.push_back({items[pi].t0, items[pi].inst});
                } else {
                    refs[i] = (int32_t)out.nodes.size();
                    coll(c[i], depth + 1);
                }
            }
            W4Node& n = out.nodes[idx];
            std::memset(&n, 0, sizeof(n));
            for (int q = 0; q < 4; ++q) {
                const bool has = q < (int)c.size();
                const double* lo = !has ? nullptr : c[q] >= 0 ? &B.lo[3 * c[q]] : items[~c[q]].lo;
                const double* hi = !has ? nullptr : c[q] >= 0 ? &B.hi[3 * c[q]] : items[~c[q]].hi;
                for (int y = 0; y < 3; ++y) {
                    n.pnear[y][q] = has ? WideBuilder::down(lo[y]) : HUGE_VALF;
                    n.pfar[y][q] = has ? WideBuilder::up(hi[y]) : HUGE_VALF;
                }
                n.ref[q] = refs[q];
            }
        };
        out.nodes.reserve(items.size() / 2 + 4);
        coll(0, 1);
    }
    if (3 * out.depth + 2 > kStackCap) return;
    const int64_t node_base = (int64_t)S.wnodes.size();
    for (W4Node n : out.nodes) {                         // node refs relative to the whole array
        for (int q = 0; q < 4; ++q)
            if (n.pnear[0][q] < HUGE_VALF && n.ref[q] >= 0) n.ref[q] += (int32_t)node_base;
        S.wnodes.push_back(n);
    }
    S.fpairs = std::move(out.pairs);
    S.fit_root = (int32_t)node_base;
    S.fit_nodes = (int64_t)out.nodes.size();
    S.fit_depth = out.depth;
    S.fit_coord = coord;
    S.fit_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
}

// Transformed scenes (instances with transforms; static, triangles only): the TLAS collapsed
// into four-wide nodes whose terminal slots are instance markers carrying their TLAS leaf's box
// (world space), and every BLAS collapsed on its own (local space; instances of one mesh share
// it).  The walk (wide.h tw_walk) enters an instance at its marker: the exact FP64 tests of the
// TLAS leaf box (world ray) and the BLAS root box (local ray) the reference does there
// (RTContext.swift:632-673, 567-571), then the BLAS's nodes with the instance's local ray.
static void build_wide_tw(HostScene& S) {
    S.wnodes.clear(); S.lbox.clear(); S.winst.clear();
    S.wide_root = -1; S.wide_leaves = 0; S.wide_coord = 0.0; S.tw_tlas_nodes = 0;
    S.fpairs.clear(); S.fit_root = -1; S.fit_nodes = 0; S.fit_depth = 0; S.fit_coord = 0.0;
    if (S.has_special || !S.has_tlas || S.max_motion != 0.0 || S.insts.empty()) return;
    for (const DInstance& I : S.insts)
        if (I.kind != kPrimTriangles) return;
    S.lbox.assign(6 * S.tris.size(), 0.0);
    S.winst.assign(S.insts.size(), DWideInst{});
    WideBuilder B(S);
    B.tw = true;
    WItem root{};
    for (int k = 0; k < 3; ++k) { root.lo[k] = S.tlas_root_lo[k]; root.hi[k] = S.tlas_root_hi[k]; }
    root.ref = S.tlas_root_ref;
    root.group = -1;
    S.wnodes.reserve(S.recs.size() / 2 + 16);
    S.wide_root = B.build(root);
    S.wide_coord = B.coord;
    S.tw_tlas_nodes = (int64_t)S.wnodes.size();
    const int tlas_depth = B.max_depth;
    B.max_depth = 0;
    std::vector<std::pair<int32_t, std::pair<int32_t, double>>> built;   // BLAS root ref -> (wide root, coord)
    for (size_t k = 0; k < S.insts.size(); ++k) {
        const DInstance& I = S.insts[k];
        int32_t wr = 0;
        double bc = 0.0;
        bool found = false;
        for (const auto& x : built)
            if (x.first == I.root_ref) { wr = x.second.first; bc = x.second.second; found = true; break; }
        if (!found) {
            WItem b{};
            for (int a = 0; a < 3; ++a) { b.lo[a] = I.root_lo[a]; b.hi[a] = I.root_hi[a]; }
            b.ref = I.root_ref;
            b.group = -1;
            B.coord = 0.0;
            for (int a = 0; a < 3; ++a) B.coord = std::fmax(B.coord, std::fmax(std::fabs(b.lo[a]), std::fabs(b.hi[a])));
            if (B.terminal(b)) {                         // a BLAS of one leaf run
                double* lb = &S.lbox[6 * (size_t)~b.ref];
                for (int a = 0; a < 3; ++a) { lb[a] = b.lo[a]; lb[3 + a] = b.hi[a]; }
                S.wide_leaves++;
                wr = b.ref;
            } else {
                wr = B.build(b);
            }
            bc = B.coord;
            built.push_back({I.root_ref, {wr, bc}});
        }
        S.winst[k].wroot = wr;
        S.winst[k].bcoord = bc;
    }
    // deepest walk: three deferred slots per wide level on the TLAS path and on the BLAS path,
    // plus slack; 32-bit byte offsets over the eight copies
    if (!std::isfinite(S.wide_coord) || 3 * (int64_t)(tlas_depth + B.max_depth) + 4 > kStackCap ||
        8 * S.wnodes.size() * sizeof(W4Node) >= (size_t(1) << 32)) {
        S.wnodes.clear(); S.lbox.clear(); S.winst.clear(); S.wide_root = -1; S.tw_tlas_nodes = 0;
        return;
    }
    for (const DWideInst& W : S.winst)
        if (!std::isfinite(W.bcoord)) { S.wnodes.clear(); S.lbox.clear(); S.winst.clear(); S.wide_root = -1; return; }
    build_fit(S);
    if (8 * S.wnodes.size() * sizeof(W4Node) >= (size_t(1) << 32)) {   // no room for the fit nodes
        S.wnodes.resize(S.wnodes.size() - (size_t)S.fit_nodes);
        S.fpairs.clear(); S.fit_root = -1; S.fit_nodes = 0;
    }
    wide_octant_copies(S);
}

int32_t build_host_scene(const rt_scene_desc* d, HostScene& S, std::string& err) {
    auto t0 = std::chrono::steady_clock::now();
    const bool trace = std::getenv("MYRT_BUILD_TRACE") != nullptr;   // phase timings on stderr
    auto phase = [&](const char* name) {
        if (trace) std::fprintf(stderr, "[build] %-10s %9.1f ms\n", name,
                                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    };
    S.eps = d->intersection_test_epsilon;
    S.shadow_eps = d->shadow_ray_epsilon;
    S.background[0] = d->background_color.x; S.background[1] = d->background_color.y; S.background[2] = d->background_color.z;
    S.ambient[0] = d->ambient_light.x; S.ambient[1] = d->ambient_light.y; S.ambient[2] = d->ambient_light.z;
    S.max_depth = d->max_recursion_depth;
    if (d->num_materials < 0 || (d->num_materials > 0 && !d->materials)) { err = "bad materials"; return RT_ERR_INVALID_ARG; }
    for (int i = 0; i < d->num_materials; ++i) {
        const rt_material& m = d->materials[i];
        DMaterial dm{};
        const rt_vec3* src[5] = {&m.ambient, &m.diffuse, &m.specular, &m.mirror, &m.absorption};
        double* dst[5] = {dm.ambient, dm.diffuse, dm.specular, dm.mirror, dm.absorption};
        for (int k = 0; k < 5; ++k) { dst[k][0] = src[k]->x; dst[k][1] = src[k]->y; dst[k][2] = src[k]->z; }
        dm.phong = m.phong; dm.ior = m.ior; dm.absorption_index = m.absorption_index; dm.roughness = m.roughness;
        dm.type = m.type;
        S.mats.push_back(dm);
    }
    for (int i = 0; i < d->num_point_lights; ++i) {
        DPointLight l{};
        l.position[0] = d->point_lights[i].position.x; l.position[1] = d->point_lights[i].position.y; l.position[2] = d->point_lights[i].position.z;
        l.intensity[0] = d->point_lights[i].intensity.x; l.intensity[1] = d->point_lights[i].intensity.y; l.intensity[2] = d->point_lights[i].intensity.z;
        S.plights.push_back(l);
    }
    S.num_area_lights = d->num_area_lights;
    for (int i = 0; i < d->num_area_lights; ++i) {
        const rt_area_light& a = d->area_lights[i];
        DAreaLight l{};
        l.position[0] = a.position.x; l.position[1] = a.position.y; l.position[2] = a.position.z;
        l.normal[0] = a.normal.x; l.normal[1] = a.normal.y; l.normal[2] = a.normal.z;
        l.radiance[0] = a.radiance.x; l.radiance[1] = a.radiance.y; l.radiance[2] = a.radiance.z;
        l.size = a.size;
        S.alights.push_back(l);
    }
    {   // buildStratifiedJitter (Object+Extension.swift:92-93, 646-659): PCG32(0x123456789ABCDEF),
        // cell (gx, gy) row-major, x draw then y draw
        uint64_t state = 0, inc = (0x123456789ABCDEFull << 1) | 1u;
        auto next = [&]() -> uint32_t {
            const uint64_t old = state;
            state = old * 6364136223846793005ull + inc;
            const uint32_t xs = (uint32_t)(((old >> 18) ^ old) >> 27);
            const uint32_t rot = (uint32_t)(old >> 59);
            return (xs >> rot) | (xs << ((~rot + 1u) & 31u));
        };
        next();
        state += 0x9E3779B97F4A7C15ull;
        next();
        S.jitter.assign(2 * kJitterCells, 0.0);
        int q = 0;
        for (int gy = 0; gy < 10; ++gy)
            for (int gx = 0; gx < 10; ++gx, ++q) {
                S.jitter[q] = (double)gx + (double)next() * 2.3283064365386963e-10;
                S.jitter[kJitterCells + q] = (double)gy + (double)next() * 2.3283064365386963e-10;
            }
    }
    for (int i = 0; i < d->num_cameras; ++i) S.cams.push_back(d->cameras[i]);

    // ---- flatten objects (RTContext.swift:120-378)
    std::vector<Tri> triangles;
    std::vector<BlasBuild> blases;
    std::vector<InstBuild> insts;
    struct Base { int blas; int material; double M[16]; };
    std::map<int, Base> instanceByID;
    std::vector<int> meshOrder;
    std::vector<const rt_object*> meshInstances;

    auto singleTriBlas = [&](const rt_object& o) {
        Tri t{};
        t.v0 = of(o.v[0]); t.v1 = of(o.v[1]); t.v2 = of(o.v[2]);
        t.e1 = t.v1 - t.v0; t.e2 = t.v2 - t.v0;
        D3 n = normalize(cross(t.e1, t.e2));
        t.n0 = t.n1 = t.n2 = n;
        const int64_t gi = (int64_t)triangles.size();
        triangles.push_back(t);
        BlasBuild bb;
        bb.smooth = false;
        bb.motion = of(o.motion_blur);
        bb.triIndex.push_back(gi);
        bb.prims.n = 1;
        const D3 mn = vmin(t.v0, vmin(t.v1, t.v2)), mx = vmax(t.v0, vmax(t.v1, t.v2));
        const D3 c = ((t.v0 + t.v1) + t.v2) / 3.0;
        bb.prims.bmin = {mn.x, mn.y, mn.z}; bb.prims.bmax = {mx.x, mx.y, mx.z}; bb.prims.cen = {c.x, c.y, c.z};
        return bb;
    };

    for (int oi = 0; oi < d->num_objects; ++oi) {
        const rt_object& o = d->objects[oi];
        if (o.kind == RT_OBJ_SPHERE || o.kind == RT_OBJ_PLANE) {            // RTContext.swift:122-192
            const bool sph = o.kind == RT_OBJ_SPHERE;
            (sph ? S.n_spheres : S.n_planes)++;
            S.has_special = true;
            Tri t{};
            t.v0 = of(o.center);
            t.e1 = sph ? d3(o.radius, 0, 0) : of(o.normal);
            const int64_t gi = (int64_t)triangles.size();
            triangles.push_back(t);
            BlasBuild bb;
            bb.kind = sph ? kPrimSphere : kPrimPlane;
            bb.smooth = true;                                                // shadingMode .smooth (unused)
            bb.triIndex.push_back(gi);
            bb.prims.n = 1;
            if (sph) {                                                       // center -/+ radius
                bb.pmin = t.v0 - o.radius;
                bb.pmax = t.v0 + o.radius;
            } else {                                                         // +-1e5 box, centroid 0
                bb.pmin = d3(-1e5, -1e5, -1e5);
                bb.pmax = d3(1e5, 1e5, 1e5);
            }
            const D3 c = sph ? t.v0 : d3(0, 0, 0);
            bb.prims.bmin = {bb.pmin.x, bb.pmin.y, bb.pmin.z};
            bb.prims.bmax = {bb.pmax.x, bb.pmax.y, bb.pmax.z};
            bb.prims.cen = {c.x, c.y, c.z};
            blases.push_back(std::move(bb));
            InstBuild ib{};
            ib.blas = (int)blases.size() - 1;
            std::memcpy(ib.M, o.transform, sizeof(ib.M));
            ib.material = o.material_id; ib.motion = d3(0, 0, 0);
            insts.push_back(ib);
            continue;
        }
        if (o.kind == RT_OBJ_TRIANGLE) {                                      // RTContext.swift:193-235
            S.n_tris++;
            blases.push_back(singleTriBlas(o));
            InstBuild ib{};
            ib.blas = (int)blases.size() - 1;
            std::memcpy(ib.M, o.transform, sizeof(ib.M));
            ib.material = o.material_id; ib.motion = d3(0, 0, 0);
            insts.push_back(ib);
            continue;
        }
        if (o.kind == RT_OBJ_MESH_INSTANCE) { meshInstances.push_back(&o); continue; }
        if (o.kind != RT_OBJ_MESH) { err = "unknown object kind"; return RT_ERR_INVALID_ARG; }
        // ---- Mesh (RTContext.swift:242-377)
        S.n_meshes++;
        std::vector<double> plyPos, plyNrm; std::vector<float> plyUV; std::vector<int32_t> plyIdx;
        const double* P; const int32_t* I; const double* Nn = nullptr; int64_t nPos, nIdx; int64_t off;
        if (o.ply_path) {
            std::string perr;
            int rc = ply_load(o.ply_path, plyPos, plyNrm, plyUV, plyIdx, perr);
            if (rc != RT_OK) {            // `try? PLYLoader.load` failing -> mesh skipped (RTContext.swift:255-261)
                continue;
            }
            P = plyPos.data(); nPos = (int64_t)plyPos.size() / 3;
            I = plyIdx.data(); nIdx = (int64_t)plyIdx.size();
            Nn = plyNrm.empty() ? nullptr : plyNrm.data();
            off = 0;
        } else {
            P = o.positions; nPos = o.num_positions; I = o.indices; nIdx = o.num_indices;
            Nn = o.normals; off = o.indices_one_based ? 1 : 0;
            if ((nPos > 0 && !P) || (nIdx > 0 && !I)) { err = "mesh arrays missing"; return RT_ERR_INVALID_ARG; }
            if (Nn && o.num_normals != nPos) {
                err = "mesh normals: num_normals must equal num_positions";
                return RT_ERR_INVALID_ARG;
            }
        }
        phase("ply");
        const bool isSmooth = o.smooth != 0;
        const int64_t triCount = nIdx / 3;
        for (int64_t t = 0; t < 3 * triCount; ++t) {
            const int64_t k = (int64_t)I[t] - off;
            if (k < 0 || k >= nPos) { err = "mesh index out of range"; return RT_ERR_INVALID_ARG; }
        }
        auto pos = [&](int64_t k) { return d3(P[3 * k], P[3 * k + 1], P[3 * k + 2]); };
        const int64_t start = (int64_t)triangles.size();
        S.n_tris += triCount;
        BlasBuild bb;
        bb.smooth = isSmooth;
        bb.motion = of(o.motion_blur);
        const bool blur = !(bb.motion.x == 0 && bb.motion.y == 0 && bb.motion.z == 0);
        bb.prims.n = triCount;
        bb.prims.bmin.resize(3 * triCount); bb.prims.bmax.resize(3 * triCount); bb.prims.cen.resize(3 * triCount);
        bb.triIndex.resize(triCount);
        std::vector<D3> vtx;
        std::vector<D3> faceN;
        if (!Nn) {
            faceN.resize(triCount);
            const int TF = std::max(1, std::min<int>(build_threads(), (int)(triCount / 65536)));
            run_chunks(TF, [&](int kc) {
                for (int64_t t = triCount * kc / TF, tEnd = triCount * (kc + 1) / TF; t < tEnd; ++t) {
                    D3 v0 = pos(I[3 * t] - off), v1 = pos(I[3 * t + 1] - off), v2 = pos(I[3 * t + 2] - off);
                    faceN[t] = normalize(cross(v1 - v0, v2 - v0));
                }
            });
            if (isSmooth) {
                vtx.assign(nPos, d3(0, 0, 0));
                for (int64_t t = 0; t < triCount; ++t)
                    for (int k = 0; k < 3; ++k) vtx[I[3 * t + k] - off] = vtx[I[3 * t + k] - off] + faceN[t];
                for (auto& v : vtx) v = normalize(v);
            }
        }
        phase("normals");
        triangles.resize(start + triCount);
        const int TC = std::max(1, std::min<int>(build_threads(), (int)(triCount / 65536)));
        run_chunks(TC, [&](int kc) {                      // independent per triangle
        for (int64_t t = triCount * kc / TC, tEnd = triCount * (kc + 1) / TC; t < tEnd; ++t) {
            const int64_t i0 = I[3 * t] - off, i1 = I[3 * t + 1] - off, i2 = I[3 * t + 2] - off;
            Tri& tr = triangles[start + t];
            tr.v0 = pos(i0); tr.v1 = pos(i1); tr.v2 = pos(i2);
            tr.e1 = tr.v1 - tr.v0; tr.e2 = tr.v2 - tr.v0;
            if (Nn) {
                tr.n0 = d3(Nn[3 * i0], Nn[3 * i0 + 1], Nn[3 * i0 + 2]);
                tr.n1 = d3(Nn[3 * i1], Nn[3 * i1 + 1], Nn[3 * i1 + 2]);
                tr.n2 = d3(Nn[3 * i2], Nn[3 * i2 + 1], Nn[3 * i2 + 2]);
            } else if (isSmooth) {
                tr.n0 = vtx[i0]; tr.n1 = vtx[i1]; tr.n2 = vtx[i2];
            } else {
                D3 n = normalize(faceN[t]);
                tr.n0 = tr.n1 = tr.n2 = n;
            }
            const D3 c = ((tr.v0 + tr.v1) + tr.v2) / 3.0;
            D3 mn = vmin(tr.v0, vmin(tr.v1, tr.v2)), mx = vmax(tr.v0, vmax(tr.v1, tr.v2));
            if (blur) {
                const D3 b0 = tr.v0 + bb.motion, b1 = tr.v1 + bb.motion, b2 = tr.v2 + bb.motion;
                mn = vmin(mn, vmin(b0, vmin(b1, b2)));
                mx = vmax(mx, vmax(b0, vmax(b1, b2)));
            }
            bb.prims.bmin[3 * t] = mn.x; bb.prims.bmin[3 * t + 1] = mn.y; bb.prims.bmin[3 * t + 2] = mn.z;
            bb.prims.bmax[3 * t] = mx.x; bb.prims.bmax[3 * t + 1] = mx.y; bb.prims.bmax[3 * t + 2] = mx.z;
            bb.prims.cen[3 * t] = c.x; bb.prims.cen[3 * t + 1] = c.y; bb.prims.cen[3 * t + 2] = c.z;
            bb.triIndex[t] = start + t;
        }
        });
        if (std::find(meshOrder.begin(), meshOrder.end(), o.id) == meshOrder.end()) meshOrder.push_back(o.id);
        if (triCount > 0) {
            blases.push_back(std::move(bb));
            Base base{};
            base.blas = (int)blases.size() - 1; base.material = o.material_id;
            std::memcpy(base.M, o.transform, sizeof(base.M));
            instanceByID[o.id] = base;
        } else {
            instanceByID.erase(o.id);
        }
    }
    // MeshInstance objects (RTContext.swift:384-401), then base meshes in scene order (:403-410, H11)
    for (const rt_object* mi : meshInstances) {
        auto it = instanceByID.find(mi->base_mesh_id);
        if (it == instanceByID.end()) continue;
        InstBuild ib{};
        ib.blas = it->second.blas;
        std::memcpy(ib.M, mi->transform, sizeof(ib.M));
        ib.material = mi->material_id; ib.motion = of(mi->motion_blur);
        insts.push_back(ib);
        Base nb{}; nb.blas = it->second.blas; nb.material = mi->material_id; std::memcpy(nb.M, mi->transform, sizeof(nb.M));
        instanceByID[mi->id] = nb;
    }
    for (int meshID : meshOrder) {
        auto it = instanceByID.find(meshID);
        if (it == instanceByID.end()) continue;
        InstBuild ib{};
        ib.blas = it->second.blas;
        std::memcpy(ib.M, it->second.M, sizeof(ib.M));
        ib.material = it->second.material; ib.motion = d3(0, 0, 0);
        insts.push_back(ib);
    }

    phase("flatten");
    // ---- BLAS builds (buildBLASForMesh: maxLeaf 2, SAH, 12 bins; RTContext.swift:430-435)
    int64_t maxBlasDepth = 0, tlasDepth = 0;
    for (auto& bb : blases) {
        bb.bvh = build_ref_bvh(bb.prims, 2, 12);
        bb.hash = ref_bvh_hash(bb.bvh, bb.triIndex);
        bb.depth = ref_bvh_depth(bb.bvh);
        maxBlasDepth = std::max(maxBlasDepth, bb.depth);
    }

    phase("blas_bvh");
    // ---- device layout: BLAS records + leaf-ordered triangles
    {
        size_t nt = 0, nr = 0;
        for (const auto& bb : blases) { nt += bb.triIndex.size(); nr += bb.triIndex.size(); }
        S.tris.reserve(nt);
        S.normals.reserve(9 * nt);
        S.recs.reserve(nr + insts.size() + 1);
    }
    for (auto& bb : blases) {
        auto emit = [&](int64_t firstSlot, int64_t count) -> int64_t {
            const int64_t first = (int64_t)S.tris.size();
            for (int64_t q = 0; q < count; ++q) {
                const int64_t g = bb.triIndex[bb.bvh.primIdx[firstSlot + q]];
                const Tri& t = triangles[g];
                TriRec r{};
                r.v0[0] = t.v0.x; r.v0[1] = t.v0.y; r.v0[2] = t.v0.z;
                r.e1[0] = t.e1.x; r.e1[1] = t.e1.y; r.e1[2] = t.e1.z;
                r.e2[0] = t.e2.x; r.e2[1] = t.e2.y; r.e2[2] = t.e2.z;
                r.last = (q == count - 1) ? 1 : 0;
                r.prim = (int32_t)g;
                S.tris.push_back(r);
                const D3 ns[3] = {t.n0, t.n1, t.n2};
                for (int k = 0; k < 3; ++k) { S.normals.push_back(ns[k].x); S.normals.push_back(ns[k].y); S.normals.push_back(ns[k].z); }
            }
            return first;
        };
        bb.tri_first = (int64_t)S.tris.size();
        // the first BLAS starts at record 0 with a breadth-first prefix of its top levels
        constexpr int64_t kTopRecords = 127;
        const int64_t top = S.recs.empty() ? kTopRecords : 0;
        bb.root_ref = layout_bvh(bb.bvh, S.recs, emit, top);
        bb.tri_end = (int64_t)S.tris.size();
        for (int k = 0; k < 3; ++k) { bb.root_lo[k] = bb.bvh.lo[k]; bb.root_hi[k] = bb.bvh.hi[k]; }
        bb.bvh = RefBVH();   // free host copy
        bb.prims = PrimSet();
    }
    S.blas_records = (int64_t)S.recs.size();
    if (!S.has_special && !S.tris.empty()) {   // compact triangles when every vertex is a float
        bool exact = true;
        auto fx = [](double x) { return (double)(float)x == x; };
        for (size_t q = 0; q < S.tris.size() && exact; ++q) {
            const Tri& t = triangles[S.tris[q].prim];
            exact &= fx(t.v0.x) && fx(t.v0.y) && fx(t.v0.z) && fx(t.v1.x) && fx(t.v1.y) && fx(t.v1.z) &&
                     fx(t.v2.x) && fx(t.v2.y) && fx(t.v2.z);
        }
        if (exact) {
            S.ctris.resize(S.tris.size());
            for (size_t q = 0; q < S.tris.size(); ++q) {
                const Tri& t = triangles[S.tris[q].prim];
                CTri& c = S.ctris[q];
                c.v0[0] = (float)t.v0.x; c.v0[1] = (float)t.v0.y; c.v0[2] = (float)t.v0.z;
                c.v1[0] = (float)t.v1.x; c.v1[1] = (float)t.v1.y; c.v1[2] = (float)t.v1.z;
                c.v2[0] = (float)t.v2.x; c.v2[1] = (float)t.v2.y; c.v2[2] = (float)t.v2.z;
                c.last = S.tris[q].last;
                c.prim = S.tris[q].prim;          // rewritten below in identity mode
                c.pad = 0;
            }
            S.compact_tris = true;
        }
    }
    {   // compact BLAS records when every bound survives a float32 round trip exactly
        bool exact = true;
        for (int64_t q = 0; q < S.blas_records && exact; ++q)
            for (int c = 0; c < 2; ++c)
                for (int k = 0; k < 3; ++k) {
                    const double lo = S.recs[q].lo[c][k], hi = S.recs[q].hi[c][k];
                    exact &= (double)(float)lo == lo && (double)(float)hi == hi;
                }
        if (exact && S.blas_records > 0) {
            S.crecs.resize(S.blas_records);
            for (int64_t q = 0; q < S.blas_records; ++q) {
                CRec& r = S.crecs[q];
                std::memset(&r, 0, sizeof(r));
                for (int c = 0; c < 2; ++c) {
                    for (int k = 0; k < 3; ++k) { r.lo[c][k] = (float)S.recs[q].lo[c][k]; r.hi[c][k] = (float)S.recs[q].hi[c][k]; }
                    r.ref[c] = S.recs[q].ref[c];
                }
            }
            S.compact_records = S.blas_records;
        }
    }

    phase("layout");
    // ---- pruning margin (DESIGN.md "Pruning"): a culled node may only hold triangles whose
    // Moeller-Trumbore t, as computed, can not undercut the current hit.  MT's t = num/det
    // with |det| >= eps carries an absolute error below
    //   8u * |e1||e2| * (|o - v0| + t|d|) / eps      (u = 2^-53; both triple products),
    // in the instance's local frame, where |d| and |o - v0| are at most ||A||_F times their
    // world values (A = the linear part of worldToLocal).  Planes: 8u |n| (...) / eps.  The
    // scene constant prune_k = 8u/eps * max over instances of P_blas * ||A||_F is turned into
    // an absolute margin per render from the ray origins' distance to the scene (make_params).
    std::vector<double> blasP(blases.size(), 0.0);
    {
        const int TP = std::max(1, std::min<int>(build_threads(), (int)(triangles.size() / 262144)));
        for (size_t b = 0; b < blases.size(); ++b) {
            const BlasBuild& bb = blases[b];
            if (bb.kind == kPrimPlane) {
                const TriRec& t = S.tris[bb.tri_first];
                blasP[b] = std::sqrt(t.e1[0] * t.e1[0] + t.e1[1] * t.e1[1] + t.e1[2] * t.e1[2]);
                continue;
            }
            if (bb.kind != kPrimTriangles) continue;          // spheres: covered by prune_rel
            std::vector<double> part(TP, 0.0);
            const int64_t n = (int64_t)bb.triIndex.size();
            run_chunks(TP, [&](int kc) {
                double m = 0.0;
                for (int64_t q = n * kc / TP, qe = n * (kc + 1) / TP; q < qe; ++q) {
                    const Tri& t = triangles[bb.triIndex[q]];
                    m = std::fmax(m, std::sqrt(dot(t.e1, t.e1)) * std::sqrt(dot(t.e2, t.e2)));
                }
                part[kc] = m;
            });
            for (double m : part) blasP[b] = std::fmax(blasP[b], m);
        }
    }
    double pruneK = 0.0, maxMotion = 0.0;
    // ---- instances (makeInstance, RTContext.swift:437-457) and TLAS (buildTLAS :459-474)
    PrimSet tp;
    tp.n = (int64_t)insts.size();
    double wlo[3] = {kInf, kInf, kInf}, whi[3] = {-kInf, -kInf, -kInf};
    for (size_t i = 0; i < insts.size(); ++i) {
        InstBuild& ib = insts[i];
        const BlasBuild& bb = blases[ib.blas];
        // world bounds: union of every prim's transformed bounds
        D3 mn = d3(kInf, kInf, kInf), mx = d3(-kInf, -kInf, -kInf);
        if (bb.kind != kPrimTriangles) {
            double lo[3] = {bb.pmin.x, bb.pmin.y, bb.pmin.z}, hi[3] = {bb.pmax.x, bb.pmax.y, bb.pmax.z}, olo[3], ohi[3];
            aabb_transformed(lo, hi, ib.M, olo, ohi);
            mn = d3(olo[0], olo[1], olo[2]);
            mx = d3(ohi[0], ohi[1], ohi[2]);
        }
        for (size_t q = 0; q < bb.triIndex.size() && bb.kind == kPrimTriangles; ++q) {
            const Tri& t = triangles[bb.triIndex[q]];
            D3 pmn = vmin(t.v0, vmin(t.v1, t.v2)), pmx = vmax(t.v0, vmax(t.v1, t.v2));
            if (!(bb.motion.x == 0 && bb.motion.y == 0 && bb.motion.z == 0)) {
                const D3 b0 = t.v0 + bb.motion, b1 = t.v1 + bb.motion, b2 = t.v2 + bb.motion;
                pmn = vmin(pmn, vmin(b0, vmin(b1, b2)));
                pmx = vmax(pmx, vmax(b0, vmax(b1, b2)));
            }
            double lo[3] = {pmn.x, pmn.y, pmn.z}, hi[3] = {pmx.x, pmx.y, pmx.z}, olo[3], ohi[3];
            aabb_transformed(lo, hi, ib.M, olo, ohi);
            mn = vmin(mn, d3(olo[0], olo[1], olo[2]));
            mx = vmax(mx, d3(ohi[0], ohi[1], ohi[2]));
        }
        ib.wlo[0] = mn.x; ib.wlo[1] = mn.y; ib.wlo[2] = mn.z;
        ib.whi[0] = mx.x; ib.whi[1] = mx.y; ib.whi[2] = mx.z;
        for (int k = 0; k < 3; ++k) { wlo[k] = std::fmin(wlo[k], ib.wlo[k]); whi[k] = std::fmax(whi[k], ib.whi[k]); }
        tp.bmin.insert(tp.bmin.end(), ib.wlo, ib.wlo + 3);
        tp.bmax.insert(tp.bmax.end(), ib.whi, ib.whi + 3);
        const D3 c = (d3(ib.wlo[0], ib.wlo[1], ib.wlo[2]) + d3(ib.whi[0], ib.whi[1], ib.whi[2])) * 0.5;
        tp.cen.insert(tp.cen.end(), {c.x, c.y, c.z});

        DInstance di{};
        std::memcpy(di.l2w, ib.M, sizeof(di.l2w));
        m4_inverse(ib.M, di.w2l);
        {
            double fro = 0.0;
            for (int c = 0; c < 3; ++c)
                for (int r = 0; r < 3; ++r) fro += di.w2l[c * 4 + r] * di.w2l[c * 4 + r];
            pruneK = std::fmax(pruneK, blasP[ib.blas] * std::sqrt(fro));
            maxMotion = std::fmax(maxMotion, std::sqrt(dot(ib.motion, ib.motion)) + std::sqrt(dot(bb.motion, bb.motion)));
        }
        normal_matrix(ib.M, di.nmat);
        di.motion[0] = ib.motion.x; di.motion[1] = ib.motion.y; di.motion[2] = ib.motion.z;
        di.tri_motion[0] = bb.motion.x; di.tri_motion[1] = bb.motion.y; di.tri_motion[2] = bb.motion.z;
        for (int k = 0; k < 3; ++k) { di.root_lo[k] = bb.root_lo[k]; di.root_hi[k] = bb.root_hi[k]; }
        di.root_ref = bb.root_ref;
        di.material = ib.material;
        di.smooth = bb.smooth ? 1 : 0;
        di.det_neg = m3_det_of4(ib.M) < 0.0 ? 1 : 0;
        di.kind = bb.kind;
        S.insts.push_back(di);
        S.inst_bvh_hash.push_back(bb.hash);
        // dielectric frames take the full trace() passes: only when an instance shades with a
        // dielectric (the clamped material index every hit uses, Object+Extension.swift:104-106, H14) - an
        // unused dielectric in the material list does not change a frame
        if (!S.mats.empty()) {
            const int mi = std::max(0, std::min((int)S.mats.size() - 1, (int)di.material - 1));
            if (S.mats[mi].type == RT_MAT_DIELECTRIC) S.has_dielectric = true;
        }
    }
    if (!insts.empty()) {
        RefBVH tb = build_ref_bvh(tp, 2, 12);
        std::vector<int64_t> ident(tp.n);
        for (int64_t i = 0; i < tp.n; ++i) ident[i] = i;
        S.tlas_hash = ref_bvh_hash(tb, ident);
        const int64_t tdepth = ref_bvh_depth(tb);
        for (int k = 0; k < 3; ++k) { S.tlas_root_lo[k] = tb.lo[k]; S.tlas_root_hi[k] = tb.hi[k]; }
        // TLAS leaf refs are offset by the TriRec count so one ref space covers both levels
        S.tlas_leaf_base = (int64_t)S.tris.size();
        auto emit = [&](int64_t firstSlot, int64_t count) -> int64_t {
            const int64_t first = S.tlas_leaf_base + (int64_t)S.tlas_leaf.size();
            for (int64_t q = 0; q < count; ++q)
                S.tlas_leaf.push_back(DTlasLeafEntry{(int32_t)tb.primIdx[firstSlot + q], (q == count - 1) ? 1 : 0});
            return first;
        };
        S.tlas_root_ref = layout_bvh(tb, S.recs, emit);
        S.tlas_records = (int64_t)S.recs.size() - S.blas_records;
        S.has_tlas = true;
        // Stack entries a walk can hold (device.h Stack, kStackCap): one deferred far child per
        // inner node on the current path, TLAS path below BLAS path (+2 slack).  The unified
        // identity walk also pushes a whole TLAS leaf's instance roots at once.
        int64_t maxTlasLeaf = 1;
        for (int64_t n = 0; n < tb.nodesUsed; ++n)
            if (tb.isLeaf(n)) maxTlasLeaf = std::max(maxTlasLeaf, tb.count[n]);
        S.max_stack = tdepth + maxBlasDepth + 2;
        S.max_stack_unified = tdepth + maxTlasLeaf + maxBlasDepth + 2;
        tlasDepth = tdepth;
        const double dx = whi[0] - wlo[0], dy = whi[1] - wlo[1], dz = whi[2] - wlo[2];
        S.scene_extent = std::sqrt(dx * dx + dy * dy + dz * dz);
        if (!std::isfinite(S.scene_extent) || S.scene_extent <= 0) S.scene_extent = 1.0;
        for (int k = 0; k < 3; ++k) S.scene_center[k] = 0.5 * (wlo[k] + whi[k]);
        if (!std::isfinite(S.scene_center[0] + S.scene_center[1] + S.scene_center[2]))
            S.scene_center[0] = S.scene_center[1] = S.scene_center[2] = 0.0;
        S.prune_k = (S.eps > 0) ? 8.0 * std::ldexp(1.0, -53) * pruneK / S.eps : kInf;
        S.max_motion = maxMotion;
        S.det_scale = pruneK;
    }
    // Identity mode: every instance's transforms are exactly the identity and nothing moves,
    // so the world ray IS the local ray (up to the sign of zeros, which no comparison sees)
    // and TLAS + BLAS records can be walked as one tree with one stack.  Each BLAS must
    // belong to exactly one instance so a triangle identifies its instance.
    {
        bool ident = S.has_tlas;
        std::vector<int> owners(blases.size(), 0);
        for (size_t i = 0; i < insts.size() && ident; ++i) {
            const InstBuild& ib = insts[i];
            for (int k = 0; k < 16; ++k) ident &= ib.M[k] == ((k % 5 == 0) ? 1.0 : 0.0);
            ident &= ib.motion.x == 0 && ib.motion.y == 0 && ib.motion.z == 0;
            const BlasBuild& bb = blases[ib.blas];
            ident &= bb.motion.x == 0 && bb.motion.y == 0 && bb.motion.z == 0;
            owners[ib.blas]++;
        }
        for (int o : owners) ident &= (o <= 1);
        ident &= !S.has_special;                    // the unified walk tests triangles only
        ident &= S.max_stack_unified <= kStackCap;  // else the general walk (fewer entries)
        S.identity = ident;
        if (ident) {
            for (size_t i = 0; i < insts.size(); ++i) {
                const BlasBuild& bb = blases[insts[i].blas];
                for (int64_t t = bb.tri_first; t < bb.tri_end; ++t) {
                    S.tris[t].prim = (int32_t)i;
                    if (S.compact_tris) S.ctris[t].prim = (int32_t)i;
                }
            }
        }
    }
    if (S.identity) build_wide(S);
    else build_wide_tw(S);
    phase("wide");
    if (trace && S.fit_root >= 0)
        std::fprintf(stderr, "[build] fit: %zu pairs, %lld nodes, depth %lld, coord %.6g, %.1f ms\n", S.fpairs.size(),
                     (long long)S.fit_nodes, (long long)S.fit_depth, S.fit_coord, S.fit_ms);
    if (S.recs.size() >= (size_t)INT32_MAX || S.tris.size() >= (size_t)INT32_MAX) { err = "scene too large for int32 refs"; return RT_ERR_UNSUPPORTED; }
    if (maxBlasDepth + 1 > 63 || tlasDepth + 1 > 63) {
        err = "BVH deeper than the reference's 64-entry stack (RTContext.swift:550, 623)";
        return RT_ERR_STACK;
    }
    if (S.max_stack > kStackCap) {                  // unreachable while kStackCap >= 2*63+2
        err = "BVH deeper than the device traversal stack";
        return RT_ERR_STACK;
    }
    phase("tlas+inst");
    S.build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return RT_OK;
}

}  // namespace myrt
