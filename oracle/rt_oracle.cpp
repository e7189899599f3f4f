// ============================================================================
//  oracle/rt_oracle.cpp  —  TEST INFRASTRUCTURE ONLY (parity checker / CPU baseline)
//
//  A line-by-line CPU restatement, in C++17 / IEEE binary64, of the reference
//  renderer's per-pixel trace path (erndmrcn/MyRayTracer, Swift).  Only tests/,
//  __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library;
//  the product (myraytracer_amd / libmyrt.so) never links or calls it.
//
//  Every function cites the Swift it restates (paths relative to Sources/):
//    RT/ = RayTracer/, e.g. RT/Models/RTContext.swift:479-510.
//
//  PINNING.  The Swift reference cannot be built or run anywhere here (Apple-only
//  frameworks, missing ParsingKit dependency, no swift toolchain — SURVEY.md §0,
//  §8c), and it ships no tests, fixtures or golden images.  This oracle is
//  therefore pinned only by known-answer tests derived from the reference's
//  formulas (PCG32 streams, closed-form single-triangle shading, slab/MT edge
//  cases: tests/test_oracle_kat.py).  With respect to the Swift binary itself,
//  RENDER PARITY IS UNPINNED.  PLY parsing is pinned separately against the
//  reference's own CPly compiled in this container (oracle/build_ref.sh).
//
//  Documented assumptions where the Swift semantics live in Apple's simd module
//  or in the missing ParsingKit:
//    * no FMA contraction anywhere (compile with -ffp-contract=off);
//    * dot(a,b) = (a.x*b.x + a.y*b.y) + a.z*b.z; length = sqrt(dot(v,v));
//      normalize(v) = v * (1/sqrt(dot(v,v)));  cross = component formula;
//    * Mat*vec = ((c0*x + c1*y) + c2*z) (+ c3*w), no fused multiply-add;
//    * simd.min/max (vector) = IEEE minNum/maxNum (fmin/fmax); Swift.max(x,y) =
//      (y >= x ? y : x), Swift.min(x,y) = (y < x ? y : x)  (asymmetric NaN);
//    * Ray(origin:dir:time:) sets invDir = 1/dir, tMin = 0, tMax = +inf, hit.t = +inf;
//    * base-mesh instances are appended in scene-object order (H11: the Swift
//      Dictionary order is unspecified);
//    * the unused global BVH (RTContext.swift:380-382) is not built.
// ============================================================================
#include "../include/rtcore.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <map>
#include <memory>
#include <string>
#include <thread>
#include <vector>

namespace orc {

static const double kInf = std::numeric_limits<double>::infinity();

// ---------------------------------------------------------------- vector math
struct V3 { double x, y, z; };
static inline V3 v3(double x, double y, double z) { return V3{x, y, z}; }
static inline V3 operator+(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
static inline V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
static inline V3 operator-(V3 a) { return {-a.x, -a.y, -a.z}; }
static inline V3 operator*(V3 a, V3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
static inline V3 operator/(V3 a, V3 b) { return {a.x / b.x, a.y / b.y, a.z / b.z}; }
static inline V3 operator*(V3 a, double s) { return {a.x * s, a.y * s, a.z * s}; }
static inline V3 operator*(double s, V3 a) { return {s * a.x, s * a.y, s * a.z}; }
static inline V3 operator/(V3 a, double s) { return {a.x / s, a.y / s, a.z / s}; }
static inline V3 operator+(double s, V3 a) { return {s + a.x, s + a.y, s + a.z}; }
static inline V3 operator/(double s, V3 a) { return {s / a.x, s / a.y, s / a.z}; }
static inline V3 operator-(V3 a, double s) { return {a.x - s, a.y - s, a.z - s}; }
static inline V3 operator+(V3 a, double s) { return {a.x + s, a.y + s, a.z + s}; }
static inline V3& operator+=(V3& a, V3 b) { a = a + b; return a; }
static inline V3& operator*=(V3& a, V3 b) { a = a * b; return a; }
static inline double dot(V3 a, V3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
static inline V3 cross(V3 a, V3 b) {
    return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
static inline double length(V3 v) { return std::sqrt(dot(v, v)); }
static inline V3 normalize(V3 v) { double r = 1.0 / std::sqrt(dot(v, v)); return v * r; }
static inline double at(V3 v, int a) { return a == 0 ? v.x : (a == 1 ? v.y : v.z); }
// simd.min / simd.max on vectors (IEEE minNum / maxNum)
static inline V3 vmin(V3 a, V3 b) { return {std::fmin(a.x, b.x), std::fmin(a.y, b.y), std::fmin(a.z, b.z)}; }
static inline V3 vmax(V3 a, V3 b) { return {std::fmax(a.x, b.x), std::fmax(a.y, b.y), std::fmax(a.z, b.z)}; }
// Swift.max / Swift.min on scalars (stdlib: y >= x ? y : x / y < x ? y : x)
static inline double smax(double x, double y) { return (y >= x) ? y : x; }
static inline double smin(double x, double y) { return (y < x) ? y : x; }
static inline bool isfin(V3 v) { return std::isfinite(v.x) && std::isfinite(v.y) && std::isfinite(v.z); }

struct M4 { double m[16]; };   // column-major: m[c*4+r]
struct M3 { double m[9]; };    // column-major: m[c*3+r]
// simd_mul(double4x4, double4): r = c0*x; r = c1*y + r; r = c2*z + r; r = c3*w + r
static inline void m4_mul(const M4& M, double x, double y, double z, double w, double out[4]) {
    for (int r = 0; r < 4; ++r) {
        double acc = M.m[0 * 4 + r] * x;
        acc = M.m[1 * 4 + r] * y + acc;
        acc = M.m[2 * 4 + r] * z + acc;
        acc = M.m[3 * 4 + r] * w + acc;
        out[r] = acc;
    }
}
static inline V3 m3_mul(const M3& M, V3 v) {
    double o[3];
    for (int r = 0; r < 3; ++r) {
        double acc = M.m[0 * 3 + r] * v.x;
        acc = M.m[1 * 3 + r] * v.y + acc;
        acc = M.m[2 * 3 + r] * v.z + acc;
        o[r] = acc;
    }
    return {o[0], o[1], o[2]};
}
// General 4x4 inverse by cofactors (simd_inverse's algorithm is unpinned; exact for
// identity and pure translations, which is all the parity configs use).
static M4 m4_inverse(const M4& A) {
    const double* m = A.m;
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
    double det = m[0] * inv[0] + m[1] * inv[4] + m[2] * inv[8] + m[3] * inv[12];
    M4 r;
    for (int i = 0; i < 16; ++i) r.m[i] = inv[i] / det;
    return r;
}
static M3 m3_of(const M4& M) {
    M3 r;
    for (int c = 0; c < 3; ++c)
        for (int rr = 0; rr < 3; ++rr) r.m[c * 3 + rr] = M.m[c * 4 + rr];
    return r;
}
static double m3_det(const M3& A) {
    const double* a = A.m;  // a[c*3+r]
    return a[0] * (a[4] * a[8] - a[7] * a[5]) - a[3] * (a[1] * a[8] - a[7] * a[2]) + a[6] * (a[1] * a[5] - a[4] * a[2]);
}
// normalTransformMatrix(from:) = M3.inverse.transpose (RTContext.swift:23-31)
static M3 normal_matrix(const M4& M) {
    M3 a = m3_of(M);
    const double* m = a.m;  // m[c*3+r] ; element (r,c)
    auto e = [&](int r, int c) { return m[c * 3 + r]; };
    double det = m3_det(a);
    M3 inv;  // inverse (r,c) = cof(c,r)/det
    double cof[3][3];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) {
            int r1 = (r + 1) % 3, r2 = (r + 2) % 3, c1 = (c + 1) % 3, c2 = (c + 2) % 3;
            cof[r][c] = e(r1, c1) * e(r2, c2) - e(r1, c2) * e(r2, c1);
        }
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) inv.m[c * 3 + r] = cof[c][r] / det;
    M3 t;  // transpose
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) t.m[c * 3 + r] = inv.m[r * 3 + c];
    return t;
}

// --------------------------------------------------------------------- AABB
// RT/Accelearion/AABB.swift:12-92
struct AABB {
    V3 minP{kInf, kInf, kInf};
    V3 maxP{-kInf, -kInf, -kInf};
    double area() const {                                   // AABB.swift:29-33
        V3 e = maxP - minP;
        return 2.0 * ((e.x * e.y + e.y * e.z) + e.z * e.x);
    }
    void grow(const AABB& b) { minP = vmin(minP, b.minP); maxP = vmax(maxP, b.maxP); }  // :65-68
    AABB transformed(const M4& M) const {                    // AABB.swift:71-92
        V3 cOld = 0.5 * (minP + maxP);
        V3 eOld = 0.5 * (maxP - minP);
        M3 r = m3_of(M);
        V3 t = v3(M.m[12], M.m[13], M.m[14]);
        V3 cNew = m3_mul(r, cOld) + t;
        double ar[9];
        for (int i = 0; i < 9; ++i) ar[i] = std::fabs(r.m[i]);
        V3 eNew = v3(ar[0] * eOld.x + ar[3] * eOld.y + ar[6] * eOld.z,
                     ar[1] * eOld.x + ar[4] * eOld.y + ar[7] * eOld.z,
                     ar[2] * eOld.x + ar[5] * eOld.y + ar[8] * eOld.z);
        AABB o;
        o.minP = cNew - eNew;
        o.maxP = cNew + eNew;
        return o;
    }
};

// ---------------------------------------------------------------- BVH builder
// RT/Accelearion/BVH.swift:16-250
enum GeomType { G_MESH = 0, G_TRIANGLE = 1, G_SPHERE = 2, G_PLANE = 3 };
enum Shading { S_FLAT = 0, S_SMOOTH = 1 };
struct BVHNode { V3 aabbMin{0, 0, 0}, aabbMax{0, 0, 0}; uint64_t leftFirst = 0, primitiveCount = 0;
                 bool isLeaf() const { return primitiveCount > 0; } };
struct PrimitiveInfo {
    int type; int64_t primitiveIndex; AABB bounds; V3 centroid; int materialID; int shadingMode;
};

struct BVHBuilder {
    std::vector<PrimitiveInfo> primitives;
    std::vector<uint64_t> primitiveIdx;
    std::vector<BVHNode> bvhNode;
    int maxLeaf = 2;
    uint64_t rootNodeIdx = 0, nodesUsed = 0;
    int binCount = 12;

    BVHBuilder() = default;
    BVHBuilder(std::vector<PrimitiveInfo> prims, int maxLeaf_ = 2, int binCount_ = 12)   // :78-104
        : primitives(std::move(prims)), maxLeaf(maxLeaf_), binCount(std::max(2, binCount_)) {
        const int64_t n = (int64_t)primitives.size();
        primitiveIdx.resize(n);
        for (int64_t i = 0; i < n; ++i) primitiveIdx[i] = (uint64_t)i;
        int64_t nodeCount = std::max<int64_t>(1, n * 2 - 1);
        bvhNode.assign(nodeCount, BVHNode());
        bvhNode[0].leftFirst = 0;
        bvhNode[0].primitiveCount = (uint64_t)n;
        nodesUsed = 0; rootNodeIdx = 0;
        updateNodeBounds(0);
        subdivide(0);
    }
    void updateNodeBounds(uint64_t nodeIdx) {                                              // :108-124
        BVHNode node = bvhNode[nodeIdx];
        node.aabbMin = v3(kInf, kInf, kInf);
        node.aabbMax = v3(-kInf, -kInf, -kInf);
        for (uint64_t i = 0; i < node.primitiveCount; ++i) {
            const PrimitiveInfo& prim = primitives[primitiveIdx[node.leftFirst + i]];
            node.aabbMin = vmin(node.aabbMin, prim.bounds.minP);
            node.aabbMax = vmax(node.aabbMax, prim.bounds.maxP);
        }
        bvhNode[nodeIdx] = node;
    }
    void subdivide(uint64_t nodeIdx) {                                                     // :128-188
        BVHNode node = bvhNode[nodeIdx];
        const int64_t primCount = (int64_t)node.primitiveCount;
        if (primCount <= maxLeaf && nodeIdx != 0) return;
        int bestAxis = 0; double bestPos = 0;
        (void)findBestSplitPlane(node, bestAxis, bestPos);
        int64_t i = (int64_t)node.leftFirst;
        int64_t j = i + primCount - 1;
        while (i <= j) {
            const uint64_t primID = primitiveIdx[i];
            if (at(primitives[primID].centroid, bestAxis) < bestPos) {
                i += 1;
            } else {
                std::swap(primitiveIdx[i], primitiveIdx[j]);
                j -= 1;
            }
        }
        const int64_t leftCount = i - (int64_t)node.leftFirst;
        if (leftCount == 0 || leftCount == primCount) return;
        nodesUsed += 1; const uint64_t leftChild = nodesUsed;
        nodesUsed += 1; const uint64_t rightChild = nodesUsed;
        if (rightChild >= bvhNode.size()) std::abort();   // precondition "BVH node overflow" (:169)
        bvhNode[leftChild].leftFirst = node.leftFirst;
        bvhNode[leftChild].primitiveCount = (uint64_t)leftCount;
        bvhNode[rightChild].leftFirst = (uint64_t)i;
        bvhNode[rightChild].primitiveCount = (uint64_t)(primCount - leftCount);
        node.leftFirst = leftChild;
        node.primitiveCount = 0;
        bvhNode[nodeIdx] = node;
        updateNodeBounds(leftChild);
        updateNodeBounds(rightChild);
        subdivide(leftChild);
        subdivide(rightChild);
    }
    double findBestSplitPlane(const BVHNode& node, int& axis, double& splitPos) const {    // :192-250
        double bestCost = kInf;
        for (int a = 0; a < 3; ++a) {
            double boundsMin = kInf, boundsMax = -kInf;
            const int64_t count = (int64_t)node.primitiveCount;
            const int64_t first = (int64_t)node.leftFirst;
            for (int64_t i = 0; i < count; ++i) {
                const PrimitiveInfo& prim = primitives[primitiveIdx[first + i]];
                boundsMin = smin(boundsMin, at(prim.centroid, a));
                boundsMax = smax(boundsMax, at(prim.centroid, a));
            }
            if (boundsMax <= boundsMin) continue;
            const int N = binCount;
            std::vector<AABB> bin(N);
            std::vector<int64_t> cnt(N, 0);
            const double scale = double(N) / (boundsMax - boundsMin);
            for (int64_t i = 0; i < count; ++i) {
                const PrimitiveInfo& prim = primitives[primitiveIdx[first + i]];
                int64_t q = (int64_t)((at(prim.centroid, a) - boundsMin) * scale);
                int64_t idx = (q < (int64_t)(N - 1)) ? q : (int64_t)(N - 1);     // Swift.min(N-1, q)
                cnt[idx] += 1;
                bin[idx].grow(prim.bounds);
            }
            std::vector<double> leftArea(N - 1, 0), rightArea(N - 1, 0);
            std::vector<int64_t> leftCnt(N - 1, 0), rightCnt(N - 1, 0);
            AABB L, R; int64_t sL = 0, sR = 0;
            for (int i = 0; i < N - 1; ++i) {
                sL += cnt[i]; leftCnt[i] = sL; L.grow(bin[i]); leftArea[i] = L.area();
                sR += cnt[N - 1 - i]; rightCnt[N - 2 - i] = sR; R.grow(bin[N - 1 - i]);
                rightArea[N - 2 - i] = R.area();
            }
            const double step = (boundsMax - boundsMin) / double(N);
            for (int i = 0; i < N - 1; ++i) {
                if (leftCnt[i] == 0 || rightCnt[i] == 0) continue;
                const double cost = double(leftCnt[i]) * leftArea[i] + double(rightCnt[i]) * rightArea[i];
                if (cost < bestCost) {
                    bestCost = cost; axis = a; splitPos = boundsMin + step * double(i + 1);
                }
            }
        }
        return bestCost;
    }
};

// ------------------------------------------------------------- scene objects
struct Triangle { V3 v0, v1, v2, e1, e2, n0, n1, n2, centroid, motionBlur; };
struct Sphere { V3 center; double radius; };
struct Plane { V3 center, normal; };
struct BLAS { std::vector<BVHNode> nodes; std::vector<uint64_t> primIdx; std::vector<PrimitiveInfo> prims; uint64_t root; };
struct Instance {                                                     // RTContext.swift:43-61
    std::shared_ptr<BLAS> blas; M4 localToWorld, worldToLocal; AABB worldBounds;
    int materialOverride; V3 instanceMotion; M3 normalMatrix;
};
struct Hit { double t = kInf; V3 p{0, 0, 0}, n{0, 0, 0}; int kind = -1; int mat = 0; };
struct Ray {                                                          // ParsingKit Ray (assumed init)
    V3 origin, dir, invDir; double tMin = 0, tMax = kInf, time = 0; Hit hit;
    Ray() = default;
    Ray(V3 o, V3 d, double t) : origin(o), dir(d), invDir(1.0 / d), tMin(0), tMax(kInf), time(t) {}
};

struct Counters {
    int64_t primary = 0, shadow = 0, secondary = 0, visits = 0;
    int64_t nodeFetch = 0, triTest = 0, smoothHit = 0, pixels = 0;
    int64_t shadowUsed = 0;   // shadow rays whose result trace() uses (point lights: N.L > 0)
    void add(const Counters& o) {
        primary += o.primary; shadow += o.shadow; secondary += o.secondary; visits += o.visits;
        nodeFetch += o.nodeFetch; triTest += o.triTest; smoothHit += o.smoothHit; pixels += o.pixels;
        shadowUsed += o.shadowUsed;
    }
};

struct Material {
    V3 ambient, diffuse, specular, mirror, absorption;
    double phong, ior, absorptionIndex, roughness; int type;
};
struct PointLight { V3 position, intensity; };
struct AreaLight { V3 position, normal, radiance; double size; };
struct Camera {
    int type, width, height, numSamples; V3 position, gazePoint, gaze, up; double fovy, nearDistance;
    double nearPlane[4]; double apertureSize, focusDistance;
};

static V3 fromc(rt_vec3 v) { return V3{v.x, v.y, v.z}; }

// ------------------------------------------------------------------ RTContext
struct Context {
    double intersectionTestEpsilon = 0, shadowRayEpsilon = 0;
    std::vector<Material> materials;
    std::vector<Sphere> spheres;
    std::vector<Plane> planes;
    std::vector<Triangle> triangles;
    std::vector<PointLight> pointLights;
    std::vector<AreaLight> areaLights;
    std::vector<Instance> instances;
    bool hasTlas = false;
    BVHBuilder tlasBuilder;
    // scene-level parameters (ParsingKit Scene)
    V3 backgroundColor{0, 0, 0}, ambientLight{0, 0, 0};
    int maxRecursionDepth = 0;
    std::vector<Camera> cameras;
    int64_t nMeshes = 0, nTris = 0, nSpheres = 0, nPlanes = 0;
};

// buildBLASForMesh (RTContext.swift:430-435)
static BLAS buildBLASForMesh(const std::vector<PrimitiveInfo>& prims, int64_t lo, int64_t hi) {
    std::vector<PrimitiveInfo> subset;
    for (const auto& p : prims)
        if (p.type == G_TRIANGLE && p.primitiveIndex >= lo && p.primitiveIndex < hi) subset.push_back(p);
    BVHBuilder b(subset, 2, 12);
    return BLAS{b.bvhNode, b.primitiveIdx, subset, b.rootNodeIdx};
}
// makeInstance (RTContext.swift:437-457)
static Instance makeInstance(std::shared_ptr<BLAS> base, const M4& M, int materialOverride, V3 motion) {
    V3 minW = v3(kInf, kInf, kInf), maxW = v3(-kInf, -kInf, -kInf);
    for (const auto& p : base->prims) {
        AABB wb = p.bounds.transformed(M);
        minW = vmin(minW, wb.minP);
        maxW = vmax(maxW, wb.maxP);
    }
    Instance inst;
    inst.blas = base; inst.localToWorld = M; inst.worldToLocal = m4_inverse(M);
    inst.worldBounds.minP = minW; inst.worldBounds.maxP = maxW;
    inst.materialOverride = materialOverride; inst.instanceMotion = motion;
    inst.normalMatrix = normal_matrix(M);
    return inst;
}
static BLAS singlePrimBLAS(const PrimitiveInfo& prim) {
    BVHBuilder b(std::vector<PrimitiveInfo>{prim});
    return BLAS{b.bvhNode, b.primitiveIdx, {prim}, b.rootNodeIdx};
}
static M4 m4_from(const double* t) { M4 r; std::memcpy(r.m, t, sizeof(r.m)); return r; }

// RTContext.init(scene:) restricted to what the descriptor carries (RTContext.swift:94-418)
static int buildContext(const rt_scene_desc* d, Context& C, std::string& err) {
    C.intersectionTestEpsilon = d->intersection_test_epsilon;
    C.shadowRayEpsilon = d->shadow_ray_epsilon;
    C.backgroundColor = fromc(d->background_color);
    C.ambientLight = fromc(d->ambient_light);
    C.maxRecursionDepth = d->max_recursion_depth;
    for (int i = 0; i < d->num_materials; ++i) {
        const rt_material& m = d->materials[i];
        C.materials.push_back(Material{fromc(m.ambient), fromc(m.diffuse), fromc(m.specular), fromc(m.mirror),
                                       fromc(m.absorption), m.phong, m.ior, m.absorption_index, m.roughness, m.type});
    }
    for (int i = 0; i < d->num_point_lights; ++i)
        C.pointLights.push_back(PointLight{fromc(d->point_lights[i].position), fromc(d->point_lights[i].intensity)});
    for (int i = 0; i < d->num_area_lights; ++i) {
        const rt_area_light& a = d->area_lights[i];
        C.areaLights.push_back(AreaLight{fromc(a.position), fromc(a.normal), fromc(a.radiance), a.size});
    }
    for (int i = 0; i < d->num_cameras; ++i) {
        const rt_camera& c = d->cameras[i];
        Camera cam;
        cam.type = c.type; cam.width = c.width; cam.height = c.height; cam.numSamples = c.num_samples;
        cam.position = fromc(c.position); cam.gazePoint = fromc(c.gaze_point); cam.gaze = fromc(c.gaze);
        cam.up = fromc(c.up); cam.fovy = c.fovy; cam.nearDistance = c.near_distance;
        for (int k = 0; k < 4; ++k) cam.nearPlane[k] = c.near_plane[k];
        cam.apertureSize = c.aperture_size; cam.focusDistance = c.focus_distance;
        C.cameras.push_back(cam);
    }

    std::vector<PrimitiveInfo> bvhPrims;
    int64_t currentSphereIndex = 0, currentPlaneIndex = 0, currentTriangleIndex = 0;
    struct Base { std::shared_ptr<BLAS> blas; int material; M4 transform; };
    std::map<int, Base> instanceByID;
    std::vector<int> meshOrder;     // H11: base meshes in scene order (first appearance)
    std::vector<Instance> instArray;
    std::vector<const rt_object*> meshInstances;

    for (int oi = 0; oi < d->num_objects; ++oi) {
        const rt_object& o = d->objects[oi];
        const int matID = o.material_id;
        const M4 M = m4_from(o.transform);
        if (o.kind == RT_OBJ_SPHERE) {                                        // :122-160
            C.nSpheres++;
            Sphere sph{fromc(o.center), o.radius};
            C.spheres.push_back(sph);
            PrimitiveInfo prim{G_SPHERE, currentSphereIndex, AABB(), sph.center, matID, S_SMOOTH};
            prim.bounds.minP = sph.center - sph.radius; prim.bounds.maxP = sph.center + sph.radius;
            auto blas = std::make_shared<BLAS>(singlePrimBLAS(prim));
            instArray.push_back(makeInstance(blas, M, matID, v3(0, 0, 0)));
            currentSphereIndex++;
        } else if (o.kind == RT_OBJ_PLANE) {                                  // :161-192
            C.nPlanes++;
            Plane pl{fromc(o.center), fromc(o.normal)};
            C.planes.push_back(pl);
            PrimitiveInfo prim{G_PLANE, currentPlaneIndex, AABB(), v3(0, 0, 0), matID, S_SMOOTH};
            prim.bounds.minP = v3(-1e5, -1e5, -1e5); prim.bounds.maxP = v3(1e5, 1e5, 1e5);
            auto blas = std::make_shared<BLAS>(singlePrimBLAS(prim));
            instArray.push_back(makeInstance(blas, M, matID, v3(0, 0, 0)));
            currentPlaneIndex++;
        } else if (o.kind == RT_OBJ_TRIANGLE) {                               // :193-235
            C.nTris++;
            Triangle tri{};
            tri.v0 = fromc(o.v[0]); tri.v1 = fromc(o.v[1]); tri.v2 = fromc(o.v[2]);
            tri.e1 = tri.v1 - tri.v0; tri.e2 = tri.v2 - tri.v0;
            tri.centroid = ((tri.v0 + tri.v1) + tri.v2) / 3.0;
            V3 n = normalize(cross(tri.e1, tri.e2));
            tri.n0 = tri.n1 = tri.n2 = n;
            tri.motionBlur = fromc(o.motion_blur);
            C.triangles.push_back(tri);
            PrimitiveInfo prim{G_TRIANGLE, currentTriangleIndex, AABB(), tri.centroid, matID, S_FLAT};
            prim.bounds.minP = vmin(tri.v0, vmin(tri.v1, tri.v2));
            prim.bounds.maxP = vmax(tri.v0, vmax(tri.v1, tri.v2));
            auto blas = std::make_shared<BLAS>(singlePrimBLAS(prim));
            instArray.push_back(makeInstance(blas, M, matID, v3(0, 0, 0)));
            currentTriangleIndex++;
        } else if (o.kind == RT_OBJ_MESH_INSTANCE) {                          // :236-241
            meshInstances.push_back(&o);
        } else if (o.kind == RT_OBJ_MESH) {                                   // :242-377
            C.nMeshes++;
            if (o.ply_path != nullptr) { err = "oracle: PLY-path meshes unsupported; pass inline arrays"; return RT_ERR_UNSUPPORTED; }
            const int64_t start = (int64_t)C.triangles.size();
            const bool isSmooth = o.smooth != 0;
            const double* P = o.positions;
            const int32_t* I = o.indices;
            const int64_t triCount = o.num_indices / 3;
            auto pos = [&](int64_t k) { return v3(P[3 * k], P[3 * k + 1], P[3 * k + 2]); };
            const V3 mb = fromc(o.motion_blur);
            const bool blur = !(mb.x == 0 && mb.y == 0 && mb.z == 0);
            C.nTris += triCount;
            auto pushPrim = [&](const Triangle& t) {
                V3 bv0 = blur ? t.v0 + mb : t.v0, bv1 = blur ? t.v1 + mb : t.v1, bv2 = blur ? t.v2 + mb : t.v2;
                AABB bnd;
                bnd.minP = vmin(vmin(t.v0, vmin(t.v1, t.v2)), vmin(bv0, vmin(bv1, bv2)));
                bnd.maxP = vmax(vmax(t.v0, vmax(t.v1, t.v2)), vmax(bv0, vmax(bv1, bv2)));
                bvhPrims.push_back(PrimitiveInfo{G_TRIANGLE, currentTriangleIndex, bnd, t.centroid, matID,
                                                 isSmooth ? S_SMOOTH : S_FLAT});
                currentTriangleIndex++;
            };
            if (o.normals != nullptr) {                                      // :267-297
                const double* Nn = o.normals;
                auto nrm = [&](int64_t k) { return v3(Nn[3 * k], Nn[3 * k + 1], Nn[3 * k + 2]); };
                for (int64_t t = 0; t < triCount; ++t) {
                    int64_t i0 = I[3 * t], i1 = I[3 * t + 1], i2 = I[3 * t + 2];
                    Triangle tr{};
                    tr.v0 = pos(i0); tr.v1 = pos(i1); tr.v2 = pos(i2);
                    tr.e1 = tr.v1 - tr.v0; tr.e2 = tr.v2 - tr.v0;
                    tr.centroid = ((tr.v0 + tr.v1) + tr.v2) / 3.0;
                    tr.n0 = nrm(i0); tr.n1 = nrm(i1); tr.n2 = nrm(i2);
                    tr.motionBlur = mb;
                    C.triangles.push_back(tr);
                    pushPrim(tr);
                }
            } else {                                                         // :298-363
                const int64_t off = o.indices_one_based ? 1 : 0;
                std::vector<V3> faceNormals(triCount);
                for (int64_t t = 0; t < triCount; ++t) {
                    V3 v0 = pos(I[3 * t] - off), v1 = pos(I[3 * t + 1] - off), v2 = pos(I[3 * t + 2] - off);
                    faceNormals[t] = normalize(cross(v1 - v0, v2 - v0));
                }
                std::vector<V3> vtx(o.num_positions, v3(0, 0, 0));
                if (isSmooth) {
                    for (int64_t t = 0; t < triCount; ++t) {
                        V3 fn = faceNormals[t];
                        vtx[I[3 * t] - off] += fn;
                        vtx[I[3 * t + 1] - off] += fn;
                        vtx[I[3 * t + 2] - off] += fn;
                    }
                    for (auto& v : vtx) v = normalize(v);
                }
                for (int64_t t = 0; t < triCount; ++t) {
                    int64_t i0 = I[3 * t] - off, i1 = I[3 * t + 1] - off, i2 = I[3 * t + 2] - off;
                    Triangle tr{};
                    tr.v0 = pos(i0); tr.v1 = pos(i1); tr.v2 = pos(i2);
                    tr.e1 = tr.v1 - tr.v0; tr.e2 = tr.v2 - tr.v0;
                    tr.centroid = ((tr.v0 + tr.v1) + tr.v2) / 3.0;
                    tr.motionBlur = mb;
                    if (isSmooth) { tr.n0 = vtx[i0]; tr.n1 = vtx[i1]; tr.n2 = vtx[i2]; }
                    else { V3 n = normalize(faceNormals[t]); tr.n0 = tr.n1 = tr.n2 = n; }
                    C.triangles.push_back(tr);
                    pushPrim(tr);
                }
            }
            const int64_t end = (int64_t)C.triangles.size();
            if (std::find(meshOrder.begin(), meshOrder.end(), o.id) == meshOrder.end()) meshOrder.push_back(o.id);
            if (end > start) {
                auto blas = std::make_shared<BLAS>(buildBLASForMesh(bvhPrims, start, end));
                instanceByID[o.id] = Base{blas, matID, M};
            } else {
                instanceByID.erase(o.id);
            }
        }
    }
    // MeshInstances (RTContext.swift:384-401)
    std::map<int, Base> baseByMesh = instanceByID;   // meshes only, captured before instances cascade
    for (const rt_object* mi : meshInstances) {
        auto it = instanceByID.find(mi->base_mesh_id);
        if (it == instanceByID.end()) continue;
        const M4 T = m4_from(mi->transform);
        instArray.push_back(makeInstance(it->second.blas, T, mi->material_id, fromc(mi->motion_blur)));
        instanceByID[mi->id] = Base{it->second.blas, mi->material_id, T};
    }
    // base-mesh instances (RTContext.swift:403-410), scene order (H11)
    for (int meshID : meshOrder) {
        auto it = instanceByID.find(meshID);
        if (it == instanceByID.end()) continue;
        instArray.push_back(makeInstance(it->second.blas, it->second.transform, it->second.material, v3(0, 0, 0)));
    }
    (void)baseByMesh;
    if (!instArray.empty()) {                                                // buildTLAS :459-474
        std::vector<PrimitiveInfo> tlasPrims;
        for (size_t i = 0; i < instArray.size(); ++i) {
            const AABB& b = instArray[i].worldBounds;
            V3 c = (b.minP + b.maxP) * 0.5;
            tlasPrims.push_back(PrimitiveInfo{G_MESH, (int64_t)i, b, c, instArray[i].materialOverride, S_SMOOTH});
        }
        C.tlasBuilder = BVHBuilder(tlasPrims, 2, 12);
        C.instances = std::move(instArray);
        C.hasTlas = true;
    }
    return RT_OK;
}

// --------------------------------------------------------------- intersection
// hitAABB closure (RTContext.swift:557-565, :632-640, :731-739, :791-799)
static inline double hitAABB(const BVHNode& n, const Ray& r, double eps) {
    V3 t1 = (n.aabbMin - r.origin) * r.invDir;
    V3 t2 = (n.aabbMax - r.origin) * r.invDir;
    V3 tminv = vmin(t1, t2);
    V3 tmaxv = vmax(t1, t2);
    double tmin = smax(smax(tminv.x, tminv.y), tminv.z);
    double tmax = smin(tmaxv.x, smin(tmaxv.y, tmaxv.z));
    return (tmax >= smax(tmin, eps)) ? tmin : kInf;
}
// intersectTriangle (RTContext.swift:479-510)
static inline void intersectTriangle(Ray& ray, const Triangle& tri, bool isSmooth, int matIdx, double eps) {
    V3 offset = tri.motionBlur * ray.time;
    V3 origin = ray.origin - offset;
    V3 pvec = cross(ray.dir, tri.e2);
    double det = dot(tri.e1, pvec);
    if (std::fabs(det) < eps) return;
    double invDet = 1.0 / det;
    V3 tvec = origin - tri.v0;
    double u = dot(tvec, pvec) * invDet;
    if (u < 0.0 || u > 1.0) return;
    V3 q = cross(tvec, tri.e1);
    double v = dot(ray.dir, q) * invDet;
    if (v < 0.0 || u + v > 1.0) return;
    double t = dot(tri.e2, q) * invDet;
    if (t <= smax(eps, ray.tMin) || t >= ray.hit.t) return;
    double w = 1.0 - u - v;
    V3 n;
    if (isSmooth) n = normalize(((w * tri.n0) + (u * tri.n1)) + (v * tri.n2));
    else n = normalize(cross(tri.e1, tri.e2));
    V3 p = (tri.v0 + (u * tri.e1)) + (v * tri.e2);
    ray.hit.t = t; ray.hit.p = p; ray.hit.n = n; ray.hit.kind = G_TRIANGLE; ray.hit.mat = matIdx;
}
// intersectSphere (RTContext.swift:513-527)
static inline void intersectSphere(Ray& ray, const Sphere& s, int matIdx, double eps) {
    V3 oc = ray.origin - s.center;
    double a = dot(ray.dir, ray.dir);
    double b = 2.0 * dot(oc, ray.dir);
    double c = dot(oc, oc) - s.radius * s.radius;
    double disc = b * b - (4 * a) * c;
    if (disc < 0) return;
    double sd = std::sqrt(disc);
    double t = (-b - sd) / (2 * a);
    if (t < eps) t = (-b + sd) / (2 * a);
    if (t <= smax(eps, ray.tMin) || t >= ray.hit.t) return;
    V3 p = ray.origin + ray.dir * t;
    V3 n = normalize(p - s.center);
    ray.hit.t = t; ray.hit.p = p; ray.hit.n = n; ray.hit.kind = G_SPHERE; ray.hit.mat = matIdx;
}
// intersectPlane (RTContext.swift:530-538)
static inline void intersectPlane(Ray& ray, const Plane& pl, int matIdx, double eps) {
    double denom = dot(pl.normal, ray.dir);
    if (std::fabs(denom) < eps) return;
    double t = dot(pl.center - ray.origin, pl.normal) / denom;
    if (t <= smax(eps, ray.tMin) || t >= ray.hit.t) return;
    V3 p = ray.origin + ray.dir * t;
    V3 n = normalize(pl.normal);
    ray.hit.t = t; ray.hit.p = p; ray.hit.n = n; ray.hit.kind = G_PLANE; ray.hit.mat = matIdx;
}
static inline bool triShadowHit(const Ray& ray, const Triangle& tri, double eps) {   // :832-848
    V3 offset = tri.motionBlur * ray.time;
    V3 origin = ray.origin - offset;
    V3 pvec = cross(ray.dir, tri.e2);
    double det = dot(tri.e1, pvec);
    if (std::fabs(det) < eps) return false;
    double invDet = 1.0 / det;
    V3 tvec = origin - tri.v0;
    double u = dot(tvec, pvec) * invDet;
    if (u < 0.0 || u > 1.0) return false;
    V3 q = cross(tvec, tri.e1);
    double v = dot(ray.dir, q) * invDet;
    if (v < 0.0 || u + v > 1.0) return false;
    double t = dot(tri.e2, q) * invDet;
    return (t > smax(eps, ray.tMin) && t < ray.tMax);
}
static inline bool sphereShadowHit(const Ray& ray, const Sphere& s, double eps) {   // :851-862
    V3 oc = ray.origin - s.center;
    double a = dot(ray.dir, ray.dir);
    double b = 2.0 * dot(oc, ray.dir);
    double c = dot(oc, oc) - s.radius * s.radius;
    double disc = b * b - (4 * a) * c;
    if (disc < 0) return false;
    double sd = std::sqrt(disc);
    double t = (-b - sd) / (2 * a);
    if (t < smax(eps, ray.tMin)) t = (-b + sd) / (2 * a);
    return (t > smax(eps, ray.tMin) && t < ray.tMax);
}
static inline bool planeShadowHit(const Ray& ray, const Plane& pl, double eps) {     // :865-870
    double denom = dot(pl.normal, ray.dir);
    if (std::fabs(denom) < eps) return false;
    double t = dot(pl.center - ray.origin, pl.normal) / denom;
    return (t > smax(eps, ray.tMin) && t < ray.tMax);
}

// intersectBLAS (RTContext.swift:544-610)
static void intersectBLAS(const Context& C, Ray& ray, const Instance& inst, double eps, Counters& k) {
    const BLAS& B = *inst.blas;
    uint64_t stack[64];
    int sp = 0;
    stack[sp] = B.root;
    k.nodeFetch += 1;                       // the root's bounds
    while (sp >= 0) {
        k.visits += 1;
        const uint64_t idx = stack[sp]; sp -= 1;
        const BVHNode& node = B.nodes[idx];
        if (hitAABB(node, ray, eps) == kInf) continue;
        if (node.isLeaf()) {
            for (uint64_t q = 0; q < node.primitiveCount; ++q) {
                const PrimitiveInfo& p = B.prims[B.primIdx[node.leftFirst + q]];
                switch (p.type) {
                case G_TRIANGLE: {
                    k.triTest += 1;
                    double before = ray.hit.t;
                    intersectTriangle(ray, C.triangles[p.primitiveIndex], p.shadingMode == S_SMOOTH, p.materialID, eps);
                    if (ray.hit.t != before && p.shadingMode == S_SMOOTH) k.smoothHit += 1;
                    break;
                }
                case G_SPHERE: intersectSphere(ray, C.spheres[p.primitiveIndex], p.materialID, eps); break;
                case G_PLANE: intersectPlane(ray, C.planes[p.primitiveIndex], p.materialID, eps); break;
                default: break;
                }
            }
            continue;
        }
        uint64_t L = node.leftFirst, R = L + 1;
        k.nodeFetch += 2;
        double d1 = hitAABB(B.nodes[L], ray, eps), d2 = hitAABB(B.nodes[R], ray, eps);
        if (d1 > d2) { std::swap(d1, d2); std::swap(L, R); }
        if (d2 != kInf) { sp += 1; if (sp >= 64) std::abort(); stack[sp] = R; }
        if (d1 != kInf) { sp += 1; if (sp >= 64) std::abort(); stack[sp] = L; }
    }
}

// world <-> local helpers shared by intersectTLAS / occludedTLAS (RTContext.swift:657-673, 754-769)
static inline Ray toLocal(const Ray& worldRay, const Instance& inst) {
    V3 instOffset = inst.instanceMotion * worldRay.time;
    Ray rL = worldRay;
    rL.time = worldRay.time;
    rL.origin = rL.origin - instOffset;
    double o4[4], d4[4];
    m4_mul(inst.worldToLocal, rL.origin.x, rL.origin.y, rL.origin.z, 1.0, o4);
    m4_mul(inst.worldToLocal, rL.dir.x, rL.dir.y, rL.dir.z, 0.0, d4);
    rL.origin = v3(o4[0], o4[1], o4[2]);
    rL.dir = v3(d4[0], d4[1], d4[2]);
    rL.invDir = 1.0 / rL.dir;
    rL.tMax = worldRay.tMax;
    rL.hit = worldRay.hit;
    rL.hit.t = worldRay.hit.t;
    return rL;
}

// intersectTLAS (RTContext.swift:619-720)
static void intersectTLAS(const Context& C, Ray& worldRay, double eps, Counters& k) {
    const BVHBuilder& T = C.tlasBuilder;
    uint64_t stack[64];
    int sp = 0;
    stack[sp] = T.rootNodeIdx;
    k.nodeFetch += 1;
    while (sp >= 0) {
        k.visits += 1;
        const uint64_t idx = stack[sp]; sp -= 1;
        const BVHNode& node = T.bvhNode[idx];
        if (hitAABB(node, worldRay, eps) == kInf) continue;
        if (node.isLeaf()) {
            for (uint64_t q = 0; q < node.primitiveCount; ++q) {
                const PrimitiveInfo& p = T.primitives[T.primitiveIdx[node.leftFirst + q]];
                if (p.type != G_MESH) continue;
                const Instance& inst = C.instances[p.primitiveIndex];
                Ray tmp = toLocal(worldRay, inst);
                intersectBLAS(C, tmp, inst, eps, k);
                if (tmp.hit.t < worldRay.hit.t) {
                    V3 instOffset = inst.instanceMotion * worldRay.time;
                    double wp[4];
                    m4_mul(inst.localToWorld, tmp.hit.p.x, tmp.hit.p.y, tmp.hit.p.z, 1.0, wp);
                    V3 wn = normalize(m3_mul(inst.normalMatrix, tmp.hit.n));
                    if (m3_det(m3_of(inst.localToWorld)) < 0.0) wn = -wn;
                    worldRay.hit.t = tmp.hit.t;
                    worldRay.hit.p = v3(wp[0], wp[1], wp[2]) + instOffset;
                    worldRay.hit.n = wn;
                    worldRay.hit.kind = tmp.hit.kind;
                    worldRay.hit.mat = inst.materialOverride;   // materialOverride ?? hit.mat; always set
                }
            }
            continue;
        }
        uint64_t L = node.leftFirst, R = L + 1;
        k.nodeFetch += 2;
        double d1 = hitAABB(T.bvhNode[L], worldRay, eps), d2 = hitAABB(T.bvhNode[R], worldRay, eps);
        if (d1 > d2) { std::swap(d1, d2); std::swap(L, R); }
        if (d2 != kInf) { sp += 1; stack[sp] = R; }
        if (d1 != kInf) { sp += 1; stack[sp] = L; }
    }
}

// occludedBLAS (RTContext.swift:784-829)
static bool occludedBLAS(const Context& C, const Ray& r, const Instance& inst, double eps, Counters& k) {
    const BLAS& B = *inst.blas;
    uint64_t stack[256]; int sp = 0;        // the Swift [UInt] heap stack, fixed-size here
    stack[sp++] = B.root;
    while (sp > 0) {
        const uint64_t idx = stack[--sp];
        k.nodeFetch += 1;
        const BVHNode& node = B.nodes[idx];
        if (hitAABB(node, r, eps) == kInf) continue;
        if (node.isLeaf()) {
            for (uint64_t q = 0; q < node.primitiveCount; ++q) {
                const PrimitiveInfo& p = B.prims[B.primIdx[node.leftFirst + q]];
                switch (p.type) {
                case G_TRIANGLE: k.triTest += 1; if (triShadowHit(r, C.triangles[p.primitiveIndex], eps)) return true; break;
                case G_SPHERE: if (sphereShadowHit(r, C.spheres[p.primitiveIndex], eps)) return true; break;
                case G_PLANE: if (planeShadowHit(r, C.planes[p.primitiveIndex], eps)) return true; break;
                default: break;
                }
            }
        } else {
            if (sp + 2 > 256) std::abort();
            stack[sp++] = node.leftFirst + 1;
            stack[sp++] = node.leftFirst;
        }
    }
    return false;
}
// occludedTLAS (RTContext.swift:724-781)
static bool occludedTLAS(const Context& C, const Ray& worldRay, double eps, Counters& k) {
    const BVHBuilder& T = C.tlasBuilder;
    std::vector<uint64_t> stack{T.rootNodeIdx};
    while (!stack.empty()) {
        const uint64_t idx = stack.back(); stack.pop_back();
        k.nodeFetch += 1;
        const BVHNode& node = T.bvhNode[idx];
        if (hitAABB(node, worldRay, eps) == kInf) continue;
        if (node.isLeaf()) {
            for (uint64_t q = 0; q < node.primitiveCount; ++q) {
                const PrimitiveInfo& p = T.primitives[T.primitiveIdx[node.leftFirst + q]];
                if (p.type != G_MESH) continue;
                const Instance& inst = C.instances[p.primitiveIndex];
                Ray rL = toLocal(worldRay, inst);
                if (occludedBLAS(C, rL, inst, eps, k)) return true;
            }
        } else {
            stack.push_back(node.leftFirst + 1);
            stack.push_back(node.leftFirst);
        }
    }
    return false;
}

// ------------------------------------------------------------------------ RNG
// PCG32 (Object+Extension.swift:556-589)
struct PCG32 {
    uint64_t state, inc;
    explicit PCG32(uint64_t seed) {
        state = 0; inc = (seed << 1) | 1u;
        (void)next();
        state += 0x9E3779B97F4A7C15ull;
        (void)next();
    }
    uint32_t next() {
        uint64_t old = state;
        state = old * 6364136223846793005ull + inc;
        uint32_t xorshifted = (uint32_t)(((old >> 18) ^ old) >> 27);
        uint32_t rot = (uint32_t)(old >> 59);
        return (xorshifted >> rot) | (xorshifted << ((~rot + 1u) & 31u));
    }
    double nextFloat() { return double(next()) * 2.3283064365386963e-10; }
};

// ------------------------------------------------------------------- renderer
struct CamBasis { V3 eye, u, v, w; double l, r, b, t, nd; bool isLookAt; };
// makeCameraBasis (Object+Extension.swift:382-427)
static CamBasis makeCameraBasis(const Camera& cam, double aspect) {
    CamBasis B;
    B.eye = cam.position; B.nd = cam.nearDistance;
    if (cam.type == RT_CAM_LOOKAT) {
        V3 gaze = cam.gazePoint - cam.position;
        V3 gazeNorm = normalize(gaze);
        B.w = -gazeNorm;
        V3 upNorm = normalize(cam.up);
        B.u = normalize(cross(upNorm, B.w));
        B.v = normalize(cross(B.w, B.u));
        if (!std::isnan(cam.fovy)) {
            double fovYRad = (cam.fovy * M_PI) / (2.0 * 180.0);
            B.t = B.nd * std::tan(fovYRad);
        } else {
            B.t = B.nd * 0.5;
        }
        B.b = -B.t; B.r = B.t * aspect; B.l = -B.r;
        B.isLookAt = true;
    } else {
        B.l = cam.nearPlane[0]; B.r = cam.nearPlane[1]; B.b = cam.nearPlane[2]; B.t = cam.nearPlane[3];
        V3 gazeNorm = normalize(cam.gaze);
        B.w = -gazeNorm;
        V3 upNorm = normalize(cam.up);
        B.u = normalize(cross(upNorm, B.w));
        B.v = normalize(cross(B.w, B.u));
        B.isLookAt = false;
    }
    return B;
}
// reflect (:467), orthonormalBasis (:531-552), fresnel helpers (:477-505), beerAttenuate (:470-474)
static inline V3 reflect(V3 d, V3 n) { return d - (2.0 * dot(d, n)) * n; }
static inline void orthonormalBasis(V3 n, V3& tangent, V3& bitangent) {
    double sign = n.z >= 0 ? 1.0 : -1.0;
    double a = -1.0 / (sign + n.z);
    double b = (n.x * n.y) * a;
    tangent = normalize(v3(1.0 + ((sign * n.x) * n.x) * a, sign * b, (-sign) * n.x));
    bitangent = normalize(v3(b, sign + (n.y * n.y) * a, -n.y));
}
static inline void fresnelDielectric(double n1, double n2, double cosI, double& R, bool& hasCosT, double& cosT, double& sin2T) {
    double cosTheta = smax(0.0, smin(1.0, std::fabs(cosI)));
    double eta = n1 / n2;
    sin2T = (eta * eta) * smax(0.0, 1.0 - cosTheta * cosTheta);
    if (sin2T > 1.0) { R = 1.0; hasCosT = false; cosT = 0; return; }
    double cosPhi = std::sqrt(smax(0.0, 1.0 - sin2T));
    double Rs = (n2 * cosTheta - n1 * cosPhi) / (n2 * cosTheta + n1 * cosPhi);
    double Rp = (n1 * cosTheta - n2 * cosPhi) / (n1 * cosTheta + n2 * cosPhi);
    R = 0.5 * (Rs * Rs + Rp * Rp); hasCosT = true; cosT = cosPhi;
}
static inline V3 fresnelConductorRGB(double eta, double k, double cosI_) {
    double cosI = smax(0.0, smin(1.0, std::fabs(cosI_)));
    double cos2 = cosI * cosI;
    V3 one = v3(1, 1, 1);
    double eta2 = eta * eta, k2 = k * k, eta2k2 = eta2 + k2;
    double twoEtaCos = (2.0 * eta) * cosI;
    V3 cos2v = v3(cos2, cos2, cos2);
    V3 Rs = ((eta2k2 - twoEtaCos) + cos2v) / ((eta2k2 + twoEtaCos) + cos2v);
    V3 Rp = (((eta2k2 * cos2v) - twoEtaCos) + one) / (((eta2k2 * cos2v) + twoEtaCos) + one);
    return 0.5 * (Rs + Rp);
}
static inline V3 vexp(V3 a) { return {std::exp(a.x), std::exp(a.y), std::exp(a.z)}; }

struct Renderer {
    const Context& C;
    int maxDepth;
    double eps, shadowEps;
    std::vector<double> jitterX, jitterY;

    explicit Renderer(const Context& c) : C(c), maxDepth(c.maxRecursionDepth), eps(c.intersectionTestEpsilon),
                                          shadowEps(c.shadowRayEpsilon), jitterX(100), jitterY(100) {
        PCG32 rng(0x123456789ABCDEFull);                       // :92-93, buildStratifiedJitter :646-659
        int q = 0;
        for (int gy = 0; gy < 10; ++gy)
            for (int gx = 0; gx < 10; ++gx) {
                jitterX[q] = double(gx) + rng.nextFloat();
                jitterY[q] = double(gy) + rng.nextFloat();
                q++;
            }
    }
    bool occluded(const Ray& r, Counters& k) const {           // :429-433
        if (!C.hasTlas) return false;
        return occludedTLAS(C, r, eps, k);
    }
    // trace (Object+Extension.swift:96-283)
    V3 trace(Ray& inRay, int depth, PCG32& rng, int64_t& jitterIndex, Counters& k) const {
        if (depth > maxDepth) return C.backgroundColor;
        if (!C.hasTlas) return v3(0, 0, 0);
        intersectTLAS(C, inRay, eps, k);
        if (inRay.hit.kind == -1) return C.backgroundColor;
        const int nm = (int)C.materials.size();
        const int matIndex = std::max(0, std::min(nm - 1, inRay.hit.mat - 1));
        const Material& mat = C.materials[matIndex];
        const V3 p = inRay.hit.p;
        const V3 Ngeo = inRay.hit.n;
        const bool frontFacing = dot(inRay.dir, Ngeo) < 0;
        const V3 N = frontFacing ? Ngeo : -Ngeo;
        const bool hasRefraction = (mat.ior > 0);
        const bool computeDirectLight = !hasRefraction || frontFacing;
        V3 Lo = computeDirectLight ? C.ambientLight * mat.ambient : v3(0, 0, 0);
        if (computeDirectLight) {
            for (const PointLight& pl : C.pointLights) {                   // :118-143
                V3 wi = pl.position - p;
                double dist = length(wi);
                wi = normalize(wi);
                Ray sRay(p + wi * shadowEps, wi, inRay.time);
                sRay.tMax = dist;
                k.shadow += 1;
                if (smax(0.0, dot(N, wi)) > 0) k.shadowUsed += 1;   // (instrumentation only)
                bool blocked = occluded(sRay, k);
                if (!blocked) {
                    double NdotL = smax(0.0, dot(N, wi));
                    if (NdotL > 0) {
                        V3 kd = mat.diffuse, ks = mat.specular;
                        double shininess = smax(1.0, mat.phong);
                        V3 Ld = kd * NdotL;
                        V3 view = normalize(-inRay.dir);
                        V3 h = normalize(wi + view);
                        double NdotH = smax(0.0, dot(N, h));
                        V3 Ls = ks * std::pow(NdotH, shininess);
                        V3 atten = pl.intensity / smax(dist * dist, 1e-12);
                        Lo += (Ld + Ls) * atten;
                    }
                }
            }
            for (const AreaLight& al : C.areaLights) {                     // :145-186
                V3 nL = normalize(al.normal);
                V3 t, b;
                orthonormalBasis(nL, t, b);
                double size = al.size;
                double area = size * size;
                double r1 = jitterX[jitterIndex % 100] / 10.0 - 0.5;
                double r2 = jitterY[jitterIndex % 100] / 10.0 - 0.5;
                jitterIndex += 1;
                V3 samplePos = (al.position + t * (r1 * size)) + b * (r2 * size);
                V3 wi = samplePos - p;
                double dist2 = dot(wi, wi);
                double dist = std::sqrt(dist2);
                wi = wi / dist;
                double NdotL = dot(N, wi);
                if (NdotL <= 0) continue;
                double Ln = std::fabs(dot(nL, -wi));
                if (Ln <= 0) continue;
                Ray sRay(p + wi * shadowEps, wi, inRay.time);
                sRay.tMax = dist - shadowEps;
                k.shadow += 1;
                k.shadowUsed += 1;
                if (occluded(sRay, k)) continue;
                V3 view = normalize(-inRay.dir);
                V3 h = normalize(wi + view);
                V3 Ld = mat.diffuse * NdotL;
                V3 Ls = mat.specular * std::pow(smax(0.0, dot(N, h)), mat.phong);
                V3 brdf = Ld + Ls;
                V3 contrib = ((brdf * al.radiance) * (Ln / dist2)) * area;
                Lo += contrib;
            }
        }
        if (mat.type == RT_MAT_MIRROR && depth < maxDepth) {                // :189-206
            V3 rd = normalize(reflect(inRay.dir, N));
            if (mat.roughness != 0.0) {
                V3 t, b;
                orthonormalBasis(rd, t, b);
                double rand1 = rng.nextFloat() - 0.5;
                double rand2 = rng.nextFloat() - 0.5;
                rd = (rd + (mat.roughness * rand1) * b) + (mat.roughness * rand2) * t;
                rd = normalize(rd);
            }
            Ray rRay = inRay;
            rRay.tMin = 0; rRay.origin = p + N * shadowEps; rRay.dir = rd; rRay.invDir = 1.0 / rd; rRay.hit = Hit();
            k.secondary += 1;
            V3 Li = trace(rRay, depth + 1, rng, jitterIndex, k);
            Lo += mat.mirror * Li;
        } else if (mat.type == RT_MAT_DIELECTRIC && depth < maxDepth) {    // :207-251
            V3 microfacetN = N;
            if (mat.roughness != 0.0) {
                V3 t, b;
                orthonormalBasis(N, t, b);
                double r1 = (rng.nextFloat() * 2.0) - 1.0;
                double r2 = (rng.nextFloat() * 2.0) - 1.0;
                microfacetN = normalize((N + ((t * r1) * mat.roughness)) + ((b * r2) * mat.roughness));
            }
            const bool entering = frontFacing;
            const double n1 = entering ? 1.0 : mat.ior;
            const double n2 = entering ? mat.ior : 1.0;
            const double cosI = -dot(inRay.dir, microfacetN);
            double R, cosT, sin2T; bool hasCosT;
            fresnelDielectric(n1, n2, cosI, R, hasCosT, cosT, sin2T);
            V3 rd = normalize(reflect(inRay.dir, microfacetN));
            Ray rRay = inRay;
            rRay.tMin = 0; rRay.origin = p + rd * shadowEps; rRay.dir = rd; rRay.invDir = 1.0 / rd; rRay.hit = Hit();
            k.secondary += 1;
            V3 LiR = trace(rRay, depth + 1, rng, jitterIndex, k);
            if (!hasCosT || sin2T > 1) {
                Lo += LiR;
            } else {
                const double eta = n1 / n2;
                V3 td = normalize((inRay.dir * eta) + (microfacetN * (eta * cosI - cosT)));
                Ray tRay(p + td * shadowEps, td, inRay.time);
                k.secondary += 1;
                V3 LiT = trace(tRay, depth + 1, rng, jitterIndex, k);
                const bool absNonZero = !(mat.absorption.x == 0 && mat.absorption.y == 0 && mat.absorption.z == 0);
                if (entering && absNonZero && tRay.hit.kind != -1 && tRay.hit.mat == inRay.hit.mat) {
                    double dd = smax(tRay.hit.t, 0.0);
                    V3 att = (std::isfinite(dd) && dd > 0) ? vexp((-mat.absorption) * dd) : LiT;  // beerAttenuate quirk
                    LiT *= att;
                }
                Lo += LiR * R + LiT * (1.0 - R);
            }
        } else if (mat.type == RT_MAT_CONDUCTOR && depth < maxDepth) {     // :252-275
            const double cosI = smax(0.0, -dot(inRay.dir, N));
            V3 Rf = fresnelConductorRGB(mat.ior, mat.absorptionIndex, cosI);
            V3 rd = normalize(reflect(inRay.dir, N));
            if (mat.roughness != 0.0) {
                V3 t, b;
                orthonormalBasis(rd, t, b);
                double rand1 = rng.nextFloat() - 0.5;
                double rand2 = rng.nextFloat() - 0.5;
                rd = (rd + (mat.roughness * rand1) * b) + (mat.roughness * rand2) * t;
                rd = normalize(rd);
            }
            Ray rRay = inRay;
            rRay.tMin = 0; rRay.origin = p + N * shadowEps; rRay.dir = rd; rRay.invDir = 1.0 / rd; rRay.hit = Hit();
            k.secondary += 1;
            V3 Li = trace(rRay, depth + 1, rng, jitterIndex, k);
            Lo += (Rf * mat.mirror) * Li;
        }
        if (!isfin(Lo)) return v3(0, 0, 0);                                 // :277-280
        return Lo;
    }

    // one 8-row chunk of Renderer.render (Object+Extension.swift:287-360)
    void renderChunk(const Camera& cam, const CamBasis& B, double du, double dv, V3 q00, int startRow, int endRow,
                     double* out, Counters& k) const {
        const int width = std::max(1, cam.width);
        int64_t jitterIndex = 0;
        const double apertureSize = cam.apertureSize, focusDistance = cam.focusDistance;
        for (int j = startRow; j < endRow; ++j) {
            for (int i = 0; i < width; ++i) {
                PCG32 rng((((uint64_t)j << 32) ^ (uint64_t)i) + 0x9E3779B97F4A7C15ull);   // H7
                V3 pixelColor = v3(0, 0, 0);
                const int samples = std::max(1, cam.numSamples);
                const int n = (int)std::sqrt((double)samples);
                int sampleIndex = 0;
                for (int sy = 0; sy < n && sampleIndex < samples; ++sy) {
                    for (int sx = 0; sx < n; ++sx) {
                        double xi1 = rng.nextFloat();
                        double xi2 = rng.nextFloat();
                        double iOffset = (double(sx) + xi1) / double(n);
                        double jOffset = (double(sy) + xi2) / double(n);
                        double currentI = double(i) + iOffset;
                        double currentJ = double(j) + jOffset;
                        V3 vOff = B.v * (currentJ * dv);
                        V3 rowTopLeft = q00 - vOff;
                        V3 uOff = B.u * (currentI * du);
                        V3 s = rowTopLeft + uOff;
                        V3 dir0 = normalize(s - B.eye);
                        V3 dir = dir0;
                        V3 camEye = B.eye;
                        if (apertureSize > 0 && focusDistance > 0) {               // :325-338
                            V3 forward = -B.w;
                            double denom = dot(dir0, forward);
                            double tFocus = std::fabs(denom) < 1e-6 ? focusDistance : (focusDistance / denom);
                            V3 pFocus = B.eye + dir0 * tFocus;
                            double uRand = rng.nextFloat() - 0.5;
                            double vRand = rng.nextFloat() - 0.5;
                            V3 lensOffset = ((uRand * B.u) + (vRand * B.v)) * apertureSize;
                            V3 a = B.eye + lensOffset;
                            dir = normalize(pFocus - a);
                            camEye = a;
                        }
                        Ray ray(camEye, dir, rng.nextFloat());
                        double denom = dot(dir, B.w);
                        double tImg = dot((B.eye - B.w * B.nd) - camEye, B.w) /
                                      (denom == 0.0 ? std::numeric_limits<double>::denorm_min() : denom);
                        ray.tMin = smax(tImg, 0.0);
                        k.primary += 1;
                        V3 sampleColor = trace(ray, 0, rng, jitterIndex, k);
                        pixelColor += sampleColor;
                        sampleIndex += 1;
                        if (sampleIndex >= samples) break;
                    }
                }
                V3 px = pixelColor / double(samples);
                double* o = out + ((int64_t)(j - startRow) * width + i) * 3;
                o[0] = px.x; o[1] = px.y; o[2] = px.z;
                k.pixels += 1;
            }
        }
    }
};

struct OracleScene { Context C; };

static thread_local std::string g_err;

}  // namespace orc

// ============================================================================ C ABI
extern "C" {

typedef struct oracle_stats {
    int64_t primary_rays, shadow_rays, secondary_rays, node_visits;
    int64_t node_fetches, tri_tests, smooth_hits, pixels;
    double milliseconds;
    int32_t threads;
    int64_t shadow_rays_used;   /* shadow rays whose result is used (the GPU's shadow_rays_traced) */
} oracle_stats;

const char* oracle_last_error(void) { return orc::g_err.c_str(); }

int32_t oracle_scene_create(const rt_scene_desc* desc, void** out) {
    if (!desc || !out) return RT_ERR_INVALID_ARG;
    try {
        auto* s = new orc::OracleScene();
        int rc = orc::buildContext(desc, s->C, orc::g_err);
        if (rc != RT_OK) { delete s; return rc; }
        *out = s;
        return RT_OK;
    } catch (const std::exception& e) {
        orc::g_err = e.what();
        return RT_ERR_INVALID_ARG;
    }
}

void oracle_scene_destroy(void* s) { delete static_cast<orc::OracleScene*>(s); }

// Renders chunks chunk_first, chunk_first+chunk_step, ... (8 rows each) with `nthreads`
// workers pulling chunks like the reference's TaskGroup (Object+Extension.swift:285-376).
int32_t oracle_render(void* scene, int32_t camera_index, int32_t chunk_first, int32_t chunk_step,
                      int32_t nthreads, double* out_rgb, uint8_t* out_rgba8, oracle_stats* stats) {
    using namespace orc;
    if (!scene) return RT_ERR_NO_SCENE;
    const Context& C = static_cast<OracleScene*>(scene)->C;
    if (camera_index < 0 || camera_index >= (int)C.cameras.size()) return RT_ERR_INVALID_CAMERA;
    if (chunk_step < 1 || chunk_first < 0) return RT_ERR_INVALID_ARG;
    const Camera& cam = C.cameras[camera_index];
    const int width = std::max(1, cam.width), height = std::max(1, cam.height);
    CamBasis B = makeCameraBasis(cam, double(width) / double(height));
    const double du = (B.r - B.l) / double(width);
    const double dv = (B.t - B.b) / double(height);
    const V3 m = B.eye - B.w * B.nd;
    const V3 q00 = (m + B.u * B.l) + B.v * B.t;
    Renderer R(C);
    const int CH = 8;
    const int nChunksTotal = (height + CH - 1) / CH;
    std::vector<int> chunks;
    for (int c = chunk_first; c < nChunksTotal; c += chunk_step) chunks.push_back(c);
    std::vector<int64_t> rowOffset(chunks.size() + 1, 0);
    for (size_t q = 0; q < chunks.size(); ++q) {
        int s0 = chunks[q] * CH, e0 = std::min(s0 + CH, height);
        rowOffset[q + 1] = rowOffset[q] + (e0 - s0);
    }
    std::vector<double> local;
    double* out = out_rgb;
    if (!out) { local.resize((size_t)rowOffset.back() * width * 3); out = local.data(); }
    if (nthreads <= 0) nthreads = (int)std::max(1u, std::thread::hardware_concurrency());
    std::atomic<size_t> next{0};
    std::vector<Counters> perThread(nthreads);
    auto t0 = std::chrono::steady_clock::now();
    auto worker = [&](int tid) {
        for (;;) {
            size_t q = next.fetch_add(1);
            if (q >= chunks.size()) break;
            int s0 = chunks[q] * CH, e0 = std::min(s0 + CH, height);
            R.renderChunk(cam, B, du, dv, q00, s0, e0, out + rowOffset[q] * width * 3, perThread[tid]);
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nthreads; ++t) th.emplace_back(worker, t);
    worker(0);
    for (auto& t : th) t.join();
    auto t1 = std::chrono::steady_clock::now();
    if (out_rgba8) {                                   // RayTracer.swift:186-195
        const int64_t npx = rowOffset.back() * width;
        for (int64_t px = 0; px < npx; ++px) {
            for (int c = 0; c < 3; ++c) {
                double v = out[px * 3 + c];
                double cl = std::fmin(std::fmax(v, 0.0), 255.0);   // simd_clamp
                out_rgba8[px * 4 + c] = (uint8_t)cl;
            }
            out_rgba8[px * 4 + 3] = 255;
        }
    }
    if (stats) {
        Counters tot;
        for (auto& c : perThread) tot.add(c);
        stats->primary_rays = tot.primary; stats->shadow_rays = tot.shadow; stats->secondary_rays = tot.secondary;
        stats->node_visits = tot.visits; stats->node_fetches = tot.nodeFetch; stats->tri_tests = tot.triTest;
        stats->smooth_hits = tot.smoothHit; stats->pixels = tot.pixels;
        stats->milliseconds = std::chrono::duration<double, std::milli>(t1 - t0).count();
        stats->threads = nthreads;
        stats->shadow_rays_used = tot.shadowUsed;
    }
    return RT_OK;
}

// Canonical hash of BLAS `instance`'s BVH (preorder: bounds bits, leaf prim order) and of the
// TLAS (instance = -1), used to check the product builder's topology against this restatement.
uint64_t oracle_bvh_hash(void* scene, int32_t instance) {
    using namespace orc;
    const Context& C = static_cast<OracleScene*>(scene)->C;
    const std::vector<BVHNode>* nodes; const std::vector<uint64_t>* pidx; const std::vector<PrimitiveInfo>* prims; uint64_t root;
    if (instance < 0) { nodes = &C.tlasBuilder.bvhNode; pidx = &C.tlasBuilder.primitiveIdx; prims = &C.tlasBuilder.primitives; root = C.tlasBuilder.rootNodeIdx; }
    else {
        if (instance >= (int)C.instances.size()) return 0;
        const BLAS& b = *C.instances[instance].blas; nodes = &b.nodes; pidx = &b.primIdx; prims = &b.prims; root = b.root;
    }
    uint64_t h = 1469598103934665603ull;
    auto mix = [&](uint64_t x) { for (int i = 0; i < 8; ++i) { h ^= (x >> (8 * i)) & 0xff; h *= 1099511628211ull; } };
    auto mixd = [&](double d) { uint64_t u; std::memcpy(&u, &d, 8); mix(u); };
    std::vector<uint64_t> st{root};
    while (!st.empty()) {
        uint64_t i = st.back(); st.pop_back();
        const BVHNode& n = (*nodes)[i];
        mixd(n.aabbMin.x); mixd(n.aabbMin.y); mixd(n.aabbMin.z); mixd(n.aabbMax.x); mixd(n.aabbMax.y); mixd(n.aabbMax.z);
        if (n.isLeaf()) {
            mix(0xABCDull); mix(n.primitiveCount);
            for (uint64_t q = 0; q < n.primitiveCount; ++q) mix((uint64_t)(*prims)[(*pidx)[n.leftFirst + q]].primitiveIndex);
        } else {
            mix(0x1234ull);
            st.push_back(n.leftFirst + 1);
            st.push_back(n.leftFirst);
        }
    }
    return h;
}

int32_t oracle_num_instances(void* scene) {
    return (int32_t) static_cast<orc::OracleScene*>(scene)->C.instances.size();
}

// Known-answer helpers (tests/test_oracle_kat.py)
void oracle_pcg32_stream(uint64_t seed, int32_t n, uint32_t* out) {
    orc::PCG32 r(seed);
    for (int i = 0; i < n; ++i) out[i] = r.next();
}
double oracle_hit_aabb(const double* bmin, const double* bmax, const double* origin, const double* dir, double eps) {
    using namespace orc;
    BVHNode n; n.aabbMin = v3(bmin[0], bmin[1], bmin[2]); n.aabbMax = v3(bmax[0], bmax[1], bmax[2]);
    Ray r(v3(origin[0], origin[1], origin[2]), v3(dir[0], dir[1], dir[2]), 0.0);
    return hitAABB(n, r, eps);
}
// Moeller-Trumbore closest-hit on one triangle: returns t (or +inf), writes u-weighted normal/point.
double oracle_intersect_triangle(const double* v0, const double* v1, const double* v2, const double* origin,
                                 const double* dir, double tmin, double eps, double* p_out, double* n_out) {
    using namespace orc;
    Triangle tri{};
    tri.v0 = v3(v0[0], v0[1], v0[2]); tri.v1 = v3(v1[0], v1[1], v1[2]); tri.v2 = v3(v2[0], v2[1], v2[2]);
    tri.e1 = tri.v1 - tri.v0; tri.e2 = tri.v2 - tri.v0; tri.motionBlur = v3(0, 0, 0);
    Ray r(v3(origin[0], origin[1], origin[2]), v3(dir[0], dir[1], dir[2]), 0.0);
    r.tMin = tmin;
    intersectTriangle(r, tri, false, 1, eps);
    if (p_out) { p_out[0] = r.hit.p.x; p_out[1] = r.hit.p.y; p_out[2] = r.hit.p.z; }
    if (n_out) { n_out[0] = r.hit.n.x; n_out[1] = r.hit.n.y; n_out[2] = r.hit.n.z; }
    return r.hit.t;
}

// Explicit-ray queries (tests/test_gpu_rays.py): intersectTLAS / occludedTLAS
// (RTContext.swift:619-781) on caller-given rays, Ray(origin:dir:time:) + tMin / tMax.
int32_t oracle_trace_rays(void* scene, int32_t n, const double* o, const double* d, const double* tmin,
                          const double* time, double* out_t, double* out_p, double* out_n, int32_t* out_mat) {
    using namespace orc;
    const Context& C = static_cast<OracleScene*>(scene)->C;
    Counters k;
    for (int32_t i = 0; i < n; ++i) {
        Ray r(v3(o[3 * i], o[3 * i + 1], o[3 * i + 2]), v3(d[3 * i], d[3 * i + 1], d[3 * i + 2]), time[i]);
        r.tMin = tmin[i];
        if (C.hasTlas) intersectTLAS(C, r, C.intersectionTestEpsilon, k);
        out_t[i] = r.hit.kind == -1 ? kInf : r.hit.t;
        out_p[3 * i] = r.hit.p.x; out_p[3 * i + 1] = r.hit.p.y; out_p[3 * i + 2] = r.hit.p.z;
        out_n[3 * i] = r.hit.n.x; out_n[3 * i + 1] = r.hit.n.y; out_n[3 * i + 2] = r.hit.n.z;
        out_mat[i] = r.hit.kind == -1 ? -1 : r.hit.mat;
    }
    return RT_OK;
}
int32_t oracle_occluded_rays(void* scene, int32_t n, const double* o, const double* d, const double* tmax,
                             const double* time, uint8_t* out) {
    using namespace orc;
    const Context& C = static_cast<OracleScene*>(scene)->C;
    Counters k;
    for (int32_t i = 0; i < n; ++i) {
        Ray r(v3(o[3 * i], o[3 * i + 1], o[3 * i + 2]), v3(d[3 * i], d[3 * i + 1], d[3 * i + 2]), time[i]);
        r.tMax = tmax[i];
        out[i] = (C.hasTlas && occludedTLAS(C, r, C.intersectionTestEpsilon, k)) ? 1 : 0;
    }
    return RT_OK;
}

}  // extern "C"
