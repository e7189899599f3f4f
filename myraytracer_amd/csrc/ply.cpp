// ply.cpp — host PLY reader for the renderer core (product code).
//
// Produces exactly what the reference's PLYLoader.load (RT/Helpers/PLYReader.swift:54-210)
// gets back from its CPly/miniply layer (CPly/miniply.cpp), but is a fresh
// implementation: the whole file is read once and parsed from memory.
//   * ASCII, binary_little_endian and binary_big_endian bodies;
//   * vertex x/y/z extracted as float32 and widened to double (PLYReader.swift:85-102);
//     optional nx/ny/nz likewise, then normalized (:105-123);
//   * face "vertex_indices" | "vertex_index" list extracted as int32; when any face is
//     not a triangle, faces are triangulated like miniply's triangulate_polygon
//     (quads -> (0,1,3),(2,3,1); n>4 -> ear clipping in float32), including its
//     destination-advance quirk for n>4 faces (miniply.cpp:1268-1290 advances by the
//     function's return value, which is 1 for n>4).
//   * ASCII numbers use miniply's digit-accumulating parser (miniply.cpp:199-354),
//     which is not correctly rounded; results are bit-identical to it.
// Verified against the reference's own CPly compiled in this container
// (oracle/build_ref.sh -> tests/golden/ply/*.json).
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "scene.h"

namespace myrt {
namespace {

enum PType { T_CHAR = 0, T_UCHAR, T_SHORT, T_USHORT, T_INT, T_UINT, T_FLOAT, T_DOUBLE, T_NONE };
static const int kSize[] = {1, 1, 2, 2, 4, 4, 4, 8, 0};

struct Prop {
    std::string name;
    PType type = T_NONE, countType = T_NONE;   // countType != T_NONE => list
    // loaded data
    std::vector<double> scal;       // scalar values widened (exact for every PLY type)
    std::vector<uint8_t> raw;       // raw scalar bytes, host endianness (for bit-exact conversions)
    std::vector<uint32_t> counts;   // list row counts
    std::vector<uint8_t> listRaw;   // list items, host endianness
};
struct Elem { std::string name; int64_t count = 0; std::vector<Prop> props; };

static bool parse_type(const std::string& s, PType& t) {
    static const struct { const char* n; PType t; } tab[] = {
        {"char", T_CHAR}, {"uchar", T_UCHAR}, {"short", T_SHORT}, {"ushort", T_USHORT}, {"int", T_INT},
        {"uint", T_UINT}, {"float", T_FLOAT}, {"float32", T_FLOAT}, {"float64", T_DOUBLE}, {"double", T_DOUBLE},
        {"uint8", T_UCHAR}, {"uint16", T_USHORT}, {"uint32", T_UINT}, {"int8", T_CHAR}, {"int16", T_SHORT},
        {"int32", T_INT}};
    for (auto& e : tab) if (s == e.n) { t = e.t; return true; }
    return false;
}

static inline bool is_ws(char c) { return c == ' ' || c == '\t' || c == '\r'; }
static inline bool is_digit(char c) { return c >= '0' && c <= '9'; }
static inline bool is_letter(char c) { c |= 32; return c >= 'a' && c <= 'z'; }
static inline bool is_alnum(char c) { return is_digit(c) || is_letter(c); }

// miniply's int_literal (miniply.cpp:199-248)
static bool int_lit(const char*& p, int& val) {
    const char* s = p;
    bool neg = false;
    if (*s == '-') { neg = true; ++s; } else if (*s == '+') { ++s; }
    bool lead0 = *s == '0';
    if (lead0) { do { ++s; } while (*s == '0'); }
    int nd = 0; int v = 0;
    while (is_digit(*s)) { v = (int)((unsigned)v * 10u + (unsigned)(*s - '0')); ++nd; ++s; }
    if (nd == 0 && lead0) nd = 1;
    if (nd == 0 || is_letter(*s) || *s == '_') return false;
    if (nd > 10) return false;
    val = neg ? -v : v;
    p = s;
    return true;
}
// miniply's double_literal (miniply.cpp:251-343): digit accumulation, not correctly rounded
static bool dbl_lit(const char*& p, double& val) {
    static const double kDigits[10] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9};
    const char* s = p;
    bool neg = false;
    if (*s == '-') { neg = true; ++s; } else if (*s == '+') { ++s; }
    double v = 0.0;
    bool hasInt = is_digit(*s);
    if (hasInt) { do { v = v * 10.0 + kDigits[*s - '0']; ++s; } while (is_digit(*s)); }
    else if (*s != '.') return false;
    if (*s == '.') {
        ++s;
        bool hasFrac = is_digit(*s);
        if (hasFrac) {
            double scale = 0.1;
            do { v += scale * kDigits[*s - '0']; scale *= 0.1; ++s; } while (is_digit(*s));
        } else if (!hasInt) return false;
    }
    if (*s == 'e' || *s == 'E') {
        ++s;
        bool negE = false;
        if (*s == '-') { negE = true; ++s; } else if (*s == '+') { ++s; }
        if (!is_digit(*s)) return false;
        double e = 0.0;
        do { e = e * 10.0 + kDigits[*s - '0']; ++s; } while (is_digit(*s));
        if (negE) e = -e;
        v *= std::pow(10.0, e);
    }
    if (*s == '.' || *s == '_' || is_alnum(*s)) return false;
    if (neg) v = -v;
    val = v;
    p = s;
    return true;
}

template <class T> static inline T rd(const uint8_t* p) { T v; std::memcpy(&v, p, sizeof(T)); return v; }
static double raw_to_double(const uint8_t* p, PType t) {
    switch (t) {
    case T_CHAR: return (double)rd<int8_t>(p);
    case T_UCHAR: return (double)rd<uint8_t>(p);
    case T_SHORT: return (double)rd<int16_t>(p);
    case T_USHORT: return (double)rd<uint16_t>(p);
    case T_INT: return (double)rd<int32_t>(p);
    case T_UINT: return (double)rd<uint32_t>(p);
    case T_FLOAT: return (double)rd<float>(p);
    case T_DOUBLE: return rd<double>(p);
    default: return 0;
    }
}
// miniply copy_and_convert to float / compatible_types memcpy semantics
static float raw_to_float(const uint8_t* p, PType t) {
    switch (t) {
    case T_CHAR: return (float)rd<int8_t>(p);
    case T_UCHAR: return (float)rd<uint8_t>(p);
    case T_SHORT: return (float)rd<int16_t>(p);
    case T_USHORT: return (float)rd<uint16_t>(p);
    case T_INT: return (float)rd<int32_t>(p);
    case T_UINT: return (float)rd<uint32_t>(p);
    case T_FLOAT: return rd<float>(p);
    case T_DOUBLE: return (float)rd<double>(p);
    default: return 0;
    }
}
static int32_t raw_to_int(const uint8_t* p, PType t) {
    switch (t) {
    case T_CHAR: return (int32_t)rd<int8_t>(p);
    case T_UCHAR: return (int32_t)rd<uint8_t>(p);
    case T_SHORT: return (int32_t)rd<int16_t>(p);
    case T_USHORT: return (int32_t)rd<uint16_t>(p);
    case T_INT: return rd<int32_t>(p);
    case T_UINT: return (int32_t)rd<uint32_t>(p);        // int/uint are "compatible": bit copy
    case T_FLOAT: return (int32_t)rd<float>(p);
    case T_DOUBLE: return (int32_t)rd<double>(p);
    default: return 0;
    }
}
static void swap_bytes(uint8_t* p, int n) { for (int i = 0; i < n / 2; ++i) std::swap(p[i], p[n - 1 - i]); }

// ASCII value -> raw bytes of its declared type (miniply ascii_value, miniply.cpp:1896-1943)
static bool ascii_value(const char*& p, PType t, uint8_t out[8]) {
    int iv = 0;
    switch (t) {
    case T_CHAR: case T_UCHAR: case T_SHORT: case T_USHORT:
        if (!int_lit(p, iv)) return false;
        if (t == T_CHAR) { int8_t v = (int8_t)iv; std::memcpy(out, &v, 1); }
        else if (t == T_UCHAR) { uint8_t v = (uint8_t)iv; std::memcpy(out, &v, 1); }
        else if (t == T_SHORT) { int16_t v = (int16_t)iv; std::memcpy(out, &v, 2); }
        else { uint16_t v = (uint16_t)iv; std::memcpy(out, &v, 2); }
        return true;
    case T_INT: case T_UINT:
        if (!int_lit(p, iv)) return false;
        std::memcpy(out, &iv, 4);
        return true;
    case T_FLOAT: {
        double d; if (!dbl_lit(p, d)) return false;
        float f = (float)d; std::memcpy(out, &f, 4); return true;
    }
    default: {
        double d; if (!dbl_lit(p, d)) return false;
        std::memcpy(out, &d, 8); return true;
    }
    }
}

// ---- float32 geometry used by miniply's triangulation (miniply.cpp:1965-2055)
struct F2 { float x, y; };
struct F3 { float x, y, z; };
static inline F2 sub(F2 a, F2 b) { return {a.x - b.x, a.y - b.y}; }
static inline F3 sub(F3 a, F3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
static inline float dot(F2 a, F2 b) { return a.x * b.x + a.y * b.y; }
static inline float dot(F3 a, F3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline F2 nrm(F2 v) { float l = std::sqrt(dot(v, v)); return {v.x / l, v.y / l}; }
static inline F3 nrm(F3 v) { float l = std::sqrt(dot(v, v)); return {v.x / l, v.y / l, v.z / l}; }
static inline F3 crs(F3 a, F3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
static const float kPiF = 3.14159265358979323846f;

static float angle_at(uint32_t i, const std::vector<F2>& pts, const std::vector<uint32_t>& prev, const std::vector<uint32_t>& next) {
    F2 xa = nrm(sub(pts[next[i]], pts[i]));
    F2 ya = {-xa.y, xa.x};
    F2 p = sub(pts[prev[i]], pts[i]);
    float a = std::atan2(dot(p, ya), dot(p, xa));
    if (a <= 0.0f || a >= kPiF) a = 10000.0f;
    return a;
}
// Returns the value miniply's triangulate_polygon returns (1 for n > 4 after clipping).
static uint32_t triangulate(uint32_t n, const float* pos, uint32_t numVerts, const int* idx, int* dst) {
    if (n < 3) return 0;
    if (n == 3) { dst[0] = idx[0]; dst[1] = idx[1]; dst[2] = idx[2]; return 1; }
    if (n == 4) {
        dst[0] = idx[0]; dst[1] = idx[1]; dst[2] = idx[3];
        dst[3] = idx[2]; dst[4] = idx[3]; dst[5] = idx[1];
        return 2;
    }
    for (uint32_t i = 0; i < n; ++i) if (idx[i] < 0 || (uint32_t)idx[i] >= numVerts) return 0;
    auto V = [&](int k) { return F3{pos[3 * k], pos[3 * k + 1], pos[3 * k + 2]}; };
    F3 origin = V(idx[0]);
    F3 fu = nrm(sub(V(idx[1]), origin));
    F3 fn = nrm(crs(fu, nrm(sub(V(idx[n - 1]), origin))));
    F3 fv = nrm(crs(fn, fu));
    std::vector<F2> pts(n, F2{0.0f, 0.0f});
    for (uint32_t i = 1; i < n; ++i) { F3 p = sub(V(idx[i]), origin); pts[i] = F2{dot(p, fu), dot(p, fv)}; }
    std::vector<uint32_t> next(n, 0u), prev(n, 0u);
    uint32_t first = 0;
    for (uint32_t i = 0, j = n - 1; i < n; ++i) { next[j] = i; prev[i] = j; j = i; }
    while (n > 3) {
        uint32_t bestI = first;
        float bestA = angle_at(first, pts, prev, next);
        for (uint32_t i = next[first]; i != first; i = next[i]) {
            float a = angle_at(i, pts, prev, next);
            if (a < bestA) { bestI = i; bestA = a; }
        }
        uint32_t nI = next[bestI], pI = prev[bestI];
        dst[0] = idx[bestI]; dst[1] = idx[nI]; dst[2] = idx[pI];
        dst += 3;
        if (bestI == first) first = nI;
        next[pI] = nI; prev[nI] = pI;
        --n;
    }
    dst[0] = idx[first]; dst[1] = idx[next[first]]; dst[2] = idx[prev[first]];
    return n - 2;
}

struct Parser {
    std::vector<char> buf;
    size_t pos = 0;
    int fileType = 0;   // 0 ascii, 1 LE, 2 BE
    std::vector<Elem> elems;
    std::string err;

    bool read_file(const char* path) {
        FILE* f = std::fopen(path, "rb");
        if (!f) { err = "Cannot open PLY file at: " + std::string(path); return false; }
        std::fseek(f, 0, SEEK_END);
        long n = std::ftell(f);
        std::fseek(f, 0, SEEK_SET);
        buf.resize((size_t)std::max(0L, n) + 1);
        size_t got = n > 0 ? std::fread(buf.data(), 1, (size_t)n, f) : 0;
        std::fclose(f);
        buf.resize(got);
        buf.push_back('\0');
        return true;
    }
    // header line tokens (the header is small; tokens split on blanks)
    bool header() {
        auto line = [&](std::vector<std::string>& toks) -> bool {
            toks.clear();
            if (pos >= buf.size() - 1) return false;
            size_t e = pos;
            while (e < buf.size() - 1 && buf[e] != '\n') ++e;
            std::string s(buf.data() + pos, buf.data() + e);
            pos = (e < buf.size() - 1) ? e + 1 : e;
            size_t i = 0;
            while (i < s.size()) {
                while (i < s.size() && is_ws(s[i])) ++i;
                size_t j = i;
                while (j < s.size() && !is_ws(s[j])) ++j;
                if (j > i) toks.emplace_back(s.substr(i, j - i));
                i = j;
            }
            return true;
        };
        std::vector<std::string> t;
        if (!line(t) || t.size() != 1 || t[0] != "ply") { err = "not a PLY file"; return false; }
        auto next_meaningful = [&](std::vector<std::string>& tk) -> bool {
            while (line(tk)) {
                if (!tk.empty() && (tk[0] == "comment" || tk[0] == "obj_info")) continue;
                return true;
            }
            return false;
        };
        if (!next_meaningful(t) || t.size() < 3 || t[0] != "format") { err = "bad format line"; return false; }
        if (t[1] == "ascii") fileType = 0;
        else if (t[1] == "binary_little_endian") fileType = 1;
        else if (t[1] == "binary_big_endian") fileType = 2;
        else { err = "unknown PLY format"; return false; }
        while (next_meaningful(t)) {
            if (t.empty()) { err = "blank header line"; return false; }
            if (t[0] == "end_header") return t.size() == 1;
            if (t[0] == "element") {
                if (t.size() != 3) { err = "bad element line"; return false; }
                Elem e; e.name = t[1];
                const char* c = t[2].c_str(); int cnt = 0;
                if (!int_lit(c, cnt) || cnt < 0) { err = "bad element count"; return false; }
                e.count = cnt;
                elems.push_back(e);
            } else if (t[0] == "property") {
                if (elems.empty()) { err = "property before element"; return false; }
                Prop p;
                if (t.size() == 5 && t[1] == "list") {
                    if (!parse_type(t[2], p.countType) || !parse_type(t[3], p.type)) { err = "bad list type"; return false; }
                    p.name = t[4];
                } else if (t.size() == 3) {
                    if (!parse_type(t[1], p.type)) { err = "bad property type"; return false; }
                    p.name = t[2];
                } else { err = "bad property line"; return false; }
                elems.back().props.push_back(p);
            } else { err = "unexpected header line"; return false; }
        }
        err = "missing end_header";
        return false;
    }
    bool load_elem(Elem& e) {
        const bool big = fileType == 2;
        for (auto& p : e.props) {
            if (p.countType == T_NONE) { p.raw.reserve((size_t)e.count * kSize[p.type]); }
            else { p.counts.reserve(e.count); p.listRaw.reserve((size_t)e.count * 3 * kSize[p.type]); }
        }
        if (fileType == 0) {
            const char* s = buf.data() + pos;
            const char* end = buf.data() + buf.size() - 1;
            for (int64_t r = 0; r < e.count; ++r) {
                for (auto& p : e.props) {
                    while (is_ws(*s)) ++s;
                    uint8_t v[8];
                    if (p.countType == T_NONE) {
                        if (!ascii_value(s, p.type, v)) { err = "bad ascii value"; return false; }
                        p.raw.insert(p.raw.end(), v, v + kSize[p.type]);
                    } else {
                        int cnt = 0;
                        if (p.countType >= T_FLOAT || !int_lit(s, cnt) || cnt < 0) { err = "bad list count"; return false; }
                        p.counts.push_back((uint32_t)cnt);
                        for (int k = 0; k < cnt; ++k) {
                            while (is_ws(*s)) ++s;
                            if (!ascii_value(s, p.type, v)) { err = "bad list value"; return false; }
                            p.listRaw.insert(p.listRaw.end(), v, v + kSize[p.type]);
                        }
                    }
                }
                // next_line: skip the rest of the row, then comment/obj_info lines
                for (;;) {
                    while (s < end && *s != '\n') ++s;
                    if (s < end) ++s;
                    if (std::strncmp(s, "comment", 7) == 0 || std::strncmp(s, "obj_info", 8) == 0) continue;
                    break;
                }
            }
            pos = (size_t)(s - buf.data());
            return true;
        }
        // binary: values are copied straight into each property's column (no per-byte
        // container appends); byte order is fixed up in place
        const size_t avail = buf.size() - 1;
        for (auto& p : e.props)
            if (p.countType == T_NONE) p.raw.resize((size_t)e.count * kSize[p.type]);
        const uint8_t* src = reinterpret_cast<const uint8_t*>(buf.data());
        for (int64_t r = 0; r < e.count; ++r) {
            for (auto& p : e.props) {
                if (p.countType == T_NONE) {
                    const int n = kSize[p.type];
                    if (pos + n > avail) { err = "truncated binary PLY"; return false; }
                    uint8_t* v = p.raw.data() + (size_t)r * n;
                    std::memcpy(v, src + pos, n); pos += n;
                    if (big) swap_bytes(v, n);
                } else {
                    const int cn = kSize[p.countType];
                    if (pos + cn > avail) { err = "truncated binary PLY"; return false; }
                    uint8_t c[8]; std::memcpy(c, src + pos, cn); pos += cn;
                    if (big) swap_bytes(c, cn);
                    const int32_t cnt = raw_to_int(c, p.countType);
                    if (cnt < 0) { err = "negative list count"; return false; }
                    p.counts.push_back((uint32_t)cnt);
                    const int n = kSize[p.type];
                    const size_t bytes = (size_t)n * cnt;
                    if (pos + bytes > avail) { err = "truncated binary PLY"; return false; }
                    const size_t at = p.listRaw.size();
                    p.listRaw.resize(at + bytes);
                    std::memcpy(p.listRaw.data() + at, src + pos, bytes); pos += bytes;
                    if (big) for (int k = 0; k < cnt; ++k) swap_bytes(p.listRaw.data() + at + (size_t)k * n, n);
                }
            }
        }
        return true;
    }
};

static int find_prop(const Elem& e, const char* name) {
    for (size_t i = 0; i < e.props.size(); ++i) if (e.props[i].name == name) return (int)i;
    return -1;
}

}  // namespace

int32_t ply_load(const char* path, std::vector<double>& positions, std::vector<double>& normals,
                 std::vector<float>& texcoords, std::vector<int32_t>& indices, std::string& err) {
    positions.clear(); normals.clear(); texcoords.clear(); indices.clear();
    Parser P;
    if (!path || !P.read_file(path)) { err = P.err.empty() ? "no path" : P.err; return RT_ERR_PLY; }
    if (!P.header()) { err = "Corrupted or unsupported PLY file: " + P.err; return RT_ERR_PLY; }
    bool gotVerts = false, gotFaces = false;
    for (auto& e : P.elems) {
        if (!P.load_elem(e)) { err = "Corrupted or unsupported PLY file: " + P.err; return RT_ERR_PLY; }
        if (e.name == "vertex") {                                       // PLYReader.swift:78-144
            int ix = find_prop(e, "x"), iy = find_prop(e, "y"), iz = find_prop(e, "z");
            if (ix < 0 || iy < 0 || iz < 0) continue;
            const int idx3[3] = {ix, iy, iz};
            bool anyList = false;
            for (int k : idx3) anyList |= e.props[k].countType != T_NONE;
            if (anyList) continue;
            positions.resize((size_t)e.count * 3);
            for (int64_t r = 0; r < e.count; ++r)
                for (int k = 0; k < 3; ++k) {
                    const Prop& p = e.props[idx3[k]];
                    positions[3 * r + k] = (double)raw_to_float(p.raw.data() + (size_t)r * kSize[p.type], p.type);
                }
            int nx = find_prop(e, "nx"), ny = find_prop(e, "ny"), nz = find_prop(e, "nz");
            if (nx >= 0 && ny >= 0 && nz >= 0) {
                const int n3[3] = {nx, ny, nz};
                normals.resize((size_t)e.count * 3);
                for (int64_t r = 0; r < e.count; ++r) {
                    double v[3];
                    for (int k = 0; k < 3; ++k) {
                        const Prop& p = e.props[n3[k]];
                        v[k] = (double)raw_to_float(p.raw.data() + (size_t)r * kSize[p.type], p.type);
                    }
                    const double s = 1.0 / std::sqrt((v[0] * v[0] + v[1] * v[1]) + v[2] * v[2]);
                    for (int k = 0; k < 3; ++k) normals[3 * r + k] = v[k] * s;
                }
            }
            static const char* uvNames[4][2] = {{"u", "v"}, {"s", "t"}, {"texture_u", "texture_v"}, {"texture_s", "texture_t"}};
            for (auto& nm : uvNames) {
                int a = find_prop(e, nm[0]), b = find_prop(e, nm[1]);
                if (a < 0 || b < 0) continue;
                texcoords.resize((size_t)e.count * 2);
                for (int64_t r = 0; r < e.count; ++r) {
                    texcoords[2 * r] = raw_to_float(e.props[a].raw.data() + (size_t)r * kSize[e.props[a].type], e.props[a].type);
                    texcoords[2 * r + 1] = raw_to_float(e.props[b].raw.data() + (size_t)r * kSize[e.props[b].type], e.props[b].type);
                }
                break;
            }
            gotVerts = true;
        } else if (e.name == "face") {                                  // PLYReader.swift:149-201
            int ip = find_prop(e, "vertex_indices");
            if (ip < 0) ip = find_prop(e, "vertex_index");
            if (ip < 0) continue;
            const Prop& p = e.props[ip];
            if (p.countType == T_NONE) continue;
            bool needsTri = false;
            uint64_t total = 0, triCount = 0;
            for (uint32_t c : p.counts) { needsTri |= (c != 3); total += c; if (c >= 3) triCount += c - 2; }
            const int isz = kSize[p.type];
            if (needsTri && !gotVerts) { err = "Need vertex positions to triangulate faces."; return RT_ERR_PLY; }
            if (!needsTri) {
                indices.resize(total);
                for (uint64_t k = 0; k < total; ++k) indices[k] = raw_to_int(p.listRaw.data() + k * isz, p.type);
            } else {
                const uint32_t numVerts = (uint32_t)(positions.size() / 3);
                std::vector<float> posF(positions.size());
                for (size_t k = 0; k < positions.size(); ++k) posF[k] = (float)positions[k];
                indices.assign(triCount * 3 + 64, 0);      // slack: the n>4 quirk can write past the count
                std::vector<int> faceIdx;
                std::vector<int> tmp;
                size_t off = 0;
                int64_t to = 0;
                for (size_t f = 0; f < p.counts.size(); ++f) {
                    const uint32_t c = p.counts[f];
                    faceIdx.resize(c);
                    for (uint32_t k = 0; k < c; ++k) faceIdx[k] = raw_to_int(p.listRaw.data() + (off + k) * isz, p.type);
                    off += c;
                    tmp.assign(c >= 3 ? (size_t)(c - 2) * 3 : 0, 0);
                    const uint32_t nt = triangulate(c, posF.data(), numVerts, faceIdx.data(), tmp.data());
                    // miniply writes every produced triangle at `to` but advances by the return value
                    const size_t written = (nt == 0) ? 0 : (c > 4 ? tmp.size() : (size_t)nt * 3);
                    for (size_t k = 0; k < written && to + (int64_t)k < (int64_t)indices.size(); ++k) indices[to + k] = tmp[k];
                    to += (int64_t)nt * 3;
                }
                indices.resize(triCount * 3);
            }
            gotFaces = true;
        }
    }
    if (!gotVerts) { err = "Vertex element missing."; return RT_ERR_PLY; }
    if (!gotFaces) { err = "Face element missing."; return RT_ERR_PLY; }
    return RT_OK;
}

}  // namespace myrt
