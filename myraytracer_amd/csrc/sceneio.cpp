// sceneio.cpp — scene files -> rt_scene_desc, for compiled hosts (rt_scene_file_*, rtcore.h).
//
// The reference reads a scene through ParsingKit's `SceneLoader.load(.url / .data(format:))`
// (RayTracer.swift:30-49; SceneFormat auto/json/xml, Models/SceneFormat.swift:8-10).  ParsingKit's
// scene model is not in the container; only its v1.0.0 decoding helpers survive in
// the SwiftPM mirror pack, and this decoder follows their conventions exactly as the Python
// mirror myraytracer_amd/sceneio.py does (the two are checked against each other,
// tests/test_sceneio_native.py):
//   * the document's "Scene" object is the root (RootDecoding.swift:12-26);
//   * a scalar is a JSON number or a numeric string (Flexible<T>, pkDouble/pkInt,
//     PropertyWrapper.swift:13-30, FlexibleDecoding.swift:31-44);
//   * a vector is a whitespace-separated string or an array (FlexibleVec3, pkVectorStrings);
//   * OneOrMany<T>: one object or an array of them (PropertyWrapper.swift:36-44);
//   * XML becomes the same tree: attributes are "_name" keys, the text of an element with
//     attributes or children is "_data", repeated children become arrays.
// Where the format is unpinned (object order, composeTransform, the rotation convention,
// material ids, PLY path resolution) the decisions are the ones sceneio.py's docstring lists.
#include <unistd.h>

#include <cctype>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>
#include <memory>
#include <sstream>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "../../include/rtcore.h"

namespace myrt {
namespace sio {

// ----------------------------------------------------------------------------- value tree
struct Value {
    enum Kind { Null, Bool, Num, Str, Arr, Obj } kind = Null;
    bool b = false;
    double num = 0.0;
    bool is_int = false;                 // a JSON number literal without '.', 'e' or 'E'
    std::string str;                     // Str, or the literal text of a Num
    std::vector<Value> arr;
    std::vector<std::pair<std::string, Value>> obj;   // keys in document order
    const Value* get(const char* key) const {
        if (kind != Obj) return nullptr;
        for (const auto& kv : obj)
            if (kv.first == key) return &kv.second;
        return nullptr;
    }
    Value* get_mut(const std::string& key) {
        for (auto& kv : obj)
            if (kv.first == key) return &kv.second;
        return nullptr;
    }
};

struct Error {
    std::string msg;
};
[[noreturn]] static void fail(const std::string& m) { throw Error{m}; }
static bool space(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }
static std::string trim(const std::string& s) {
    size_t a = 0, b = s.size();
    while (a < b && std::isspace((unsigned char)s[a])) ++a;
    while (b > a && std::isspace((unsigned char)s[b - 1])) --b;
    return s.substr(a, b - a);
}
static void put_utf8(std::string& out, unsigned long cp) {
    if (cp < 0x80) {
        out += (char)cp;
    } else if (cp < 0x800) {
        out += (char)(0xC0 | (cp >> 6)); out += (char)(0x80 | (cp & 0x3F));
    } else if (cp < 0x10000) {
        out += (char)(0xE0 | (cp >> 12)); out += (char)(0x80 | ((cp >> 6) & 0x3F)); out += (char)(0x80 | (cp & 0x3F));
    } else {
        out += (char)(0xF0 | (cp >> 18)); out += (char)(0x80 | ((cp >> 12) & 0x3F));
        out += (char)(0x80 | ((cp >> 6) & 0x3F)); out += (char)(0x80 | (cp & 0x3F));
    }
}

// Deepest array/object (JSON) or element (XML) nesting the decoders accept: they recurse once
// per level, so an unbounded '[[[[...' would overflow the host stack instead of failing.
constexpr int kMaxNesting = 512;

// ----------------------------------------------------------------------------- JSON
class Json {
  public:
    Json(const char* p, size_t n) : p_(p), e_(p + n) {}
    Value parse() {
        Value v = value();
        ws();
        if (p_ != e_) bad("trailing characters after the JSON value");
        return v;
    }

  private:
    const char *p_, *e_;
    int depth_ = 0;
    void ws() { while (p_ < e_ && space(*p_)) ++p_; }
    [[noreturn]] void bad(const char* what) { fail(std::string("scene decode failed: ") + what); }
    Value nested(bool obj) {
        if (++depth_ > kMaxNesting) bad("nesting too deep");
        Value v = obj ? object() : array();
        --depth_;
        return v;
    }
    Value value() {
        ws();
        if (p_ >= e_) bad("unexpected end of JSON");
        const char c = *p_;
        if (c == '{') return nested(true);
        if (c == '[') return nested(false);
        if (c == '"') { Value v; v.kind = Value::Str; v.str = string(); return v; }
        if (c == 't' || c == 'f' || c == 'n') return literal();
        return number();
    }
    bool take(const char* w) {
        const size_t n = std::strlen(w);
        if ((size_t)(e_ - p_) >= n && std::strncmp(p_, w, n) == 0) { p_ += n; return true; }
        return false;
    }
    Value literal() {
        Value v;
        if (take("true")) { v.kind = Value::Bool; v.b = true; return v; }
        if (take("false")) { v.kind = Value::Bool; v.b = false; return v; }
        if (take("null")) return v;
        bad("invalid literal");
    }
    Value number() {
        const char* s = p_;
        bool frac = false;
        while (p_ < e_ && ((*p_ >= '0' && *p_ <= '9') || *p_ == '.' || *p_ == 'e' || *p_ == 'E' || *p_ == '-' ||
                           *p_ == '+')) {
            if (*p_ == '.' || *p_ == 'e' || *p_ == 'E') frac = true;
            ++p_;
        }
        if (p_ == s) bad("unexpected character");
        Value v;
        v.kind = Value::Num;
        v.str.assign(s, p_);
        char* end = nullptr;
        v.num = std::strtod(v.str.c_str(), &end);
        if (!end || *end != '\0') bad("invalid number");
        v.is_int = !frac;
        return v;
    }
    unsigned hex4() {
        if (e_ - p_ < 4) bad("bad \\u escape");
        unsigned v = 0;
        for (int k = 0; k < 4; ++k) {
            const char c = *p_++;
            v <<= 4;
            if (c >= '0' && c <= '9') v |= (unsigned)(c - '0');
            else if (c >= 'a' && c <= 'f') v |= (unsigned)(c - 'a' + 10);
            else if (c >= 'A' && c <= 'F') v |= (unsigned)(c - 'A' + 10);
            else bad("bad \\u escape");
        }
        return v;
    }
    std::string string() {
        ++p_;   // opening quote
        std::string out;
        while (p_ < e_ && *p_ != '"') {
            char c = *p_++;
            if (c != '\\') { out += c; continue; }
            if (p_ >= e_) bad("unterminated string");
            c = *p_++;
            switch (c) {
                case '"': out += '"'; break;
                case '\\': out += '\\'; break;
                case '/': out += '/'; break;
                case 'b': out += '\b'; break;
                case 'f': out += '\f'; break;
                case 'n': out += '\n'; break;
                case 'r': out += '\r'; break;
                case 't': out += '\t'; break;
                case 'u': {
                    unsigned long cp = hex4();
                    if (cp >= 0xD800 && cp < 0xDC00 && e_ - p_ >= 6 && p_[0] == '\\' && p_[1] == 'u') {
                        p_ += 2;
                        const unsigned lo = hex4();
                        cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
                    }
                    put_utf8(out, cp);
                    break;
                }
                default: bad("bad escape");
            }
        }
        if (p_ >= e_) bad("unterminated string");
        ++p_;
        return out;
    }
    Value array() {
        ++p_;
        Value v;
        v.kind = Value::Arr;
        ws();
        if (p_ < e_ && *p_ == ']') { ++p_; return v; }
        for (;;) {
            v.arr.push_back(value());
            ws();
            if (p_ < e_ && *p_ == ',') { ++p_; continue; }
            if (p_ < e_ && *p_ == ']') { ++p_; return v; }
            bad("expected , or ]");
        }
    }
    Value object() {
        ++p_;
        Value v;
        v.kind = Value::Obj;
        ws();
        if (p_ < e_ && *p_ == '}') { ++p_; return v; }
        for (;;) {
            ws();
            if (p_ >= e_ || *p_ != '"') bad("expected a key");
            std::string k = string();
            ws();
            if (p_ >= e_ || *p_ != ':') bad("expected :");
            ++p_;
            Value x = value();
            if (Value* old = v.get_mut(k)) *old = std::move(x);   // a repeated key keeps the last value
            else v.obj.emplace_back(std::move(k), std::move(x));
            ws();
            if (p_ < e_ && *p_ == ',') { ++p_; continue; }
            if (p_ < e_ && *p_ == '}') { ++p_; return v; }
            bad("expected , or }");
        }
    }
};

// ----------------------------------------------------------------------------- XML
// Elements, attributes, text, comments, <?...?> and <!...> declarations, CDATA, the five
// predefined entities and numeric character references.
class Xml {
  public:
    Xml(const char* p, size_t n) : p_(p), e_(p + n) {}
    Value parse() {
        misc();
        if (p_ >= e_ || *p_ != '<') bad("no root element");
        std::string tag;
        Value root = element(tag);
        misc();
        if (p_ != e_) bad("junk after the root element");
        Value doc;
        doc.kind = Value::Obj;
        doc.obj.emplace_back(tag, std::move(root));
        return doc;
    }

  private:
    const char *p_, *e_;
    int depth_ = 0;
    [[noreturn]] void bad(const char* what) { fail(std::string("scene decode failed: XML: ") + what); }
    bool starts(const char* w) const {
        const size_t n = std::strlen(w);
        return (size_t)(e_ - p_) >= n && std::strncmp(p_, w, n) == 0;
    }
    void skip_until(const char* w) {
        const size_t n = std::strlen(w);
        while (p_ < e_ && !starts(w)) ++p_;
        if (p_ >= e_) bad("unterminated construct");
        p_ += n;
    }
    void ws() { while (p_ < e_ && space(*p_)) ++p_; }
    void misc() {                                    // whitespace, comments, PIs, doctype
        for (;;) {
            ws();
            if (starts("<?")) skip_until("?>");
            else if (starts("<!--")) skip_until("-->");
            else if (starts("<!")) skip_until(">");
            else return;
        }
    }
    std::string name() {
        const char* s = p_;
        while (p_ < e_ && !space(*p_) && *p_ != '>' && *p_ != '/' && *p_ != '=') ++p_;
        if (p_ == s) bad("expected a name");
        return std::string(s, p_);
    }
    void entity(std::string& out) {
        const char* s = ++p_;
        while (p_ < e_ && *p_ != ';') ++p_;
        if (p_ >= e_) bad("unterminated entity");
        const std::string ent(s, p_);
        ++p_;
        if (ent == "lt") out += '<';
        else if (ent == "gt") out += '>';
        else if (ent == "amp") out += '&';
        else if (ent == "quot") out += '"';
        else if (ent == "apos") out += '\'';
        else if (ent.size() > 1 && ent[0] == '#')
            put_utf8(out, (ent[1] == 'x' || ent[1] == 'X') ? std::strtoul(ent.c_str() + 2, nullptr, 16)
                                                            : std::strtoul(ent.c_str() + 1, nullptr, 10));
        else bad("unknown entity");
    }
    // One element -> Str (no attributes and no children: its text) or Obj ("_attr" keys, the
    // children by tag - repeats become an Arr - and "_data" = the text before the first child)
    Value element(std::string& tag) {
        if (++depth_ > kMaxNesting) bad("nesting too deep");
        struct Leave { int& d; ~Leave() { --d; } } leave{depth_};
        ++p_;   // '<'
        tag = name();
        Value v;
        v.kind = Value::Obj;
        bool attrs = false;
        for (;;) {
            ws();
            if (p_ >= e_) bad("unterminated tag");
            if (*p_ == '/' || *p_ == '>') break;
            const std::string an = name();
            ws();
            if (p_ >= e_ || *p_ != '=') bad("expected = after an attribute name");
            ++p_;
            ws();
            if (p_ >= e_ || (*p_ != '"' && *p_ != '\'')) bad("expected a quoted attribute value");
            const char q = *p_++;
            Value x;
            x.kind = Value::Str;
            while (p_ < e_ && *p_ != q) {
                if (*p_ == '&') entity(x.str);
                else x.str += *p_++;
            }
            if (p_ >= e_) bad("unterminated attribute value");
            ++p_;
            v.obj.emplace_back("_" + an, std::move(x));
            attrs = true;
        }
        if (*p_ == '/') {                           // <tag ... />
            ++p_;
            if (p_ >= e_ || *p_ != '>') bad("expected >");
            ++p_;
            if (!attrs) { Value s; s.kind = Value::Str; return s; }
            return v;
        }
        ++p_;   // '>'
        std::string text;
        bool kids = false;
        for (;;) {
            if (p_ >= e_) bad("unterminated element");
            if (starts("</")) {
                p_ += 2;
                if (name() != tag) bad("mismatched closing tag");
                ws();
                if (p_ >= e_ || *p_ != '>') bad("expected >");
                ++p_;
                break;
            }
            if (starts("<!--")) { skip_until("-->"); continue; }
            if (starts("<![CDATA[")) {
                p_ += 9;
                const char* s = p_;
                while (p_ < e_ && !starts("]]>")) ++p_;
                if (p_ >= e_) bad("unterminated CDATA");
                if (!kids) text.append(s, p_);
                p_ += 3;
                continue;
            }
            if (starts("<?")) { skip_until("?>"); continue; }
            if (*p_ == '<') {
                std::string ct;
                Value child = element(ct);
                kids = true;                          // ElementTree's text: before the first child
                if (Value* prev = v.get_mut(ct)) {
                    if (prev->kind == Value::Arr) {
                        prev->arr.push_back(std::move(child));
                    } else {
                        Value a;
                        a.kind = Value::Arr;
                        a.arr.push_back(std::move(*prev));
                        a.arr.push_back(std::move(child));
                        *prev = std::move(a);
                    }
                } else {
                    v.obj.emplace_back(ct, std::move(child));
                }
                continue;
            }
            if (*p_ == '&') {
                std::string ch;
                entity(ch);
                if (!kids) text += ch;
                continue;
            }
            if (!kids) text += *p_;
            ++p_;
        }
        text = trim(text);
        if (!attrs && !kids) { Value s; s.kind = Value::Str; s.str = text; return s; }
        if (!text.empty()) { Value s; s.kind = Value::Str; s.str = text; v.obj.emplace_back("_data", std::move(s)); }
        return v;
    }
};

// ----------------------------------------------------------------------------- flexible scalars
static const Value* text_of(const Value* v) {          // "_data" of an element given with attributes
    if (v && v->kind == Value::Obj)
        if (const Value* d = v->get("_data")) return d;
    return v;
}
// sceneio._opt: the key is there, not null and not empty text
static bool present(const Value* obj, const char* key) {
    const Value* v = obj ? obj->get(key) : nullptr;
    if (!v || v->kind == Value::Null) return false;
    const Value* t = text_of(v);
    return !(t->kind == Value::Str && t->str.empty());
}
static bool parse_double(const std::string& s0, double& out) {   // Python float(str)
    const std::string s = trim(s0);
    if (s.empty()) return false;
    char* end = nullptr;
    out = std::strtod(s.c_str(), &end);
    return end && *end == '\0';
}
static double to_double(const Value* v, const char* key) {       // pkDouble / Flexible<Double>
    v = text_of(v);
    if (v && v->kind == Value::Num) return v->num;
    double d;
    if (v && v->kind == Value::Str && parse_double(v->str, d)) return d;
    fail(std::string("Expected double-like value for ") + key);
}
static long long to_int(const Value* v, const char* key) {       // pkInt: int, numeric string, double truncated
    v = text_of(v);
    if (v && v->kind == Value::Num) return v->is_int ? std::strtoll(v->str.c_str(), nullptr, 10) : (long long)v->num;
    if (v && v->kind == Value::Str) {
        const std::string s = trim(v->str);
        char* end = nullptr;
        const long long x = std::strtoll(s.c_str(), &end, 10);
        if (!s.empty() && end && *end == '\0') return x;
    }
    fail(std::string("Expected int-like value for ") + key);
}
static std::vector<std::string> strings(const Value* v, const char* key) {   // pkVectorStrings
    v = text_of(v);
    std::vector<std::string> out;
    if (v && v->kind == Value::Str) {
        std::istringstream is(v->str);
        std::string w;
        while (is >> w) out.push_back(w);
        return out;
    }
    if (v && v->kind == Value::Arr) {
        for (const Value& x : v->arr)
            if (x.kind == Value::Num || x.kind == Value::Str) out.push_back(x.str);
        return out;
    }
    if (v && v->kind == Value::Num) { out.push_back(v->str); return out; }
    fail(std::string("Expected vector-like value for ") + key);
}
static std::vector<double> doubles(const Value* v, const char* key, size_t n = 0) {
    std::vector<double> out;
    for (const std::string& s : strings(v, key)) {
        double d;
        if (!parse_double(s, d)) fail(std::string("Invalid vector element for ") + key);
        out.push_back(d);
    }
    if (out.size() < n) fail(std::string(key) + " requires " + std::to_string(n) + " components");
    return out;
}
static rt_vec3 vec3(const Value* v, const char* key) {             // FlexibleVec3: the first three
    const auto x = doubles(v, key, 3);
    return rt_vec3{x[0], x[1], x[2]};
}
static rt_vec3 opt_vec3(const Value* o, const char* key, rt_vec3 def) {
    return present(o, key) ? vec3(o->get(key), key) : def;
}
static double opt_double(const Value* o, const char* key, double def) {
    return present(o, key) ? to_double(o->get(key), key) : def;
}
static long long opt_int(const Value* o, const char* key, long long def) {
    return present(o, key) ? to_int(o->get(key), key) : def;
}
static std::vector<const Value*> one_or_many(const Value* v) {   // OneOrMany<T>
    std::vector<const Value*> out;
    if (!v || v->kind == Value::Null) return out;
    if (v->kind == Value::Arr) {
        for (const Value& x : v->arr) out.push_back(&x);
    } else {
        out.push_back(v);
    }
    return out;
}
static std::string str_of(const Value* v) {                     // Python str(_text(v))
    v = text_of(v);
    if (!v) return "";
    if (v->kind == Value::Str || v->kind == Value::Num) return v->str;
    if (v->kind == Value::Bool) return v->b ? "True" : "False";
    return "";
}
static bool opt_bool(const Value* o, const char* key) {
    const Value* v = o ? o->get(key) : nullptr;
    if (!v) return false;
    const Value* t = text_of(v);
    if (t->kind == Value::Bool) return t->b;
    std::string s = trim(str_of(t));
    for (auto& c : s) c = (char)std::tolower((unsigned char)c);
    return s == "true" || s == "1" || s == "yes";
}
static bool id_of(const Value* o, std::string& id) {
    const Value* v = o->get("_id");
    if (!v) v = o->get("id");
    if (!v) return false;
    id = str_of(v);
    return true;
}
static bool full_int(const std::string& s, long long& x) {      // Python int(s, 10) on a stripped string
    if (s.empty() || std::isspace((unsigned char)s[0])) return false;
    char* end = nullptr;
    x = std::strtoll(s.c_str(), &end, 10);
    return end && *end == '\0';
}

// ----------------------------------------------------------------------------- transforms
// Row-major 4x4 (numpy's layout in sceneio.py); rt_object.transform is its column-major copy.
struct M4 {
    double m[16];
    static M4 eye() {
        M4 r{};
        r.m[0] = r.m[5] = r.m[10] = r.m[15] = 1.0;
        return r;
    }
    M4 operator*(const M4& b) const {
        M4 r{};
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) {
                double acc = 0.0;
                for (int k = 0; k < 4; ++k) acc += m[4 * i + k] * b.m[4 * k + j];
                r.m[4 * i + j] = acc;
            }
        return r;
    }
};

class Transforms {
  public:
    explicit Transforms(const Value* d) {
        static const struct { const char* kind; char letter; } kinds[] = {
            {"Translation", 't'}, {"Scaling", 's'}, {"Rotation", 'r'}, {"Composite", 'c'}};
        for (const auto& k : kinds) {
            for (const Value* e : one_or_many(d ? d->get(k.kind) : nullptr)) {
                if (e->kind != Value::Obj) fail(std::string(k.kind) + " needs an _id");
                std::string id;
                if (!id_of(e, id)) id = "None";
                const auto v = doubles(e->get("_data"), k.kind);
                M4 m = M4::eye();
                if (k.letter == 't') {
                    if (v.size() < 3) fail("Translation needs 3 numbers");
                    m.m[3] = v[0]; m.m[7] = v[1]; m.m[11] = v[2];
                } else if (k.letter == 's') {
                    if (v.size() < 3) fail("Scaling needs 3 numbers");
                    m.m[0] = v[0]; m.m[5] = v[1]; m.m[10] = v[2];
                } else if (k.letter == 'r') {
                    if (v.size() < 4) fail("Rotation needs angle and axis");
                    m = rotation(v[0], v[1], v[2], v[3]);
                } else {
                    if (v.size() < 16) fail("Composite needs 16 numbers");
                    for (int q = 0; q < 16; ++q) m.m[q] = v[q];
                }
                table_[std::string(1, k.letter) + id] = m;
            }
        }
    }
    // Scene.composeTransform(tokens:reset:base:): tokens applied in order (M = T_n ... T_1),
    // on top of `base` unless `reset`
    M4 compose(const std::string& tokens, const M4* base, bool reset) const {
        M4 m = (base && !reset) ? *base : M4::eye();
        std::istringstream is(tokens);
        std::string tok;
        while (is >> tok) {
            std::string key = tok;
            key[0] = (char)std::tolower((unsigned char)key[0]);
            auto it = table_.find(key);
            if (it == table_.end()) fail("unknown transformation '" + tok + "'");
            m = it->second * m;
        }
        return m;
    }

  private:
    std::unordered_map<std::string, M4> table_;
    static M4 rotation(double deg, double ax, double ay, double az) {   // degrees about the unit axis
        const double n = std::sqrt(ax * ax + ay * ay + az * az);
        if (n == 0.0) fail("rotation axis is zero");
        const double x = ax / n, y = ay / n, z = az / n;
        const double th = deg * (M_PI / 180.0);                          // math.radians
        const double c = std::cos(th), s = std::sin(th), C = 1.0 - std::cos(th);
        const double r[9] = {c + x * x * C, x * y * C - z * s, x * z * C + y * s,
                             y * x * C + z * s, c + y * y * C, y * z * C - x * s,
                             z * x * C - y * s, z * y * C + x * s, c + z * z * C};
        M4 m = M4::eye();
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) m.m[4 * i + j] = r[3 * i + j];
        return m;
    }
};

static void colmajor(const M4& m, double out[16]) {
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r) out[4 * c + r] = m.m[4 * r + c];
}

// rt_object.id is an int; scene-file ids are strings: Int(id), else a CRC32-derived id
static uint32_t crc32(const std::string& s) {
    uint32_t c = 0xFFFFFFFFu;
    for (unsigned char ch : s) {
        c ^= ch;
        for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
    }
    return ~c;
}
static int32_t numeric_id(bool has, const std::string& id) {
    if (!has) return -1;
    long long x;
    if (full_int(id, x)) return (int32_t)x;
    return (int32_t)((crc32(id) & 0x3FFFFFFFu) | 0x40000000u);
}
// RTContext.materialIndex(for:) (RTContext.swift:423-426): Int(id) or -1
static int32_t material_index(bool has, const std::string& m) {
    long long x;
    return (has && full_int(m, x)) ? (int32_t)x : -1;
}

static rt_vec3 vertex(const std::vector<double>& vd, long long idx, const char* what) {
    const long long n = (long long)vd.size() / 3;
    if (idx < 1 || idx > n)
        fail(std::string(what) + ": vertex index " + std::to_string(idx) + " out of range 1.." + std::to_string(n));
    return rt_vec3{vd[3 * (idx - 1)], vd[3 * (idx - 1) + 1], vd[3 * (idx - 1) + 2]};
}

static std::vector<long long> int_list(const Value* v, const char* key) {   // [int(float(x)) for x in ...]
    std::vector<long long> out;
    for (const std::string& s : strings(v, key)) {
        double d;
        if (!parse_double(s, d)) fail(std::string("Invalid vector element for ") + key);
        out.push_back((long long)d);
    }
    return out;
}

}  // namespace sio
}  // namespace myrt

// ----------------------------------------------------------------------------- the decoded scene
struct rt_scene_file {
    rt_scene_desc desc{};
    std::vector<rt_camera> cams;
    std::vector<rt_material> mats;
    std::vector<rt_point_light> plights;
    std::vector<rt_area_light> alights;
    std::vector<rt_object> objs;
    std::vector<double> vertex_data;                  // VertexData (xyz triples, 1-based in the file)
    std::vector<std::unique_ptr<std::vector<int32_t>>> faces;
    std::vector<std::unique_ptr<std::string>> paths;
    std::vector<std::string> image_names;             // per camera (ImageName)
};

namespace {
thread_local std::string g_sio_err;
int32_t sio_fail(int32_t code, const std::string& m) { g_sio_err = m; return code; }
}  // namespace

namespace myrt {
namespace sio {

static const char* kObjectOrder[] = {"Mesh", "Triangle", "Sphere", "Plane", "MeshInstance"};

// ParsingKit.decode(Scene.self, from:, rootKey: "Scene"), then the fields RTContext reads
static void decode(const Value& root, const std::string& base_dir, rt_scene_file& F) {
    const Value* doc = root.get("Scene");
    if (!doc || doc->kind != Value::Obj) fail("Root key not found: Scene");
    const Transforms tf(doc->get("Transformations"));
    if (const Value* vdv = doc->get("VertexData")) {
        if (vdv->kind != Value::Null) F.vertex_data = doubles(vdv, "VertexData");
        if (F.vertex_data.size() % 3) fail("VertexData length is not a multiple of 3");
    }
    const std::vector<double>& vd = F.vertex_data;

    const Value* camsV = doc->get("Cameras");
    for (const Value* c : one_or_many(camsV ? camsV->get("Camera") : nullptr)) {
        rt_camera cc{};
        Value defRes;
        defRes.kind = Value::Str;
        defRes.str = "0 0";
        const auto res = strings(c->get("ImageResolution") ? c->get("ImageResolution") : &defRes, "ImageResolution");
        if (res.size() < 2) fail("ImageResolution requires 2 components");
        double w, h;
        if (!parse_double(res[0], w) || !parse_double(res[1], h)) fail("Invalid vector element for ImageResolution");
        cc.width = (int32_t)w;
        cc.height = (int32_t)h;
        std::string type = str_of(c->get("_type"));
        if (type.empty()) type = "simple";
        for (auto& ch : type) ch = (char)std::tolower((unsigned char)ch);
        cc.type = type == "lookat" ? RT_CAM_LOOKAT : RT_CAM_NEARPLANE;
        cc.position = c->get("Position") ? vec3(c->get("Position"), "Position") : rt_vec3{0, 0, 0};
        cc.up = c->get("Up") ? vec3(c->get("Up"), "Up") : rt_vec3{0, 1, 0};
        cc.gaze_point = opt_vec3(c, "GazePoint", rt_vec3{0, 0, -1});
        cc.gaze = opt_vec3(c, "Gaze", rt_vec3{0, 0, -1});
        cc.fovy = present(c, "FovY") ? to_double(c->get("FovY"), "FovY") : std::nan("");
        cc.near_distance = opt_double(c, "NearDistance", 1.0);
        double np[4] = {-1.0, 1.0, -1.0, 1.0};
        if (present(c, "NearPlane")) {
            const auto v = doubles(c->get("NearPlane"), "NearPlane", 4);
            for (int k = 0; k < 4; ++k) np[k] = v[k];
        }
        for (int k = 0; k < 4; ++k) cc.near_plane[k] = np[k];
        cc.num_samples = (int32_t)opt_int(c, "NumSamples", 1);
        cc.aperture_size = opt_double(c, "ApertureSize", 0.0);
        cc.focus_distance = opt_double(c, "FocusDistance", 0.0);
        F.cams.push_back(cc);
        F.image_names.push_back(present(c, "ImageName") ? trim(str_of(c->get("ImageName"))) : std::string());
    }
    const Value* matsV = doc->get("Materials");
    for (const Value* m : one_or_many(matsV ? matsV->get("Material") : nullptr)) {
        const rt_vec3 z{0, 0, 0};
        rt_material mm{};
        mm.ambient = opt_vec3(m, "AmbientReflectance", z);
        mm.diffuse = opt_vec3(m, "DiffuseReflectance", z);
        mm.specular = opt_vec3(m, "SpecularReflectance", z);
        mm.mirror = opt_vec3(m, "MirrorReflectance", z);
        mm.phong = opt_double(m, "PhongExponent", 1.0);
        mm.ior = opt_double(m, "RefractionIndex", 0.0);
        mm.absorption_index = opt_double(m, "AbsorptionIndex", 0.0);
        mm.roughness = opt_double(m, "Roughness", 0.0);
        mm.absorption = opt_vec3(m, "AbsorptionCoefficient", z);
        const std::string t = trim(str_of(m->get("_type")));
        mm.type = t == "mirror" ? RT_MAT_MIRROR : t == "dielectric" ? RT_MAT_DIELECTRIC
                : t == "conductor" ? RT_MAT_CONDUCTOR : RT_MAT_DEFAULT;
        F.mats.push_back(mm);
    }
    const Value* lights = doc->get("Lights");
    for (const Value* p : one_or_many(lights ? lights->get("PointLight") : nullptr))
        F.plights.push_back(rt_point_light{vec3(p->get("Position"), "Position"), vec3(p->get("Intensity"), "Intensity")});
    for (const Value* a : one_or_many(lights ? lights->get("AreaLight") : nullptr))
        F.alights.push_back(rt_area_light{vec3(a->get("Position"), "Position"), vec3(a->get("Normal"), "Normal"),
                                          vec3(a->get("Radiance"), "Radiance"), to_double(a->get("Size"), "Size")});

    const Value* objsIn = doc->get("Objects");
    std::unordered_map<std::string, M4> meshTransform;                      // id -> composed transform
    std::unordered_map<int32_t, std::pair<bool, std::string>> baseMaterial;  // mesh id -> its material
    for (const char* kind : kObjectOrder) {
        const std::string k(kind);
        for (const Value* o : one_or_many(objsIn ? objsIn->get(kind) : nullptr)) {
            if (o->kind != Value::Obj) fail(k + " must be an object");
            std::string oid;
            const bool hasId = id_of(o, oid);
            const Value* mv = o->get("Material");
            const bool hasMat = mv != nullptr && mv->kind != Value::Null;
            const std::string mat = hasMat ? trim(str_of(mv)) : std::string();
            const bool reset = opt_bool(o, "_resetTransform");
            const std::string tokens = str_of(o->get("Transformations"));
            rt_object r{};
            r.id = numeric_id(hasId, oid);
            r.indices_one_based = 1;
            if (k == "Mesh") {
                const M4 M = tf.compose(tokens, nullptr, reset);
                colmajor(M, r.transform);
                r.kind = RT_OBJ_MESH;
                r.material_id = material_index(hasMat, mat);
                r.smooth = (o->get("_shadingMode") ? str_of(o->get("_shadingMode")) : std::string("flat")) == "smooth";
                r.motion_blur = opt_vec3(o, "MotionBlur", rt_vec3{0, 0, 0});
                const Value* faces = o->get("Faces");
                const Value* ply = (faces && faces->kind == Value::Obj) ? faces->get("_plyFile") : nullptr;
                if (ply) {
                    std::string path = str_of(ply);
                    if (path.empty() || path[0] != '/') path = base_dir + "/" + path;   // os.path.join
                    F.paths.push_back(std::make_unique<std::string>(path));
                    r.ply_path = F.paths.back()->c_str();
                } else {
                    const std::vector<long long> idx = faces ? int_list(faces, "Faces") : std::vector<long long>();
                    if (idx.size() % 3) fail("Mesh " + oid + ": face index count is not a multiple of 3");
                    const long long off = (faces && faces->kind == Value::Obj) ? opt_int(faces, "_vertexOffset", 0) : 0;
                    const long long nv = (long long)vd.size() / 3;
                    auto fv = std::make_unique<std::vector<int32_t>>();
                    fv->reserve(idx.size());
                    for (long long x : idx) {
                        x += off;
                        if (x < 1 || x > nv) fail("Mesh " + oid + ": face index out of range 1.." + std::to_string(nv));
                        fv->push_back((int32_t)x);
                    }
                    r.positions = vd.empty() ? nullptr : vd.data();
                    r.num_positions = nv;
                    r.indices = fv->empty() ? nullptr : fv->data();
                    r.num_indices = (int64_t)fv->size();
                    F.faces.push_back(std::move(fv));
                }
                meshTransform[oid] = M;
                baseMaterial[r.id] = {hasMat, mat};
            } else if (k == "Triangle") {
                const auto ii = int_list(o->get("Indices"), "Indices");
                if (ii.size() < 3) fail("Triangle needs 3 indices");
                for (int q = 0; q < 3; ++q) r.v[q] = vertex(vd, ii[q], "Triangle");
                colmajor(tf.compose(tokens, nullptr, reset), r.transform);
                r.kind = RT_OBJ_TRIANGLE;
                r.material_id = material_index(hasMat, mat);
            } else if (k == "Sphere") {
                r.kind = RT_OBJ_SPHERE;
                r.center = vertex(vd, to_int(o->get("Center"), "Center"), "Sphere");
                r.radius = to_double(o->get("Radius"), "Radius");
                r.material_id = material_index(hasMat, mat);
                colmajor(tf.compose(tokens, nullptr, reset), r.transform);
            } else if (k == "Plane") {
                r.kind = RT_OBJ_PLANE;
                r.center = vertex(vd, to_int(o->get("Point") ? o->get("Point") : o->get("Center"), "Point"), "Plane");
                r.normal = vec3(o->get("Normal"), "Normal");
                r.material_id = material_index(hasMat, mat);
                colmajor(tf.compose(tokens, nullptr, reset), r.transform);
            } else {                                          // MeshInstance
                const std::string base = str_of(o->get("_baseMeshId"));
                auto it = meshTransform.find(base);
                // RTContext.swift:386: `guard let baseData = instanceByID[baseMeshID] else { continue }`
                if (it == meshTransform.end()) continue;
                const M4 M = tf.compose(tokens, &it->second, reset);
                meshTransform[oid] = M;
                colmajor(M, r.transform);
                r.kind = RT_OBJ_MESH_INSTANCE;
                r.base_mesh_id = numeric_id(true, base);
                if (hasMat && !mat.empty()) {
                    r.material_id = material_index(true, mat);
                } else {                                      // the base mesh's material
                    auto bm = baseMaterial.find(r.base_mesh_id);
                    r.material_id = bm == baseMaterial.end() ? -1 : material_index(bm->second.first, bm->second.second);
                }
                r.motion_blur = opt_vec3(o, "MotionBlur", rt_vec3{0, 0, 0});
            }
            F.objs.push_back(r);
        }
    }
    rt_scene_desc& d = F.desc;
    d.background_color = opt_vec3(doc, "BackgroundColor", rt_vec3{0, 0, 0});
    d.ambient_light = opt_vec3(lights, "AmbientLight", rt_vec3{0, 0, 0});
    d.shadow_ray_epsilon = opt_double(doc, "ShadowRayEpsilon", 1e-3);
    d.intersection_test_epsilon = opt_double(doc, "IntersectionTestEpsilon", 1e-6);
    d.max_recursion_depth = (int32_t)opt_int(doc, "MaxRecursionDepth", 6);
    d.num_materials = (int32_t)F.mats.size();
    d.materials = F.mats.empty() ? nullptr : F.mats.data();
    d.num_point_lights = (int32_t)F.plights.size();
    d.point_lights = F.plights.empty() ? nullptr : F.plights.data();
    d.num_area_lights = (int32_t)F.alights.size();
    d.area_lights = F.alights.empty() ? nullptr : F.alights.data();
    d.num_objects = (int32_t)F.objs.size();
    d.objects = F.objs.empty() ? nullptr : F.objs.data();
    d.num_cameras = (int32_t)F.cams.size();
    d.cameras = F.cams.empty() ? nullptr : F.cams.data();
}

static size_t bom(const char* p, size_t n) {
    return (n >= 3 && (unsigned char)p[0] == 0xEF && (unsigned char)p[1] == 0xBB && (unsigned char)p[2] == 0xBF) ? 3 : 0;
}
// SceneFormat.auto: '<' -> XML, '{' / '[' -> JSON
static int32_t detect(const char* p, size_t n) {
    size_t k = bom(p, n);
    while (k < n && std::isspace((unsigned char)p[k])) ++k;
    if (k < n && p[k] == '<') return RT_SCENE_FORMAT_XML;
    if (k < n && (p[k] == '{' || p[k] == '[')) return RT_SCENE_FORMAT_JSON;
    return -1;
}

}  // namespace sio
}  // namespace myrt

extern "C" {

const char* rt_scene_file_last_error(void) { return g_sio_err.c_str(); }

int32_t rt_scene_file_parse(const void* data, uint64_t size, int32_t format, const char* base_dir,
                            rt_scene_file** out) {
    using namespace myrt::sio;
    if (!out) return sio_fail(RT_ERR_INVALID_ARG, "out is NULL");
    *out = nullptr;
    if (!data && size > 0) return sio_fail(RT_ERR_INVALID_ARG, "data is NULL");
    const char* p = static_cast<const char*>(data);
    const size_t n = (size_t)size;
    const int32_t fmt = format == RT_SCENE_FORMAT_AUTO ? detect(p, n) : format;
    if (fmt != RT_SCENE_FORMAT_JSON && fmt != RT_SCENE_FORMAT_XML)
        return sio_fail(RT_ERR_SCENE_FILE, format == RT_SCENE_FORMAT_AUTO
                                               ? "cannot detect scene format (expected JSON or XML)"
                                               : "unknown scene format");
    std::string dir = base_dir ? std::string(base_dir) : std::string();
    if (dir.empty()) {                                         // os.getcwd()
        char buf[4096];
        dir = getcwd(buf, sizeof(buf)) ? std::string(buf) : std::string(".");
    }
    try {
        const size_t skip = bom(p, n);
        const Value doc = fmt == RT_SCENE_FORMAT_JSON ? Json(p + skip, n - skip).parse() : Xml(p + skip, n - skip).parse();
        auto F = std::make_unique<rt_scene_file>();
        decode(doc, dir, *F);
        *out = F.release();
        return RT_OK;
    } catch (const Error& e) {
        return sio_fail(RT_ERR_SCENE_FILE, e.msg);
    } catch (const std::bad_alloc&) {
        return sio_fail(RT_ERR_OOM, "host allocation failed");
    } catch (const std::exception& e) {
        return sio_fail(RT_ERR_SCENE_FILE, e.what());
    }
}

int32_t rt_scene_file_load(const char* path, int32_t format, rt_scene_file** out) {
    if (!out) return sio_fail(RT_ERR_INVALID_ARG, "out is NULL");
    *out = nullptr;
    if (!path) return sio_fail(RT_ERR_INVALID_ARG, "path is NULL");
    std::ifstream f(path, std::ios::binary);
    if (!f) return sio_fail(RT_ERR_SCENE_FILE, std::string("cannot open scene file ") + path);
    const std::string data((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    const std::string sp(path);
    int32_t fmt = format;
    if (fmt == RT_SCENE_FORMAT_AUTO) {                       // the extension first, then the content
        const size_t dot = sp.find_last_of('.');
        std::string ext = dot == std::string::npos ? std::string() : sp.substr(dot);
        for (auto& c : ext) c = (char)std::tolower((unsigned char)c);
        if (ext == ".json") fmt = RT_SCENE_FORMAT_JSON;
        else if (ext == ".xml") fmt = RT_SCENE_FORMAT_XML;
    }
    // Scene.path = the file's directory (RayTracer.swift:33-34): PLY paths resolve against it
    char* rp = realpath(path, nullptr);
    const std::string abs = rp ? std::string(rp) : sp;
    std::free(rp);
    const size_t slash = abs.find_last_of('/');
    const std::string dir = slash == std::string::npos ? std::string(".") : (slash == 0 ? std::string("/") : abs.substr(0, slash));
    return rt_scene_file_parse(data.data(), data.size(), fmt, dir.c_str(), out);
}

const rt_scene_desc* rt_scene_file_desc(const rt_scene_file* f) { return f ? &f->desc : nullptr; }

const char* rt_scene_file_image_name(const rt_scene_file* f, int32_t camera_index) {
    if (!f || camera_index < 0 || camera_index >= (int32_t)f->image_names.size()) return nullptr;
    return f->image_names[camera_index].c_str();
}

void rt_scene_file_destroy(rt_scene_file* f) { delete f; }

}  // extern "C"
