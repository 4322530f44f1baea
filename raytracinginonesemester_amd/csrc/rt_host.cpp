// rt_host.cpp — host side of the drop-in boundary: the pieces the reference keeps in C++
// around render() (scene JSON, OBJ meshes, object transforms, camera basis, CPU LBVH,
// ppm_p6), re-implemented with identical float results so the device scene built from
// them is byte-identical to the reference's arrays.  Citations use
//   G/   = HW2/HW2/GPUandCPU     HW1/ = HW1     (relative to the reference repo)
#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <memory>
#include <new>
#include <random>
#include <sstream>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "rt_common.hpp"

namespace rt {

namespace {
thread_local std::string g_last_error;
}

int set_error(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}
void clear_error() { g_last_error.clear(); }

namespace {
// rt_tuning_set's table: per knob, the bits of the value set XOR a quiet NaN's, so that the
// zero-initialised table reads NaN (= the default) everywhere
std::atomic<uint64_t> g_tuning[RT_TUNE_COUNT];
constexpr uint64_t kTuneNaN = 0x7ff8000000000000ull;
}  // namespace

double tuning(int id, double dflt) {
    if (id < 0 || id >= RT_TUNE_COUNT) return dflt;
    const uint64_t b = g_tuning[id].load(std::memory_order_relaxed) ^ kTuneNaN;
    double v;
    std::memcpy(&v, &b, sizeof v);
    return v == v ? v : dflt;
}

}  // namespace rt

using namespace rt;

extern "C" const char* rt_last_error(void) { return rt::g_last_error.c_str(); }
extern "C" int rt_abi_version(void) { return RT_ABI_VERSION; }

extern "C" int rt_tuning_set(int id, double value) {
    if (id < 0 || id >= RT_TUNE_COUNT) return set_error(RT_ERR_ARG, "rt_tuning_set: unknown knob");
    uint64_t b;
    std::memcpy(&b, &value, sizeof b);
    rt::g_tuning[id].store(value == value ? b ^ rt::kTuneNaN : 0);
    return RT_OK;
}
extern "C" int rt_tuning_get(int id, double* value) {
    if (id < 0 || id >= RT_TUNE_COUNT || !value) return set_error(RT_ERR_ARG, "rt_tuning_get: unknown knob");
    *value = rt::tuning(id, NAN);
    return RT_OK;
}
extern "C" void rt_tuning_reset(void) {
    for (auto& v : rt::g_tuning) v.store(0);
}

// ---------------------------------------------------------------------------------------
// Material defaults, camera, jitter
// ---------------------------------------------------------------------------------------
extern "C" void rt_material_default(rt_material* m) {
    // G/include/material.h:8-19
    m->albedo = v3(0.8f, 0.8f, 0.8f);
    m->kd = 1.0f;
    m->specular_color = v3(0.04f, 0.04f, 0.04f);
    m->ks = 0.0f;
    m->shininess = 32.0f;
    m->kr = 0.0f;
    m->emission = v3(0.0f, 0.0f, 0.0f);
}

namespace {
// Camera::unit_vector with its 1e-12 fallback (G/include/camera.h:218-223).
rt_vec3 cam_unit(rt_vec3 v) {
    const float len = sqrtf(v.x * v.x + v.y * v.y + v.z * v.z);
    if (double(len) < 1e-12) return v3(0.0f, 0.0f, 1.0f);
    return div_d(v, double(len));
}
}  // namespace

extern "C" int rt_camera_init(rt_camera* cam, const float pos[3], const float look_at[3],
                              const float up[3], double focal_length_mm, double sensor_height_mm,
                              int width, int height, int hw1) {
    if (!cam || !pos || !look_at || !up) return set_error(RT_ERR_ARG, "rt_camera_init: null argument");
    if (hw1 && (width < 1 || height < 1))  // HW1/include/camera.h:57-62 throws
        return set_error(RT_ERR_ARG, "Error: pixel_width/pixel_height must be >= 1");
    if (width < 1) width = 1;  // G/include/camera.h:73-74
    if (height < 1) height = 1;
    // G/include/camera.h:72-94: float vectors, double scalars narrowed at each Vec3 product.
    const rt_vec3 center = v3(pos[0], pos[1], pos[2]);
    const rt_vec3 forward = cam_unit(v3(look_at[0], look_at[1], look_at[2]) - center);
    const rt_vec3 right = cam_unit(cross(forward, v3(up[0], up[1], up[2])));
    const rt_vec3 up_corrected = cross(right, forward);
    const double focal_m = focal_length_mm / 1000.0;
    const double sensor_m = sensor_height_mm / 1000.0;
    const double vh = sensor_m;
    const double vw = vh * (double(width) / double(height));
    const rt_vec3 vu = right * float(vw);
    const rt_vec3 vv = up_corrected * float(-vh);
    cam->pixel_delta_u = div_d(vu, double(width));
    cam->pixel_delta_v = div_d(vv, double(height));
    const rt_vec3 vcenter = center + forward * float(focal_m);
    const rt_vec3 vul = (vcenter - vu * 0.5f) - vv * 0.5f;
    cam->pixel00_loc = vul + (cam->pixel_delta_u + cam->pixel_delta_v) * 0.5f;
    cam->center = center;
    cam->pixel_width = width;
    cam->pixel_height = height;
    return RT_OK;
}

extern "C" int rt_jittered_samples(int spp, uint32_t seed, int centered, float* out) {
    if (spp < 0 || (spp > 0 && !out)) return set_error(RT_ERR_ARG, "rt_jittered_samples: bad args");
    // G/include/antialias.h:12-27 — the same libstdc++ engine and distribution.
    std::mt19937 rng(seed);
    std::uniform_real_distribution<float> uni(0.0f, 1.0f);
    for (int s = 0; s < spp; ++s) {
        float dx = uni(rng), dy = uni(rng);
        if (centered) { dx = dx - 0.5f; dy = dy - 0.5f; }
        out[2 * s] = dx;
        out[2 * s + 1] = dy;
    }
    return RT_OK;
}

// ---------------------------------------------------------------------------------------
// OBJ loading: G/ LoadOBJ_ToMesh (MeshOBJ.h:260-427) and HW1 LoadOBJ_ToMeshSOA
// (HW1/src/MeshOBJ.cpp:143-281).  Unified vertices are created in first-reference order
// for each distinct (position, uv, normal) triple; quads split (i0,i1,i2),(i0,i2,i3).
// ---------------------------------------------------------------------------------------
namespace {

struct Mesh {
    std::vector<rt_vec3> positions;
    std::vector<rt_vec3> normals;
    std::vector<float> uvs;            // 2 per vertex when present
    std::vector<uint32_t> indices;
    std::vector<int32_t> tri_obj_ids;
    bool has_uvs() const { return !uvs.empty(); }
    bool has_normals() const { return !normals.empty(); }
};

struct VKey {
    int p, t, n;
    bool operator==(const VKey& o) const { return p == o.p && t == o.t && n == o.n; }
};
struct VKeyHash {
    size_t operator()(const VKey& k) const {
        uint64_t h = uint64_t(uint32_t(k.p)) * 0x9E3779B97F4A7C15ull;
        h ^= uint64_t(uint32_t(k.t)) + 0x7F4A7C159E3779B9ull + (h << 6) + (h >> 2);
        h ^= uint64_t(uint32_t(k.n)) + 0x94D049BB133111EBull + (h << 6) + (h >> 2);
        return size_t(h);
    }
};

inline void skip_ws(const char*& s) { while (*s == ' ' || *s == '\t') ++s; }

bool parse_int(const char*& s, int& out) {
    skip_ws(s);
    bool neg = false;
    if (*s == '-') { neg = true; ++s; }
    if (*s < '0' || *s > '9') return false;
    // digits past int's range make no index (the reference's std::stoi throws out_of_range):
    // the token is refused instead of overflowing (UBSan, tests/test_host_fuzz.py)
    long long v = 0;
    bool big = false;
    while (*s >= '0' && *s <= '9') {
        if (!big) v = v * 10 + (*s - '0');
        big = big || v > 2147483647LL;
        ++s;
    }
    if (big) return false;
    out = neg ? -int(v) : int(v);
    return true;
}

bool parse_float(const char*& s, float& out) {
    skip_ws(s);
    char* end = nullptr;
    out = std::strtof(s, &end);
    if (end == s) return false;
    s = end;
    return true;
}

// One face token "v", "v/vt", "v//vn", "v/vt/vn".  relative = G/ negative-index support.
bool parse_face_vertex(const char*& s, VKey& k, bool relative, size_t np, size_t nt, size_t nn) {
    int v = 0;
    if (!parse_int(s, v)) return false;
    k.p = (relative && v < 0) ? int(np) + v : v - 1;
    k.t = -1;
    k.n = -1;
    if (*s != '/') return true;
    ++s;
    if (*s == '/') {
        ++s;
        int n = 0;
        if (!parse_int(s, n)) return false;
        k.n = (relative && n < 0) ? int(nn) + n : n - 1;
        return true;
    }
    int t = 0;
    if (parse_int(s, t)) k.t = (relative && t < 0) ? int(nt) + t : t - 1;
    if (*s != '/') return true;
    ++s;
    int n = 0;
    if (parse_int(s, n)) k.n = (relative && n < 0) ? int(nn) + n : n - 1;
    return true;
}

// g_dialect: G/ semantics (negative indices, 'o'/'g' object ids); else HW1 semantics.
int load_obj(const std::string& path, Mesh& out, int& next_object_id, bool g_dialect) {
    out = Mesh{};
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) return set_error(RT_ERR_IO, "cannot open OBJ: " + path);
    std::vector<rt_vec3> raw_pos, raw_nrm;
    std::vector<float> raw_uv;
    bool file_has_uv = false, file_has_nrm = false;
    std::unordered_map<VKey, uint32_t, VKeyHash> dedup;
    dedup.reserve(10000);
    int current_obj = next_object_id;
    bool first_tag = false;
    char line[1024];  // fgets chunking as in the reference loaders
    int rc = RT_OK;

    auto get_or_create = [&](const VKey& k, uint32_t& idx) -> bool {
        auto it = dedup.find(k);
        if (it != dedup.end()) { idx = it->second; return true; }
        if (k.p < 0 || size_t(k.p) >= raw_pos.size()) return false;  // rawPos.at() throws
        idx = uint32_t(out.positions.size());
        dedup.emplace(k, idx);
        out.positions.push_back(raw_pos[size_t(k.p)]);
        if (file_has_uv) {
            float u = 0.0f, v = 0.0f;
            if (k.t >= 0 && k.t < int(raw_uv.size() / 2)) { u = raw_uv[2 * k.t]; v = raw_uv[2 * k.t + 1]; }
            out.uvs.push_back(u);
            out.uvs.push_back(v);
        }
        if (file_has_nrm) {
            rt_vec3 n = v3(0.0f, 0.0f, 0.0f);
            if (k.n >= 0 && k.n < int(raw_nrm.size())) n = raw_nrm[size_t(k.n)];
            out.normals.push_back(n);
        }
        return true;
    };

    while (std::fgets(line, sizeof(line), f)) {
        const char* s = line;
        skip_ws(s);
        if (*s == '\0' || *s == '\n' || *s == '#') continue;
        if (g_dialect && (*s == 'o' || *s == 'g')) {  // MeshOBJ.h:292-311
            if (first_tag) {
                next_object_id++;
                current_obj = next_object_id;
            } else {
                if (!out.indices.empty()) {
                    next_object_id++;
                    current_obj = next_object_id;
                }
                first_tag = true;
            }
            continue;
        }
        if (s[0] == 'v' && (s[1] == ' ' || s[1] == '\t')) {
            s += 1;
            rt_vec3 p{};
            if (!parse_float(s, p.x) || !parse_float(s, p.y) || !parse_float(s, p.z)) {
                rc = set_error(RT_ERR_PARSE, "bad vertex line in " + path);
                break;
            }
            raw_pos.push_back(p);
            continue;
        }
        if (s[0] == 'v' && s[1] == 't' && (s[2] == ' ' || s[2] == '\t')) {
            s += 2;
            float u = 0, v = 0;
            if (!parse_float(s, u) || !parse_float(s, v)) {
                rc = set_error(RT_ERR_PARSE, "bad vt line in " + path);
                break;
            }
            raw_uv.push_back(u);
            raw_uv.push_back(v);
            file_has_uv = true;
            continue;
        }
        if (s[0] == 'v' && s[1] == 'n' && (s[2] == ' ' || s[2] == '\t')) {
            s += 2;
            rt_vec3 n{};
            if (!parse_float(s, n.x) || !parse_float(s, n.y) || !parse_float(s, n.z)) {
                rc = set_error(RT_ERR_PARSE, "bad vn line in " + path);
                break;
            }
            raw_nrm.push_back(n);
            file_has_nrm = true;
            continue;
        }
        if (s[0] == 'f' && (s[1] == ' ' || s[1] == '\t')) {
            s += 1;
            VKey keys[4];
            int count = 0;
            while (count < 4) {
                skip_ws(s);
                if (*s == '\0' || *s == '\n') break;
                VKey k{};
                if (!parse_face_vertex(s, k, g_dialect, raw_pos.size(), raw_uv.size() / 2, raw_nrm.size())) break;
                if (k.t >= 0) file_has_uv = true;
                if (k.n >= 0) file_has_nrm = true;
                keys[count++] = k;
                while (*s != '\0' && *s != '\n' && *s != ' ' && *s != '\t') ++s;
            }
            if (count < 3) {
                rc = set_error(RT_ERR_PARSE, "face with fewer than 3 vertices in " + path);
                break;
            }
            uint32_t i0, i1, i2;
            if (!get_or_create(keys[0], i0) || !get_or_create(keys[1], i1) || !get_or_create(keys[2], i2)) {
                rc = set_error(RT_ERR_PARSE, "face index out of range in " + path);
                break;
            }
            out.indices.insert(out.indices.end(), {i0, i1, i2});
            out.tri_obj_ids.push_back(current_obj);
            if (count == 4) {
                uint32_t i3;
                if (!get_or_create(keys[3], i3)) {
                    rc = set_error(RT_ERR_PARSE, "face index out of range in " + path);
                    break;
                }
                out.indices.insert(out.indices.end(), {i0, i2, i3});
                out.tri_obj_ids.push_back(current_obj);
            }
            continue;
        }
    }
    std::fclose(f);
    if (rc != RT_OK) return rc;
    if (out.positions.empty() || out.indices.empty()) return set_error(RT_ERR_PARSE, "OBJ has no faces: " + path);
    if (g_dialect) next_object_id++;  // MeshOBJ.h:420
    if (file_has_uv && out.uvs.size() / 2 != out.positions.size())
        return set_error(RT_ERR_PARSE, "OBJ uv stream does not cover every vertex: " + path);
    if (file_has_nrm && out.normals.size() != out.positions.size())
        return set_error(RT_ERR_PARSE, "OBJ normal stream does not cover every vertex: " + path);
    return RT_OK;
}

// G/include/MeshOBJ.h:429-466
void append_mesh(Mesh& dst, const Mesh& src) {
    const uint32_t offset = uint32_t(dst.positions.size());
    dst.positions.insert(dst.positions.end(), src.positions.begin(), src.positions.end());
    if (dst.has_normals() || src.has_normals()) {
        if (!dst.has_normals() && !dst.positions.empty()) dst.normals.resize(offset, v3(0, 0, 0));
        if (src.has_normals()) dst.normals.insert(dst.normals.end(), src.normals.begin(), src.normals.end());
        else dst.normals.resize(dst.normals.size() + src.positions.size(), v3(0, 0, 0));
    }
    if (dst.has_uvs() || src.has_uvs()) {
        if (!dst.has_uvs() && !dst.positions.empty()) dst.uvs.resize(size_t(offset) * 2, 0.0f);
        if (src.has_uvs()) dst.uvs.insert(dst.uvs.end(), src.uvs.begin(), src.uvs.end());
        else dst.uvs.resize(dst.uvs.size() + src.positions.size() * 2, 0.0f);
    }
    const size_t old = dst.indices.size();
    dst.indices.resize(old + src.indices.size());
    for (size_t i = 0; i < src.indices.size(); ++i) dst.indices[old + i] = src.indices[i] + offset;
    dst.tri_obj_ids.insert(dst.tri_obj_ids.end(), src.tri_obj_ids.begin(), src.tri_obj_ids.end());
}

// G/src/main.cu:53-96
inline float deg2rad(float d) { return d * 0.01745329251994329577f; }
rt_vec3 rotate_xyz(rt_vec3 v, rt_vec3 rdeg) {
    const float rx = deg2rad(rdeg.x), ry = deg2rad(rdeg.y), rz = deg2rad(rdeg.z);
    const float cx = cosf(rx), sx = sinf(rx);
    const float cy = cosf(ry), sy = sinf(ry);
    const float cz = cosf(rz), sz = sinf(rz);
    v = v3(v.x, cx * v.y - sx * v.z, sx * v.y + cx * v.z);
    v = v3(cy * v.x + sy * v.z, v.y, -sy * v.x + cy * v.z);
    v = v3(cz * v.x - sz * v.y, sz * v.x + cz * v.y, v.z);
    return v;
}

struct SceneObject {
    std::string name, type, path;
    rt_vec3 position{0, 0, 0}, rotation{0, 0, 0}, scale{1, 1, 1};
    rt_material material;
    SceneObject() { rt_material_default(&material); }
};

void apply_object_transform(Mesh& mesh, const SceneObject& obj) {
    for (auto& p : mesh.positions) {
        const rt_vec3 scaled = v3(p.x * obj.scale.x, p.y * obj.scale.y, p.z * obj.scale.z);
        p = rotate_xyz(scaled, obj.rotation) + obj.position;
    }
    for (auto& n : mesh.normals) {
        rt_vec3 ns = n;
        if (fabsf(obj.scale.x) > 1e-8f) ns.x /= obj.scale.x;
        if (fabsf(obj.scale.y) > 1e-8f) ns.y /= obj.scale.y;
        if (fabsf(obj.scale.z) > 1e-8f) ns.z /= obj.scale.z;
        const rt_vec3 nr = rotate_xyz(ns, obj.rotation);
        const float len2 = dot(nr, nr);
        if (len2 > 1e-12f) {
            const float inv = 1.0f / sqrtf(len2);
            n = nr * inv;
        } else {
            n = v3(0.0f, 0.0f, 1.0f);
        }
    }
}

// ---------------------------------------------------------------------------------------
// Minimal JSON reader (the G/ scene dialect, G/include/scene.h:47-217): numbers via
// strtod, strings with the standard escapes.
// ---------------------------------------------------------------------------------------
struct Json {
    enum Type { Null, Bool, Number, String, Array, Object } type = Null;
    bool b = false;
    double num = 0.0;
    std::string str;
    std::vector<Json> arr;
    std::vector<std::pair<std::string, Json>> obj;
    const Json* get(const char* key) const {
        if (type != Object) return nullptr;
        for (auto& kv : obj)
            if (kv.first == key) return &kv.second;
        return nullptr;
    }
};

class JsonReader {
public:
    explicit JsonReader(const std::string& s) : s_(s) {}
    bool parse(Json& out, std::string& err) {
        if (!value(out, 0)) { err = err_; return false; }
        ws();
        if (i_ != s_.size()) { err = "Trailing characters"; return false; }
        return true;
    }

private:
    const std::string& s_;
    size_t i_ = 0;
    std::string err_;
    bool fail(const char* m) { err_ = m; return false; }
    void ws() { while (i_ < s_.size() && std::isspace(static_cast<unsigned char>(s_[i_]))) ++i_; }
    // Nesting is bounded (the scene dialect needs 4 levels): the reader recurses per level, and
    // an unbounded depth let a file of 10^5 '[' overflow the C stack (tests/test_host_fuzz.py).
    static constexpr int kMaxDepth = 256;
    bool value(Json& o, int depth) {
        ws();
        if (i_ >= s_.size()) return fail("Unexpected end of input");
        const char c = s_[i_];
        if ((c == '{' || c == '[') && depth >= kMaxDepth) return fail("Nesting too deep");
        if (c == '{') return object(o, depth);
        if (c == '[') return array(o, depth);
        if (c == '"') return string(o);
        if (c == 't' || c == 'f') return boolean(o);
        if (c == 'n') {
            if (s_.compare(i_, 4, "null") == 0) { i_ += 4; o.type = Json::Null; return true; }
            return fail("Bad null");
        }
        if (c == '-' || (c >= '0' && c <= '9')) return number(o);
        return fail("Unexpected character");
    }
    bool object(Json& o, int depth) {
        o.type = Json::Object;
        ++i_;
        ws();
        if (i_ < s_.size() && s_[i_] == '}') { ++i_; return true; }
        while (i_ < s_.size()) {
            Json key;
            if (i_ >= s_.size() || s_[i_] != '"') return fail("Expected '\"'");
            if (!string(key)) return false;
            ws();
            if (i_ >= s_.size() || s_[i_] != ':') return fail("Expected ':'");
            ++i_;
            Json v;
            if (!value(v, depth + 1)) return false;
            o.obj.emplace_back(key.str, std::move(v));
            ws();
            if (i_ < s_.size() && s_[i_] == ',') { ++i_; ws(); continue; }
            if (i_ < s_.size() && s_[i_] == '}') { ++i_; return true; }
            return fail("Expected ',' or '}'");
        }
        return fail("Unterminated object");
    }
    bool array(Json& o, int depth) {
        o.type = Json::Array;
        ++i_;
        ws();
        if (i_ < s_.size() && s_[i_] == ']') { ++i_; return true; }
        while (i_ < s_.size()) {
            Json v;
            if (!value(v, depth + 1)) return false;
            o.arr.push_back(std::move(v));
            ws();
            if (i_ < s_.size() && s_[i_] == ',') { ++i_; ws(); continue; }
            if (i_ < s_.size() && s_[i_] == ']') { ++i_; return true; }
            return fail("Expected ',' or ']'");
        }
        return fail("Unterminated array");
    }
    bool string(Json& o) {
        o.type = Json::String;
        ++i_;
        while (i_ < s_.size()) {
            const char c = s_[i_++];
            if (c == '"') return true;
            if (c != '\\') { o.str.push_back(c); continue; }
            if (i_ >= s_.size()) return fail("Bad escape");
            const char e = s_[i_++];
            switch (e) {
                case '"': o.str.push_back('"'); break;
                case '\\': o.str.push_back('\\'); break;
                case '/': o.str.push_back('/'); break;
                case 'b': o.str.push_back('\b'); break;
                case 'f': o.str.push_back('\f'); break;
                case 'n': o.str.push_back('\n'); break;
                case 'r': o.str.push_back('\r'); break;
                case 't': o.str.push_back('\t'); break;
                case 'u': {
                    if (i_ + 4 > s_.size()) return fail("Bad unicode escape");
                    unsigned code = 0;
                    for (int k = 0; k < 4; ++k) {
                        const char h = s_[i_++];
                        code <<= 4;
                        if (h >= '0' && h <= '9') code |= unsigned(h - '0');
                        else if (h >= 'a' && h <= 'f') code |= unsigned(h - 'a' + 10);
                        else if (h >= 'A' && h <= 'F') code |= unsigned(h - 'A' + 10);
                        else return fail("Bad unicode escape");
                    }
                    o.str.push_back(code <= 0x7F ? char(code) : '?');
                } break;
                default: return fail("Bad escape");
            }
        }
        return fail("Unterminated string");
    }
    bool number(Json& o) {
        o.type = Json::Number;
        const char* start = s_.c_str() + i_;
        char* end = nullptr;
        o.num = std::strtod(start, &end);
        if (end == start) return fail("Bad number");
        i_ = size_t(end - s_.c_str());
        return true;
    }
    bool boolean(Json& o) {
        if (s_.compare(i_, 4, "true") == 0) { o.type = Json::Bool; o.b = true; i_ += 4; return true; }
        if (s_.compare(i_, 5, "false") == 0) { o.type = Json::Bool; o.b = false; i_ += 5; return true; }
        return fail("Bad boolean");
    }
};

// int(x) of a JSON number, as the reference's int conversions give for every value in int's
// range; outside it (and NaN) the C++ conversion is undefined, so it saturates here instead.
int json_int(double d) {
    if (!(d == d)) return 0;
    if (d >= 2147483647.0) return 2147483647;
    if (d <= -2147483648.0) return -2147483647 - 1;
    return int(d);
}

bool as_vec3(const Json* v, rt_vec3& out) {  // scene.h:230-240
    if (!v || v->type != Json::Array || v->arr.size() != 3) return false;
    for (int k = 0; k < 3; ++k)
        if (v->arr[k].type != Json::Number) return false;
    out = v3(float(v->arr[0].num), float(v->arr[1].num), float(v->arr[2].num));
    return true;
}

struct SceneDesc {
    int max_depth = 1, spp = 1;
    bool diffuse_bounce = true;
    rt_vec3 miss_color{0, 0, 0};
    // Camera() defaults (G/include/camera.h:13-20)
    rt_vec3 cam_pos{0, 0, 0}, cam_look{0, 1, 0}, cam_up{0, 0, 1};
    double focal_mm = 50.0, sensor_mm = 24.0;
    int width = 100, height = 100;
    std::vector<rt_light> lights;
    std::vector<SceneObject> objects;
};

rt_light default_light() {
    rt_light l;
    l.position = v3(0, 0, 0);
    l.color = v3(1, 1, 1);
    l.intensity = 1;
    return l;
}

bool read_light(const Json& item, rt_light& lc) {  // scene.h:307-316, 322-330
    lc = default_light();
    as_vec3(item.get("position"), lc.position);
    as_vec3(item.get("color"), lc.color);
    const Json* v = item.get("intensity");
    if (v && v->type == Json::Number) lc.intensity = json_int(v->num);
    return true;
}

// G/include/scene.h:242-380
int parse_scene(const Json& root, SceneDesc& sc) {
    if (root.type != Json::Object) return set_error(RT_ERR_PARSE, "Root is not an object");
    if (const Json* st = root.get("settings")) {
        const Json* v;
        if ((v = st->get("max_bounces")) && v->type == Json::Number) sc.max_depth = json_int(v->num);
        if ((v = st->get("spp")) && v->type == Json::Number) {
            sc.spp = json_int(v->num);
            if (sc.spp < 1) sc.spp = 1;
        }
        if ((v = st->get("diffuse_bounce")) && v->type == Json::Bool) sc.diffuse_bounce = v->b;
    }
    if (const Json* mc = root.get("miss_color")) as_vec3(mc, sc.miss_color);
    if (const Json* cam = root.get("camera")) {
        const Json* v;
        if ((v = cam->get("focal_length_mm")) && v->type == Json::Number) sc.focal_mm = v->num;
        if ((v = cam->get("sensor_height_mm")) && v->type == Json::Number) sc.sensor_mm = v->num;
        if ((v = cam->get("pixel_width")) && v->type == Json::Number) sc.width = json_int(v->num);
        if ((v = cam->get("pixel_height")) && v->type == Json::Number) sc.height = json_int(v->num);
        as_vec3(cam->get("position"), sc.cam_pos);
        as_vec3(cam->get("look_at"), sc.cam_look);
        as_vec3(cam->get("up"), sc.cam_up);
        // Camera::initialize clamps < 1 (camera.h:73-74); the stored dims follow it.
        if (sc.width < 1) sc.width = 1;
        if (sc.height < 1) sc.height = 1;
    }
    sc.lights.clear();
    if (const Json* ls = root.get("lights"); ls && ls->type == Json::Array) {
        for (const auto& item : ls->arr) {
            if (item.type != Json::Object) continue;
            rt_light lc;
            read_light(item, lc);
            sc.lights.push_back(lc);
        }
    }
    if (sc.lights.empty()) {
        if (const Json* l = root.get("light"); l && l->type == Json::Object) {
            rt_light lc;
            read_light(*l, lc);
            sc.lights.push_back(lc);
        }
    }
    const Json* arr = root.get("scene");
    if (!arr || arr->type != Json::Array) return set_error(RT_ERR_PARSE, "Missing 'scene' array");
    sc.objects.clear();
    for (const auto& item : arr->arr) {
        if (item.type != Json::Object) continue;
        SceneObject obj;
        const Json* v;
        if ((v = item.get("name")) && v->type == Json::String) obj.name = v->str;
        if ((v = item.get("type")) && v->type == Json::String) obj.type = v->str;
        if ((v = item.get("path")) && v->type == Json::String) obj.path = v->str;
        if (const Json* tr = item.get("transform"); tr && tr->type == Json::Object) {
            as_vec3(tr->get("position"), obj.position);
            as_vec3(tr->get("rotation"), obj.rotation);
            as_vec3(tr->get("scale"), obj.scale);
        }
        if (const Json* m = item.get("material"); m && m->type == Json::Object) {
            as_vec3(m->get("albedo"), obj.material.albedo);
            as_vec3(m->get("specular_color"), obj.material.specular_color);
            as_vec3(m->get("emission"), obj.material.emission);
            if ((v = m->get("kd")) && v->type == Json::Number) obj.material.kd = float(v->num);
            if ((v = m->get("ks")) && v->type == Json::Number) obj.material.ks = float(v->num);
            if ((v = m->get("shininess")) && v->type == Json::Number) obj.material.shininess = float(v->num);
            if ((v = m->get("kr")) && v->type == Json::Number) obj.material.kr = float(v->num);
        }
        if (!obj.path.empty()) sc.objects.push_back(obj);
    }
    if (sc.objects.empty()) return set_error(RT_ERR_PARSE, "Scene contains no valid objects");
    return RT_OK;
}

std::string dirname_of(const std::string& p) {  // scene.h:395-399
    const size_t pos = p.find_last_of("/\\");
    if (pos == std::string::npos) return ".";
    return p.substr(0, pos);
}
bool is_abs_path(const std::string& p) {  // scene.h:401-406
    if (p.empty()) return false;
    if (p[0] == '/' || p[0] == '\\') return true;
    return p.size() >= 2 && std::isalpha(static_cast<unsigned char>(p[0])) && p[1] == ':';
}
std::string join_path(const std::string& base, const std::string& rel) {  // scene.h:408-412
    if (base.empty() || base == ".") return rel;
    if (base.back() == '/' || base.back() == '\\') return base + rel;
    return base + "/" + rel;
}
bool file_exists(const std::string& p) { std::ifstream f(p); return bool(f); }

}  // namespace

// ---------------------------------------------------------------------------------------
// CPU LBVH (G/include/bvh.h:131-151, 292-406; G/include/bvh.cu:60-89, 209-317)
// ---------------------------------------------------------------------------------------
namespace {

inline rt_aabb aabb_empty() {
    return rt_aabb{v3(INFINITY, INFINITY, INFINITY), v3(-INFINITY, -INFINITY, -INFINITY)};
}
inline rt_aabb aabb_merge(const rt_aabb& a, const rt_aabb& b) {
    return rt_aabb{v3(fminf(a.min_corner.x, b.min_corner.x), fminf(a.min_corner.y, b.min_corner.y),
                      fminf(a.min_corner.z, b.min_corner.z)),
                   v3(fmaxf(a.max_corner.x, b.max_corner.x), fmaxf(a.max_corner.y, b.max_corner.y),
                      fmaxf(a.max_corner.z, b.max_corner.z))};
}
inline rt_aabb aabb_of_triangle(rt_vec3 a, rt_vec3 b, rt_vec3 c) {
    rt_aabb box;
    box.min_corner = v3(fminf(a.x, fminf(b.x, c.x)), fminf(a.y, fminf(b.y, c.y)), fminf(a.z, fminf(b.z, c.z)));
    box.max_corner = v3(fmaxf(a.x, fmaxf(b.x, c.x)), fmaxf(a.y, fmaxf(b.y, c.y)), fmaxf(a.z, fmaxf(b.z, c.z)));
    const float eps = 0.0f;
    box.min_corner = v3(box.min_corner.x - eps, box.min_corner.y - eps, box.min_corner.z - eps);
    box.max_corner = v3(box.max_corner.x + eps, box.max_corner.y + eps, box.max_corner.z + eps);
    return box;
}
inline uint32_t bit_expansion(uint32_t v) {
    v = (v * 0x00010001u) & 0xFF0000FFu;
    v = (v * 0x00000101u) & 0x0F00F00Fu;
    v = (v * 0x00000011u) & 0xC30C30C3u;
    v = (v * 0x00000005u) & 0x49249249u;
    return v;
}
inline uint32_t morton30(rt_vec3 p) {
    const float res = 1024.0f;
    p.x = fminf(fmaxf(p.x * res, 0.0f), res - 1.0f);
    p.y = fminf(fmaxf(p.y * res, 0.0f), res - 1.0f);
    p.z = fminf(fmaxf(p.z * res, 0.0f), res - 1.0f);
    return bit_expansion(uint32_t(p.x)) * 4 + bit_expansion(uint32_t(p.y)) * 2 + bit_expansion(uint32_t(p.z));
}
inline int clz_common(uint64_t a, uint64_t b) {
    const uint64_t d = a ^ b;
    return d == 0 ? 64 : __builtin_clzll(d);
}

// Karras 2012 range determination (bvh.h:303-361), types as in the reference.
void determine_range(const uint64_t* code, unsigned n, unsigned idx, unsigned& first, unsigned& last) {
    if (idx == 0) { first = 0; last = n - 1; return; }
    const uint64_t self = code[idx];
    const int L = clz_common(self, code[idx - 1]);
    const int R = clz_common(self, code[idx + 1]);
    const int d = (R > L) ? 1 : -1;
    const int delta_min = std::min(L, R);
    int l_max = 2;
    int delta = -1;
    int i_tmp = int(idx + unsigned(d * l_max));
    if (0 <= i_tmp && unsigned(i_tmp) < n) delta = clz_common(self, code[i_tmp]);
    while (delta > delta_min) {
        l_max <<= 1;
        i_tmp = int(idx + unsigned(d * l_max));
        delta = -1;
        if (0 <= i_tmp && unsigned(i_tmp) < n) delta = clz_common(self, code[i_tmp]);
    }
    int l = 0;
    int t = l_max >> 1;
    while (t > 0) {
        i_tmp = int(idx + unsigned((l + t) * d));
        delta = -1;
        if (0 <= i_tmp && unsigned(i_tmp) < n) delta = clz_common(self, code[i_tmp]);
        if (delta > delta_min) l += t;
        t >>= 1;
    }
    unsigned jdx = idx + unsigned(l * d);
    if (d < 0) std::swap(idx, jdx);
    first = idx;
    last = jdx;
}

// bvh.h:363-394
unsigned find_split(const uint64_t* code, unsigned first, unsigned last) {
    const uint64_t fc = code[first], lc = code[last];
    if (fc == lc) return (first + last) >> 1;
    const int delta_node = clz_common(fc, lc);
    int split = int(first);
    int stride = int(last - first);
    do {
        stride = (stride + 1) >> 1;
        const int middle = split + stride;
        if (middle < int(last)) {
            if (clz_common(fc, code[middle]) > delta_node) split = middle;
        }
    } while (stride > 1);
    return unsigned(split);
}

// Leaves' AABBs must already sit at [P-1, 2P-1) (calculateAABBs).
void build_lbvh(rt_bvh_node* nodes, rt_aabb* aabbs, rt_aabb scene_box, int P) {
    if (P <= 0) return;
    const int total = 2 * P - 1;
    for (int i = 0; i < total; ++i) nodes[i] = rt_bvh_node{0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
    std::vector<std::pair<uint64_t, uint32_t>> pairs(static_cast<size_t>(P));
    const rt_vec3 extent = scene_box.max_corner - scene_box.min_corner;
    for (int i = 0; i < P; ++i) {
        const rt_aabb& b = aabbs[(P - 1) + i];
        const rt_vec3 centroid = (b.min_corner + b.max_corner) * 0.5f;
        const rt_vec3 nrm = div_v(centroid - scene_box.min_corner, extent);
        const uint64_t key = (uint64_t(morton30(nrm)) << 32) | uint64_t(uint32_t(i));
        pairs[size_t(i)] = {key, uint32_t(i)};
    }
    std::sort(pairs.begin(), pairs.end());
    std::vector<uint64_t> codes(static_cast<size_t>(P));
    std::vector<rt_aabb> leaf_copy(static_cast<size_t>(P));
    for (int i = 0; i < P; ++i) {
        codes[size_t(i)] = pairs[size_t(i)].first;
        leaf_copy[size_t(i)] = aabbs[(P - 1) + pairs[size_t(i)].second];
    }
    for (int i = 0; i < P; ++i) {
        aabbs[(P - 1) + i] = leaf_copy[size_t(i)];
        nodes[(P - 1) + i].object_idx = pairs[size_t(i)].second;
    }
    for (int idx = 0; idx < P - 1; ++idx) {
        nodes[idx].object_idx = 0xFFFFFFFFu;
        unsigned a, b;
        determine_range(codes.data(), unsigned(P), unsigned(idx), a, b);
        const unsigned gamma = find_split(codes.data(), a, b);
        nodes[idx].left_idx = gamma;
        nodes[idx].right_idx = gamma + 1;
        if (std::min(a, b) == gamma) nodes[idx].left_idx += unsigned(P - 1);
        if (std::max(a, b) == gamma + 1) nodes[idx].right_idx += unsigned(P - 1);
        nodes[nodes[idx].left_idx].parent_idx = unsigned(idx);
        nodes[nodes[idx].right_idx].parent_idx = unsigned(idx);
    }
    // refit_cpu (bvh.h:396-406): children before parent; iterative post-order.
    if (P > 1) {
        std::vector<std::pair<uint32_t, bool>> st;
        st.push_back({0u, false});
        while (!st.empty()) {
            auto [n, expanded] = st.back();
            st.pop_back();
            if (int(n) >= P - 1) continue;
            if (expanded) {
                aabbs[n] = aabb_merge(aabbs[nodes[n].left_idx], aabbs[nodes[n].right_idx]);
            } else {
                st.push_back({n, true});
                st.push_back({nodes[n].right_idx, false});
                st.push_back({nodes[n].left_idx, false});
            }
        }
    }
}

int build_bvh_from_mesh(const rt_vec3* pos, size_t nv, const uint32_t* idx, size_t P,
                        rt_bvh_node* nodes, rt_aabb* aabbs) {
    if (P == 0) return set_error(RT_ERR_ARG, "no triangles");
    if (P > 0x7FFFFFFFull) return set_error(RT_ERR_UNSUPPORTED, "more than 2^31-1 triangles");
    // calculateAABBs (bvh.cu:73-88)
    for (size_t i = 0; i < P; ++i) {
        const uint32_t a = idx[3 * i], b = idx[3 * i + 1], c = idx[3 * i + 2];
        if (a >= nv || b >= nv || c >= nv) return set_error(RT_ERR_ARG, "triangle index out of range");
        aabbs[(P - 1) + i] = aabb_of_triangle(pos[a], pos[b], pos[c]);
    }
    // std::accumulate(AABB::merge) from AABB() (main.cu:296-302)
    rt_aabb scene = aabb_empty();
    for (size_t i = 0; i < P; ++i) scene = aabb_merge(scene, aabbs[(P - 1) + i]);
    build_lbvh(nodes, aabbs, scene, int(P));
    return RT_OK;
}

}  // namespace

extern "C" int rt_build_bvh(const rt_vec3* positions, size_t num_vertices, const uint32_t* indices,
                            size_t num_triangles, rt_bvh_node* nodes, rt_aabb* aabbs) {
    if (!positions || !indices || !nodes || !aabbs) return set_error(RT_ERR_ARG, "rt_build_bvh: null argument");
    return build_bvh_from_mesh(positions, num_vertices, indices, num_triangles, nodes, aabbs);
}

// ---------------------------------------------------------------------------------------
// Host scene
// ---------------------------------------------------------------------------------------
struct rt_host_scene {
    SceneDesc desc;
    Mesh mesh;
    std::vector<rt_material> materials;
    std::vector<rt_light> lights;
    std::vector<rt_bvh_node> nodes;
    std::vector<rt_aabb> aabbs;
    std::vector<rt_triangle> tris;
    int objects_loaded = 0;
    int max_stack = 0, height = 0;
};

namespace {

// DFS stack depth needed by SearchBVH's push-left-push-right / pop-right-first order
// (no pruning): S(leaf) = 0, S(n) = max(2, 1 + S(right), S(left)); whole = max(1, S(root)).
void tree_stats(const std::vector<rt_bvh_node>& nodes, int& max_stack, int& height) {
    const size_t n = nodes.size();
    std::vector<int> S(n, 0), Hh(n, 0);
    std::vector<std::pair<uint32_t, bool>> st{{0u, false}};
    while (!st.empty()) {
        auto [v, done] = st.back();
        st.pop_back();
        const rt_bvh_node& nd = nodes[v];
        if (nd.object_idx != 0xFFFFFFFFu) { S[v] = 0; Hh[v] = 0; continue; }
        if (!done) {
            st.push_back({v, true});
            st.push_back({nd.left_idx, false});
            st.push_back({nd.right_idx, false});
        } else {
            S[v] = std::max({2, 1 + S[nd.right_idx], S[nd.left_idx]});
            Hh[v] = 1 + std::max(Hh[nd.left_idx], Hh[nd.right_idx]);
        }
    }
    max_stack = std::max(1, S[0]);
    height = Hh[0];
}

int finish_scene(rt_host_scene* hs) {
    Mesh& gm = hs->mesh;
    if (gm.positions.empty()) return set_error(RT_ERR_PARSE, "No valid geometry loaded.");
    const size_t P = gm.indices.size() / 3;
    hs->nodes.resize(2 * P - 1);
    hs->aabbs.resize(2 * P - 1);
    int rc = build_bvh_from_mesh(gm.positions.data(), gm.positions.size(), gm.indices.data(), P,
                                 hs->nodes.data(), hs->aabbs.data());
    if (rc != RT_OK) return rc;
    // main.cu:388-404
    hs->tris.resize(P);
    for (size_t i = 0; i < P; ++i) {
        const uint32_t a = gm.indices[3 * i], b = gm.indices[3 * i + 1], c = gm.indices[3 * i + 2];
        rt_triangle t;
        t.v0 = gm.positions[a];
        t.v1 = gm.positions[b];
        t.v2 = gm.positions[c];
        if (!gm.normals.empty()) {
            t.n0 = gm.normals[a]; t.n1 = gm.normals[b]; t.n2 = gm.normals[c];
        } else {
            t.n0 = t.n1 = t.n2 = v3(0, 0, 0);
        }
        hs->tris[i] = t;
    }
    // main.cu:328-336: fallback light when the scene has none
    hs->lights = hs->desc.lights;
    if (hs->lights.empty()) {
        rt_light l;
        l.position = v3(-3.0f, 0.0f, 1.0f);
        l.color = v3(1.0f, 1.0f, 1.0f);
        l.intensity = 1;
        hs->lights.push_back(l);
    }
    tree_stats(hs->nodes, hs->max_stack, hs->height);
    return RT_OK;
}

int load_objects(rt_host_scene* hs, const std::vector<SceneObject>& objs) {
    int next_id = 0;
    for (const auto& obj : objs) {  // main.cu:168-190
        Mesh tmp;
        const int id_begin = next_id;
        int rc = load_obj(obj.path, tmp, next_id, true);
        if (rc != RT_OK) continue;  // the reference skips objects that fail to load
        apply_object_transform(tmp, obj);
        if (hs->materials.size() < size_t(next_id)) {
            rt_material d;
            rt_material_default(&d);
            hs->materials.resize(size_t(next_id), d);
        }
        for (int oid = id_begin; oid < next_id; ++oid) hs->materials[size_t(oid)] = obj.material;
        append_mesh(hs->mesh, tmp);
        hs->objects_loaded++;
    }
    return RT_OK;
}

}  // namespace

extern "C" int rt_host_scene_load_json(const char* scene_path, const char* project_dir, rt_host_scene** out) {
    if (!scene_path || !out) return set_error(RT_ERR_ARG, "rt_host_scene_load_json: null argument");
    *out = nullptr;
    std::ifstream f(scene_path);
    if (!f) return set_error(RT_ERR_IO, std::string("Failed to open scene file: ") + scene_path);
    std::stringstream buf;
    buf << f.rdbuf();
    const std::string text = buf.str();
    Json root;
    std::string err;
    if (!JsonReader(text).parse(root, err)) return set_error(RT_ERR_PARSE, "scene JSON: " + err);
    std::unique_ptr<rt_host_scene> hs(new (std::nothrow) rt_host_scene());
    if (!hs) return set_error(RT_ERR_NOMEM, "out of memory");
    int rc = parse_scene(root, hs->desc);
    if (rc != RT_OK) return rc;
    // main.cu:119-150
    const std::string base_dir = dirname_of(scene_path);
    const std::string proj = project_dir ? std::string(project_dir) : dirname_of(dirname_of(base_dir));
    std::vector<SceneObject> objs;
    for (const auto& o : hs->desc.objects) {
        if (!o.type.empty() && o.type != "mesh") continue;
        SceneObject r = o;
        if (!is_abs_path(r.path)) {
            const std::string scene_rel = join_path(base_dir, r.path);
            std::string proj_rel = r.path;
            if (proj_rel.rfind("./", 0) == 0) proj_rel = proj_rel.substr(2);
            proj_rel = join_path(proj, proj_rel);
            if (file_exists(scene_rel)) r.path = scene_rel;
            else if (file_exists(r.path)) { /* cwd-relative */ }
            else if (file_exists(proj_rel)) r.path = proj_rel;
            else r.path = scene_rel;
        }
        objs.push_back(r);
    }
    load_objects(hs.get(), objs);
    rc = finish_scene(hs.get());
    if (rc != RT_OK) return rc;
    *out = hs.release();
    clear_error();
    return RT_OK;
}

extern "C" int rt_host_scene_load_objs(const char* const* obj_paths, int n, rt_host_scene** out) {
    if (!obj_paths || n < 1 || !out) return set_error(RT_ERR_ARG, "rt_host_scene_load_objs: bad args");
    *out = nullptr;
    std::unique_ptr<rt_host_scene> hs(new (std::nothrow) rt_host_scene());
    if (!hs) return set_error(RT_ERR_NOMEM, "out of memory");
    std::vector<SceneObject> objs;
    for (int i = 0; i < n; ++i) {
        SceneObject o;
        o.path = obj_paths[i];
        objs.push_back(o);
    }
    load_objects(hs.get(), objs);
    int rc = finish_scene(hs.get());
    if (rc != RT_OK) return rc;
    *out = hs.release();
    return RT_OK;
}

extern "C" int rt_host_scene_info(const rt_host_scene* s, rt_scene_info* o) {
    if (!s || !o) return set_error(RT_ERR_ARG, "rt_host_scene_info: null argument");
    const SceneDesc& d = s->desc;
    o->max_depth = d.max_depth;
    o->spp = d.spp;
    o->diffuse_bounce = d.diffuse_bounce ? 1 : 0;
    o->miss_color = d.miss_color;
    o->cam_position = d.cam_pos;
    o->cam_look_at = d.cam_look;
    o->cam_up = d.cam_up;
    o->focal_length_mm = d.focal_mm;
    o->sensor_height_mm = d.sensor_mm;
    o->pixel_width = d.width;
    o->pixel_height = d.height;
    o->num_triangles = s->tris.size();
    o->num_vertices = s->mesh.positions.size();
    o->num_materials = int32_t(s->materials.size());
    o->num_lights = int32_t(s->lights.size());
    o->num_objects_loaded = s->objects_loaded;
    o->bvh_max_stack = s->max_stack;
    o->bvh_height = s->height;
    return RT_OK;
}

extern "C" int rt_host_scene_arrays(const rt_host_scene* s, rt_scene_arrays* o) {
    if (!s || !o) return set_error(RT_ERR_ARG, "rt_host_scene_arrays: null argument");
    o->nodes = s->nodes.data();
    o->aabbs = s->aabbs.data();
    o->triangles = s->tris.data();
    o->tri_object_ids = s->mesh.tri_obj_ids.data();
    o->materials = s->materials.data();
    o->lights = s->lights.data();
    o->positions = s->mesh.positions.data();
    o->normals = s->mesh.normals.empty() ? nullptr : s->mesh.normals.data();
    o->indices = s->mesh.indices.data();
    return RT_OK;
}

extern "C" void rt_host_scene_free(rt_host_scene* s) { delete s; }

// ---------------------------------------------------------------------------------------
// HW1 mesh
// ---------------------------------------------------------------------------------------
struct rt_mesh {
    Mesh m;
};

extern "C" int rt_mesh_load_obj_hw1(const char* path, rt_mesh** out) {
    if (!path || !out) return set_error(RT_ERR_ARG, "rt_mesh_load_obj_hw1: null argument");
    *out = nullptr;
    std::unique_ptr<rt_mesh> m(new (std::nothrow) rt_mesh());
    if (!m) return set_error(RT_ERR_NOMEM, "out of memory");
    int ids = 0;
    int rc = load_obj(path, m->m, ids, false);
    if (rc != RT_OK) return rc;
    *out = m.release();
    return RT_OK;
}

extern "C" int rt_mesh_view_get(const rt_mesh* m, rt_mesh_view* o) {
    if (!m || !o) return set_error(RT_ERR_ARG, "rt_mesh_view_get: null argument");
    o->positions = m->m.positions.data();
    o->normals = m->m.normals.empty() ? nullptr : m->m.normals.data();
    o->indices = m->m.indices.data();
    o->num_vertices = m->m.positions.size();
    o->num_triangles = m->m.indices.size() / 3;
    o->has_normals = m->m.has_normals();
    o->has_uvs = m->m.has_uvs();
    return RT_OK;
}

extern "C" void rt_mesh_free(rt_mesh* m) { delete m; }

// ---------------------------------------------------------------------------------------
// ppm_p6 (HW1/ppm_p6_lib/src/ppm_p6.cpp)
// ---------------------------------------------------------------------------------------
extern "C" void rt_ppm_options_default(rt_ppm_options* o) {
    o->maxval = 255;  // ppm_p6.hpp:46-51
    o->clamp = 1;
    o->gamma2 = 1;
    o->flip_y = 0;
}

namespace {
uint16_t float_to_sample(double linear, int maxval, bool clamp, bool gamma2) {  // ppm_p6.cpp:137-155
    if (gamma2) {
        if (linear < 0.0) linear = 0.0;
        linear = std::sqrt(linear);
    }
    if (clamp) {
        if (linear < 0.0) linear = 0.0;
        else if (linear > 1.0) linear = 1.0;
    }
    long r = std::lround(linear * double(maxval));
    if (r < 0) r = 0;
    if (r > maxval) r = maxval;
    return uint16_t(r);
}
}  // namespace

extern "C" int rt_ppm_encode(const float* rgb, int W, int H, const rt_ppm_options* opt,
                             uint8_t* buf, size_t cap, size_t* written) {
    rt_ppm_options d;
    rt_ppm_options_default(&d);
    if (!opt) opt = &d;
    if (!rgb || W <= 0 || H <= 0) return set_error(RT_ERR_ARG, "Image has non-positive dimensions.");
    if (opt->maxval <= 0 || opt->maxval > 65535) return set_error(RT_ERR_ARG, "Invalid maxval (must be 1..65535).");
    char header[64];
    const int hl = std::snprintf(header, sizeof(header), "P6\n%d %d\n%d\n", W, H, opt->maxval);
    const size_t bps = opt->maxval < 256 ? 1 : 2;
    const size_t need = size_t(hl) + size_t(W) * size_t(H) * 3 * bps;
    if (written) *written = need;
    if (!buf) return RT_OK;
    if (cap < need) return set_error(RT_ERR_ARG, "rt_ppm_encode: buffer too small");
    std::memcpy(buf, header, size_t(hl));
    uint8_t* p = buf + hl;
    for (int y = 0; y < H; ++y) {
        const int sy = opt->flip_y ? (H - 1 - y) : y;
        for (int x = 0; x < W; ++x)
            for (int c = 0; c < 3; ++c) {
                const uint16_t s = float_to_sample(double(rgb[(size_t(sy) * W + x) * 3 + c]), opt->maxval,
                                                   opt->clamp != 0, opt->gamma2 != 0);
                if (bps == 1) *p++ = uint8_t(s & 0xFF);
                else { *p++ = uint8_t(s >> 8); *p++ = uint8_t(s & 0xFF); }
            }
    }
    return RT_OK;
}

extern "C" int rt_ppm_write(const char* path, const float* rgb, int W, int H, const rt_ppm_options* opt) {
    if (!path) return set_error(RT_ERR_ARG, "rt_ppm_write: null path");
    size_t need = 0;
    int rc = rt_ppm_encode(rgb, W, H, opt, nullptr, 0, &need);
    if (rc != RT_OK) return rc;
    std::vector<uint8_t> buf(need);
    rc = rt_ppm_encode(rgb, W, H, opt, buf.data(), buf.size(), &need);
    if (rc != RT_OK) return rc;
    FILE* f = std::fopen(path, "wb");
    if (!f) return set_error(RT_ERR_IO, std::string("Failed to open output file: ") + path);
    const size_t w = std::fwrite(buf.data(), 1, need, f);
    const int cl = std::fclose(f);
    if (w != need || cl != 0) return set_error(RT_ERR_IO, "Failed while writing PPM");
    return RT_OK;
}

extern "C" int rt_ppm_read(const char* path, float* rgb_out, size_t cap_floats, int* width, int* height, int* maxval_out) {
    if (!path) return set_error(RT_ERR_ARG, "rt_ppm_read: null path");
    std::ifstream in(path, std::ios::binary);
    if (!in) return set_error(RT_ERR_IO, std::string("Failed to open input file: ") + path);
    auto is_ws = [](int ch) { return ch != EOF && std::isspace(static_cast<unsigned char>(ch)) != 0; };
    auto next_token = [&](std::string& tok) -> bool {  // ppm_p6.cpp:31-98
        for (;;) {
            const int p = in.peek();
            if (p == EOF) break;
            if (is_ws(p)) { in.get(); continue; }
            if (p == '#') { in.get(); in.ignore(std::numeric_limits<std::streamsize>::max(), '\n'); continue; }
            break;
        }
        tok.clear();
        for (;;) {
            const int p = in.peek();
            if (p == EOF || is_ws(p) || p == '#') break;
            tok.push_back(char(in.get()));
        }
        return !tok.empty();
    };
    auto to_int = [](const std::string& s, int& v) -> bool {
        try { v = std::stoi(s); return true; } catch (...) { return false; }
    };
    std::string tok;
    if (!next_token(tok) || tok != "P6") return set_error(RT_ERR_PARSE, "Unsupported magic number (expected P6)");
    int w = 0, h = 0, mv = 0;
    if (!next_token(tok) || !to_int(tok, w)) return set_error(RT_ERR_PARSE, "Invalid width token");
    if (!next_token(tok) || !to_int(tok, h)) return set_error(RT_ERR_PARSE, "Invalid height token");
    if (!next_token(tok) || !to_int(tok, mv)) return set_error(RT_ERR_PARSE, "Invalid maxval token");
    if (w <= 0 || h <= 0) return set_error(RT_ERR_PARSE, "Invalid image dimensions in header.");
    if (mv <= 0 || mv > 65535) return set_error(RT_ERR_PARSE, "Invalid maxval in header (must be 1..65535).");
    const int ws = in.get();
    if (ws == EOF || !is_ws(ws)) return set_error(RT_ERR_PARSE, "Expected whitespace after maxval");
    // The samples must all be there before the size is reported (a caller sizes its buffer by
    // it: a forged header of 99999 x 99999 on a short file is refused here, not allocated for).
    // The reference's reader fails the same file while reading the samples (ppm_p6.cpp:340-366).
    {
        const std::streampos at = in.tellg();
        in.seekg(0, std::ios::end);
        const std::streampos end = in.tellg();
        in.seekg(at);
        const unsigned long long need = (unsigned long long)w * (unsigned long long)h * 3ull * (mv < 256 ? 1ull : 2ull);
        if (at < 0 || end < at || (unsigned long long)(end - at) < need)
            return set_error(RT_ERR_PARSE, mv < 256 ? "Failed while reading 8-bit sample byte."
                                                    : "Failed while reading 16-bit sample bytes.");
    }
    if (width) *width = w;
    if (height) *height = h;
    if (maxval_out) *maxval_out = mv;
    if (!rgb_out) return RT_OK;
    if (cap_floats < size_t(w) * size_t(h) * 3) return set_error(RT_ERR_ARG, "rt_ppm_read: buffer too small");
    for (size_t i = 0; i < size_t(w) * size_t(h) * 3; ++i) {
        uint16_t s;
        if (mv < 256) {
            const int b = in.get();
            if (b == EOF) return set_error(RT_ERR_PARSE, "Failed while reading 8-bit sample byte.");
            s = uint16_t(b);
        } else {
            const int hi = in.get(), lo = in.get();
            if (hi == EOF || lo == EOF) return set_error(RT_ERR_PARSE, "Failed while reading 16-bit sample bytes.");
            s = uint16_t((hi << 8) | lo);
        }
        rgb_out[i] = float(double(s) / double(mv));
    }
    return RT_OK;
}
