// gltf.cpp -- host glTF (embedded/ASCII) scene loader behind tpt_gltf_load.
//
// Semantics of Scene::readFromGLTF (src/mesh.cu:80-307) and
// Scene::copySceneToDevice (src/mesh.cu:309-397): node walk order, tinygltf
// defaults (metallic = roughness = 1, baseColor = 1), std::map (byte-wise name)
// order for materials and lights, LUT of first faces, T*R*S object matrices and
// normal matrices transpose(M3)^-1 through the reference's Mat4::inverse
// cofactor formula (include/math/mat.h:203-282), all in fp32 with the
// reference's rounding order.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "json_lite.hpp"
#include "tpt.h"
#include "tpt_internal.hpp"

namespace tpt {
namespace {

using M4 = std::array<std::array<float, 4>, 4>;   // [column][row]

M4 identity() {
    M4 m{};
    for (int i = 0; i < 4; ++i) m[i][i] = 1.0f;
    return m;
}

// MatrixMultiply (mat.h:17-35): res[j][i] = sum_k lhs[k][i] * rhs[j][k] from 0
M4 mul(const M4& l, const M4& r) {
    M4 o{};
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            float acc = 0.0f;
            for (int k = 0; k < 4; ++k) acc += l[k][i] * r[j][k];
            o[j][i] = acc;
        }
    return o;
}

void mul_vec(const M4& m, const float v[4], float out[4]) {
    for (int i = 0; i < 4; ++i) {
        float acc = 0.0f;
        for (int j = 0; j < 4; ++j) acc += m[j][i] * v[j];
        out[i] = acc;
    }
}

M4 transpose(const M4& m) {
    M4 o{};
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) o[j][i] = m[i][j];
    return o;
}

// One signed product chain: sign, then (col,row) pairs.  Terms accumulate left
// to right exactly like the reference's long expressions.
struct Term3 { int8_t s; uint8_t a, b, c; };      // indices packed col*4+row
struct Term4 { int8_t s; uint8_t a, b, c, d; };

#define CR(c, r) (uint8_t)((c) * 4 + (r))
// Mat4::determinant (mat.h:203-228)
const Term4 kDet[24] = {
    {+1, CR(0,3), CR(1,2), CR(2,1), CR(3,0)}, {-1, CR(0,2), CR(1,3), CR(2,1), CR(3,0)},
    {-1, CR(0,3), CR(1,1), CR(2,2), CR(3,0)}, {+1, CR(0,1), CR(1,3), CR(2,2), CR(3,0)},
    {+1, CR(0,2), CR(1,1), CR(2,3), CR(3,0)}, {-1, CR(0,1), CR(1,2), CR(2,3), CR(3,0)},
    {-1, CR(0,3), CR(1,2), CR(2,0), CR(3,1)}, {+1, CR(0,2), CR(1,3), CR(2,0), CR(3,1)},
    {+1, CR(0,3), CR(1,0), CR(2,2), CR(3,1)}, {-1, CR(0,0), CR(1,3), CR(2,2), CR(3,1)},
    {-1, CR(0,2), CR(1,0), CR(2,3), CR(3,1)}, {+1, CR(0,0), CR(1,2), CR(2,3), CR(3,1)},
    {+1, CR(0,3), CR(1,1), CR(2,0), CR(3,2)}, {-1, CR(0,1), CR(1,3), CR(2,0), CR(3,2)},
    {-1, CR(0,3), CR(1,0), CR(2,1), CR(3,2)}, {+1, CR(0,0), CR(1,3), CR(2,1), CR(3,2)},
    {+1, CR(0,1), CR(1,0), CR(2,3), CR(3,2)}, {-1, CR(0,0), CR(1,1), CR(2,3), CR(3,2)},
    {-1, CR(0,2), CR(1,1), CR(2,0), CR(3,3)}, {+1, CR(0,1), CR(1,2), CR(2,0), CR(3,3)},
    {+1, CR(0,2), CR(1,0), CR(2,1), CR(3,3)}, {-1, CR(0,0), CR(1,2), CR(2,1), CR(3,3)},
    {-1, CR(0,1), CR(1,0), CR(2,2), CR(3,3)}, {+1, CR(0,0), CR(1,1), CR(2,2), CR(3,3)},
};
// Mat4::inverse (mat.h:229-282): entry r[col][row] = six signed triple products.
struct InvEntry { uint8_t col, row; Term3 t[6]; };
const InvEntry kInv[16] = {
    {0, 0, {{+1, CR(1,2), CR(2,3), CR(3,1)}, {-1, CR(1,3), CR(2,2), CR(3,1)}, {+1, CR(1,3), CR(2,1), CR(3,2)},
            {-1, CR(1,1), CR(2,3), CR(3,2)}, {-1, CR(1,2), CR(2,1), CR(3,3)}, {+1, CR(1,1), CR(2,2), CR(3,3)}}},
    {0, 1, {{+1, CR(0,3), CR(2,2), CR(3,1)}, {-1, CR(0,2), CR(2,3), CR(3,1)}, {-1, CR(0,3), CR(2,1), CR(3,2)},
            {+1, CR(0,1), CR(2,3), CR(3,2)}, {+1, CR(0,2), CR(2,1), CR(3,3)}, {-1, CR(0,1), CR(2,2), CR(3,3)}}},
    {0, 2, {{+1, CR(0,2), CR(1,3), CR(3,1)}, {-1, CR(0,3), CR(1,2), CR(3,1)}, {+1, CR(0,3), CR(1,1), CR(3,2)},
            {-1, CR(0,1), CR(1,3), CR(3,2)}, {-1, CR(0,2), CR(1,1), CR(3,3)}, {+1, CR(0,1), CR(1,2), CR(3,3)}}},
    {0, 3, {{+1, CR(0,3), CR(1,2), CR(2,1)}, {-1, CR(0,2), CR(1,3), CR(2,1)}, {-1, CR(0,3), CR(1,1), CR(2,2)},
            {+1, CR(0,1), CR(1,3), CR(2,2)}, {+1, CR(0,2), CR(1,1), CR(2,3)}, {-1, CR(0,1), CR(1,2), CR(2,3)}}},
    {1, 0, {{+1, CR(1,3), CR(2,2), CR(3,0)}, {-1, CR(1,2), CR(2,3), CR(3,0)}, {-1, CR(1,3), CR(2,0), CR(3,2)},
            {+1, CR(1,0), CR(2,3), CR(3,2)}, {+1, CR(1,2), CR(2,0), CR(3,3)}, {-1, CR(1,0), CR(2,2), CR(3,3)}}},
    {1, 1, {{+1, CR(0,2), CR(2,3), CR(3,0)}, {-1, CR(0,3), CR(2,2), CR(3,0)}, {+1, CR(0,3), CR(2,0), CR(3,2)},
            {-1, CR(0,0), CR(2,3), CR(3,2)}, {-1, CR(0,2), CR(2,0), CR(3,3)}, {+1, CR(0,0), CR(2,2), CR(3,3)}}},
    {1, 2, {{+1, CR(0,3), CR(1,2), CR(3,0)}, {-1, CR(0,2), CR(1,3), CR(3,0)}, {-1, CR(0,3), CR(1,0), CR(3,2)},
            {+1, CR(0,0), CR(1,3), CR(3,2)}, {+1, CR(0,2), CR(1,0), CR(3,3)}, {-1, CR(0,0), CR(1,2), CR(3,3)}}},
    {1, 3, {{+1, CR(0,2), CR(1,3), CR(2,0)}, {-1, CR(0,3), CR(1,2), CR(2,0)}, {+1, CR(0,3), CR(1,0), CR(2,2)},
            {-1, CR(0,0), CR(1,3), CR(2,2)}, {-1, CR(0,2), CR(1,0), CR(2,3)}, {+1, CR(0,0), CR(1,2), CR(2,3)}}},
    {2, 0, {{+1, CR(1,1), CR(2,3), CR(3,0)}, {-1, CR(1,3), CR(2,1), CR(3,0)}, {+1, CR(1,3), CR(2,0), CR(3,1)},
            {-1, CR(1,0), CR(2,3), CR(3,1)}, {-1, CR(1,1), CR(2,0), CR(3,3)}, {+1, CR(1,0), CR(2,1), CR(3,3)}}},
    {2, 1, {{+1, CR(0,3), CR(2,1), CR(3,0)}, {-1, CR(0,1), CR(2,3), CR(3,0)}, {-1, CR(0,3), CR(2,0), CR(3,1)},
            {+1, CR(0,0), CR(2,3), CR(3,1)}, {+1, CR(0,1), CR(2,0), CR(3,3)}, {-1, CR(0,0), CR(2,1), CR(3,3)}}},
    {2, 2, {{+1, CR(0,1), CR(1,3), CR(3,0)}, {-1, CR(0,3), CR(1,1), CR(3,0)}, {+1, CR(0,3), CR(1,0), CR(3,1)},
            {-1, CR(0,0), CR(1,3), CR(3,1)}, {-1, CR(0,1), CR(1,0), CR(3,3)}, {+1, CR(0,0), CR(1,1), CR(3,3)}}},
    {2, 3, {{+1, CR(0,3), CR(1,1), CR(2,0)}, {-1, CR(0,1), CR(1,3), CR(2,0)}, {-1, CR(0,3), CR(1,0), CR(2,1)},
            {+1, CR(0,0), CR(1,3), CR(2,1)}, {+1, CR(0,1), CR(1,0), CR(2,3)}, {-1, CR(0,0), CR(1,1), CR(2,3)}}},
    {3, 0, {{+1, CR(1,2), CR(2,1), CR(3,0)}, {-1, CR(1,1), CR(2,2), CR(3,0)}, {-1, CR(1,2), CR(2,0), CR(3,1)},
            {+1, CR(1,0), CR(2,2), CR(3,1)}, {+1, CR(1,1), CR(2,0), CR(3,2)}, {-1, CR(1,0), CR(2,1), CR(3,2)}}},
    {3, 1, {{+1, CR(0,1), CR(2,2), CR(3,0)}, {-1, CR(0,2), CR(2,1), CR(3,0)}, {+1, CR(0,2), CR(2,0), CR(3,1)},
            {-1, CR(0,0), CR(2,2), CR(3,1)}, {-1, CR(0,1), CR(2,0), CR(3,2)}, {+1, CR(0,0), CR(2,1), CR(3,2)}}},
    {3, 2, {{+1, CR(0,2), CR(1,1), CR(3,0)}, {-1, CR(0,1), CR(1,2), CR(3,0)}, {-1, CR(0,2), CR(1,0), CR(3,1)},
            {+1, CR(0,0), CR(1,2), CR(3,1)}, {+1, CR(0,1), CR(1,0), CR(3,2)}, {-1, CR(0,0), CR(1,1), CR(3,2)}}},
    {3, 3, {{+1, CR(0,1), CR(1,2), CR(2,0)}, {-1, CR(0,2), CR(1,1), CR(2,0)}, {+1, CR(0,2), CR(1,0), CR(2,1)},
            {-1, CR(0,0), CR(1,2), CR(2,1)}, {-1, CR(0,1), CR(1,0), CR(2,2)}, {+1, CR(0,0), CR(1,1), CR(2,2)}}},
};
#undef CR

inline float at(const M4& m, uint8_t cr) { return m[cr >> 2][cr & 3]; }

float determinant(const M4& m) {
    float acc = 0.0f;
    for (int t = 0; t < 24; ++t) {
        const Term4& x = kDet[t];
        float p = at(m, x.a) * at(m, x.b) * at(m, x.c) * at(m, x.d);
        acc = (t == 0) ? (x.s > 0 ? p : -p) : (x.s > 0 ? acc + p : acc - p);
    }
    return acc;
}

M4 inverse(const M4& m) {
    M4 r{};
    for (const InvEntry& e : kInv) {
        float acc = 0.0f;
        for (int t = 0; t < 6; ++t) {
            const Term3& x = e.t[t];
            float p = at(m, x.a) * at(m, x.b) * at(m, x.c);
            acc = (t == 0) ? (x.s > 0 ? p : -p) : (x.s > 0 ? acc + p : acc - p);
        }
        r[e.col][e.row] = acc;
    }
    float s = 1.0f / determinant(m);
    for (auto& c : r)
        for (auto& v : c) v = v * s;
    return r;
}

// Quat::RotateFromQuat (quat.h:52-69) embedded by Mat4(const Mat3&) (mat.h:175)
M4 rotation(float w, float x, float y, float z) {
    float x2 = x * x, y2 = y * y, z2 = z * z;
    float xy = x * y, xz = x * z, yz = y * z;
    float wx = w * x, wy = w * y, wz = w * z;
    M4 m = identity();
    m[0][0] = 1.0f - 2.0f * (y2 + z2); m[0][1] = 2.0f * (xy + wz);        m[0][2] = 2.0f * (xz - wy);
    m[1][0] = 2.0f * (xy - wz);        m[1][1] = 1.0f - 2.0f * (x2 + z2); m[1][2] = 2.0f * (yz + wx);
    m[2][0] = 2.0f * (xz + wy);        m[2][1] = 2.0f * (yz - wx);        m[2][2] = 1.0f - 2.0f * (x2 + y2);
    return m;
}

struct TRS {
    float t[3] = {0.0f, 0.0f, 0.0f};
    float q[4] = {0.0f, 0.0f, 0.0f, 0.0f};   // w, x, y, z; Quat() == 0 (quat.h:10)
    float s[3] = {1.0f, 1.0f, 1.0f};
};

// readTransform (mesh.cu:102-138)
TRS read_trs(const json::Value& node) {
    TRS r;
    if (const json::Value* q = node.find("rotation"); q && q->size() == 4) {
        r.q[0] = (float)(*q)[3].num; r.q[1] = (float)(*q)[0].num;
        r.q[2] = (float)(*q)[1].num; r.q[3] = (float)(*q)[2].num;
    }
    if (const json::Value* s = node.find("scale"); s && s->size() == 3)
        for (int i = 0; i < 3; ++i) r.s[i] = (float)(*s)[i].num;
    if (const json::Value* t = node.find("translation"); t && t->size() == 3)
        for (int i = 0; i < 3; ++i) r.t[i] = (float)(*t)[i].num;
    return r;
}

// Transform::localToParent (transform.h:28-33): (T * R) * S
M4 local_to_world(const TRS& x) {
    M4 t = identity();
    t[3] = {x.t[0], x.t[1], x.t[2], 1.0f};
    M4 s = identity();
    s[0][0] = x.s[0]; s[1][1] = x.s[1]; s[2][2] = x.s[2];
    return mul(mul(t, rotation(x.q[0], x.q[1], x.q[2], x.q[3])), s);
}

// normal_to_world lambda (mesh.cu:370-378)
M4 normal_to_world(const M4& l2w) {
    M4 m{};
    for (int c = 0; c < 3; ++c) m[c] = {l2w[c][0], l2w[c][1], l2w[c][2], 0.0f};
    m[3] = {0.0f, 0.0f, 0.0f, 1.0f};
    return inverse(transpose(m));
}

void flatten(const M4& m, float* out) {
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r) out[4 * c + r] = m[c][r];
}

std::vector<uint8_t> b64decode(const std::string& s) {
    auto val = [](char c) -> int {
        if (c >= 'A' && c <= 'Z') return c - 'A';
        if (c >= 'a' && c <= 'z') return c - 'a' + 26;
        if (c >= '0' && c <= '9') return c - '0' + 52;
        if (c == '+' || c == '-') return 62;
        if (c == '/' || c == '_') return 63;
        return -1;
    };
    std::vector<uint8_t> out;
    out.reserve(s.size() * 3 / 4);
    uint32_t acc = 0;
    int bits = 0;
    for (char c : s) {
        int v = val(c);
        if (v < 0) continue;   // '=', whitespace
        acc = (acc << 6) | (uint32_t)v;
        bits += 6;
        if (bits >= 8) {
            bits -= 8;
            out.push_back((uint8_t)((acc >> bits) & 0xFF));
        }
    }
    return out;
}

std::string read_file(const std::string& path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw io_error("cannot open " + path);
    std::ostringstream ss;
    ss << f.rdbuf();
    return ss.str();
}

struct MeshData {
    std::vector<float> pos, nrm;
    std::vector<uint32_t> ind;
    std::string material;
    M4 l2w;
};

}  // namespace

// Accessor view (tightly packed; the reference ignores byteStride, mesh.cu:165-222)
static const uint8_t* accessor_ptr(const json::Value& model, const std::vector<std::vector<uint8_t>>& bufs,
                                   long long acc_idx, long long* count, long long* ctype, int* ncomp) {
    const json::Value* accs = model.find("accessors");
    const json::Value* views = model.find("bufferViews");
    if (!accs || !views || acc_idx < 0 || (size_t)acc_idx >= accs->size()) throw parse_error("bad accessor index");
    const json::Value& a = (*accs)[(size_t)acc_idx];
    long long bv = a.int_or("bufferView", -1);
    if (bv < 0 || (size_t)bv >= views->size()) throw parse_error("accessor without bufferView");
    const json::Value& v = (*views)[(size_t)bv];
    long long b = v.int_or("buffer", 0);
    if (b < 0 || (size_t)b >= bufs.size()) throw parse_error("bad buffer index");
    const long long aoff = a.int_or("byteOffset", 0), voff = v.int_or("byteOffset", 0);
    *count = a.int_or("count", 0);
    *ctype = a.int_or("componentType", 0);
    std::string type = a.string_or("type", "SCALAR");
    *ncomp = type == "VEC2" ? 2 : type == "VEC3" ? 3 : type == "VEC4" ? 4 : 1;
    size_t csize = (*ctype == 5120 || *ctype == 5121) ? 1 : (*ctype == 5122 || *ctype == 5123) ? 2 : 4;
    // untrusted offsets and counts: non-negative, and off + count * ncomp * csize
    // within the buffer without overflowing
    const size_t size = bufs[(size_t)b].size();
    if (aoff < 0 || voff < 0 || *count < 0) throw parse_error("negative accessor offset or count");
    if ((unsigned long long)aoff > size || (unsigned long long)voff > size - (size_t)aoff)
        throw parse_error("accessor exceeds buffer");
    const size_t off = (size_t)aoff + (size_t)voff;
    const size_t elem = (size_t)(*ncomp) * csize;
    if ((unsigned long long)*count > (size - off) / elem) throw parse_error("accessor exceeds buffer");
    return bufs[(size_t)b].data() + off;
}

static std::vector<float> read_vec3(const json::Value& model, const std::vector<std::vector<uint8_t>>& bufs,
                                    long long acc) {
    long long count, ctype;
    int ncomp;
    const uint8_t* p = accessor_ptr(model, bufs, acc, &count, &ctype, &ncomp);
    if (ctype != 5126 || ncomp != 3) throw parse_error("expected float VEC3 accessor");
    std::vector<float> out((size_t)count * 3);
    if (!out.empty()) std::memcpy(out.data(), p, out.size() * 4);
    return out;
}

static std::vector<uint32_t> read_indices(const json::Value& model, const std::vector<std::vector<uint8_t>>& bufs,
                                          long long acc) {
    long long count, ctype;
    int ncomp;
    const uint8_t* p = accessor_ptr(model, bufs, acc, &count, &ctype, &ncomp);
    std::vector<uint32_t> out((size_t)count);
    for (long long i = 0; i < count; ++i) {   // static_cast<uint32_t>(ptr[i]) (mesh.cuh:44-52)
        switch (ctype) {
            case 5120: { int8_t v; std::memcpy(&v, p + i, 1); out[i] = (uint32_t)(int32_t)v; break; }
            case 5121: out[i] = p[i]; break;
            case 5122: { int16_t v; std::memcpy(&v, p + 2 * i, 2); out[i] = (uint32_t)(int32_t)v; break; }
            case 5123: { uint16_t v; std::memcpy(&v, p + 2 * i, 2); out[i] = v; break; }
            case 5124: { int32_t v; std::memcpy(&v, p + 4 * i, 4); out[i] = (uint32_t)v; break; }
            case 5125: { uint32_t v; std::memcpy(&v, p + 4 * i, 4); out[i] = v; break; }
            default: throw parse_error("unsupported index component type");
        }
    }
    return out;
}

void load_gltf(const std::string& path, HostScene& hs) {
    json::Value model = json::parse(read_file(path));
    std::string dir;
    if (size_t k = path.find_last_of('/'); k != std::string::npos) dir = path.substr(0, k + 1);

    std::vector<std::vector<uint8_t>> bufs;
    if (const json::Value* b = model.find("buffers")) {
        for (const auto& buf : b->arr) {
            std::string uri = buf.string_or("uri", "");
            if (uri.rfind("data:", 0) == 0) {
                size_t comma = uri.find(',');
                bufs.push_back(b64decode(comma == std::string::npos ? "" : uri.substr(comma + 1)));
            } else {
                std::string raw = read_file(dir + uri);
                bufs.emplace_back(raw.begin(), raw.end());
            }
        }
    }

    std::vector<MeshData> meshes;
    std::map<std::string, tpt_material> materials;   // std::map order (mesh.cuh:113)
    std::map<std::string, tpt_light> lights;
    bool have_cam = false;
    const json::Value* mats = model.find("materials");
    const json::Value* nodes = model.find("nodes");
    hs.missing_material = false;

    for (size_t ni = 0; nodes && ni < nodes->size(); ++ni) {
        const json::Value& node = (*nodes)[ni];
        long long cam = node.int_or("camera", -1), mesh = node.int_or("mesh", -1);
        if (cam > -1) {
            const json::Value* cams = model.find("cameras");
            if (!cams || (size_t)cam >= cams->size()) throw parse_error("bad camera index");
            const json::Value& ci = (*cams)[(size_t)cam];
            if (ci.string_or("type", "") == "perspective") {
                const json::Value* p = ci.find("perspective");
                json::Value empty;
                empty.kind = json::Value::Object;
                if (!p) p = &empty;
                flatten(local_to_world(read_trs(node)), hs.camera.c2w);
                hs.camera.vfov = (float)p->number_or("yfov", 0.0);
                hs.camera.aspect = (float)p->number_or("aspectRatio", 0.0);
                hs.camera.znear = (float)p->number_or("znear", 0.0);
                have_cam = true;
            }
        } else if (mesh > -1) {
            const json::Value* ms = model.find("meshes");
            if (!ms || (size_t)mesh >= ms->size()) throw parse_error("bad mesh index");
            const json::Value* prims = (*ms)[(size_t)mesh].find("primitives");
            if (!prims || prims->size() == 0) throw parse_error("mesh without primitives");
            const json::Value& prim = (*prims)[0];            // only primitives[0] (App. A.10)
            const json::Value* attrs = prim.find("attributes");
            if (!attrs) throw parse_error("primitive without attributes");
            MeshData md;
            md.pos = read_vec3(model, bufs, attrs->int_or("POSITION", -1));
            md.ind = read_indices(model, bufs, prim.int_or("indices", -1));
            md.nrm = read_vec3(model, bufs, attrs->int_or("NORMAL", -1));
            if (md.nrm.size() != md.pos.size()) throw parse_error("NORMAL count != POSITION count");
            if (md.ind.size() % 3) throw parse_error("index count not a multiple of 3");
            if (mats && mats->size() > 0) {
                long long mi = prim.int_or("material", -1);
                if (mi < 0 || (size_t)mi >= mats->size()) {
                    hs.missing_material = true;                // reference: materials[-1] (UB)
                } else {
                    const json::Value& m = (*mats)[(size_t)mi];
                    md.material = m.string_or("name", "");
                    if (!materials.count(md.material)) {
                        tpt_material cm = default_material();
                        const json::Value* pbr = m.find("pbrMetallicRoughness");
                        json::Value empty;
                        empty.kind = json::Value::Object;
                        if (!pbr) pbr = &empty;
                        cm.roughness = (float)pbr->number_or("roughnessFactor", 1.0);
                        cm.metallic = (float)pbr->number_or("metallicFactor", 1.0);
                        const json::Value* bc = pbr->find("baseColorFactor");
                        if (bc && bc->size() == 4) {
                            for (int c = 0; c < 3; ++c) cm.base_color[c] = (float)(*bc)[(size_t)c].num;
                        } else {
                            cm.base_color[0] = cm.base_color[1] = cm.base_color[2] = 1.0f;
                        }
                        if (const json::Value* ext = m.find("extensions")) {
                            for (const auto& kv : ext->obj) {
                                if (kv.first == "KHR_materials_transmission")
                                    cm.specular = 1.0f - (float)kv.second.number_or("transmissionFactor", 0.0) / 5.0f;
                                if (kv.first == "KHR_materials_emissive_strength")
                                    cm.emission_factor = (float)kv.second.number_or("emissiveStrength", 0.0);
                                if (kv.first == "KHR_materials_ior")
                                    cm.eta = (float)kv.second.number_or("ior", 0.0);
                            }
                        }
                        materials[md.material] = cm;
                    }
                }
            } else {
                hs.missing_material = true;
            }
            md.l2w = local_to_world(read_trs(node));
            meshes.push_back(std::move(md));
        } else {
            const json::Value* ext = node.find("extensions");
            const json::Value* lp = ext ? ext->find("KHR_lights_punctual") : nullptr;
            if (!lp) continue;
            long long li = lp->int_or("light", -1);
            const json::Value* mext = model.find("extensions");
            const json::Value* mlp = mext ? mext->find("KHR_lights_punctual") : nullptr;
            const json::Value* ll = mlp ? mlp->find("lights") : nullptr;
            if (!ll || li < 0 || (size_t)li >= ll->size()) throw parse_error("bad light index");
            const json::Value& L = (*ll)[(size_t)li];
            M4 m = local_to_world(read_trs(node));
            tpt_light out{};
            const json::Value* col = L.find("color");
            for (int c = 0; c < 3; ++c) out.color[c] = (col && col->size() == 3) ? (float)(*col)[(size_t)c].num : 1.0f;
            std::string type = L.string_or("type", "");
            const float wpl = 1.0f / 683.0f;                    // WATTS_PER_LUMEN (delta_light.h:6)
            const float org[4] = {0.0f, 0.0f, 0.0f, 1.0f}, fwd[4] = {0.0f, 0.0f, -1.0f, 0.0f};
            float v[4];
            if (type == "point") {
                out.type = 0;
                out.intensity = (float)L.number_or("intensity", 1.0) * wpl;
                mul_vec(m, org, v);
                out.pos[0] = v[0]; out.pos[1] = v[1]; out.pos[2] = v[2];
            } else if (type == "directional") {
                out.type = 1;
                out.intensity = (float)L.number_or("intensity", 1.0);
                mul_vec(m, fwd, v);
                out.direction[0] = v[0]; out.direction[1] = v[1]; out.direction[2] = v[2];
            } else if (type == "spot") {
                out.type = 2;
                out.intensity = (float)L.number_or("intensity", 1.0) * wpl;
                const json::Value* sp = L.find("spot");
                float inner = sp ? (float)sp->number_or("innerConeAngle", 0.0) : 0.0f;
                float outer = sp ? (float)sp->number_or("outerConeAngle", 0.7853981634) : (float)0.7853981634;
                float co = (float)std::cos((double)outer), ci = (float)std::cos((double)inner);
                out.cos_outer = co;
                out.inv_cos_cone_diff = 1.0f / (ci - co);
                mul_vec(m, fwd, v);
                out.direction[0] = v[0]; out.direction[1] = v[1]; out.direction[2] = v[2];
                mul_vec(m, org, v);
                out.pos[0] = v[0]; out.pos[1] = v[1]; out.pos[2] = v[2];
            } else {
                throw parse_error("Unsupported light type");
            }
            lights[node.string_or("name", "")] = out;
        }
    }
    if (!have_cam) {   // Camera() (camera.h:11-14)
        flatten(identity(), hs.camera.c2w);
        hs.camera.vfov = 60.0f;
        hs.camera.aspect = 1.77778f;
        hs.camera.znear = 0.1f;
    }
    if (meshes.empty()) throw parse_error("scene has no meshes");

    // copySceneToDevice (mesh.cu:309-397)
    std::map<std::string, int32_t> mat_index;
    hs.materials.clear();
    for (const auto& kv : materials) {
        mat_index[kv.first] = (int32_t)hs.materials.size();
        hs.materials.push_back(kv.second);
    }
    if (materials.empty()) hs.missing_material = true;
    hs.indices.clear(); hs.vertices.clear(); hs.normals.clear(); hs.lut.clear();
    hs.vert_trans.clear(); hs.normal_trans.clear();
    uint32_t icount = 0, vcount = 0;
    for (const MeshData& md : meshes) {
        for (uint32_t id : md.ind) hs.indices.push_back(id + vcount);
        hs.vertices.insert(hs.vertices.end(), md.pos.begin(), md.pos.end());
        hs.normals.insert(hs.normals.end(), md.nrm.begin(), md.nrm.end());
        auto it = mat_index.find(md.material);
        hs.lut.push_back(tpt_interval{(int32_t)(icount / 3), it == mat_index.end() ? 0 : it->second});
        icount += (uint32_t)md.ind.size();
        vcount += (uint32_t)(md.pos.size() / 3);
        float f[16];
        flatten(md.l2w, f);
        hs.vert_trans.insert(hs.vert_trans.end(), f, f + 16);
        flatten(normal_to_world(md.l2w), f);
        hs.normal_trans.insert(hs.normal_trans.end(), f, f + 16);
    }
    hs.lights.clear();
    for (const auto& kv : lights) hs.lights.push_back(kv.second);
    for (uint32_t id : hs.indices)
        if (id >= vcount) throw parse_error("vertex index out of range");
}

}  // namespace tpt
