// MagicaVoxel .vox import: BoxTree::load_vox_file (src/convert/magicavoxel.rs:234-374) over a from-scratch reader
// of the .vox chunk format.
//
// The reference reads files with the `dot_vox = "5.1.1"` crate (Cargo.toml:24), which is not vendored. This file
// restates the part of its data model the reference uses: models in SIZE/XYZI order, the 256-entry RGBA palette with
// a voxel's colour index = file index - 1 (saturating), and the scene graph nodes nTRN (attributes, child, frames
// with "_t"/"_r"), nGRP (children) and nSHP (models with "_f"), stored in file order and referenced by position.
// Other chunks (MATL, LAYR, rOBJ, rCAM, NOTE, IMAP, PACK) are skipped. Files without an RGBA chunk (dot_vox would
// substitute MagicaVoxel's default palette) or without a scene graph (the reference panics on `scenes[0]`) are
// rejected with VHX_E_VOX_FORMAT.
#include <algorithm>
#include <array>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

#include "../../include/vhx_boxtree.h"
#include "boxtree.hpp"

namespace {

using Dict = std::vector<std::pair<std::string, std::string>>;

const std::string *dict_get(const Dict &d, const char *key) {
    for (const auto &kv : d)
        if (kv.first == key) return &kv.second;
    return nullptr;
}

struct VoxModel {
    int32_t sx = 0, sy = 0, sz = 0;
    std::vector<std::array<uint8_t, 4>> voxels;  // x, y, z, colour index (already file index - 1)
};

struct SceneNode {
    enum Kind { Transform, Group, Shape } kind = Transform;
    uint32_t child = 0;                          // Transform
    std::vector<Dict> frames;                    // Transform
    std::vector<uint32_t> children;              // Group
    std::vector<std::pair<uint32_t, Dict>> models;  // Shape: model id + attributes
};

struct VoxData {
    std::vector<VoxModel> models;
    std::array<uint32_t, 256> palette{};  // r | g << 8 | b << 16 | a << 24
    bool has_palette = false;
    std::vector<SceneNode> scenes;
};

struct Reader {
    const uint8_t *p, *end;
    bool ok = true;
    bool need(size_t n) {
        if ((size_t)(end - p) < n) ok = false;
        return ok;
    }
    int32_t i32() {
        if (!need(4)) return 0;
        int32_t v;
        std::memcpy(&v, p, 4);
        p += 4;
        return v;
    }
    std::string str() {
        const int32_t n = i32();
        if (n < 0 || !need((size_t)n)) {
            ok = false;
            return {};
        }
        std::string s((const char *)p, (size_t)n);
        p += n;
        return s;
    }
    Dict dict() {
        Dict d;
        const int32_t n = i32();
        if (n < 0 || n > (1 << 20)) {
            ok = false;
            return d;
        }
        for (int32_t k = 0; k < n && ok; ++k) {
            std::string key = str();
            std::string val = str();
            d.emplace_back(std::move(key), std::move(val));
        }
        return d;
    }
};

bool parse(const uint8_t *data, size_t size, VoxData &out) {
    if (size < 8 || std::memcmp(data, "VOX ", 4) != 0) return false;
    Reader top{data + 8, data + size};
    // MAIN chunk: id, content bytes, children bytes
    if (!top.need(12) || std::memcmp(top.p, "MAIN", 4) != 0) return false;
    top.p += 4;
    const int32_t main_content = top.i32(), main_children = top.i32();
    if (!top.ok || main_content < 0 || main_children < 0 || !top.need((size_t)main_content + (size_t)main_children))
        return false;
    const uint8_t *c = top.p + main_content, *cend = c + main_children;
    int32_t pending_sx = -1, pending_sy = 0, pending_sz = 0;
    while (c < cend) {
        if (cend - c < 12) return false;
        char id[5] = {0};
        std::memcpy(id, c, 4);
        int32_t n, m;
        std::memcpy(&n, c + 4, 4);
        std::memcpy(&m, c + 8, 4);
        if (n < 0 || m < 0 || (size_t)(cend - c - 12) < (size_t)n + (size_t)m) return false;
        Reader r{c + 12, c + 12 + n};
        const std::string cid(id);
        if (cid == "SIZE") {
            pending_sx = r.i32();
            pending_sy = r.i32();
            pending_sz = r.i32();
        } else if (cid == "XYZI") {
            if (pending_sx < 0) return false;
            VoxModel mdl;
            mdl.sx = pending_sx;
            mdl.sy = pending_sy;
            mdl.sz = pending_sz;
            pending_sx = -1;
            const int32_t nv = r.i32();
            if (nv < 0 || !r.need((size_t)nv * 4)) return false;
            mdl.voxels.resize((size_t)nv);
            for (int32_t k = 0; k < nv; ++k) {
                const uint8_t *v = r.p + 4 * (size_t)k;
                mdl.voxels[(size_t)k] = {v[0], v[1], v[2], (uint8_t)(v[3] > 0 ? v[3] - 1 : 0)};
            }
            out.models.push_back(std::move(mdl));
        } else if (cid == "RGBA") {
            if (!r.need(256 * 4)) return false;
            for (int k = 0; k < 256; ++k) {
                const uint8_t *q = r.p + 4 * k;
                out.palette[(size_t)k] = (uint32_t)q[0] | ((uint32_t)q[1] << 8) | ((uint32_t)q[2] << 16) |
                                         ((uint32_t)q[3] << 24);
            }
            out.has_palette = true;
        } else if (cid == "nTRN") {
            SceneNode s;
            s.kind = SceneNode::Transform;
            r.i32();  // node id
            r.dict();
            s.child = (uint32_t)r.i32();
            r.i32();  // reserved
            r.i32();  // layer id
            const int32_t nf = r.i32();
            if (nf < 0 || nf > (1 << 16)) return false;
            for (int32_t k = 0; k < nf && r.ok; ++k) s.frames.push_back(r.dict());
            if (!r.ok) return false;
            out.scenes.push_back(std::move(s));
        } else if (cid == "nGRP") {
            SceneNode s;
            s.kind = SceneNode::Group;
            r.i32();
            r.dict();
            const int32_t nc = r.i32();
            if (nc < 0 || !r.need((size_t)nc * 4)) return false;
            for (int32_t k = 0; k < nc; ++k) s.children.push_back((uint32_t)r.i32());
            out.scenes.push_back(std::move(s));
        } else if (cid == "nSHP") {
            SceneNode s;
            s.kind = SceneNode::Shape;
            r.i32();
            r.dict();
            const int32_t nm = r.i32();
            if (nm < 0 || nm > (1 << 20)) return false;
            for (int32_t k = 0; k < nm && r.ok; ++k) {
                const uint32_t mid = (uint32_t)r.i32();
                s.models.emplace_back(mid, r.dict());
            }
            if (!r.ok) return false;
            out.scenes.push_back(std::move(s));
        }
        if (!r.ok) return false;
        c += 12 + (size_t)n + (size_t)m;
    }
    return true;
}

// nalgebra Matrix3<i8>, row-major here: m[r][c]
using Mat3 = std::array<std::array<int32_t, 3>, 3>;
const Mat3 kIdentity = {{{1, 0, 0}, {0, 1, 0}, {0, 0, 1}}};

// parse_rotation_matrix, magicavoxel.rs:62-90; false for a byte that is not a rotation (column index 3 or two rows on
// one column: the reference asserts in debug builds and indexes out of bounds otherwise)
bool rotation(uint8_t b, Mat3 &m) {
    m = Mat3{};
    const int r0 = b & 0x3, r1 = ((b & (0x3 << 2)) >> 2) & 0x3, r2 = (~(r0 ^ r1)) & 0x3;
    if (r0 > 2 || r1 > 2 || r2 > 2 || r0 == r1 || r0 == r2 || r1 == r2) return false;
    m[0][r0] = (b & 0x10) ? -1 : 1;
    m[1][r1] = (b & 0x20) ? -1 : 1;
    m[2][r2] = (b & 0x40) ? -1 : 1;
    return true;
}

Mat3 mul(const Mat3 &a, const Mat3 &b) {
    Mat3 r{};
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) r[i][j] = a[i][0] * b[0][j] + a[i][1] * b[1][j] + a[i][2] * b[2][j];
    return r;
}

struct I3 {
    int32_t x, y, z;
};
// V3c::transformed, magicavoxel.rs:92-104
I3 transformed(I3 v, const Mat3 &m) {
    return {v.x * m[0][0] + v.y * m[0][1] + v.z * m[0][2], v.x * m[1][0] + v.y * m[1][1] + v.z * m[1][2],
            v.x * m[2][0] + v.y * m[2][1] + v.z * m[2][2]};
}
// convert_coordinate Rzup <-> Lyup (src/spatial/math/mod.rs:189-192): (x, z, y)
I3 swap_yz(I3 v) { return {v.x, v.z, v.y}; }

bool parse_i32(const std::string &s, size_t &pos, int32_t &v) {
    while (pos < s.size() && s[pos] == ' ') ++pos;
    if (pos >= s.size()) return false;
    size_t start = pos;
    if (s[pos] == '-' || s[pos] == '+') ++pos;
    long long acc = 0;
    bool digits = false;
    while (pos < s.size() && s[pos] >= '0' && s[pos] <= '9') {
        acc = acc * 10 + (s[pos] - '0');
        if (acc > 0x7FFFFFFFll + 1) return false;
        ++pos;
        digits = true;
    }
    if (!digits) return false;
    if (s[start] == '-') acc = -acc;
    if (acc > 0x7FFFFFFFll || acc < -0x80000000ll) return false;
    v = (int32_t)acc;
    return true;
}

// iterate_vox_tree, magicavoxel.rs:106-202 (frame 0); returns false on a malformed graph (the reference panics)
template <class F>
bool iterate(const VoxData &vd, F &&fun) {
    if (vd.scenes.empty() || vd.scenes[0].kind != SceneNode::Transform) return false;
    struct Item {
        uint32_t node;
        I3 t;
        Mat3 rot;
        uint32_t index;
    };
    std::vector<Item> stack;
    stack.push_back({vd.scenes[0].child, {0, 0, 0}, kIdentity, 0});
    size_t guard = 0;
    while (!stack.empty()) {
        if (++guard > (size_t)1 << 26) return false;  // cyclic graph
        const Item cur = stack.back();
        if (cur.node >= vd.scenes.size()) return false;
        const SceneNode &s = vd.scenes[cur.node];
        if (s.kind == SceneNode::Transform) {
            if (s.frames.empty()) return false;
            const Dict &fr = s.frames[0];
            I3 t = cur.t;
            if (const std::string *ts = dict_get(fr, "_t")) {
                size_t pos = 0;
                int32_t a, b, c;
                if (!parse_i32(*ts, pos, a) || !parse_i32(*ts, pos, b) || !parse_i32(*ts, pos, c)) return false;
                t = {t.x + a, t.y + b, t.z + c};
            }
            Mat3 orient = kIdentity;  // the reference resets to identity when "_r" is absent
            if (const std::string *rs = dict_get(fr, "_r")) {
                size_t pos = 0;
                int32_t v;
                Mat3 r;
                if (!parse_i32(*rs, pos, v) || v < 0 || v > 255 || !rotation((uint8_t)v, r)) return false;
                orient = mul(cur.rot, r);
            }
            if (cur.index == 0) {
                stack.back().index += 1;
                stack.push_back({s.child, t, orient, 0});
            } else {
                stack.pop_back();
            }
        } else if (s.kind == SceneNode::Group) {
            if (cur.index < s.children.size()) {
                stack.back().index += 1;
                stack.push_back({s.children[cur.index], cur.t, cur.rot, 0});
            } else {
                stack.pop_back();
            }
        } else {
            for (const auto &m : s.models) {
                int32_t f = 0;
                if (const std::string *fs = dict_get(m.second, "_f")) {
                    size_t pos = 0;
                    if (!parse_i32(*fs, pos, f) || f < 0) return false;
                }
                if (f == 0) {
                    if (m.first >= vd.models.size()) return false;
                    fun(vd.models[m.first], cur.t, cur.rot);
                }
            }
            stack.pop_back();
            if (!stack.empty()) stack.back().index += 1;
        }
    }
    return true;
}

}  // namespace

extern "C" {

// model_size_to_tree_size, magicavoxel.rs:55-60
uint32_t vhx_vox_tree_size(int32_t sx, int32_t sy, int32_t sz, uint32_t brick_dim) {
    int32_t m = sx > sy ? sx : sy;
    m = m > sz ? m : sz;
    const float l = std::ceil(std::log((float)m / (float)brick_dim) / std::log(4.0f));
    const uint32_t e = l <= 0.0f ? 0u : (uint32_t)l;
    uint32_t r = 1;
    for (uint32_t k = 0; k < e; ++k) r *= 4;
    return r * brick_dim;
}

int vhx_vox_rotation(uint8_t b, int32_t m[9]) {
    if (!m) return VHX_E_INVALID_ARG;
    Mat3 r;
    if (!rotation(b, r)) return VHX_E_VOX_FORMAT;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) m[i * 3 + j] = r[i][j];
    return VHX_OK;
}

int vhx_boxtree_load_vox_memory(const uint8_t *data, uint64_t size, uint32_t brick_dim, vhx_boxtree **out) {
    if (!data || !out) return VHX_E_INVALID_ARG;
    *out = nullptr;
    VoxData vd;
    if (!parse(data, (size_t)size, vd) || !vd.has_palette) return VHX_E_VOX_FORMAT;
    // load_vox_file_internal (magicavoxel.rs:267-323): model bounds in Rzup, converted to Lyup
    I3 mn{INT32_MAX, INT32_MAX, INT32_MAX}, mx{INT32_MIN, INT32_MIN, INT32_MIN};
    size_t nvox = 0;
    const bool ok = iterate(vd, [&](const VoxModel &m, I3 pos, const Mat3 &rot) {
        const I3 s = transformed({m.sx, m.sy, m.sz}, rot);
        const I3 h{s.x / 2, s.y / 2, s.z / 2};
        mn.x = std::min(std::min(mn.x, pos.x - h.x), pos.x + h.x);
        mn.y = std::min(std::min(mn.y, pos.y - h.y), pos.y + h.y);
        mn.z = std::min(std::min(mn.z, pos.z - h.z), pos.z + h.z);
        mx.x = std::max(std::max(mx.x, pos.x + h.x), pos.x - h.x);
        mx.y = std::max(std::max(mx.y, pos.y + h.y), pos.y - h.y);
        mx.z = std::max(std::max(mx.z, pos.z + h.z), pos.z - h.z);
        nvox += m.voxels.size();
    });
    if (!ok || nvox == 0) return VHX_E_VOX_FORMAT;
    const I3 min_lyup = swap_yz(mn), max_lyup = swap_yz(mx);
    const I3 extent{max_lyup.x - min_lyup.x, max_lyup.y - min_lyup.y, max_lyup.z - min_lyup.z};
    const uint32_t tree_size = vhx_vox_tree_size(extent.x, extent.y, extent.z, brick_dim);
    vhx::BoxTree *t = nullptr;
    int rc = vhx::BoxTree::create(tree_size, brick_dim, &t);
    if (rc != 0) return rc;
    // load_vox_data_internal (magicavoxel.rs:325-374)
    const bool auto_simplify = t->auto_simplify;
    t->auto_simplify = false;
    const I3 min_rzup = swap_yz(min_lyup);
    rc = 0;
    iterate(vd, [&](const VoxModel &m, I3 pos, const Mat3 &rot) {
        if (rc) return;
        const I3 s = transformed({m.sx, m.sy, m.sz}, rot);
        const I3 h{s.x / 2, s.y / 2, s.z / 2};
        const I3 bl{pos.x - h.x - min_rzup.x + (h.x < 0 ? -1 : 0), pos.y - h.y - min_rzup.y + (h.y < 0 ? -1 : 0),
                    pos.z - h.z - min_rzup.z + (h.z < 0 ? -1 : 0)};
        for (const auto &v : m.voxels) {
            const I3 tv = transformed({v[0], v[1], v[2]}, rot);
            const I3 p = swap_yz({bl.x + tv.x, bl.y + tv.y, bl.z + tv.z});
            const uint32_t albedo = vd.palette[v[3]];
            // V3c<i32> -> V3c<u32> is `as u32` (vector.rs:357-362): negatives wrap and are rejected by insert
            rc = t->insert(vhx::U3{(uint32_t)p.x, (uint32_t)p.y, (uint32_t)p.z},
                           vhx::Entry{VHX_ENTRY_VISUAL, albedo, 0});
            if (rc) return;
        }
    });
    if (rc) {
        delete t;
        return rc;
    }
    if (auto_simplify) {
        t->simplify(0, true);
        t->auto_simplify = true;
    }
    *out = new vhx_boxtree{t};
    return VHX_OK;
}

int vhx_boxtree_load_vox(const char *path, uint32_t brick_dim, vhx_boxtree **out) {
    if (!path || !out) return VHX_E_INVALID_ARG;
    *out = nullptr;
    FILE *f = std::fopen(path, "rb");
    if (!f) return VHX_E_VOX_IO;
    std::vector<uint8_t> buf;
    uint8_t tmp[1 << 16];
    size_t n;
    while ((n = std::fread(tmp, 1, sizeof(tmp), f)) > 0) buf.insert(buf.end(), tmp, tmp + n);
    const bool err = std::ferror(f) != 0;
    std::fclose(f);
    if (err) return VHX_E_VOX_IO;
    return vhx_boxtree_load_vox_memory(buf.data(), buf.size(), brick_dim, out);
}

}  // extern "C"
