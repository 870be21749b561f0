// Host-side BoxTree<u32>: see boxtree.hpp for the list of restated reference functions.
// Float arithmetic follows the reference op order (compiled with -ffp-contract=off).
#include "boxtree.hpp"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <cmath>
#include <functional>
#include <atomic>
#include <climits>
#include <cstdint>
#include <system_error>
#include <thread>

#include "../../include/vhx_boxtree.h"

namespace vhx {

// ---------------------------------------------------------------------------------------------- scalar helpers
static inline F3 f3(float x, float y, float z) { return F3{x, y, z}; }
static inline F3 add(F3 a, F3 b) { return f3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline F3 sub(F3 a, F3 b) { return f3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline F3 mul(F3 a, float s) { return f3(a.x * s, a.y * s, a.z * s); }
static inline F3 divs(F3 a, float s) { return f3(a.x / s, a.y / s, a.z / s); }
static inline F3 floor3(F3 a) { return f3(std::floor(a.x), std::floor(a.y), std::floor(a.z)); }
static inline F3 from_u3(U3 a) { return f3((float)a.x, (float)a.y, (float)a.z); }
static inline uint32_t as_u32(float f) {  // Rust `as u32` (saturating, NaN -> 0)
    if (std::isnan(f) || f <= 0.f) return 0;
    if (f >= 4294967296.0f) return 0xFFFFFFFFu;
    return (uint32_t)f;
}
static inline size_t as_usize(float f) {
    if (std::isnan(f) || f <= 0.f) return 0;
    if (f >= 18446744073709551616.0f) return SIZE_MAX;
    return (size_t)f;
}
static inline uint8_t as_u8(float f) {
    if (std::isnan(f) || f <= 0.f) return 0;
    if (f >= 255.f) return 255;
    return (uint8_t)f;
}
// From<V3c<f32>> for V3c<u32>/V3c<usize> rounds (src/spatial/math/vector.rs:325-355)
static inline U3 round_u3(F3 a) { return U3{as_u32(std::round(a.x)), as_u32(std::round(a.y)), as_u32(std::round(a.z))}; }
// derived PartialOrd on V3c compares lexicographically (src/spatial/math/vector.rs:3)
static inline bool lex_le(F3 a, F3 b) {
    if (a.x != b.x) return a.x < b.x;
    if (a.y != b.y) return a.y < b.y;
    return a.z <= b.z;
}
static inline size_t flat_projection(size_t x, size_t y, size_t z, size_t size) { return x + (y * size) + (z * size * size); }

static float SECTANT_OFFSET_LUT[64][3];
static const bool kLutInit = [] {
    for (int x = 0; x < 4; ++x)
        for (int y = 0; y < 4; ++y)
            for (int z = 0; z < 4; ++z) {
                int s = x + y * 4 + z * 16;
                SECTANT_OFFSET_LUT[s][0] = (float)x / 4.f;
                SECTANT_OFFSET_LUT[s][1] = (float)y / 4.f;
                SECTANT_OFFSET_LUT[s][2] = (float)z / 4.f;
            }
    return true;
}();
const float *sectant_offset(uint32_t s) { return SECTANT_OFFSET_LUT[s]; }
static inline F3 lut(uint32_t s) { return f3(SECTANT_OFFSET_LUT[s][0], SECTANT_OFFSET_LUT[s][1], SECTANT_OFFSET_LUT[s][2]); }

// offset_sectant, src/spatial/math/mod.rs:27-44
uint8_t offset_sectant(F3 off, float size) {
    F3 idx = floor3(divs(mul(off, 4.f), size));
    idx = f3(std::fmin(idx.x, 3.f), std::fmin(idx.y, 3.f), std::fmin(idx.z, 3.f));
    return as_u8(idx.x + (idx.y * 4.f) + (idx.z * 16.f));
}
// Cube::child_bounds_for, src/spatial/mod.rs:72-77
Cube child_bounds_for(const Cube &c, uint8_t s) { return Cube{add(c.min, mul(lut(s), c.size)), c.size / 4.f}; }
static inline bool cube_contains(const Cube &c, F3 p) {  // src/spatial/mod.rs:54-61
    return p.x >= c.min.x && p.y >= c.min.y && p.z >= c.min.z && p.x < (c.min.x + c.size) &&
           p.y < (c.min.y + c.size) && p.z < (c.min.z + c.size);
}
static inline uint8_t sectant_for(const Cube &c, F3 p) { return offset_sectant(sub(p, c.min), c.size); }
// matrix_index_for, src/spatial/math/mod.rs:64-96
static inline std::array<size_t, 3> matrix_index_for(const Cube &b, U3 pos, uint32_t dim) {
    F3 m = floor3(divs(mul(sub(from_u3(pos), b.min), (float)dim), b.size));
    return {as_usize(std::round(m.x)), as_usize(std::round(m.y)), as_usize(std::round(m.z))};
}
// `(x as f32).log(base).fract() != 0.0` (src/boxtree/mod.rs:189, 194); Rust f32::log = ln(x) / ln(base)
bool rust_log_is_integral(float x, float base) {
    float l = std::log(x) / std::log(base);
    return (l - std::trunc(l)) == 0.f;
}

// pix_* (src/boxtree/node.rs:260-309)
static inline uint32_t pix_visual(uint32_t c) { return c | (0xFFFFu << 16); }
static inline uint32_t pix_informal(uint32_t d) { return 0xFFFFu | (d << 16); }
static inline uint32_t pix_complex(uint32_t c, uint32_t d) { return c | (d << 16); }
static inline uint32_t pix_color_index(uint32_t v) { return v & 0xFFFFu; }
static inline uint32_t pix_data_index(uint32_t v) { return (v & 0xFFFF0000u) >> 16; }
static inline bool pix_color_is_some(uint32_t v) { return pix_color_index(v) < 0xFFFFu; }
static inline bool pix_data_is_some(uint32_t v) { return pix_data_index(v) != 0xFFFFu; }

// execute_for_relevant_sectants, src/boxtree/iterate.rs:40-121
using SectantFn = std::function<void(U3, U3, uint8_t, const Cube &)>;
std::array<size_t, 3> execute_for_relevant_sectants(const Cube &nb, U3 position_, uint32_t update_size_,
                                                    const SectantFn &fun) {
    return relevant_sectants(nb, position_, update_size_, fun);  // boxtree.hpp
}

// ---------------------------------------------------------------------------------------------- ObjectPool
bool ObjectPool::try_set_next_available() {  // src/object_pool.rs:168-183
    if ((first_available_ + 1) < buffer_.size() && !reserved_[first_available_]) return true;
    if ((first_available_ + 1) < buffer_.size() && !reserved_[first_available_ + 1]) {
        first_available_ += 1;
        return true;
    }
    return false;
}
size_t ObjectPool::allocate() {  // src/object_pool.rs:198-222
    size_t key;
    if (try_set_next_available()) {
        size_t fa = first_available_;
        reserved_[fa] = true;
        try_set_next_available();
        key = fa;
    } else {
        reserved_.push_back(true);
        buffer_.emplace_back();
        key = buffer_.size() - 1;
    }
    try_set_next_available();
    return key;
}
size_t ObjectPool::push(Node item) {
    size_t key = allocate();
    buffer_[key] = std::move(item);
    return key;
}
bool ObjectPool::free(size_t key) {
    if (!key_is_valid(key)) return false;
    reserved_[key] = false;
    first_available_ = std::min(first_available_, key);
    return true;
}

// ---------------------------------------------------------------------------------------------- node constructors
static Node empty_node() { return Node{}; }
static Node uniform_solid_node(uint32_t v) {
    Node n;
    n.content = Content::UniformLeaf;
    n.bricks.resize(1);
    n.bricks[0].kind = BrickKind::Solid;
    n.bricks[0].solid = v;
    n.mip.kind = BrickKind::Solid;  // node.rs:191-199: a uniform solid node is its own MIP
    n.mip.solid = v;
    n.occupied_bits = ~0ull;
    return n;
}
static Node uniform_parted_node(std::vector<uint32_t> brick, uint64_t occ) {
    Node n;
    n.content = Content::UniformLeaf;
    n.bricks.resize(1);
    n.bricks[0].kind = BrickKind::Parted;
    n.bricks[0].parted = std::move(brick);
    n.occupied_bits = occ;
    return n;
}
static Brick parted(std::vector<uint32_t> v) {
    Brick b;
    b.kind = BrickKind::Parted;
    b.parted = std::move(v);
    return b;
}
static Brick solid(uint32_t v) {
    Brick b;
    b.kind = BrickKind::Solid;
    b.solid = v;
    return b;
}

// ---------------------------------------------------------------------------------------------- BoxTree
int BoxTree::create(uint32_t size, uint32_t bd, BoxTree **out) {  // src/boxtree/mod.rs:188-219
    if (0 == size || !rust_log_is_integral((float)bd, 2.0f)) return VHX_E_TREE_INVALID_BRICK_DIMENSION;
    if (bd > size || 0 == size || !rust_log_is_integral((float)size / (float)bd, 4.0f)) return VHX_E_TREE_INVALID_SIZE;
    if (size < bd * 4u) return VHX_E_TREE_INVALID_STRUCTURE;
    BoxTree *t = new BoxTree();
    t->boxtree_size = size;
    t->brick_dim = bd;
    size_t root = t->nodes.push(empty_node());
    (void)root;
    *out = t;
    return 0;
}

bool BoxTree::points_to_empty(uint32_t v) const {  // src/boxtree/node.rs:311-333
    uint32_t ci = pix_color_index(v), di = pix_data_index(v);
    bool color_none = !pix_color_is_some(v) || ci >= color_palette.size() || ((color_palette[ci] >> 24) & 0xFFu) == 0;
    bool data_none = !pix_data_is_some(v) || di >= data_palette.size() || data_palette[di] == 0;
    return color_none && data_none;
}

size_t BoxTree::child(size_t key, uint8_t s) const {  // src/boxtree/node.rs:214-219
    const Node &n = nodes.get(key);
    return n.has_children ? (size_t)n.children[s] : SIZE_MAX;
}
uint32_t &BoxTree::child_mut(size_t key, size_t index) {  // src/boxtree/node.rs:222-230
    Node &n = nodes.get(key);
    if (!n.has_children) {
        n.has_children = true;
        n.children.fill(kEmpty32);
    }
    return n.children[index];
}

static bool entry_is_none(const Entry &e) {  // src/boxtree/mod.rs:99-106
    switch (e.kind) {
        case VHX_ENTRY_EMPTY: return true;
        case VHX_ENTRY_VISUAL: return ((e.albedo >> 24) & 0xFFu) == 0;
        case VHX_ENTRY_INFORMATIVE: return e.data == 0;
        default: return ((e.albedo >> 24) & 0xFFu) == 0 && e.data == 0;
    }
}

uint32_t BoxTree::add_to_palette(Entry e) {  // src/boxtree/update/mod.rs:39-120
    auto color = [&](uint32_t albedo) {
        size_t potential = color_index_.size();
        auto it = color_index_.find(albedo);
        if (it == color_index_.end()) {
            color_index_.emplace(albedo, potential);
            color_palette.push_back(albedo);
            return potential;
        }
        return it->second;
    };
    auto data = [&](uint32_t d) {
        size_t potential = data_index_.size();
        auto it = data_index_.find(d);
        if (it == data_index_.end()) {
            data_index_.emplace(d, potential);
            data_palette.push_back(d);
            return potential;
        }
        return it->second;
    };
    switch (e.kind) {
        case VHX_ENTRY_EMPTY: return kEmpty32;
        case VHX_ENTRY_VISUAL:
            if (e.albedo == 0) return kEmpty32;
            return pix_visual((uint32_t)color(e.albedo));
        case VHX_ENTRY_INFORMATIVE:
            if (e.data == 0) return kEmpty32;
            return pix_informal((uint32_t)data(e.data));
        default:
            if (e.albedo == 0) return add_to_palette(Entry{VHX_ENTRY_INFORMATIVE, 0, e.data});
            if (e.data == 0) return add_to_palette(Entry{VHX_ENTRY_VISUAL, e.albedo, 0});
            {
                size_t ci = color(e.albedo);
                size_t di = data(e.data);
                return pix_complex((uint32_t)ci, (uint32_t)di);
            }
    }
}

// ------------------------------------------------------------------------------------- BrickData (node.rs:34-145)
uint64_t BoxTree::calculate_brick_occupied_bits(const std::vector<uint32_t> &brick) const {
    uint64_t bitmap = 0;
    size_t bd = brick_dim;
    for (size_t x = 0; x < bd; ++x)
        for (size_t y = 0; y < bd; ++y)
            for (size_t z = 0; z < bd; ++z) {
                if (points_to_empty(brick[flat_projection(x, y, z, bd)])) continue;
                // set_occupied_bitmap_value(&V3c(x,y,z), 1, bd, true, bitmap), src/spatial/math/mod.rs:104-155
                if (bd == 1) {
                    bitmap = ~0ull;
                    continue;
                }
                size_t count = (size_t)std::ceil((float)1 * 4.f / (float)bd);
                size_t sx = as_usize(std::round(std::floor((float)(x * 4) / (float)bd)));
                size_t sy = as_usize(std::round(std::floor((float)(y * 4) / (float)bd)));
                size_t sz = as_usize(std::round(std::floor((float)(z * 4) / (float)bd)));
                for (size_t ax = sx; ax < std::min(sx + count, (size_t)4); ++ax)
                    for (size_t ay = sy; ay < std::min(sy + count, (size_t)4); ++ay)
                        for (size_t az = sz; az < std::min(sz + count, (size_t)4); ++az)
                            bitmap |= 1ull << offset_sectant(f3((float)ax, (float)ay, (float)az), 4.f);
            }
    return bitmap;
}
uint64_t BoxTree::calculate_occupied_bits(const Brick &b) const {
    switch (b.kind) {
        case BrickKind::Empty: return 0;
        case BrickKind::Solid: return points_to_empty(b.solid) ? 0 : ~0ull;
        default: return calculate_brick_occupied_bits(b.parted);
    }
}
static const uint32_t *homogeneous(const Brick &b) {
    switch (b.kind) {
        case BrickKind::Empty: return nullptr;
        case BrickKind::Solid: return &b.solid;
        default:
            for (uint32_t v : b.parted)
                if (v != b.parted[0]) return nullptr;
            return &b.parted[0];
    }
}
bool BoxTree::brick_contains_nothing(const Brick &b) const {
    switch (b.kind) {
        case BrickKind::Empty: return true;
        case BrickKind::Solid: return points_to_empty(b.solid);
        default:
            for (uint32_t v : b.parted)
                if (!points_to_empty(v)) return false;
            return true;
    }
}
bool BoxTree::brick_simplify(Brick &b) const {
    const uint32_t *h = homogeneous(b);
    if (!h) return false;
    uint32_t v = *h;
    if (points_to_empty(v)) {
        b = Brick{};
    } else {
        b = solid(v);
    }
    return true;
}
bool BoxTree::content_is_all(const Node &n, uint32_t data) const {  // node.rs:424-458
    auto brick_is = [&](const Brick &b) {
        switch (b.kind) {
            case BrickKind::Empty: return false;
            case BrickKind::Solid: return b.solid == data;
            default: {
                const uint32_t *h = homogeneous(b);
                return h && *h == data;
            }
        }
    };
    switch (n.content) {
        case Content::UniformLeaf: return brick_is(n.bricks[0]);
        case Content::Leaf:
            for (const Brick &b : n.bricks)
                if (!brick_is(b)) return false;
            return true;
        default: return false;
    }
}

// ------------------------------------------------------------------------------------- detail.rs
bool BoxTree::node_empty_at(size_t key, uint8_t s) const {  // detail.rs:156-224
    const Node &n = nodes.get(key);
    switch (n.content) {
        case Content::Nothing: return true;
        case Content::Leaf: {
            const Brick &b = n.bricks[s];
            if (b.kind == BrickKind::Empty) return true;
            if (b.kind == BrickKind::Solid) return points_to_empty(b.solid);
            const uint32_t *h = homogeneous(b);
            return h ? points_to_empty(*h) : false;
        }
        case Content::UniformLeaf: {
            const Brick &b = n.bricks[0];
            if (b.kind == BrickKind::Empty) return true;
            if (b.kind == BrickKind::Solid) return points_to_empty(b.solid);
            const float *o = sectant_offset(s);
            F3 cs = floor3(f3(o[0] * (float)brick_dim, o[1] * (float)brick_dim, o[2] * (float)brick_dim));
            U3 start = round_u3(cs);
            size_t check = as_usize(std::fmax((float)brick_dim / 4.f, 1.f));
            for (size_t x = start.x; x < start.x + check; ++x)
                for (size_t y = start.y; y < start.y + check; ++y)
                    for (size_t z = start.z; z < start.z + check; ++z)
                        if (!points_to_empty(b.parted[flat_projection(x, y, z, brick_dim)])) return false;
            return true;
        }
        default: {
            size_t ck = child(key, s);
            if (!nodes.key_is_valid(ck)) return true;
            for (uint32_t cs = 0; cs < kChildren; ++cs)
                if (!node_empty_at(ck, (uint8_t)cs)) return false;
            return true;
        }
    }
}
bool BoxTree::compare_nodes(size_t l, size_t r) const {  // detail.rs:229-243, node.rs:460-479
    if (nodes.key_is_valid(l) != nodes.key_is_valid(r)) return false;
    if (!nodes.key_is_valid(l)) return true;
    const Node &a = nodes.get(l), &b = nodes.get(r);
    switch (a.content) {
        case Content::Nothing: return b.content == Content::Nothing;
        case Content::Internal: return false;
        case Content::UniformLeaf: return b.content == Content::UniformLeaf && a.bricks[0] == b.bricks[0];
        default: return b.content == Content::Leaf && a.bricks == b.bricks;
    }
}
void BoxTree::deallocate_children_of(size_t key) {  // detail.rs:352-370
    if (!nodes.key_is_valid(key)) return;
    std::vector<size_t> to_free;
    const Node &n = nodes.get(key);
    if (n.has_children)
        for (uint32_t c : n.children)
            if (nodes.key_is_valid(c)) to_free.push_back(c);
    for (size_t c : to_free) {
        deallocate_children_of(c);
        nodes.free(c);
    }
}
Brick BoxTree::try_brick_from_node(size_t key) const {  // detail.rs:340-349
    if (!nodes.key_is_valid(key)) return Brick{};
    const Node &n = nodes.get(key);
    if (n.content == Content::UniformLeaf) return n.bricks[0];
    return Brick{};
}

std::array<std::vector<uint32_t>, kChildren> BoxTree::dilute_brick_data(const std::vector<uint32_t> &bdata) const {
    // src/boxtree/update/mod.rs:478-555
    std::array<std::vector<uint32_t>, kChildren> result;
    size_t bd = brick_dim, n3 = bd * bd * bd;
    if (bd == 1) {
        for (auto &r : result) r = bdata;
        return result;
    }
    if (bd == 2) {
        for (uint32_t s = 0; s < kChildren; ++s) {
            // octant_in_sectants (src/spatial/math/mod.rs:56-59)
            const float *o = sectant_offset(s);
            float ox = o[0] * 2.f, oy = o[1] * 2.f, oz = o[2] * 2.f;
            size_t oct = (size_t)(ox >= 1.f) + (size_t)(oz >= 1.f) * 2 + (size_t)(oy >= 1.f) * 4;
            result[s].assign(n3, bdata[oct]);
        }
        return result;
    }
    for (uint32_t s = 0; s < kChildren; ++s) result[s].assign(n3, bdata[s]);
    if (bd == 4) return result;
    for (uint32_t s = 0; s < kChildren; ++s) {
        const float *o = sectant_offset(s);
        U3 off = round_u3(f3(o[0] * (float)bd, o[1] * (float)bd, o[2] * (float)bd));
        std::vector<uint32_t> nb(n3, bdata[flat_projection(off.x, off.y, off.z, bd)]);
        for (size_t x = 0; x < bd; ++x)
            for (size_t y = 0; y < bd; ++y)
                for (size_t z = 0; z < bd; ++z) {
                    if (x < 4 && y < 4 && z < 4) continue;
                    nb[flat_projection(x, y, z, bd)] = bdata[flat_projection(off.x + x / 4, off.y + y / 4, off.z + z / 4, bd)];
                }
        result[s] = std::move(nb);
    }
    return result;
}

void BoxTree::update_brick(bool overwrite, std::vector<uint32_t> &brick, const Cube &bb, U3 position, U3 size,
                           uint32_t data) const {  // src/boxtree/update/mod.rs:564-603
    auto mi = matrix_index_for(bb, position, brick_dim);
    size_t bd = brick_dim;
    for (size_t x = mi[0]; x < std::min(mi[0] + size.x, bd); ++x)
        for (size_t y = mi[1]; y < std::min(mi[1] + size.y, bd); ++y)
            for (size_t z = mi[2]; z < std::min(mi[2] + size.z, bd); ++z) {
                size_t f = flat_projection(x, y, z, bd);
                if (overwrite) {
                    brick[f] = data;
                } else {
                    if (pix_color_is_some(data)) brick[f] = (brick[f] & 0xFFFF0000u) | (data & 0x0000FFFFu);
                    if (pix_data_is_some(data)) brick[f] = (brick[f] & 0x0000FFFFu) | (data & 0xFFFF0000u);
                }
            }
}

void BoxTree::subdivide_leaf_to_nodes(size_t key, size_t target_sectant) {  // detail.rs:248-337
    Node &n0 = nodes.get(key);
    Content content = n0.content;
    std::vector<Brick> bricks = std::move(n0.bricks);
    n0.content = Content::Internal;
    n0.bricks.clear();
    std::array<uint32_t, kChildren> new_children;
    new_children.fill(kEmpty32);
    if (content == Content::Leaf) {
        for (size_t s = 0; s < kChildren; ++s) {
            Brick brick = std::move(bricks[s]);
            bricks[s] = Brick{};  // std::mem::swap leaves BrickData::Empty behind
            if (!brick_contains_nothing(brick) || s == target_sectant)
                new_children[s] = (uint32_t)nodes.push(empty_node());
            if (brick.kind == BrickKind::Solid) {
                Node &c = nodes.get(new_children[s]);
                c.occupied_bits = ~0ull;
                c.content = Content::UniformLeaf;
                c.bricks.assign(1, solid(brick.solid));
            } else if (brick.kind == BrickKind::Parted) {
                // detail.rs:283-289 computes the occupancy of bricks[sectant] after the swap, i.e. of Empty -> 0
                uint64_t occ = calculate_occupied_bits(bricks[s]);
                Node &c = nodes.get(new_children[s]);
                c.occupied_bits = occ;
                c.content = Content::UniformLeaf;
                c.bricks.assign(1, parted(brick.parted));
            }
        }
    } else if (content == Content::UniformLeaf) {
        Brick brick = std::move(bricks[0]);
        if (brick.kind == BrickKind::Empty) {
            new_children[target_sectant] = (uint32_t)nodes.push(empty_node());
        } else if (brick.kind == BrickKind::Solid) {
            for (size_t s = 0; s < kChildren; ++s) new_children[s] = (uint32_t)nodes.push(uniform_solid_node(brick.solid));
        } else {
            auto cb = dilute_brick_data(brick.parted);
            for (size_t s = 0; s < kChildren; ++s) {
                uint64_t occ = calculate_brick_occupied_bits(cb[s]);
                new_children[s] = (uint32_t)nodes.push(uniform_parted_node(std::move(cb[s]), occ));
            }
        }
    }  // Nothing / Internal: the reference panics
    Node &n = nodes.get(key);
    n.has_children = true;
    n.children = new_children;
}

size_t BoxTree::get_node_internal(size_t key, Cube &bounds, F3 position) const {  // iterate.rs:293-343
    for (;;) {
        const Node &n = nodes.get(key);
        if (n.content != Content::Internal) return key;
        uint8_t s = sectant_for(bounds, position);
        size_t c = child(key, s);
        if (!nodes.key_is_valid(c)) return key;
        key = c;
        bounds = child_bounds_for(bounds, s);
    }
}

uint32_t BoxTree::get_internal(size_t key, Cube bounds, U3 pos) const {  // src/boxtree/mod.rs:247-317
    F3 p = from_u3(pos);
    if (!cube_contains(bounds, p)) return kEmpty32;
    key = get_node_internal(key, bounds, p);
    const Node &n = nodes.get(key);
    switch (n.content) {
        case Content::Leaf: {
            uint8_t s = sectant_for(bounds, p);
            const Brick &b = n.bricks[s];
            if (b.kind == BrickKind::Empty) return kEmpty32;
            if (b.kind == BrickKind::Solid) return b.solid;
            Cube cb = child_bounds_for(bounds, s);
            auto mi = matrix_index_for(cb, pos, brick_dim);
            uint32_t v = b.parted[flat_projection(mi[0], mi[1], mi[2], brick_dim)];
            return points_to_empty(v) ? kEmpty32 : v;
        }
        case Content::UniformLeaf: {
            const Brick &b = n.bricks[0];
            if (b.kind == BrickKind::Empty) return kEmpty32;
            if (b.kind == BrickKind::Solid) return b.solid;
            auto mi = matrix_index_for(bounds, pos, brick_dim);
            return b.parted[flat_projection(mi[0], mi[1], mi[2], brick_dim)];
        }
        default: return kEmpty32;
    }
}
uint32_t BoxTree::get_raw(U3 pos) const {  // src/boxtree/mod.rs:223-233
    return get_internal(0, Cube{f3(0.f, 0.f, 0.f), (float)boxtree_size}, pos);
}
Entry BoxTree::get(U3 pos) const { return entry_of(get_raw(pos)); }
Entry BoxTree::entry_of(uint32_t v) const {  // pix_get_ref, src/boxtree/node.rs:335-373
    bool cn = !pix_color_is_some(v), dn = !pix_data_is_some(v);
    Entry e{VHX_ENTRY_EMPTY, 0, 0};
    if (cn && dn) return e;
    if (!cn) e.albedo = pix_color_index(v) < color_palette.size() ? color_palette[pix_color_index(v)] : 0;
    if (!dn) e.data = pix_data_index(v) < data_palette.size() ? data_palette[pix_data_index(v)] : 0;
    e.kind = dn ? VHX_ENTRY_VISUAL : (cn ? VHX_ENTRY_INFORMATIVE : VHX_ENTRY_COMPLEX);
    return e;
}

bool BoxTree::leaf_update(bool overwrite, size_t key, const Cube &node_bounds, const Cube &target_bounds, size_t tcs,
                          U3 position, U3 size, uint32_t tc) {  // src/boxtree/update/mod.rs:144-464
    Node &node = nodes.get(key);
    switch (node.content) {
        case Content::Leaf: {
            Brick &b = node.bricks[tcs];
            if (b.kind == BrickKind::Empty) {
                std::vector<uint32_t> nb((size_t)brick_dim * brick_dim * brick_dim, kEmpty32);
                update_brick(overwrite, nb, target_bounds, position, size, tc);
                nodes.get(key).bricks[tcs] = parted(std::move(nb));
                return true;
            }
            if (b.kind == BrickKind::Solid) {
                uint32_t v = b.solid;
                if ((points_to_empty(tc) && !points_to_empty(v)) || (!points_to_empty(tc) && v != tc)) {
                    std::vector<uint32_t> nb((size_t)brick_dim * brick_dim * brick_dim, v);
                    update_brick(overwrite, nb, target_bounds, position, size, tc);
                    nodes.get(key).bricks[tcs] = parted(std::move(nb));
                    return true;
                }
                return false;
            }
            update_brick(overwrite, b.parted, target_bounds, position, size, tc);
            return true;
        }
        case Content::UniformLeaf: {
            Brick &mat = node.bricks[0];
            if (mat.kind == BrickKind::Empty) {
                if (!points_to_empty(tc)) {
                    std::vector<Brick> leaf(kChildren);
                    std::vector<uint32_t> nb((size_t)brick_dim * brick_dim * brick_dim, add_to_palette(Entry{VHX_ENTRY_EMPTY, 0, 0}));
                    update_brick(overwrite, nb, target_bounds, position, size, tc);
                    leaf[tcs] = parted(std::move(nb));
                    Node &n = nodes.get(key);
                    n.content = Content::Leaf;
                    n.bricks = std::move(leaf);
                    return true;
                }
                break;  // falls through to the recursive call below (unreachable for insert: data is never empty)
            }
            if (mat.kind == BrickKind::Solid) {
                uint32_t v = mat.solid;
                if (points_to_empty(tc) && points_to_empty(v)) {
                    node.content = Content::Nothing;
                    node.bricks.clear();
                    return false;
                }
                if ((!points_to_empty(tc) && v != tc) || (points_to_empty(tc) && !points_to_empty(v))) {
                    mat = parted(std::vector<uint32_t>((size_t)brick_dim * brick_dim * brick_dim, v));
                    return leaf_update(overwrite, key, node_bounds, target_bounds, tcs, position, size, tc);
                }
                return false;
            }
            {
                auto mi = matrix_index_for(node_bounds, position, brick_dim);
                size_t f = flat_projection(mi[0], mi[1], mi[2], brick_dim);
                if (1 < brick_dim && ((points_to_empty(tc) && points_to_empty(mat.parted[f])) ||
                                      (!points_to_empty(tc) && mat.parted[f] == tc)))
                    return false;
                if (node_bounds.size <= (float)brick_dim && brick_dim > 1) {
                    update_brick(overwrite, mat.parted, node_bounds, position, size, tc);
                    return true;
                }
                std::vector<Brick> leaf(kChildren);
                std::vector<uint32_t> taken = std::move(mat.parted);
                mat.parted.clear();
                auto cb = dilute_brick_data(taken);
                bool updated = false;
                for (size_t s = 0; s < kChildren; ++s) {
                    if (s == tcs) {
                        update_brick(overwrite, cb[s], target_bounds, position, size, tc);
                        updated = true;
                    }
                    leaf[s] = parted(std::move(cb[s]));
                }
                Node &n = nodes.get(key);
                n.content = Content::Leaf;
                n.bricks = std::move(leaf);
                return updated;
            }
        }
        case Content::Internal: {
            node.has_children = false;  // children = NoChildren before the bricks are gathered (update/mod.rs:420)
            std::vector<Brick> leaf(kChildren);
            for (size_t s = 0; s < kChildren; ++s) leaf[s] = try_brick_from_node(child(key, (uint8_t)s));
            Node &n = nodes.get(key);
            n.content = Content::Leaf;
            n.bricks = std::move(leaf);
            deallocate_children_of(key);
            return leaf_update(overwrite, key, node_bounds, target_bounds, tcs, position, size, tc);
        }
        case Content::Nothing: {
            std::vector<Brick> leaf(kChildren);
            for (size_t s = 0; s < kChildren; ++s) leaf[s] = try_brick_from_node(child(key, (uint8_t)s));
            Node &n = nodes.get(key);
            n.content = Content::Leaf;
            n.bricks = std::move(leaf);
            deallocate_children_of(key);
            return leaf_update(overwrite, key, node_bounds, target_bounds, tcs, position, size, tc);
        }
    }
    return leaf_update(overwrite, key, node_bounds, target_bounds, tcs, position, size, tc);
}

uint8_t step_sectant_i(uint8_t s, int dx, int dy, int dz) {
    const int x = (s & 3) + dx, y = ((s >> 2) & 3) + dy, z = (s >> 4) + dz;
    const int out = (x < 0 || x > 3 || y < 0 || y > 3 || z < 0 || z > 3) ? 64 : 0;
    return (uint8_t)(out + (x & 3) + ((y & 3) << 2) + ((z & 3) << 4));
}

// get_sibling_by_stack, src/boxtree/iterate.rs:186-290 (direction given as unit integer steps)
bool BoxTree::get_sibling_by_stack(int dx, int dy, int dz, const std::vector<std::pair<size_t, uint8_t>> &ns_in,
                                   size_t &sibling, uint8_t &sibling_sectant) const {
    std::vector<std::pair<size_t, uint8_t>> ns = ns_in;
    uint8_t current = ns.back().second;
    uint8_t next = step_sectant_i(current, dx, dy, dz);
    std::vector<uint8_t> mirror;  // front = mirror[0]
    bool uniform_sibling = false;
    uint8_t uniform_sibling_sectant = 0;
    if (!ns.empty() && nodes.get(ns.back().first).content == Content::UniformLeaf) {
        uint8_t ts = ns.back().second;
        ns.pop_back();
        while (ts < kChildren) ts = step_sectant_i(ts, dx, dy, dz);
        uniform_sibling = true;
        uniform_sibling_sectant = (uint8_t)(ts - kChildren);
        if (!ns.empty()) next = step_sectant_i(ns.back().second, dx, dy, dz);
    }
    while (!ns.empty() && next >= kChildren) {
        mirror.insert(mirror.begin(), (uint8_t)(next - kChildren));
        const auto parent = ns.back();
        ns.pop_back();
        current = parent.second;
        next = step_sectant_i(current, dx, dy, dz);
        if (next < kChildren) ns.push_back({parent.first, next});
    }
    if (ns.empty()) return false;
    mirror.insert(mirror.begin(), next);
    if (uniform_sibling) {
        const size_t sn = child(ns.back().first, next);
        if (nodes.key_is_valid(sn)) {
            sibling = sn;
            sibling_sectant = uniform_sibling_sectant;
            return true;
        }
        return false;
    }
    size_t key = ns.back().first;
    for (uint8_t ts : mirror) {
        const size_t c = child(key, ts);
        if (nodes.key_is_valid(c)) {
            key = c;
            next = ts;
        } else if (nodes.get(key).content == Content::Leaf) {
            sibling = key;
            sibling_sectant = ts;
            return true;
        } else if (nodes.get(key).content == Content::UniformLeaf) {
            sibling = key;
            sibling_sectant = kChildren;
            return true;
        } else {
            return false;
        }
    }
    sibling = key;
    sibling_sectant = next;
    return true;
}

void BoxTree::post_process_node_insert(const std::vector<std::pair<size_t, uint8_t>> &node_stack, const Cube &nb,
                                       const std::array<size_t, 3> &aus, U3 pos,
                                       uint32_t insert_size) {  // src/boxtree/update/insert.rs:411-495
    const size_t key = node_stack.back().first;
    Node &n = nodes.get(key);
    if (n.content == Content::Nothing) {
        n.content = Content::Internal;
        n.occupied_bits = 0;
    }
    uint64_t occ = n.occupied_bits;
    size_t ns = as_usize(nb.size);
    if (ns == aus[0] && ns == aus[1] && ns == aus[2]) {
        occ = ~0ull;
    } else {
        execute_for_relevant_sectants(nb, pos, insert_size, [&](U3, U3, uint8_t cs, const Cube &) {
            if (!node_empty_at(key, cs)) occ |= 1ull << cs;
        });
    }
    if (occ == ~0ull) {  // a full node occludes the facing side of each sibling (insert.rs:451-468)
        static const int dirs[6][4] = {{-1, 0, 0, 5 /*Right*/}, {1, 0, 0, 4 /*Left*/},  {0, -1, 0, 2 /*Top*/},
                                       {0, 1, 0, 3 /*Bottom*/}, {0, 0, -1, 1 /*Front*/}, {0, 0, 1, 0 /*Back*/}};
        for (const auto &dv : dirs) {
            size_t sib;
            uint8_t ss;
            if (get_sibling_by_stack(dv[0], dv[1], dv[2], node_stack, sib, ss))
                nodes.get(sib).occlusion_bits |= (uint8_t)(1u << dv[3]);
        }
    }
    nodes.get(key).occupied_bits = occ;
    update_mip(key, nb, pos);  // insert.rs:494
}

int BoxTree::insert_at_lod_internal(bool overwrite, U3 pos_u32, uint32_t insert_size, Entry data) {
    // src/boxtree/update/insert.rs:73-407
    Cube root{f3(0.f, 0.f, 0.f), (float)boxtree_size};
    F3 position = from_u3(pos_u32);
    if (!cube_contains(root, position)) return VHX_E_TREE_INVALID_POSITION;
    if (entry_is_none(data) || insert_size == 0) return 0;

    std::vector<std::pair<size_t, uint8_t>> node_stack{{0, sectant_for(root, position)}};
    std::vector<Cube> bounds_stack{root};
    std::vector<uint8_t> modified_bottom;
    std::array<size_t, 3> actual_update_size{0, 0, 0};
    bool updated = false;
    uint32_t tc = add_to_palette(data);
    for (;;) {
        size_t cur = node_stack.back().first;
        uint8_t tcs = node_stack.back().second;
        Cube cb = bounds_stack.back();
        Cube tb = child_bounds_for(cb, tcs);
        size_t tck = child(cur, tcs);

        if (tb.size > 1.f && insert_size > 1 && tb.size <= (float)insert_size && lex_le(position, tb.min)) {
            actual_update_size = execute_for_relevant_sectants(cb, pos_u32, insert_size, [&](U3 pit, U3 uit, uint8_t cs, const Cube &ctb) {
                U3 ctb_min = round_u3(ctb.min);
                uint32_t csz = as_u32(ctb.size);
                if (pit.x == ctb_min.x && pit.y == ctb_min.y && pit.z == ctb_min.z && uit.x == csz && uit.y == csz && uit.z == csz) {
                    updated = true;
                    tck = child(cur, cs);
                    if (nodes.get(cur).content == Content::Leaf || nodes.get(cur).content == Content::UniformLeaf) {
                        subdivide_leaf_to_nodes(cur, cs);
                        tck = child(cur, cs);
                    }
                    if (nodes.key_is_valid(tck)) {
                        deallocate_children_of(tck);
                        Node &t = nodes.get(tck);
                        t.content = Content::UniformLeaf;
                        t.bricks.assign(1, solid(tc));
                        t.occupied_bits = ~0ull;
                    } else {
                        uint32_t nk = (uint32_t)nodes.push(uniform_solid_node(tc));
                        child_mut(cur, cs) = nk;
                    }
                    modified_bottom.push_back(cs);
                }
            });
            break;
        }

        if (tb.size > 1.f && (tb.size > (float)brick_dim || nodes.key_is_valid(tck))) {
            if (nodes.key_is_valid(tck)) {
                node_stack.push_back({child(cur, tcs), sectant_for(tb, position)});
                bounds_stack.push_back(tb);
            } else {
                const Node &cn = nodes.get(cur);
                if (cn.content == Content::Leaf || cn.content == Content::UniformLeaf) {
                    bool target_match = false;
                    if (cn.content == Content::UniformLeaf) {
                        const Brick &b = cn.bricks[0];
                        if (b.kind == BrickKind::Solid) target_match = b.solid == tc;
                        else if (b.kind == BrickKind::Parted) {
                            auto mi = matrix_index_for(cb, round_u3(position), brick_dim);
                            target_match = b.parted[flat_projection(mi[0], mi[1], mi[2], brick_dim)] == tc;
                        }
                    } else {
                        const Brick &b = cn.bricks[tcs];
                        if (b.kind == BrickKind::Solid) target_match = b.solid == tc;
                        else if (b.kind == BrickKind::Parted) {
                            auto mi = matrix_index_for(tb, round_u3(position), brick_dim);
                            target_match = b.parted[flat_projection(mi[0], mi[1], mi[2], brick_dim)] == tc;
                        }
                    }
                    if (target_match || content_is_all(cn, tc)) break;
                    subdivide_leaf_to_nodes(cur, tcs);
                    node_stack.push_back({child(cur, tcs), sectant_for(tb, position)});
                    bounds_stack.push_back(tb);
                } else {
                    Node &n = nodes.get(cur);
                    if (n.content == Content::Nothing) {
                        n.content = Content::Internal;
                        n.occupied_bits = 0;
                    }
                    size_t nc = nodes.push(empty_node());
                    child_mut(cur, tcs) = (uint32_t)nc;
                    node_stack.push_back({nc, sectant_for(tb, position)});
                    bounds_stack.push_back(tb);
                }
            }
        } else {
            actual_update_size = execute_for_relevant_sectants(cb, pos_u32, insert_size, [&](U3 pit, U3 uit, uint8_t cs, const Cube &ctb) {
                updated |= leaf_update(overwrite, cur, cb, ctb, cs, pit, uit, tc);
                modified_bottom.push_back(cs);
            });
            break;
        }
    }

    if (!updated) return 0;
    bool simplifyable = auto_simplify;
    const std::vector<std::pair<size_t, uint8_t>> node_stack_clone = node_stack;  // insert.rs:329
    for (uint8_t mbs : modified_bottom) {
        size_t node_key = node_stack.back().first;
        uint8_t original = node_stack.back().second;
        Cube nbounds = bounds_stack.back();
        size_t ck = child(node_key, mbs);
        if (nodes.key_is_valid(ck)) {
            Cube cbounds = child_bounds_for(nbounds, mbs);
            node_stack.push_back({ck, sectant_for(cbounds, f3(std::fmax(position.x, cbounds.min.x),
                                                              std::fmax(position.y, cbounds.min.y),
                                                              std::fmax(position.z, cbounds.min.z)))});
            post_process_node_insert(node_stack, cbounds, actual_update_size, pos_u32, insert_size);
            node_stack.pop_back();
        } else {
            node_stack.back().second = mbs;
            post_process_node_insert(node_stack, nbounds, actual_update_size, pos_u32, insert_size);
            node_stack.back().second = original;
        }
        if (simplifyable) simplifyable &= simplify(ck, false);
    }
    while (!node_stack.empty()) {
        size_t node_key = node_stack.back().first;
        if (!nodes.key_is_valid(node_key)) {  // the reference `continue`s here without popping (never reached)
            node_stack.pop_back();
            bounds_stack.pop_back();
            continue;
        }
        post_process_node_insert(node_stack, bounds_stack.back(), actual_update_size, pos_u32, insert_size);
        if (simplifyable) simplifyable = simplify(node_key, false);
        node_stack.pop_back();
        bounds_stack.pop_back();
    }
    ++edit_seq;
    if (track_changes > 0) changes.push_back(Change{node_stack_clone, modified_bottom});  // insert.rs:401-404
    return 0;
}

bool BoxTree::simplify(size_t key, bool recursive) {  // src/boxtree/update/mod.rs:617-867
    if (!nodes.key_is_valid(key)) return false;
    ++edit_seq;
    Node &node = nodes.get(key);
    switch (node.content) {
        case Content::Nothing: return true;
        case Content::UniformLeaf: {
            Brick &b = node.bricks[0];
            if (b.kind == BrickKind::Empty) return true;
            if (b.kind == BrickKind::Solid) {
                if (points_to_empty(b.solid)) {
                    node.content = Content::Nothing;
                    node.bricks.clear();
                    node.has_children = false;
                    return true;
                }
                return false;
            }
            return brick_simplify(b);
        }
        case Content::Leaf: {
            bool simplified = false, uniform_solid = true, have_usv = false;
            uint32_t usv = 0;
            for (Brick &b : node.bricks) {
                simplified |= brick_simplify(b);
                if (uniform_solid) {
                    if (b.kind == BrickKind::Solid) {
                        if (have_usv) {
                            if (usv != b.solid) uniform_solid = false;
                        } else {
                            usv = b.solid;
                            have_usv = true;
                        }
                    } else {
                        uniform_solid = false;
                    }
                }
            }
            if (uniform_solid) {
                node.content = Content::UniformLeaf;
                node.bricks.assign(1, solid(usv));
                return true;
            }
            if (brick_dim == 1) return false;  // update/mod.rs:721-723 (even if bricks were simplified)
            size_t bd = brick_dim;
            std::vector<uint32_t> unified(bd * bd * bd, kEmpty32);
            bool uniform = true;
            float sbs = (float)brick_dim * 4.f;
            auto voxel_of = [&](size_t s, F3 pic) -> uint32_t {
                const Brick &b = node.bricks[s];
                if (b.kind == BrickKind::Empty) return kEmpty32;
                if (b.kind == BrickKind::Solid) return b.solid;
                return b.parted[flat_projection(as_usize(pic.x), as_usize(pic.y), as_usize(pic.z), bd)];
            };
            for (size_t x = 0; x < bd && uniform; ++x)
                for (size_t y = 0; y < bd && uniform; ++y)
                    for (size_t z = 0; z < bd && uniform; ++z) {
                        F3 cell_start = mul(f3((float)x, (float)y, (float)z), 4.f);
                        uint8_t rs = offset_sectant(cell_start, sbs);
                        F3 pic = sub(cell_start, mul(lut(rs), sbs));
                        uint32_t ref = voxel_of(rs, pic);
                        for (int cx = 0; cx < 4 && uniform; ++cx)
                            for (int cy = 0; cy < 4 && uniform; ++cy)
                                for (int cz = 0; cz < 4 && uniform; ++cz) {
                                    F3 p = add(cell_start, f3((float)cx, (float)cy, (float)cz));
                                    uint8_t s = offset_sectant(p, sbs);
                                    F3 pc = sub(p, mul(lut(s), sbs));
                                    uniform = uniform && (ref == voxel_of(s, pc));
                                }
                        if (uniform) unified[flat_projection(x, y, z, bd)] = ref;
                    }
            if (uniform) {
                node.content = Content::UniformLeaf;
                node.bricks.assign(1, parted(std::move(unified)));
                simplified = true;
            }
            return simplified;
        }
        case Content::Internal: {
            if (node.occupied_bits == 0 || !node.has_children) {
                node.content = Content::Nothing;
                return true;
            }
            std::array<uint32_t, kChildren> ck = node.children;
            if (recursive)
                for (uint32_t c : ck) simplify(c, true);
            // update/mod.rs:833-844 tests the *parent's* content for UniformLeaf(Solid); the parent is Internal,
            // so the collapse below never happens and the function returns false.
            for (size_t s = 1; s < kChildren; ++s) {
                size_t c0 = ck[0];
                const Node &self = nodes.get(key);
                bool parent_uniform_solid = self.content == Content::UniformLeaf && self.bricks[0].kind == BrickKind::Solid;
                if (!nodes.key_is_valid(c0) || !parent_uniform_solid || !compare_nodes(c0, ck[s])) return false;
            }
            nodes.swap(key, ck[0]);
            deallocate_children_of(key);
            nodes.get(key).has_children = false;
            return true;
        }
    }
    return false;
}

// ---------------------------------------------------------------------------------------------- MIP maps
// src/boxtree/mipmap.rs and the resampling functions of src/boxtree/iterate.rs:349-560. Albedo is packed
// r | g<<8 | b<<16 | a<<24 here; the reference's u32 arithmetic on Albedou32 wraps like release builds (in a debug
// build the reference panics on the subtraction in Posterize whenever a channel of the candidate is brighter).
struct Alb {
    uint32_t r, g, b, a;
};
static inline Alb alb_of(uint32_t c) { return Alb{c & 0xFFu, (c >> 8) & 0xFFu, (c >> 16) & 0xFFu, c >> 24}; }
static inline uint32_t alb_pack_u8(uint32_t r, uint32_t g, uint32_t b, uint32_t a) {
    return (r & 0xFFu) | ((g & 0xFFu) << 8) | ((b & 0xFFu) << 16) | ((a & 0xFFu) << 24);
}
// From<Albedou32> for Albedo: min(255) as u8
static inline uint32_t alb_pack(Alb v) {
    return alb_pack_u8(std::min(v.r, 255u), std::min(v.g, 255u), std::min(v.b, 255u), std::min(v.a, 255u));
}
static inline Alb alb_pow2(Alb v) { return Alb{v.r * v.r, v.g * v.g, v.b * v.b, v.a * v.a}; }
static inline Alb alb_add(Alb x, Alb y) { return Alb{x.r + y.r, x.g + y.g, x.b + y.b, x.a + y.a}; }
static inline Alb alb_sub(Alb x, Alb y) { return Alb{x.r - y.r, x.g - y.g, x.b - y.b, x.a - y.a}; }
static inline uint32_t round_u32(float f) { return as_u32(std::round(f)); }
static inline Alb alb_div(Alb v, uint32_t d) {  // Div<u32>: (x as f32 / d as f32).round() as u32
    const float fd = (float)d;
    return Alb{round_u32((float)v.r / fd), round_u32((float)v.g / fd), round_u32((float)v.b / fd),
               round_u32((float)v.a / fd)};
}
static inline Alb alb_sqrt(Alb v) {  // (x as f32).sqrt().round() as u32
    return Alb{round_u32(std::sqrt((float)v.r)), round_u32(std::sqrt((float)v.g)), round_u32(std::sqrt((float)v.b)),
               round_u32(std::sqrt((float)v.a))};
}
static inline float alb_length(Alb v) {
    return std::sqrt((float)(v.r * v.r + v.g * v.g + v.b * v.b + v.a * v.a));
}
// Albedo::distance_from, src/boxtree/detail.rs:62-69
static inline float alb_distance(uint32_t x, uint32_t y) {
    const Alb a = alb_of(x), b = alb_of(y);
    const float dr = (float)a.r - (float)b.r, dg = (float)a.g - (float)b.g, db = (float)a.b - (float)b.b,
                da = (float)a.a - (float)b.a;
    return std::sqrt(dr * dr + dg * dg + db * db + da * da);
}

// Process-wide MIP options (vhx_boxtree_set_mip_options; the library reads no environment): `direct` (tests) runs the
// leaf resampling through get_internal and the palette matching by a full scan, the direct restatements that
// leaf_value and mip_palette_match shortcut; `threads` caps the leaf-resampling workers (0 = up to 16)
std::atomic<int> g_mip_direct{0};
std::atomic<int> g_mip_threads{0};
static bool mip_generic() { return g_mip_direct.load(std::memory_order_relaxed) != 0; }

// MIPResamplingFunction::execute (iterate.rs:434-560). `sample` returns false for None. PointFilter and Posterize keep
// their groups in first-seen order where the reference iterates a std HashMap (random order per process): results
// that depend on that order (ties of the most frequent colour, a colour within the threshold of two groups) are not
// reproducible by the reference itself; this restatement resolves them in first-seen order, the last group of the
// highest count winning like Iterator::max_by_key.
// `sample` is a template parameter rather than a std::function: the samplers capture three references, beyond
// std::function's inline buffer, and the heap allocation per call serialised the parallel leaf resampling of
// recalculate_mips on the allocator (8 threads ran at the speed of one on a fresh process)
template <class Sample>
static bool mip_execute(const MipMethodCfg &m, U3 start, uint32_t size, const Sample &sample, uint32_t &out) {
    uint32_t c = 0;
    switch (m.kind) {
        case kBoxFilter: {
            bool any = false;
            int32_t count = 0;
            float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
            for (uint32_t x = start.x; x < start.x + size; ++x)
                for (uint32_t y = start.y; y < start.y + size; ++y)
                    for (uint32_t z = start.z; z < start.z + size; ++z) {
                        if (!sample(U3{x, y, z}, c)) continue;
                        const Alb a = alb_of(c);
                        const float r = (float)a.r, g = (float)a.g, b = (float)a.b, al = (float)a.a;
                        if (!any) {
                            any = true;
                            count = 1;
                            s0 = r * r, s1 = g * g, s2 = b * b, s3 = al * al;
                        } else {
                            count += 1;
                            s0 += r * r, s1 += g * g, s2 += b * b, s3 += al * al;
                        }
                    }
            if (!any) return false;
            const float n = (float)count;
            out = alb_pack_u8(as_u8(std::fmin(std::sqrt(s0 / n), 255.f)), as_u8(std::fmin(std::sqrt(s1 / n), 255.f)),
                              as_u8(std::fmin(std::sqrt(s2 / n), 255.f)), as_u8(std::fmin(std::sqrt(s3 / n), 255.f)));
            return true;
        }
        case kPointFilter:
        case kPointFilterBD: {
            std::vector<std::pair<uint32_t, uint32_t>> counts;  // (albedo, occurrences), first-seen order
            for (uint32_t x = start.x; x < start.x + size; ++x)
                for (uint32_t y = start.y; y < start.y + size; ++y)
                    for (uint32_t z = start.z; z < start.z + size; ++z) {
                        if (!sample(U3{x, y, z}, c)) continue;
                        auto it = std::find_if(counts.begin(), counts.end(), [&](const auto &e) { return e.first == c; });
                        if (it == counts.end())
                            counts.push_back({c, 1});
                        else
                            it->second += 1;
                    }
            if (counts.empty()) return false;
            size_t best = 0;
            for (size_t i = 1; i < counts.size(); ++i)
                if (counts[i].second >= counts[best].second) best = i;
            out = counts[best].first;
            return true;
        }
        default: {  // Posterize / PosterizeBD
            std::vector<std::pair<Alb, uint32_t>> groups;  // (sum of squared albedo, count)
            const float thr = m.thr * 255.f;
            for (uint32_t x = start.x; x < start.x + size; ++x)
                for (uint32_t y = start.y; y < start.y + size; ++y)
                    for (uint32_t z = start.z; z < start.z + size; ++z) {
                        if (!sample(U3{x, y, z}, c)) continue;
                        const Alb col = alb_of(c);
                        bool merged = false;
                        for (auto &g : groups) {
                            const Alb poster = alb_sqrt(alb_div(g.first, g.second));
                            if (alb_length(alb_sub(poster, col)) < thr) {
                                g.first = alb_add(g.first, alb_pow2(col));
                                g.second += 1;
                                merged = true;
                                break;
                            }
                        }
                        if (!merged) groups.push_back({alb_pow2(col), 1});
                    }
            if (groups.empty()) return false;
            size_t best = 0;
            for (size_t i = 1; i < groups.size(); ++i)
                if (groups[i].second >= groups[best].second) best = i;
            out = alb_pack(alb_sqrt(alb_div(groups[best].first, groups[best].second)));
            return true;
        }
    }
}

// NodeContent::pix_get_ref(..).albedo() (node.rs:335-373, mod.rs:81-88): the colour of a colour-carrying value
bool BoxTree::albedo_of(uint32_t v, uint32_t &albedo) const {
    if (!pix_color_is_some(v) || pix_color_index(v) >= color_palette.size()) return false;
    albedo = color_palette[pix_color_index(v)];
    return true;
}

void BoxTree::update_mip(size_t key, const Cube &nb, U3 position) {  // src/boxtree/mipmap.rs:42-338
    if (!mip_strategy.enabled) return;
    const Content content = nodes.get(key).content;
    if (content == Content::Nothing) return;
    if (content == Content::UniformLeaf) {
        nodes.get(key).mip = Brick{};  // a uniform leaf is equivalent to its MIP
        return;
    }
    uint32_t color = 0;
    if (mip_sample(key, nb, position, color)) mip_store(key, nb, position, color);
}

// mipmap.rs:42-270: the sampled colour of the MIP cell `position` falls in (Leaf / Internal nodes only)
bool BoxTree::mip_sample(size_t key, const Cube &nb, U3 position, uint32_t &color) const {
    const uint32_t bd = brick_dim;
    const size_t level = as_usize(std::log2(nb.size / (float)bd));
    const auto mit = mip_strategy.methods.find(level);
    const MipMethodCfg sampler = mit != mip_strategy.methods.end() ? mit->second : MipMethodCfg{kBoxFilter, 0.f};
    const bool dominant_bottom = mit != mip_strategy.methods.end() && mit->second.kind == kPointFilterBD;

    const Content content = nodes.get(key).content;
    U3 start{0, 0, 0};
    uint32_t ssize = 0;
    if (content == Content::Leaf) {
        ssize = std::min(as_u32(nb.size) / bd, bd * 4u);
        auto st = [&](uint32_t p) {
            const uint32_t q = (p - p % ssize) * 4u * bd;
            return as_u32(std::round(std::floor((float)q / nb.size)));
        };
        start = U3{st(position.x), st(position.y), st(position.z)};
    } else if (dominant_bottom) {
        ssize = as_u32(nb.size) / bd;
        start = U3{position.x - position.x % ssize, position.y - position.y % ssize, position.z - position.z % ssize};
    } else {
        ssize = 4;
        const F3 pib = sub(from_u3(position), nb.min);
        const F3 v1 = divs(mul(mul(pib, 4.f), (float)bd), nb.size);
        const U3 v2 = round_u3(floor3(v1));
        start = U3{v2.x - v2.x % 4u, v2.y - v2.y % 4u, v2.z - v2.z % 4u};
    }

    if (content == Content::Leaf && !mip_generic()) {
        const Node &n = nodes.get(key);
        return mip_execute(sampler, start, ssize, [&](U3 pos, uint32_t &c) { return albedo_of(leaf_value(n, nb, pos), c); },
                           color);
    }
    if (content == Content::Leaf || dominant_bottom) {
        return mip_execute(sampler, start, ssize, [&](U3 pos, uint32_t &c) {
            return albedo_of(get_internal(key, nb, pos), c);
        }, color);
    } else {
        const float mip_edge = (float)(bd * 4u);
        return mip_execute(sampler, start, ssize, [&](U3 pos, uint32_t &c) {
            const uint8_t cs = offset_sectant(from_u3(pos), mip_edge);
            const size_t ck = child(key, cs);
            if (ck == (size_t)kEmpty32 || !nodes.key_is_valid(ck)) return false;
            const F3 pic = sub(from_u3(pos), mul(lut(cs), mip_edge));
            const size_t px = as_usize(pic.x), py = as_usize(pic.y), pz = as_usize(pic.z);
            const Brick &m = nodes.get(ck).mip;
            switch (m.kind) {
                case BrickKind::Empty: return false;
                case BrickKind::Solid: return albedo_of(m.solid, c);
                default:  // a sample outside the child's MIP (the reference would index out of bounds) reads nothing
                    if (px >= bd || py >= bd || pz >= bd) return false;
                    return albedo_of(m.parted[flat_projection(px, py, pz, bd)], c);
            }
        }, color);
    }
}

// get_internal(key, nb, pos) (src/boxtree/mod.rs:247-317) for a Leaf node `n` with bounds nb: every quantity is an
// integer below 2^24 and every cube size a power of two, so cube_contains, sectant_for (offset_sectant, clamped to 3),
// child_bounds_for and matrix_index_for reduce to integer compares, divisions and remainders with the same results
uint32_t BoxTree::leaf_value(const Node &n, const Cube &nb, U3 pos) const {
    const int64_t size = (int64_t)nb.size, sub = size / 4, bd = brick_dim;
    const int64_t rx = (int64_t)pos.x - (int64_t)nb.min.x, ry = (int64_t)pos.y - (int64_t)nb.min.y,
                  rz = (int64_t)pos.z - (int64_t)nb.min.z;
    if (rx < 0 || ry < 0 || rz < 0 || rx >= size || ry >= size || rz >= size) return kEmpty32;
    const int64_t sx = std::min<int64_t>(rx / sub, 3), sy = std::min<int64_t>(ry / sub, 3), sz = std::min<int64_t>(rz / sub, 3);
    const Brick &b = n.bricks[(size_t)(sx + sy * 4 + sz * 16)];
    if (b.kind == BrickKind::Empty) return kEmpty32;
    if (b.kind == BrickKind::Solid) return b.solid;
    const size_t mx = (size_t)((rx - sx * sub) * bd / sub), my = (size_t)((ry - sy * sub) * bd / sub),
                 mz = (size_t)((rz - sz * sub) * bd / sub);
    const uint32_t v = b.parted[flat_projection(mx, my, mz, brick_dim)];
    return points_to_empty(v) ? kEmpty32 : v;
}

uint32_t BoxTree::mip_palette_match(uint32_t color, float thr) {
    uint32_t tb;
    std::memcpy(&tb, &thr, 4);
    const uint64_t key = ((uint64_t)tb << 32) | color;
    // neighbouring MIP cells mostly carry the same colour: the last found match answers them without a map lookup
    if (key == mip_last_key_ && mip_last_index_ != UINT32_MAX) return mip_last_index_;
    MipMatch &m = mip_match_.try_emplace(key, MipMatch{UINT32_MAX, 0}).first->second;
    if (m.index != UINT32_MAX) return m.index;
    if (m.checked > color_palette.size()) m.checked = 0;  // (the palette never shrinks; defensive)
    for (size_t i = m.checked; i < color_palette.size(); ++i)
        if (alb_distance(color, color_palette[i]) < thr) {
            m.index = (uint32_t)i;
            break;
        }
    if (m.index == UINT32_MAX) m.checked = (uint32_t)color_palette.size();
    mip_last_key_ = key;
    mip_last_index_ = m.index;
    return m.index;
}

// mipmap.rs:272-338: the sampled colour matched against the palette (first entry within the level's threshold) or
// added to it, stored in the node's MIP brick
void BoxTree::mip_store(size_t key, const Cube &nb, U3 position, uint32_t color) {
    const uint32_t bd = brick_dim;
    const size_t level = as_usize(std::log2(nb.size / (float)bd));
    uint32_t entry;
    const auto tit = mip_strategy.color_thresholds.find(level);
    bool similar = false;
    if (tit != mip_strategy.color_thresholds.end()) {
        const float thr = tit->second * 255.f;
        if (mip_generic()) {
            for (size_t i = 0; i < color_palette.size(); ++i)
                if (alb_distance(color, color_palette[i]) < thr) {
                    entry = pix_visual((uint32_t)i);
                    similar = true;
                    break;
                }
        } else {
            const uint32_t i = mip_palette_match(color, thr);
            if (i != UINT32_MAX) {
                entry = pix_visual(i);
                similar = true;
            }
        }
    }
    if (!similar) entry = add_to_palette(Entry{VHX_ENTRY_VISUAL, color, 0});

    const auto mi = matrix_index_for(nb, position, bd);
    if (mi[0] >= bd || mi[1] >= bd || mi[2] >= bd) return;  // a position outside the node (the reference panics)
    const size_t f = flat_projection(mi[0], mi[1], mi[2], bd);
    Brick &mip = nodes.get(key).mip;
    const size_t n3 = (size_t)bd * bd * bd;
    if (mip.kind == BrickKind::Empty) {
        mip.parted.assign(n3, kEmpty32);
    } else if (mip.kind == BrickKind::Solid) {
        mip.parted.assign(n3, mip.solid);
    }
    mip.kind = BrickKind::Parted;
    mip.parted[f] = entry;
}

// the bd^3 positions recalculate_mip visits in a node, in its order (mipmap.rs:619-631)
static void mip_positions(const Cube &nb, uint32_t brick_dim, std::vector<U3> &out) {
    out.clear();
    const float bd = (float)brick_dim;
    for (uint32_t x = 0; x < brick_dim; ++x)
        for (uint32_t y = 0; y < brick_dim; ++y)
            for (uint32_t z = 0; z < brick_dim; ++z) {
                const F3 off = divs(mul(f3((float)x, (float)y, (float)z), nb.size), bd);
                const F3 pos = add(nb.min, f3(std::round(off.x), std::round(off.y), std::round(off.z)));
                out.push_back(round_u3(pos));
            }
}

void BoxTree::recalculate_mip(size_t key, const Cube &nb) {  // mipmap.rs:613-633
    if (!mip_strategy.enabled) return;
    nodes.get(key).mip = Brick{};
    std::vector<U3> positions;
    mip_positions(nb, brick_dim, positions);
    for (const U3 &p : positions) update_mip(key, nb, p);
}

void BoxTree::recalculate_mips() {  // mipmap.rs:536-586: depth first, children before their parent
    struct Item {
        size_t key;
        Cube bounds;
        uint32_t target;
    };
    // 1. the visiting order (post-order, children before their parent)
    std::vector<std::pair<size_t, Cube>> order;
    std::vector<Item> stack{{0, Cube{f3(0.f, 0.f, 0.f), (float)boxtree_size}, 0}};
    while (!stack.empty()) {
        Item &it = stack.back();
        if (it.target >= kChildren) {
            order.push_back({it.key, it.bounds});
            stack.pop_back();
            if (!stack.empty()) stack.back().target += 1;
            continue;
        }
        switch (nodes.get(it.key).content) {
            case Content::Internal: {
                const size_t ck = child(it.key, (uint8_t)it.target);
                if (nodes.key_is_valid(ck) && nodes.get(ck).content != Content::Nothing) {
                    const Cube cb = child_bounds_for(it.bounds, (uint8_t)it.target);
                    stack.push_back(Item{ck, cb, 0});
                } else {
                    it.target += 1;
                }
                break;
            }
            case Content::Nothing:  // the reference panics (unreachable); only an empty root gets here
                stack.pop_back();
                if (!stack.empty()) stack.back().target += 1;
                break;
            default: it.target = kChildren; break;
        }
    }
    if (!mip_strategy.enabled) return;
#ifndef VHX_MIP_TIMING
#define VHX_MIP_TIMING 0  // a diagnostic build prints the phases of recalculate_mips
#endif
    const bool tm = VHX_MIP_TIMING != 0;
    auto t0 = std::chrono::steady_clock::now();
    auto lap = [&](const char *what) {
        if (!tm) return;
        const auto t1 = std::chrono::steady_clock::now();
        fprintf(stderr, "[mips] %-28s %.3f s\n", what, std::chrono::duration<double>(t1 - t0).count());
        t0 = t1;
    };
    lap("order");
    // 2. the leaves' resampling reads their bricks only (never a MIP, never a palette entry added below), so it runs
    //    for every leaf up front, spread over threads
    const uint32_t n3 = brick_dim * brick_dim * brick_dim;
    std::vector<size_t> leaf_of(order.size(), SIZE_MAX);
    size_t nleaves = 0;
    for (size_t i = 0; i < order.size(); ++i)
        if (nodes.get(order[i].first).content == Content::Leaf) leaf_of[i] = nleaves++;
    std::vector<uint32_t> colors((size_t)nleaves * n3);
    std::vector<uint8_t> sampled((size_t)nleaves * n3);
    {
        std::vector<size_t> leaves;
        leaves.reserve(nleaves);
        for (size_t i = 0; i < order.size(); ++i)
            if (leaf_of[i] != SIZE_MAX) leaves.push_back(i);
        std::atomic<size_t> next{0};
        auto work = [&]() {
            std::vector<U3> positions;
            const auto w0 = std::chrono::steady_clock::now();
            size_t mine = 0;
            struct Report {
                bool on;
                std::chrono::steady_clock::time_point w0;
                size_t *mine;
                ~Report() {
                    timespec ts;
                    clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
                    if (on) fprintf(stderr, "[mips]   worker: %zu leaves in %.3f s (thread cpu %.3f s)\n", *mine,
                                    std::chrono::duration<double>(std::chrono::steady_clock::now() - w0).count(),
                                    ts.tv_sec + 1e-9 * ts.tv_nsec);
                }
            } rep{tm, w0, &mine};
            // runs of 64 leaves per grab: each thread writes its own contiguous stretch of `colors` / `sampled` (one
            // leaf per grab put neighbouring leaves' results, written by different threads, on shared cache lines:
            // 8 threads ran slower than one)
            constexpr size_t RUN = 64;
            for (size_t j0; (j0 = next.fetch_add(RUN)) < leaves.size();)
                for (size_t j = j0; j < std::min(j0 + RUN, leaves.size()); ++j, ++mine) {
                    const auto &[key, nb] = order[leaves[j]];
                    mip_positions(nb, brick_dim, positions);
                    for (uint32_t p = 0; p < n3; ++p)
                        sampled[j * n3 + p] = mip_sample(key, nb, positions[p], colors[j * n3 + p]) ? 1 : 0;
                }
        };
        unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
        if (const int t = g_mip_threads.load(std::memory_order_relaxed); t > 0) nt = (unsigned)t;
        std::vector<std::thread> pool;
        for (unsigned t = 1; t < nt && (size_t)t * 64 < leaves.size(); ++t) {
            try {  // a thread that cannot be created is missing: the shared queue is finished by the others
                pool.emplace_back(work);
            } catch (const std::system_error &) {
                break;
            }
        }
        work();
        for (auto &th : pool) th.join();
    }
    lap("leaf resampling");
    // 3. palette matching and stores in the reference's order (the palette grows as it goes, and a later match takes
    //    the first entry within the threshold); other nodes resample their children's finished MIPs here
    std::vector<U3> positions;
    for (size_t i = 0; i < order.size(); ++i) {
        const auto &[key, nb] = order[i];
        if (leaf_of[i] == SIZE_MAX) {
            recalculate_mip(key, nb);
            continue;
        }
        nodes.get(key).mip = Brick{};
        mip_positions(nb, brick_dim, positions);
        const size_t base = leaf_of[i] * n3;
        for (uint32_t p = 0; p < n3; ++p)
            if (sampled[base + p]) mip_store(key, nb, positions[p], colors[base + p]);
    }
    lap("stores + upper levels");
}

void BoxTree::switch_albedo_mip_maps(bool enabled) {  // mipmap.rs:588-609
    const bool before = mip_strategy.enabled;
    mip_strategy.enabled = enabled;
    if (enabled && before != enabled && nodes.get(0).content != Content::Nothing) recalculate_mips();
}

uint32_t BoxTree::sample_root_mip(uint8_t sectant, U3 position) const {  // mipmap.rs:635-668
    const size_t key = sectant >= kChildren ? 0 : child(0, sectant);
    if (!nodes.key_is_valid(key)) return kEmpty32;
    const Brick &m = nodes.get(key).mip;
    switch (m.kind) {
        case BrickKind::Empty: return kEmpty32;
        case BrickKind::Solid: return m.solid;
        default: return m.parted[flat_projection(position.x, position.y, position.z, brick_dim)];
    }
}


}  // namespace vhx
