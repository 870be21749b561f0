// Flattening of the host BoxTree into the vhx_tree_desc layout, bulk procedural-scene builder, and the C ABI of
// include/vhx_boxtree.h.
//
// The flattened layout replaces the reference's streamed GPU buffers (BoxTreeRenderData,
// src/raytracing/bevy/types.rs:203-256, filled by add_node/add_brick, src/raytracing/bevy/streaming/cache.rs:226-455,
// 608-716) with a full-residency image: nodes breadth-first from the root, bricks and solid values in node order.
//
// Bulk builder: a tree filled only through BoxTree::insert of single voxels is canonical — insert never simplifies
// (insert.rs:371-373 calls simplify on the invalid bottom child key, which returns false, so `simplifyable` drops
// to false before any node is touched), leaf nodes are exactly the nodes of edge 4*brick_dim, every brick that
// received a voxel is Parted, and occupied_bits has a bit per non-empty child (post_process_node_insert,
// insert.rs:428-449). vhx_scene_build writes that canonical image directly; tests check it buffer-equal against
// vhx_scene_insert + vhx_boxtree_flatten.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstring>
#include <deque>
#include <memory>
#include <new>
#include <system_error>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../include/vhx_boxtree.h"
#include "boxtree.hpp"

using namespace vhx;

struct vhx_flat {
    uint32_t size = 0, brick_dim = 0;
    std::vector<uint32_t> node_type;
    std::vector<uint64_t> node_ocbits;
    std::vector<uint32_t> node_children;
    std::unique_ptr<uint32_t[]> voxels;  // uninitialised storage (GB scale)
    uint64_t voxel_count = 0;
    uint32_t brick_count = 0;
    std::vector<uint32_t> solid_values;
    std::vector<uint32_t> color_palette;
    std::vector<uint32_t> data_palette;
    // per node: its MIP brick descriptor (same encoding as a leaf's child entry; node_mips of
    // src/raytracing/bevy/types.rs:245-247); empty unless the tree's MIP maps are enabled
    std::vector<uint32_t> node_mips;
};

// ---------------------------------------------------------------------------------------------- parallel helper
template <class F>
static void parallel_for(int64_t n, int threads, F &&f) {
    if (threads <= 0) threads = (int)std::max(1u, std::thread::hardware_concurrency());
    threads = (int)std::min<int64_t>(threads, std::max<int64_t>(n, 1));
    if (threads <= 1) {
        for (int64_t i = 0; i < n; ++i) f(i);
        return;
    }
    std::atomic<int64_t> next{0};
    auto worker = [&] {
        for (;;) {
            int64_t i = next.fetch_add(1);
            if (i >= n) break;
            f(i);
        }
    };
    // the calling thread is one of the workers; a helper that cannot be created (std::system_error) is missing and the
    // shared counter lets the others finish, so no exception crosses the C ABI
    std::vector<std::thread> pool;
    for (int t = 1; t < threads; ++t) {
        try {
            pool.emplace_back(worker);
        } catch (const std::system_error &) {
            break;
        }
    }
    worker();
    for (auto &th : pool) th.join();
}

// ---------------------------------------------------------------------------------------------- scenes
static inline uint32_t rgba(uint32_t r, uint32_t g, uint32_t b, uint32_t a) {
    return (r & 0xFFu) | ((g & 0xFFu) << 8) | ((b & 0xFFu) << 16) | ((a & 0xFFu) << 24);
}
static inline uint32_t u8_of(float f) {  // Rust `as u8` on f32 (saturating)
    if (std::isnan(f) || f <= 0.f) return 0;
    if (f >= 255.f) return 255;
    return (uint32_t)f;
}
static inline uint64_t splitmix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

struct Scene {
    uint32_t id, S;
    uint64_t seed;
    uint32_t extent;  // voxels are only set inside [0, extent)^3
    // value-noise heightfield cache (per (x,z) column), built lazily for VHX_SCENE_HEIGHTFIELD
    std::vector<uint16_t> height;

    // returns packed albedo, 0 = no voxel
    inline uint32_t voxel(uint32_t x, uint32_t y, uint32_t z) const {
        const uint32_t q = S / 4, h = S / 2;
        switch (id) {
            case VHX_SCENE_LATTICE_CUBE: {  // examples/gpu_render.rs:57-82
                bool set = ((x < q || y < q || z < q) && (0 == x % 2 && 0 == y % 4 && 0 == z % 2)) ||
                           (h <= x && h <= y && h <= z);
                if (!set) return 0;
                uint32_t r = (0 == x % q) ? (uint32_t)((float)x / (float)S * 255.f) : 128u;
                uint32_t g = (0 == y % q) ? (uint32_t)((float)y / (float)S * 255.f) : 128u;
                uint32_t b = (0 == z % q) ? (uint32_t)((float)z / (float)S * 255.f) : 128u;
                return rgba(r, g, b, 255);
            }
            case VHX_SCENE_BENCH_REGION: {  // benches/performance.rs:13-26, Albedo::from(0x00ABCDEF)
                if (x >= 100 || y >= 100 || z >= 100) return 0;
                bool set = x < q || y < q || z < q || (h <= x && h <= y && h <= z);
                return set ? rgba(0x00, 0xAB, 0xCD, 0xEF) : 0;
            }
            case VHX_SCENE_LATTICE: {  // src/raytracing/tests.rs:777-789
                bool set = (x < q || y < q || z < q) && (0 == x % 2 && 0 == y % 4 && 0 == z % 2);
                if (!set) return 0;
                return rgba(u8_of(255.f * (float)x / (float)S), u8_of(255.f * (float)y / (float)S),
                            u8_of(255.f * (float)z / (float)S), 255);
            }
            case VHX_SCENE_CUBE: {  // src/raytracing/tests.rs:736-748
                if (!(h <= x && h <= y && h <= z)) return 0;
                return rgba(u8_of(255.f * (float)x / (float)S), u8_of(255.f * (float)y / (float)S),
                            u8_of(255.f * (float)z / (float)S), 255);
            }
            case VHX_SCENE_BOUNDARY: {  // src/raytracing/tests.rs:692-703
                bool set = ((x < q || y < q || z < q) && (0 == x % 2 && 0 == y % 4 && 0 == z % 2)) ||
                           (h <= x && h <= y && h <= z);
                if (!set) return 0;
                return rgba(u8_of(255.f * (float)(x % 6) / 6.0f), u8_of(255.f * (float)(y % 6) / 6.0f),
                            u8_of(255.f * (float)(z % 6) / 6.0f), 255);
            }
            case VHX_SCENE_HEIGHTFIELD: {
                uint32_t hh = height[(size_t)x * S + z];
                if (y > hh) return 0;
                if (y + 2 < hh) return rgba(110, 84, 60, 255);               // soil
                if (hh > (S * 3) / 8) return rgba(235, 235, 240, 255);       // snow caps
                return rgba(70, 140 + (hh % 5) * 10, 60, 255);               // grass bands
            }
            default: return 0;
        }
    }

    void prepare() {
        extent = id == VHX_SCENE_BENCH_REGION ? std::min(S, 100u) : S;
        if (id != VHX_SCENE_HEIGHTFIELD) return;
        // seeded 4-octave value noise, height in [S/16, S/16 + S/4)
        height.assign((size_t)S * S, 0);
        auto lattice = [&](int64_t ix, int64_t iz, int oct) {
            uint64_t k = splitmix(seed ^ splitmix((uint64_t)ix * 0x9E37u + (uint64_t)oct * 0x1234567ull) ^
                                  splitmix((uint64_t)iz * 0x85EBCA77ull));
            return (float)(k >> 40) / (float)(1ull << 24);
        };
        auto smooth = [](float t) { return t * t * (3.f - 2.f * t); };
        for (uint32_t x = 0; x < S; ++x)
            for (uint32_t z = 0; z < S; ++z) {
                float n = 0.f, amp = 0.5f, cell = (float)std::max(4u, S / 4);
                for (int o = 0; o < 4; ++o) {
                    float fx = (float)x / cell, fz = (float)z / cell;
                    int64_t ix = (int64_t)std::floor(fx), iz = (int64_t)std::floor(fz);
                    float tx = smooth(fx - (float)ix), tz = smooth(fz - (float)iz);
                    float a = lattice(ix, iz, o), b = lattice(ix + 1, iz, o), c = lattice(ix, iz + 1, o),
                          d = lattice(ix + 1, iz + 1, o);
                    float v = (a + (b - a) * tx) + ((c + (d - c) * tx) - (a + (b - a) * tx)) * tz;
                    n += v * amp;
                    amp *= 0.5f;
                    cell = std::max(1.f, cell / 2.f);
                }
                height[(size_t)x * S + z] = (uint16_t)std::min<float>((float)(S - 1), (float)(S / 16) + n * (float)(S / 4));
            }
    }
};

static bool scene_valid(uint32_t id) { return id >= VHX_SCENE_LATTICE_CUBE && id <= VHX_SCENE_HEIGHTFIELD; }

// ---------------------------------------------------------------------------------------------- flatten
static uint32_t brick_desc(const Brick &b, vhx_flat &f, std::vector<const std::vector<uint32_t> *> &parted,
                           std::unordered_map<uint32_t, uint32_t> &solid_index) {
    switch (b.kind) {
        case BrickKind::Empty: return VHX_EMPTY;
        case BrickKind::Solid: {
            auto it = solid_index.find(b.solid);
            uint32_t idx;
            if (it == solid_index.end()) {
                idx = (uint32_t)f.solid_values.size();
                solid_index.emplace(b.solid, idx);
                f.solid_values.push_back(b.solid);
            } else {
                idx = it->second;
            }
            return VHX_SOLID_BIT | idx;
        }
        default:
            parted.push_back(&b.parted);
            return (uint32_t)(parted.size() - 1);
    }
}

// max_depth: nodes deeper than this (root = depth 0) are left out; their parent's child entries are VHX_EMPTY while its
// occupancy bits stay, so a MIP-enabled trace shows the parent's MIP there (the WGSL's stand-in for a child that is
// not resident, viewport_render.wgsl:438-454). MIP bricks are numbered with the bricks, after the node's own.
static vhx_flat *flatten_tree(const BoxTree &t, uint32_t max_depth = 0xFFFFFFFFu, bool with_mips = false) {
    auto *f = new vhx_flat();
    f->size = t.boxtree_size;
    f->brick_dim = t.brick_dim;
    std::unordered_map<size_t, uint32_t> index;  // pool key -> BFS index
    std::deque<size_t> queue;
    std::vector<const std::vector<uint32_t> *> parted;
    std::unordered_map<uint32_t, uint32_t> solid_index;
    std::vector<uint32_t> depth{0};  // by BFS index
    index.emplace(0, 0);
    queue.push_back(0);
    while (!queue.empty()) {
        size_t key = queue.front();
        queue.pop_front();
        const Node &n = t.nodes.get(key);
        uint32_t idx = (uint32_t)f->node_type.size();
        uint32_t type = n.content == Content::Nothing   ? VHX_NODE_NOTHING
                        : n.content == Content::Internal ? VHX_NODE_INTERNAL
                        : n.content == Content::Leaf     ? VHX_NODE_LEAF
                                                         : VHX_NODE_UNIFORM_LEAF;
        f->node_type.push_back(type);
        f->node_ocbits.push_back(n.occupied_bits);
        f->node_children.resize((size_t)(idx + 1) * 64, VHX_EMPTY);
        uint32_t *ch = &f->node_children[(size_t)idx * 64];
        if (n.content == Content::Internal && n.has_children && depth[idx] < max_depth) {
            for (int s = 0; s < 64; ++s) {
                size_t c = n.children[s];
                if (!t.nodes.key_is_valid(c)) continue;  // freed / missing child: traced as empty
                auto it = index.find(c);
                if (it == index.end()) {
                    uint32_t ni = (uint32_t)index.size();
                    index.emplace(c, ni);
                    queue.push_back(c);
                    depth.push_back(depth[idx] + 1);
                    ch[s] = ni;
                } else {
                    ch[s] = it->second;
                }
            }
        } else if (n.content == Content::Leaf) {
            for (int s = 0; s < 64; ++s) ch[s] = brick_desc(n.bricks[s], *f, parted, solid_index);
        } else if (n.content == Content::UniformLeaf) {
            ch[0] = brick_desc(n.bricks[0], *f, parted, solid_index);
        }
        if (with_mips) f->node_mips.push_back(brick_desc(n.mip, *f, parted, solid_index));
    }
    size_t n3 = (size_t)t.brick_dim * t.brick_dim * t.brick_dim;
    f->brick_count = (uint32_t)parted.size();
    f->voxel_count = (uint64_t)parted.size() * n3;
    f->voxels.reset(new uint32_t[std::max<uint64_t>(f->voxel_count, 1)]);
    for (size_t i = 0; i < parted.size(); ++i) std::memcpy(&f->voxels[i * n3], parted[i]->data(), n3 * 4);
    f->color_palette = t.color_palette;
    f->data_palette = t.data_palette;
    return f;
}

// A BoxTree holding a flattened image's nodes, bricks and palettes (pool key = breadth-first index, so the depth-first
// child order and therefore the MIP palette growth are those of the tree the image came from). Occlusion bits and the
// insert bookkeeping are not restored: the tree only serves recalculate_mips + flatten_tree inside this file.
static BoxTree *tree_of_flat(const vhx_flat &f) {
    BoxTree *t = nullptr;
    if (BoxTree::create(f.size, f.brick_dim, &t) != 0) return nullptr;
    const size_t n3 = (size_t)f.brick_dim * f.brick_dim * f.brick_dim;
    auto brick_of = [&](uint32_t desc) {
        Brick b;
        if (desc == VHX_EMPTY) return b;
        if (desc & VHX_SOLID_BIT) {
            b.kind = BrickKind::Solid;
            b.solid = f.solid_values[desc & ~VHX_SOLID_BIT];
        } else {
            b.kind = BrickKind::Parted;
            b.parted.assign(&f.voxels[(size_t)desc * n3], &f.voxels[(size_t)desc * n3] + n3);
        }
        return b;
    };
    for (size_t i = 0; i < f.node_type.size(); ++i) {
        Node n;
        const uint32_t *ch = &f.node_children[i * 64];
        n.occupied_bits = f.node_ocbits[i];
        switch (f.node_type[i]) {
            case VHX_NODE_INTERNAL:
                n.content = Content::Internal;
                n.has_children = true;
                for (int s = 0; s < 64; ++s) n.children[s] = ch[s] == VHX_EMPTY ? kEmpty32 : ch[s];
                break;
            case VHX_NODE_LEAF:
                n.content = Content::Leaf;
                for (int s = 0; s < 64; ++s) n.bricks.push_back(brick_of(ch[s]));
                break;
            case VHX_NODE_UNIFORM_LEAF:
                n.content = Content::UniformLeaf;
                n.bricks.push_back(brick_of(ch[0]));
                break;
            default: n.content = Content::Nothing; break;
        }
        if (i == 0) {
            t->nodes.get(0) = std::move(n);
        } else if (t->nodes.push(std::move(n)) != i) {
            delete t;
            return nullptr;
        }
    }
    for (uint32_t c : f.color_palette) t->add_to_palette(Entry{VHX_ENTRY_VISUAL, c, 0});
    for (uint32_t d : f.data_palette) t->add_to_palette(Entry{VHX_ENTRY_INFORMATIVE, 0, d});
    if (t->color_palette != f.color_palette || t->data_palette != f.data_palette) {
        delete t;
        return nullptr;
    }
    return t;
}

// ---------------------------------------------------------------------------------------------- bulk builder
static int build_scene(uint32_t scene_id, uint32_t S, uint32_t bd, uint64_t seed, int threads, vhx_flat **out) {
    BoxTree *probe = nullptr;
    int rc = BoxTree::create(S, bd, &probe);  // same validity rules as BoxTree::new
    if (rc != 0) return rc;
    delete probe;
    Scene sc{scene_id, S, seed, S, {}};
    sc.prepare();
    const uint32_t L = 4 * bd;         // leaf node edge
    const uint32_t nl = S / L;         // leaf nodes per axis = 4^D
    uint32_t D = 0;
    while ((1u << (2 * D)) < nl) ++D;  // nl == 4^D
    const uint64_t nleaf = 1ull << (6 * D);

    // 1) palette in first-appearance order of the reference insert loop (x outer, y, z inner)
    std::vector<std::vector<uint32_t>> slab_colors(sc.extent);
    parallel_for(sc.extent, threads, [&](int64_t x) {
        std::unordered_set<uint32_t> seen;
        uint32_t last = 0;
        for (uint32_t y = 0; y < sc.extent; ++y)
            for (uint32_t z = 0; z < sc.extent; ++z) {
                uint32_t c = sc.voxel((uint32_t)x, y, z);
                if (c == 0 || c == last) continue;
                last = c;
                if (seen.insert(c).second) slab_colors[x].push_back(c);
            }
    });
    auto *f = new vhx_flat();
    f->size = S;
    f->brick_dim = bd;
    std::unordered_map<uint32_t, uint32_t> color_index;
    for (auto &sl : slab_colors)
        for (uint32_t c : sl)
            if (color_index.emplace(c, (uint32_t)f->color_palette.size()).second) f->color_palette.push_back(c);
    slab_colors.clear();

    // leaf path code -> leaf coordinates (digit i of the code = sectant taken at depth i)
    auto leaf_coord = [&](uint64_t code, uint32_t &lx, uint32_t &ly, uint32_t &lz) {
        lx = ly = lz = 0;
        for (uint32_t i = 0; i < D; ++i) {
            uint32_t d = (uint32_t)((code >> (6 * (D - 1 - i))) & 63u);
            lx = lx * 4 + (d & 3u);
            ly = ly * 4 + ((d >> 2) & 3u);
            lz = lz * 4 + (d >> 4);
        }
    };
    // 2) brick masks of every leaf node
    std::vector<uint64_t> leaf_mask(nleaf, 0);
    parallel_for((int64_t)nleaf, threads, [&](int64_t code) {
        uint32_t lx, ly, lz;
        leaf_coord((uint64_t)code, lx, ly, lz);
        uint32_t x0 = lx * L, y0 = ly * L, z0 = lz * L;
        if (x0 >= sc.extent || y0 >= sc.extent || z0 >= sc.extent) return;
        uint64_t m = 0;
        for (uint32_t s = 0; s < 64; ++s) {
            uint32_t bx = x0 + (s & 3u) * bd, by = y0 + ((s >> 2) & 3u) * bd, bz = z0 + (s >> 4) * bd;
            bool any = false;
            for (uint32_t x = bx; x < bx + bd && !any; ++x)
                for (uint32_t y = by; y < by + bd && !any; ++y)
                    for (uint32_t z = bz; z < bz + bd && !any; ++z) any = sc.voxel(x, y, z) != 0;
            if (any) m |= 1ull << s;
        }
        leaf_mask[code] = m;
    });
    // 3) presence per level (level D = leaves), BFS numbering level by level in path order
    std::vector<std::vector<uint64_t>> occ(D + 1);  // occupancy bits of every possible node per level
    occ[D] = leaf_mask;
    for (int lv = (int)D - 1; lv >= 0; --lv) {
        occ[lv].assign(1ull << (6 * lv), 0);
        for (uint64_t c = 0; c < occ[lv + 1].size(); ++c)
            if (occ[lv + 1][c]) occ[lv][c >> 6] |= 1ull << (c & 63);
    }
    std::vector<std::vector<uint32_t>> bfs(D + 1);  // BFS index of each present node per level
    uint32_t next = 0;
    for (uint32_t lv = 0; lv <= D; ++lv) {
        bfs[lv].assign(occ[lv].size(), VHX_EMPTY);
        for (uint64_t c = 0; c < occ[lv].size(); ++c)
            if (occ[lv][c] || (lv == 0)) bfs[lv][c] = next++;
    }
    const uint32_t node_count = next;
    f->node_type.assign(node_count, VHX_NODE_INTERNAL);
    f->node_ocbits.assign(node_count, 0);
    f->node_children.assign((size_t)node_count * 64, VHX_EMPTY);
    for (uint32_t lv = 0; lv <= D; ++lv)
        for (uint64_t c = 0; c < occ[lv].size(); ++c) {
            uint32_t i = bfs[lv][c];
            if (i == VHX_EMPTY) continue;
            f->node_ocbits[i] = occ[lv][c];
            if (lv < D) {
                f->node_type[i] = occ[lv][c] ? VHX_NODE_INTERNAL : VHX_NODE_NOTHING;
                for (uint32_t s = 0; s < 64; ++s) f->node_children[(size_t)i * 64 + s] = bfs[lv + 1][(c << 6) | s];
            } else {
                f->node_type[i] = occ[lv][c] ? VHX_NODE_LEAF : VHX_NODE_NOTHING;
            }
        }
    // 4) bricks numbered in (leaf BFS order, sectant) order; fill voxels
    std::vector<uint64_t> leaf_first(nleaf + 1, 0);
    for (uint64_t c = 0; c < nleaf; ++c) leaf_first[c + 1] = leaf_first[c] + (uint64_t)__builtin_popcountll(leaf_mask[c]);
    const uint64_t nbricks = leaf_first[nleaf];
    if (nbricks >= 0x80000000ull) {
        delete f;
        return VHX_E_CAPACITY;
    }
    const size_t n3 = (size_t)bd * bd * bd;
    f->brick_count = (uint32_t)nbricks;
    f->voxel_count = nbricks * n3;
    f->voxels.reset(new (std::nothrow) uint32_t[std::max<uint64_t>(f->voxel_count, 1)]);
    if (!f->voxels) {
        delete f;
        return VHX_E_CAPACITY;
    }
    uint32_t *vox = f->voxels.get();
    parallel_for((int64_t)nleaf, threads, [&](int64_t code) {
        uint64_t m = leaf_mask[code];
        if (!m) return;
        uint32_t li = bfs[D][code];
        uint32_t lx, ly, lz;
        leaf_coord((uint64_t)code, lx, ly, lz);
        uint64_t b = leaf_first[code];
        uint32_t last_c = 0, last_v = VHX_EMPTY;
        for (uint32_t s = 0; s < 64; ++s) {
            if (!((m >> s) & 1ull)) continue;
            f->node_children[(size_t)li * 64 + s] = (uint32_t)b;
            uint32_t bx = lx * L + (s & 3u) * bd, by = ly * L + ((s >> 2) & 3u) * bd, bz = lz * L + (s >> 4) * bd;
            uint32_t *dst = vox + b * n3;
            for (uint32_t z = 0; z < bd; ++z)
                for (uint32_t y = 0; y < bd; ++y)
                    for (uint32_t x = 0; x < bd; ++x) {
                        uint32_t c = sc.voxel(bx + x, by + y, bz + z);
                        uint32_t v = VHX_EMPTY;
                        if (c != 0) {
                            if (c != last_c) {
                                last_c = c;
                                last_v = color_index.at(c) | (0xFFFFu << 16);  // pix_visual
                            }
                            v = last_v;
                        }
                        dst[x + y * bd + z * bd * bd] = v;
                    }
            ++b;
        }
    });
    *out = f;
    return 0;
}

// ---------------------------------------------------------------------------------------------- C ABI
extern "C" {

int vhx_boxtree_new(uint32_t size, uint32_t brick_dim, vhx_boxtree **out) {
    if (!out) return VHX_E_INVALID_ARG;
    BoxTree *t = nullptr;
    int rc = BoxTree::create(size, brick_dim, &t);
    if (rc != 0) return rc;
    *out = new vhx_boxtree{t};
    return VHX_OK;
}
void vhx_boxtree_free(vhx_boxtree *tree) {
    if (!tree) return;
    delete tree->tree;
    delete tree;
}
int vhx_boxtree_set_auto_simplify(vhx_boxtree *tree, int enabled) {
    if (!tree) return VHX_E_INVALID_ARG;
    tree->tree->auto_simplify = enabled != 0;
    return VHX_OK;
}
int vhx_boxtree_insert(vhx_boxtree *tree, uint32_t x, uint32_t y, uint32_t z, uint32_t kind, uint32_t albedo,
                       uint32_t data) {
    if (!tree || kind > VHX_ENTRY_COMPLEX) return VHX_E_INVALID_ARG;
    return tree->tree->insert(U3{x, y, z}, Entry{kind, albedo, data});
}
int vhx_boxtree_insert_at_lod(vhx_boxtree *tree, uint32_t x, uint32_t y, uint32_t z, uint32_t insert_size,
                              uint32_t kind, uint32_t albedo, uint32_t data) {
    if (!tree || kind > VHX_ENTRY_COMPLEX) return VHX_E_INVALID_ARG;
    return tree->tree->insert_at_lod(U3{x, y, z}, insert_size, Entry{kind, albedo, data});
}
int vhx_boxtree_update(vhx_boxtree *tree, uint32_t x, uint32_t y, uint32_t z, uint32_t kind, uint32_t albedo,
                       uint32_t data) {
    if (!tree || kind > VHX_ENTRY_COMPLEX) return VHX_E_INVALID_ARG;
    return tree->tree->update(U3{x, y, z}, Entry{kind, albedo, data});
}
int vhx_boxtree_get(const vhx_boxtree *tree, uint32_t x, uint32_t y, uint32_t z, uint32_t *kind, uint32_t *albedo,
                    uint32_t *data) {
    if (!tree || !kind || !albedo || !data) return VHX_E_INVALID_ARG;
    Entry e = tree->tree->get(U3{x, y, z});
    *kind = e.kind;
    *albedo = e.albedo;
    *data = e.data;
    return VHX_OK;
}
int vhx_boxtree_node_info(const vhx_boxtree *tree, float x, float y, float z, uint64_t *key, uint32_t *content,
                          uint64_t *occupied_bits, uint32_t *occlusion_bits) {
    if (!tree || !key || !content || !occupied_bits || !occlusion_bits) return VHX_E_INVALID_ARG;
    const BoxTree &t = *tree->tree;
    const float S = (float)t.boxtree_size;
    if (!(x >= 0.f && y >= 0.f && z >= 0.f && x < S && y < S && z < S)) return VHX_E_TREE_INVALID_POSITION;
    Cube bounds{F3{0.f, 0.f, 0.f}, S};
    const size_t k = t.get_node_internal(0, bounds, F3{x, y, z});
    if (k == SIZE_MAX) return VHX_E_TREE_INVALID_POSITION;
    const Node &n = t.nodes.get(k);
    *key = k;
    *content = (uint32_t)n.content;
    *occupied_bits = n.occupied_bits;
    *occlusion_bits = n.occlusion_bits;
    return VHX_OK;
}

int vhx_boxtree_simplify(vhx_boxtree *tree, int recursive) {
    if (!tree) return VHX_E_INVALID_ARG;
    tree->tree->simplify(0, recursive != 0);
    return VHX_OK;
}
int vhx_boxtree_info(const vhx_boxtree *tree, uint32_t info[5]) {
    if (!tree || !info) return VHX_E_INVALID_ARG;
    info[0] = tree->tree->boxtree_size;
    info[1] = tree->tree->brick_dim;
    info[2] = (uint32_t)tree->tree->nodes.len();
    info[3] = (uint32_t)tree->tree->color_palette.size();
    info[4] = (uint32_t)tree->tree->data_palette.size();
    return VHX_OK;
}
int vhx_scene_insert(vhx_boxtree *tree, uint32_t scene, uint64_t seed) {
    if (!tree || !scene_valid(scene)) return VHX_E_INVALID_ARG;
    Scene sc{scene, tree->tree->boxtree_size, seed, 0, {}};
    sc.prepare();
    for (uint32_t x = 0; x < sc.extent; ++x)
        for (uint32_t y = 0; y < sc.extent; ++y)
            for (uint32_t z = 0; z < sc.extent; ++z) {
                uint32_t c = sc.voxel(x, y, z);
                if (c == 0) continue;
                int rc = tree->tree->insert(U3{x, y, z}, Entry{VHX_ENTRY_VISUAL, c, 0});
                if (rc != 0) return rc;
            }
    return VHX_OK;
}
int vhx_boxtree_flatten(const vhx_boxtree *tree, vhx_flat **out) {
    if (!tree || !out) return VHX_E_INVALID_ARG;
    *out = flatten_tree(*tree->tree, 0xFFFFFFFFu, tree->tree->mip_strategy.enabled);
    return VHX_OK;
}
int vhx_boxtree_flatten_lod(const vhx_boxtree *tree, uint32_t max_depth, vhx_flat **out) {
    if (!tree || !out) return VHX_E_INVALID_ARG;
    *out = flatten_tree(*tree->tree, max_depth, true);
    return VHX_OK;
}
int vhx_flat_node_mips(const vhx_flat *f, const uint32_t **node_mips, uint32_t *count) {
    if (!f || !node_mips || !count) return VHX_E_INVALID_ARG;
    *node_mips = f->node_mips.empty() ? nullptr : f->node_mips.data();
    *count = (uint32_t)f->node_mips.size();
    return VHX_OK;
}
int vhx_boxtree_switch_mips(vhx_boxtree *tree, int enabled) {
    if (!tree) return VHX_E_INVALID_ARG;
    tree->tree->switch_albedo_mip_maps(enabled != 0);
    return VHX_OK;
}
int vhx_boxtree_set_mip_method(vhx_boxtree *tree, uint32_t level, uint32_t method, float threshold) {
    if (!tree || method > VHX_MIP_POSTERIZE_BD || !(threshold == threshold)) return VHX_E_INVALID_ARG;
    // set_method_at_internal (mipmap.rs:414-431): Posterize thresholds are clamped to [0, 1]
    if (method == VHX_MIP_POSTERIZE || method == VHX_MIP_POSTERIZE_BD) threshold = std::clamp(threshold, 0.f, 1.f);
    tree->tree->mip_strategy.methods[level] = MipMethodCfg{method, threshold};
    return VHX_OK;
}
int vhx_boxtree_set_mip_color_threshold(vhx_boxtree *tree, uint32_t level, float threshold) {
    if (!tree || !(threshold == threshold)) return VHX_E_INVALID_ARG;
    // set_color_similarity_thr_internal (mipmap.rs:365-379): clamped to [0, 1]
    tree->tree->mip_strategy.color_thresholds[level] = std::clamp(threshold, 0.f, 1.f);
    return VHX_OK;
}
int vhx_boxtree_set_mip_options(int direct, int threads) {
    if (threads < 0 || threads > 256) return VHX_E_INVALID_ARG;
    g_mip_direct.store(direct ? 1 : 0);
    g_mip_threads.store(threads);
    return VHX_OK;
}
int vhx_boxtree_recalculate_mips(vhx_boxtree *tree) {
    if (!tree) return VHX_E_INVALID_ARG;
    if (tree->tree->nodes.get(0).content != Content::Nothing) tree->tree->recalculate_mips();
    return VHX_OK;
}
int vhx_boxtree_sample_root_mip(const vhx_boxtree *tree, uint32_t sectant, uint32_t x, uint32_t y, uint32_t z,
                                uint32_t *kind, uint32_t *albedo, uint32_t *data) {
    const uint32_t bd = tree ? tree->tree->brick_dim : 0;
    if (!tree || !kind || !albedo || !data || sectant > 64 || x >= bd || y >= bd || z >= bd) return VHX_E_INVALID_ARG;
    const Entry e = tree->tree->entry_of(tree->tree->sample_root_mip((uint8_t)sectant, U3{x, y, z}));
    *kind = e.kind;
    *albedo = e.albedo;
    *data = e.data;
    return VHX_OK;
}
int vhx_scene_build(uint32_t scene, uint32_t size, uint32_t brick_dim, uint64_t seed, int threads, vhx_flat **out) {
    if (!out || !scene_valid(scene)) return VHX_E_INVALID_ARG;
    try {
        return build_scene(scene, size, brick_dim, seed, threads, out);
    } catch (const std::bad_alloc &) {
        return VHX_E_CAPACITY;
    }
}
int vhx_scene_build_lod(uint32_t scene, uint32_t size, uint32_t brick_dim, uint64_t seed, int threads,
                        uint32_t max_depth, vhx_flat **out) {
    if (!out || !scene_valid(scene)) return VHX_E_INVALID_ARG;
    try {
        vhx_flat *full = nullptr;
        int rc = build_scene(scene, size, brick_dim, seed, threads, &full);
        if (rc != VHX_OK) return rc;
        std::unique_ptr<vhx_flat> owned(full);
        std::unique_ptr<BoxTree> t(tree_of_flat(*full));
        if (!t) return VHX_E_STATE;
        owned.reset();
        t->switch_albedo_mip_maps(true);
        *out = flatten_tree(*t, max_depth, true);
        return VHX_OK;
    } catch (const std::bad_alloc &) {
        return VHX_E_CAPACITY;
    }
}
int vhx_scene_build_tree(uint32_t scene, uint32_t size, uint32_t brick_dim, uint64_t seed, int threads,
                         vhx_boxtree **out) {
    if (!out || !scene_valid(scene)) return VHX_E_INVALID_ARG;
    *out = nullptr;
    try {
        vhx_flat *full = nullptr;
        int rc = build_scene(scene, size, brick_dim, seed, threads, &full);
        if (rc != VHX_OK) return rc;
        std::unique_ptr<vhx_flat> owned(full);
        BoxTree *t = tree_of_flat(*full);
        if (!t) return VHX_E_STATE;
        *out = new vhx_boxtree{t};
        return VHX_OK;
    } catch (const std::bad_alloc &) {
        return VHX_E_CAPACITY;
    }
}
int vhx_flat_desc(const vhx_flat *f, vhx_tree_desc *d) {
    if (!f || !d) return VHX_E_INVALID_ARG;
    std::memset(d, 0, sizeof(*d));
    d->boxtree_size = f->size;
    d->brick_dim = f->brick_dim;
    d->node_count = (uint32_t)f->node_type.size();
    d->brick_count = f->brick_count;
    d->solid_count = (uint32_t)f->solid_values.size();
    d->color_count = (uint32_t)f->color_palette.size();
    d->data_count = (uint32_t)f->data_palette.size();
    d->node_type = f->node_type.data();
    d->node_ocbits = f->node_ocbits.data();
    d->node_children = f->node_children.data();
    d->voxels = f->voxels.get();
    d->solid_values = f->solid_values.data();
    d->color_palette = f->color_palette.data();
    d->data_palette = f->data_palette.data();
    return VHX_OK;
}
void vhx_flat_free(vhx_flat *f) { delete f; }

}  // extern "C"
