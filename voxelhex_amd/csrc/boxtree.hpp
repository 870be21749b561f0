// Host-side BoxTree<u32> — C++ restatement of VoxelHex's voxel container (the host half of the raytracing
// drop-in; the reference's Rust toolchain is not available to this build).
//
// Restated (paths relative to the VoxelHex repository):
//   ObjectPool                 src/object_pool.rs:51-266 (same key allocation, so node keys match the reference)
//   BoxTree::new / get         src/boxtree/mod.rs:188-317
//   insert / insert_at_lod     src/boxtree/update/insert.rs:21-407, post_process_node_insert 411-495
//   add_to_palette             src/boxtree/update/mod.rs:39-120
//   leaf_update                src/boxtree/update/mod.rs:144-464
//   dilute_brick_data          src/boxtree/update/mod.rs:478-555, update_brick 564-603
//   simplify                   src/boxtree/update/mod.rs:617-867
//   subdivide_leaf_to_nodes    src/boxtree/detail.rs:248-337, node_empty_at 156-224, deallocate_children_of 352-370
//   execute_for_relevant_sectants src/boxtree/iterate.rs:40-121, get_node_internal 293-343
//   BrickData helpers          src/boxtree/node.rs:34-145, NodeContent pix_* 259-373, is_all 424-458
//   update triggers            insert.rs:328-405: (node stack, modified bottom sectants) of every insert/update, queued
//                              for a stream like BoxTreeGPUHost's changes_buffer (src/raytracing/bevy/mod.rs:164-173)
//   MIP maps                   update_mip src/boxtree/mipmap.rs:42-338, MIPMapStrategy defaults 341-354,
//                              recalculate_mips / switch_albedo_mip_maps / recalculate_mip 536-633, resampling
//                              MIPResamplingFunction::execute src/boxtree/iterate.rs:434-560 (Albedou32 349-432)
#include <map>
#pragma once

#include <array>
#include <cmath>
#include <atomic>
#include <deque>
#include <functional>
#include <cstddef>
#include <utility>
#include <cstdint>
#include <unordered_map>
#include <vector>

namespace vhx {

// process-wide MIP generation options (vhx_boxtree_set_mip_options, boxtree.cpp)
extern std::atomic<int> g_mip_direct;
extern std::atomic<int> g_mip_threads;


constexpr uint32_t kChildren = 64;
constexpr uint32_t kEmpty32 = 0xFFFFFFFFu;

struct F3 {
    float x, y, z;
};
struct U3 {
    uint32_t x, y, z;
};
struct Cube {
    F3 min;
    float size;
};

enum class BrickKind : uint8_t { Empty, Parted, Solid };
struct Brick {
    BrickKind kind = BrickKind::Empty;
    uint32_t solid = 0;
    std::vector<uint32_t> parted;
    bool operator==(const Brick &o) const {
        if (kind != o.kind) return false;
        if (kind == BrickKind::Solid) return solid == o.solid;
        if (kind == BrickKind::Parted) return parted == o.parted;
        return true;
    }
};

enum class Content : uint8_t { Nothing, Internal, Leaf, UniformLeaf };
struct Node {
    Content content = Content::Nothing;
    std::vector<Brick> bricks;  // Leaf: 64, UniformLeaf: 1
    bool has_children = false;  // NodeChildren::Children vs NoChildren
    std::array<uint32_t, kChildren> children{};
    uint64_t occupied_bits = 0;
    Brick mip;                   // NodeData::mip (src/boxtree/types.rs:183-186): the node's albedo MIP brick
    uint8_t occlusion_bits = 0;  // bit CubeSides: no ray enters from that side (src/boxtree/types.rs:189-200)
    bool is_occluded() const { return (occlusion_bits & 0x3F) == 0x3F; }  // node.rs:176-178
};

// BoxTreeEntry<u32>
struct Entry {
    uint32_t kind;  // VHX_ENTRY_*
    uint32_t albedo;  // r | g<<8 | b<<16 | a<<24
    uint32_t data;
};

class ObjectPool {
   public:
    size_t push(Node item);
    size_t allocate();
    bool free(size_t key);
    void swap(size_t a, size_t b) { std::swap(buffer_[a], buffer_[b]); }
    bool key_is_valid(size_t key) const { return key < buffer_.size() && reserved_[key]; }
    Node &get(size_t key) { return buffer_[key]; }
    const Node &get(size_t key) const { return buffer_[key]; }
    size_t len() const { return buffer_.size(); }

   private:
    bool try_set_next_available();
    std::vector<Node> buffer_;
    std::vector<bool> reserved_;
    size_t first_available_ = 0;
};

// MIPResamplingMethods (src/boxtree/types.rs:113-149); the values are the C ABI's VHX_MIP_* codes
enum MipMethod : uint32_t { kBoxFilter = 0, kPointFilter = 1, kPointFilterBD = 2, kPosterize = 3, kPosterizeBD = 4 };
struct MipMethodCfg {
    uint32_t kind;
    float thr;  // Posterize / PosterizeBD similarity threshold
};
// MIPMapStrategy with its defaults (src/boxtree/mipmap.rs:341-354); a level without a method uses BoxFilter
// (MIPResamplingMethods::default, types.rs:121-122), a level without a colour threshold adds every new colour
struct MipStrategy {
    bool enabled = false;
    std::map<size_t, MipMethodCfg> methods{
        {1, {kPosterize, 0.05f}}, {2, {kBoxFilter, 0.f}}, {3, {kBoxFilter, 0.f}}, {4, {kBoxFilter, 0.f}}};
    std::map<size_t, float> color_thresholds{{2, 0.1f}, {3, 0.05f}, {4, 0.02f}};
};

class BoxTree {
   public:
    // returns 0 or a VHX_E_TREE_* code (OctreeError)
    static int create(uint32_t size, uint32_t brick_dim, BoxTree **out);

    int insert(U3 pos, Entry e) { return insert_at_lod_internal(true, pos, 1, e); }
    int insert_at_lod(U3 pos, uint32_t size, Entry e) { return insert_at_lod_internal(true, pos, size, e); }
    int update(U3 pos, Entry e) { return insert_at_lod_internal(false, pos, 1, e); }
    uint32_t get_raw(U3 pos) const;
    Entry get(U3 pos) const;
    Entry entry_of(uint32_t value) const;
    bool simplify(size_t node_key, bool recursive);
    // MIP maps (src/boxtree/mipmap.rs)
    MipStrategy mip_strategy;
    void switch_albedo_mip_maps(bool enabled);
    void recalculate_mips();
    void recalculate_mip(size_t node_key, const Cube &node_bounds);
    void update_mip(size_t node_key, const Cube &node_bounds, U3 position);
    // the two halves of update_mip: the resampling (reads the tree only; false for None) and the palette match + store
    bool mip_sample(size_t node_key, const Cube &node_bounds, U3 position, uint32_t &color) const;
    void mip_store(size_t node_key, const Cube &node_bounds, U3 position, uint32_t color);
    // sample_root_mip (mipmap.rs:635-668): sectant >= 64 samples the root's MIP, else the root's child's; raw value
    uint32_t sample_root_mip(uint8_t sectant, U3 position) const;
    // BoxTree::get_internal (src/boxtree/mod.rs:247-317) from any node and its bounds
    uint32_t get_internal(size_t node_key, Cube bounds, U3 position) const;
    bool albedo_of(uint32_t value, uint32_t &albedo) const;

    bool auto_simplify = true;
    uint32_t brick_dim = 0, boxtree_size = 0;
    // BoxTreeUpdatedSignalParams (src/boxtree/types.rs:204) of every insert/update that changed the tree, queued while
    // a stream tracks the tree (the trigger BoxTreeGPUHost::new installs, src/raytracing/bevy/mod.rs:164-173); the
    // stream pops them in its upload (handle_tree_updates, src/raytracing/bevy/streaming/mod.rs:35-286)
    struct Change {
        std::vector<std::pair<size_t, uint8_t>> node_stack;
        std::vector<uint8_t> updated_sectants;
    };
    mutable std::deque<Change> changes;
    mutable int track_changes = 0;
    // bumped by every structural edit (update_at_lod, simplify), tracked or not: a stream's cached view walk is valid
    // only for the edit_seq it was made on (vhx_stream rebuild)
    uint64_t edit_seq = 0;
    ObjectPool nodes;
    std::vector<uint32_t> color_palette;
    std::vector<uint32_t> data_palette;

    bool points_to_empty(uint32_t v) const;
    size_t get_node_internal(size_t key, Cube &bounds, F3 position) const;
    size_t child(size_t node_key, uint8_t sectant) const;

    uint32_t add_to_palette(Entry e);

   private:
    std::unordered_map<uint32_t, size_t> color_index_, data_index_;
    // mip_store's palette matching (the first entry within a level's colour threshold, mipmap.rs:252-274): per
    // (threshold bits, colour) the first matching index, or none among the first `checked` entries. Entries are never
    // changed or removed, only appended, so a found match stays the first one and a miss needs only the new entries.
    struct MipMatch {
        uint32_t index;    // UINT32_MAX: no match among the first `checked` entries
        uint32_t checked;
    };
    std::unordered_map<uint64_t, MipMatch> mip_match_;
    uint64_t mip_last_key_ = ~0ull;
    uint32_t mip_last_index_ = UINT32_MAX;
    uint32_t mip_palette_match(uint32_t color, float thr);  // index or UINT32_MAX
    // get_internal(key, nb, pos) of a Leaf node at an integer position, in integer arithmetic (the leaf resampling)
    uint32_t leaf_value(const struct Node &n, const Cube &nb, U3 pos) const;

    int insert_at_lod_internal(bool overwrite_if_empty, U3 pos, uint32_t insert_size, Entry e);
    void post_process_node_insert(const std::vector<std::pair<size_t, uint8_t>> &node_stack, const Cube &node_bounds,
                                  const std::array<size_t, 3> &aus, U3 pos, uint32_t insert_size);
    bool get_sibling_by_stack(int dx, int dy, int dz, const std::vector<std::pair<size_t, uint8_t>> &node_stack,
                              size_t &sibling, uint8_t &sibling_sectant) const;
    bool leaf_update(bool overwrite_if_empty, size_t node_key, const Cube &node_bounds, const Cube &target_bounds,
                     size_t target_child_sectant, U3 position, U3 size, uint32_t target_content);
    void subdivide_leaf_to_nodes(size_t node_key, size_t target_sectant);
    bool node_empty_at(size_t node_key, uint8_t sectant) const;
    bool compare_nodes(size_t l, size_t r) const;
    void deallocate_children_of(size_t node_key);
    Brick try_brick_from_node(size_t node_key) const;
    uint32_t &child_mut(size_t node_key, size_t index);
    uint64_t calculate_brick_occupied_bits(const std::vector<uint32_t> &brick) const;
    uint64_t calculate_occupied_bits(const Brick &b) const;
    bool brick_contains_nothing(const Brick &b) const;
    bool brick_simplify(Brick &b) const;
    bool content_is_all(const Node &n, uint32_t data) const;
    std::array<std::vector<uint32_t>, kChildren> dilute_brick_data(const std::vector<uint32_t> &brick) const;
    void update_brick(bool overwrite_if_empty, std::vector<uint32_t> &brick, const Cube &bb, U3 position, U3 size,
                      uint32_t data) const;
};

// spatial helpers shared with the flattener / scene builder (src/spatial/math/mod.rs, src/spatial/mod.rs)
const float *sectant_offset(uint32_t s);
uint8_t offset_sectant(F3 off, float size);
Cube child_bounds_for(const Cube &c, uint8_t s);
bool rust_log_is_integral(float x, float base);
// step_sectant (src/spatial/mod.rs:23-26) for integer steps in {-1, 0, 1}: >= 64 means out of the node
uint8_t step_sectant_i(uint8_t s, int dx, int dy, int dz);
// execute_for_relevant_sectants (src/boxtree/iterate.rs:40-121)
std::array<size_t, 3> execute_for_relevant_sectants(const Cube &nb, U3 position, uint32_t update_size,
                                                    const std::function<void(U3, U3, uint8_t, const Cube &)> &fun);

namespace sect {  // the scalar conversions relevant_sectants needs (Rust `as` casts: saturating, NaN -> 0)
inline uint32_t as_u32(float f) {
    if (std::isnan(f) || f <= 0.f) return 0;
    if (f >= 4294967296.0f) return 0xFFFFFFFFu;
    return (uint32_t)f;
}
inline size_t as_usize(float f) {
    if (std::isnan(f) || f <= 0.f) return 0;
    if (f >= 18446744073709551616.0f) return SIZE_MAX;
    return (size_t)f;
}
}  // namespace sect

// The body of execute_for_relevant_sectants as a template over the callback, so that a hot caller (the streaming view
// walk, stream.cpp) calls `fun` inline instead of through std::function; execute_for_relevant_sectants forwards here.
// The reference walks the whole update region, which may reach far past the node (the streaming view's include regions
// grow by 4x per MIP level): a point past the node's upper bound on an axis fails cube_contains, and so does every
// later point on that axis (shifted only grows; position >= nb.min), so the loops stop there. The calls of `fun` and
// their order are the reference's.
template <class Fn>
inline std::array<size_t, 3> relevant_sectants(const Cube &nb, U3 position_, uint32_t update_size_, Fn &&fun) {
    const float nx = nb.min.x + nb.size, ny = nb.min.y + nb.size, nz = nb.min.z + nb.size;
    if ((float)position_.x > nx || (float)position_.y > ny || (float)position_.z > nz) return {0, 0, 0};
    const F3 position{std::fmax((float)position_.x, nb.min.x), std::fmax((float)position_.y, nb.min.y),
                      std::fmax((float)position_.z, nb.min.z)};
    const float us = (float)update_size_;
    const F3 update_size{((float)position_.x + us) - position.x, ((float)position_.y + us) - position.y,
                         ((float)position_.z + us) - position.z};
    const float cell_size = nb.size / 4.f;
    const F3 end{position.x + update_size.x, position.y + update_size.y, position.z + update_size.z};
    F3 shifted = position;
    while (shifted.x <= end.x && shifted.x < nx) {
        shifted.y = position.y;
        while (shifted.y <= end.y && shifted.y < ny) {
            shifted.z = position.z;
            while (shifted.z <= end.z && shifted.z < nz) {
                // cube_contains (src/spatial/mod.rs:54-61)
                if (!(shifted.x >= nb.min.x && shifted.y >= nb.min.y && shifted.z >= nb.min.z && shifted.x < nx &&
                      shifted.y < ny && shifted.z < nz)) {
                    shifted.z += cell_size;
                    continue;
                }
                const uint8_t s = offset_sectant(F3{shifted.x - nb.min.x, shifted.y - nb.min.y, shifted.z - nb.min.z},
                                                 nb.size);  // Cube::sectant_for
                Cube tb = child_bounds_for(nb, s);
                tb = Cube{F3{std::floor(tb.min.x), std::floor(tb.min.y), std::floor(tb.min.z)}, std::ceil(tb.size)};
                const F3 pit{std::fmax(position.x, tb.min.x), std::fmax(position.y, tb.min.y),
                             std::fmax(position.z, tb.min.z)};
                const F3 remains{end.x - pit.x, end.y - pit.y, end.z - pit.z};
                const F3 uit{std::fmin((tb.min.x + tb.size) - pit.x, remains.x),
                             std::fmin((tb.min.y + tb.size) - pit.y, remains.y),
                             std::fmin((tb.min.z + tb.size) - pit.z, remains.z)};
                if (0.f < uit.x && 0.f < uit.y && 0.f < uit.z)
                    fun(U3{sect::as_u32(std::round(pit.x)), sect::as_u32(std::round(pit.y)), sect::as_u32(std::round(pit.z))},
                        U3{sect::as_u32(std::round(uit.x)), sect::as_u32(std::round(uit.y)), sect::as_u32(std::round(uit.z))},
                        s, tb);
                shifted.z += cell_size;
            }
            shifted.y += cell_size;
        }
        shifted.x += cell_size;
    }
    return {sect::as_usize(std::round(update_size.x)), sect::as_usize(std::round(update_size.y)),
            sect::as_usize(std::round(update_size.z))};
}

}  // namespace vhx

// opaque handle of the C ABI (include/vhx_boxtree.h)
struct vhx_boxtree {
    vhx::BoxTree *tree;
};
