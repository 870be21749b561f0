// Streaming producer: a device-resident *view* of a BoxTree with bounded node and brick capacity, filled around a
// viewport with ranged writes — BoxTreeGPUDataHandler and its upload queue (src/raytracing/bevy/streaming/*.rs)
// over the host BoxTree restatement, feeding vhx_update_range instead of wgpu's write_buffer.
//
//   rebuild                            upload_queue.rs:60-207   nodes to see around the viewport
//   process / next_valid_node          upload_queue.rs:218-574  node uploads, then brick uploads, per frame
//   process_node_child_bricks          upload_queue.rs:406-476
//   add_node / first_available_node    cache.rs:188-455         node slots, victim = not in view
//   add_brick / first_available_brick  cache.rs:460-716         brick slots, victim = unused / MIP / furthest
//   erase_node_child                   cache.rs:41-145
//   re_evaluate_view_size              streaming/mod.rs:292-340 grows capacities (caller re-creates buffers)
//   upload                             streaming/mod.rs:420-635 cache updates -> ranged writes
//   view sizing                        view.rs:50-69; set_viewport: bevy/mod.rs:110-155 (brick slot hysteresis)
//
// Behavioural deviations: rebuild puts the whole root -> center access path into the view set (see rebuild); after
// queued tree changes the view set is recomputed (see handle_tree_updates).
// Differences in the layout the device kernel reads (docs/DESIGN_LOG.md §9c): node type is one u32 per node (not 2 bits
// packed 16 per word), occupancy one u64, a Solid brick descriptor is 0x80000000 | index into a deduplicated solid
// value table (the reference inlines the value, losing data-palette bits), MIP data is tracked for slot accounting
// but never uploaded (the raytracer does not read MIPs). The reference computes the view set on a worker thread; here
// `rebuild` runs synchronously when the viewport leaves its brick slot, so the upload order is deterministic.
// Tree-change propagation: inserts and updates made to the tree while a stream tracks it are queued by the tree
// (BoxTree::changes, the update trigger of BoxTreeGPUHost::new) and re-uploaded by handle_tree_updates
// (streaming/mod.rs:35-286) at the start of the next upload frames, before the regular upload queue.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <system_error>
#include <thread>
#include <array>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <tuple>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../include/vhx.h"
#include "../../include/vhx_boxtree.h"
#include "../../include/vhx_stream.h"
#include "boxtree.hpp"

using namespace vhx;

namespace {

constexpr uint32_t kEmpty = 0xFFFFFFFFu;
constexpr uint32_t kSolidCapacity0 = 4096;
constexpr uint32_t kPaletteCapacity = 65536;

// BrickOwnedBy (streaming/types.rs:14-21); equality and hash ignore the brick position (streaming/mod.rs:561-590)
struct Owned {
    uint8_t kind = 0;  // 0 None, 1 NodeAsChild, 2 NodeAsMIP
    uint32_t node = 0;
    uint8_t sectant = 0;
    F3 bl{0.f, 0.f, 0.f};  // V3c<u32> brick position, kept as floats
    uint64_t key() const { return ((uint64_t)kind << 40) | ((uint64_t)sectant << 32) | node; }
};

struct CacheUpdate {  // CacheUpdatePackage (types.rs:35-47)
    std::vector<std::pair<size_t, Owned>> brick_updates;
    std::vector<std::pair<size_t, uint64_t>> modified_nodes;
};

struct StackItem {
    size_t node;
    uint8_t sectant;
    Cube bounds;
};

inline F3 f3(float x, float y, float z) { return F3{x, y, z}; }
inline F3 sub(F3 a, F3 b) { return f3(a.x - b.x, a.y - b.y, a.z - b.z); }
inline F3 add(F3 a, F3 b) { return f3(a.x + b.x, a.y + b.y, a.z + b.z); }
inline F3 unit(float v) { return f3(v, v, v); }
inline float clampf(float v, float lo, float hi) { return std::fmin(std::fmax(v, lo), hi); }  // f32::clamp
inline float length(F3 a) { return std::sqrt((a.x * a.x + a.y * a.y) + a.z * a.z); }
inline bool contains(const Cube &c, F3 p) {  // Cube::contains, spatial/mod.rs:54-61
    return p.x >= c.min.x && p.y >= c.min.y && p.z >= c.min.z && p.x < (c.min.x + c.size) &&
           p.y < (c.min.y + c.size) && p.z < (c.min.z + c.size);
}
inline uint32_t round_u32(float v) {  // f32::round() as u32 (saturating)
    const float r = std::round(v);
    if (!(r > 0.f)) return 0;
    if (r >= 4294967296.f) return 0xFFFFFFFFu;
    return (uint32_t)r;
}
inline uint32_t as_u32(float v) {
    if (!(v > 0.f)) return 0;
    if (v >= 4294967296.f) return 0xFFFFFFFFu;
    return (uint32_t)v;
}

}  // namespace

struct vhx_stream {
    const BoxTree *tree = nullptr;
    vhx_ctx *ctx = nullptr;
    // BoxTreeGPUDataHandler
    size_t node_uploads_per_frame = 25, brick_uploads_per_frame = 50, brick_unload_search_perimeter = 10;
    size_t nodes_in_view = 0, bricks_in_view = 0;
    Cube upload_range{};
    // render data: the host mirror of the device view
    std::vector<uint32_t> node_type;
    std::vector<uint64_t> node_ocbits;
    std::vector<uint32_t> node_children;
    std::vector<uint32_t> node_mips;  // host only
    std::vector<uint32_t> voxels;
    std::vector<uint32_t> solid_values;
    std::unordered_map<uint32_t, uint32_t> solid_index;
    size_t solid_capacity = kSolidCapacity0;
    std::vector<uint32_t> color_palette, data_palette;  // device-side capacity kPaletteCapacity
    // UploadQueueTargets
    std::unordered_map<size_t, Owned> brick_by_index;
    std::unordered_map<uint64_t, size_t> brick_by_owner;
    std::unordered_map<size_t, size_t> meta_by_key, key_by_meta;
    // meta_by_key's keys as a dense flag per pool key (kept with it by meta_insert / reset_targets): the upload stats
    // count the nodes to see that are not resident with one pass over the set instead of a hash lookup per node
    std::vector<uint8_t> resident_key;
    void set_resident(size_t key, bool on) {
        if (key >= resident_key.size()) {
            if (!on) return;
            resident_key.resize(std::max<size_t>(key + 1, resident_key.size() * 2), 0u);
        }
        if ((resident_key[key] != 0u) != on && nodes_to_see.count(key)) {
            if (on)
                ++nodes_to_see.n_resident;
            else
                --nodes_to_see.n_resident;
        }
        resident_key[key] = on ? 1u : 0u;
    }
    bool is_resident(size_t key) const { return key < resident_key.size() && resident_key[key] != 0u; }
    std::unordered_map<size_t, std::pair<size_t, uint8_t>> node_index_vs_parent;
    // nodes_to_see (upload_queue.rs: a HashSet of node keys): a set over the pool's dense keys, stamped by generation so
    // that the per-rebuild clear is O(1); membership and size are what the queue logic reads (no iteration order).
    // erase (the incremental rebuild) swaps the member with the last one: pos[k] is k's place in `members`
    // `resident` (the stream's resident_key flags) lets the set count its members that are resident, so that the
    // stats' "not resident" count needs no pass over the set
    struct KeySet {
        std::vector<uint32_t> stamp;
        std::vector<uint32_t> pos;
        std::vector<size_t> members;
        uint32_t gen = 1;
        const std::vector<uint8_t> *resident = nullptr;
        size_t n_resident = 0;
        bool res(size_t k) const { return resident && k < resident->size() && (*resident)[k] != 0u; }
        void clear() {
            members.clear();
            n_resident = 0;
            if (++gen == 0) {  // wrapped: reset every stamp once
                std::fill(stamp.begin(), stamp.end(), 0u);
                gen = 1;
            }
        }
        void insert(size_t k) {
            if (k >= stamp.size()) {
                stamp.resize(std::max<size_t>(k + 1, stamp.size() * 2), 0u);
                pos.resize(stamp.size(), 0u);
            }
            if (stamp[k] != gen) {
                stamp[k] = gen;
                pos[k] = (uint32_t)members.size();
                members.push_back(k);
                n_resident += res(k) ? 1u : 0u;
            }
        }
        void erase(size_t k) {
            if (k >= stamp.size() || stamp[k] != gen) return;
            stamp[k] = 0u;  // never a generation
            n_resident -= res(k) ? 1u : 0u;
            const size_t last = members.back();
            members[pos[k]] = last;
            pos[last] = pos[k];
            members.pop_back();
        }
        size_t count(size_t k) const { return k < stamp.size() && stamp[k] == gen ? 1u : 0u; }
        size_t size() const { return members.size(); }
        std::vector<size_t>::const_iterator begin() const { return members.begin(); }
        std::vector<size_t>::const_iterator end() const { return members.end(); }
    } nodes_to_see;
    // UploadQueueStatus
    std::vector<StackItem> target_node_stack;
    std::vector<Owned> bricks_to_upload;
    size_t victim_brick = 0, victim_node = 0;
    size_t uploaded_color_palette_size = 0, uploaded_data_palette_size = 0, uploaded_solid_size = 0;
    // view
    F3 origin{0.f, 0.f, 0.f};
    float view_distance = 0.f;
    bool reload = true, resize = false, device_valid = false;
    Cube brick_slot{f3(0.f, 0.f, 0.f), 0.f};
    bool brick_slot_set = false;
    // A viewport move's upload-queue rebuild (upload_queue.rs:60-142) is deferred to the next upload that reads the queue
    // and coalesced, the latest request winning: the reference runs it as a background task and keeps only the newest
    // pending request (bevy/mod.rs:110-155, upload_queue.rs:262-289), so several moves between two uploads (a renderer
    // keeping K frames in flight on one tree version, vhx_stream_upload_frames) cost one rebuild instead of K.
    bool rebuild_pending = false;
    F3 pending_origin{0.f, 0.f, 0.f};
    float pending_distance = 0.f;
    void apply_pending_rebuild() {
        if (!rebuild_pending) return;
        rebuild_pending = false;
#ifdef VHX_STREAM_TIMING
        const auto t0 = std::chrono::steady_clock::now();
#endif
        rebuild(pending_origin, pending_distance);
#ifdef VHX_STREAM_TIMING
        fprintf(stderr, "[stream] rebuild %.3f ms, %zu nodes to see, shell %lu ins %lu era %lu (full %lu inc %lu)\n",
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(), nodes_to_see.size(),
                (unsigned long)dbg_shell, (unsigned long)dbg_ins, (unsigned long)dbg_era, (unsigned long)rebuilds_full,
                (unsigned long)rebuilds_incremental);
        dbg_shell = dbg_ins = dbg_era = 0;
#endif
        target_node_stack = node_stack_init();
    }
    // statistics of the last upload
    uint64_t last_nodes = 0, last_bricks = 0, last_bytes = 0;
    // completion tracking over the cyclic node walk: new work (node adds, brick requests) found in the current and
    // in the last complete walk cycle (UINT64_MAX: no complete cycle since the last rebuild)
    uint64_t cycle_work = 0, last_cycle_work = UINT64_MAX;
    bool walk_started = false;

    ~vhx_stream() {
        if (tree && --tree->track_changes == 0) tree->changes.clear();
    }
    uint32_t bd() const { return tree->brick_dim; }
    uint32_t max_mip_level() const {  // boxtree/mod.rs:320-324
        const float l = std::ceil(std::log((float)tree->boxtree_size / (float)tree->brick_dim) / std::log(4.f));
        return l <= 0.f ? 0u : (uint32_t)l;
    }
    bool key_valid(size_t k) const { return tree->nodes.key_is_valid(k); }
    const Node &node(size_t k) const { return tree->nodes.get(k); }
    size_t child(size_t k, uint8_t s) const {
        const Node &n = node(k);
        return n.has_children ? (size_t)n.children[s] : SIZE_MAX;
    }
    bool valid_child(size_t k, uint8_t s, size_t &c) const {
        c = child(k, s);
        return key_valid(c);
    }

    // --------------------------------------------------------------------------------- ownership bimap helpers
    bool owner_has(const Owned &o) const { return brick_by_owner.count(o.key()) != 0; }
    void owner_insert(size_t idx, const Owned &o) {  // BiHashMap::insert drops both old pairs
        auto a = brick_by_index.find(idx);
        if (a != brick_by_index.end()) brick_by_owner.erase(a->second.key());
        auto b = brick_by_owner.find(o.key());
        if (b != brick_by_owner.end()) brick_by_index.erase(b->second);
        brick_by_index[idx] = o;
        brick_by_owner[o.key()] = idx;
    }
    void owner_remove_index(size_t idx) {
        auto a = brick_by_index.find(idx);
        if (a == brick_by_index.end()) return;
        brick_by_owner.erase(a->second.key());
        brick_by_index.erase(a);
    }
    void meta_insert(size_t key, size_t meta) {
        auto a = meta_by_key.find(key);
        if (a != meta_by_key.end()) key_by_meta.erase(a->second);
        auto b = key_by_meta.find(meta);
        if (b != key_by_meta.end()) {
            meta_by_key.erase(b->second);
            set_resident(b->second, false);
        }
        meta_by_key[key] = meta;
        key_by_meta[meta] = key;
        set_resident(key, true);
    }

    // ------------------------------------------------------------------------------------------ node MIPs
    // Streamed when the tree's MIP maps are enabled (tree_properties bit 16, streaming/mod.rs:288-290): a node's entry
    // follows cache.rs:435-453 (Empty -> empty marker, Solid -> a solid descriptor of this view's solid table instead
    // of the reference's inline 0x80000000 | value, Parted -> its MIP slot once uploaded) and the MIP slot's voxels
    // are written with the brick updates. Deviation: a MIP slot is taken for every node, as in the reference
    // (upload_queue.rs:332-341), but node_mips points at it only for a Parted MIP (the reference points at the slot for
    // Empty and Solid MIPs too, which leaves the shader reading a slot nothing was written to).
    bool stream_mips() const { return tree->mip_strategy.enabled; }
    bool mips_dirty = false, device_mips_on = false;
    void set_mip(size_t idx, uint32_t v) {
        if (idx < node_mips.size() && node_mips[idx] != v) {
            node_mips[idx] = v;
            mips_dirty = true;
        }
    }
    uint32_t mip_descriptor(size_t key) {
        if (!stream_mips()) return kEmpty;
        const Brick &m = node(key).mip;
        if (m.kind == BrickKind::Empty) return kEmpty;
        if (m.kind == BrickKind::Solid) return solid_descriptor(m.solid);
        Owned o;
        o.kind = 2;
        o.node = (uint32_t)key;
        auto it = brick_by_owner.find(o.key());
        return it == brick_by_owner.end() ? kEmpty : (0x7FFFFFFFu & (uint32_t)it->second);
    }
    // hands the view's node MIPs to the device (vhx_set_node_mips) when they changed, or switches them off
    int sync_device_mips(bool force) {
        if (!ctx) return VHX_OK;
        if (!stream_mips()) {
            if (!device_mips_on) return VHX_OK;
            device_mips_on = false;
            return vhx_set_node_mips(ctx, nullptr, 0);
        }
        if (!force && !mips_dirty && device_mips_on) return VHX_OK;
        const int rc = vhx_set_node_mips(ctx, node_mips.data(), (uint32_t)node_mips.size());
        if (rc) return rc;
        mips_dirty = false;
        device_mips_on = true;
        return VHX_OK;
    }

    uint32_t solid_descriptor(uint32_t value) {
        auto it = solid_index.find(value);
        if (it != solid_index.end()) return 0x80000000u | it->second;
        const uint32_t i = (uint32_t)solid_values.size();
        solid_values.push_back(value);
        solid_index[value] = i;
        return 0x80000000u | i;
    }

    // ------------------------------------------------------------------------------------------ view sizing
    void size_view() {  // view.rs:50-69
        const float dist = view_distance;
        const uint32_t levels = max_mip_level();
        size_t nodes = 0;
        for (uint32_t level = 1; level <= levels; ++level) {
            uint32_t cube = tree->brick_dim;
            for (uint32_t k = 0; k < level; ++k) cube *= 4;
            nodes += (size_t)std::pow(std::ceil(dist / (float)cube), 3.f);
        }
        const size_t per_axis = (size_t)std::ceil(dist / (float)tree->brick_dim);
        nodes_in_view = std::max<size_t>(nodes, 1);
        bricks_in_view = std::max<size_t>((per_axis * per_axis * per_axis + nodes_in_view) / 4, 1);
    }
    void alloc_mirror() {
        node_type.assign(nodes_in_view, VHX_NODE_NOTHING);
        node_ocbits.assign(nodes_in_view, 0);
        node_children.assign(nodes_in_view * kChildren, kEmpty);
        node_mips.assign(nodes_in_view, kEmpty);
        voxels.assign(bricks_in_view * (size_t)bd() * bd() * bd(), 0u);
    }
    void reset_targets() {  // UploadQueueTargets::reset + view.reload (view.rs:141-145)
        brick_by_index.clear();
        brick_by_owner.clear();
        meta_by_key.clear();
        key_by_meta.clear();
        std::fill(resident_key.begin(), resident_key.end(), 0u);
        nodes_to_see.n_resident = 0;
        node_index_vs_parent.clear();
        nodes_to_see.clear();
        view_walk.valid = false;
        bricks_to_upload.clear();
        reload = true;
        rebuild_pending = false;  // the reload rebuilds at the current viewport
    }

    // --------------------------------------------------------------------------------------------- rebuild
    // add_children_nodes_to_upload_queue (upload_queue.rs:144-207): every valid child of a relevant sectant joins the
    // view set, recursively down to min_mip. The walk only reads the tree, and the view set is a set, so subtrees run on
    // host threads into lists of their own that are merged afterwards: the same set as the serial walk (a 1024^3 tree at
    // view distance 256 holds 126 k nodes in view).
    struct ViewItem {
        size_t key;
        Cube nb;
        uint32_t mip;
    };
    // the relevant-sectant mask each exploring node of the view had in the walk that last explored it, with the box
    // corner it was computed for (incremental rebuild): written by the walks (one element per node key, so the threads
    // of a full walk write disjoint elements); sized to the node pool before a walk
    struct VMask {
        uint64_t m;
        U3 lo;
    };
    mutable std::vector<VMask> vmask;
    template <class F>
    void view_children(const ViewItem &it, F3 vc, float dist, uint32_t min_mip, F &&visit) const {
        if (it.mip < min_mip) return;
        const float include = dist * std::pow(4.f, (float)it.mip - 1.f);
        const F3 c = sub(vc, unit(include / 2.f));
        const U3 cbl{round_u32(c.x), round_u32(c.y), round_u32(c.z)};
        if (node(it.key).content != Content::Internal) return;
        uint64_t m = 0;
        relevant_sectants(it.nb, cbl, as_u32(include), [&](U3, U3, uint8_t cs, const Cube &tb) {
            m |= 1ull << cs;
            size_t ck;
            if (valid_child(it.key, cs, ck)) visit(ViewItem{ck, tb, it.mip - 1});
        });
        if (it.key < vmask.size()) vmask[it.key] = VMask{m, cbl};
    }
    void view_subtree(const ViewItem &it, F3 vc, float dist, uint32_t min_mip, std::vector<size_t> &out) const {
        view_children(it, vc, dist, min_mip, [&](const ViewItem &ch) {
            out.push_back(ch.key);
            view_subtree(ch, vc, dist, min_mip, out);
        });
    }
    void add_children_nodes_to_upload_queue(size_t key, Cube nb, uint32_t mip_level, F3 vc, float dist,
                                            uint32_t min_mip) {
        // breadth-first until there are enough subtrees to share out (each level's children join the set here)
        std::vector<ViewItem> front{ViewItem{key, nb, mip_level}}, next;
        for (int level = 0; level < 2 && !front.empty() && front.size() < 64; ++level) {
            next.clear();
            for (const ViewItem &it : front)
                view_children(it, vc, dist, min_mip, [&](const ViewItem &ch) {
                    nodes_to_see.insert(ch.key);
                    next.push_back(ch);
                });
            front.swap(next);
        }
        const unsigned nt = (unsigned)std::min<size_t>(
            front.size(), std::max(1u, std::min(16u, std::thread::hardware_concurrency())));
        // each thread collects into a vector of its own, handed over at its end (per-subtree vectors side by side had
        // their headers share cache lines between threads: every push_back bounced a line)
        std::vector<std::vector<size_t>> lists(std::max(1u, nt));
        std::atomic<size_t> at{0};
        auto work = [&](unsigned k) {
            std::vector<size_t> mine;
            for (size_t i; (i = at.fetch_add(1)) < front.size();) view_subtree(front[i], vc, dist, min_mip, mine);
            lists[k] = std::move(mine);
        };
        if (nt <= 1) {
            work(0);
        } else {
            // threads 1..nt-1 help the calling thread, which takes part itself (slot 0); a thread that cannot be created
            // (std::system_error under a thread limit) is simply missing: the work queue is shared, so the threads that
            // exist finish it, and no exception crosses the C ABI
            std::vector<std::thread> pool;
            for (unsigned k = 1; k < nt; ++k) {
                try {
                    pool.emplace_back(work, k);
                } catch (const std::system_error &) {
                    break;
                }
            }
            work(0);
            for (auto &th : pool) th.join();
        }
        for (const auto &l : lists)
            for (size_t k : l) nodes_to_see.insert(k);
    }
    // Incremental rebuild: the view set of a rebuild is the root path to the walk root plus every
    // node reached from the walk root through relevant sectants (view_children: a node at MIP level m >= min_mip takes
    // its children that overlap the include box B_m, of edge dist * 4^(m - 1) around the clamped viewport centre). When
    // the walk root, its path, the view distance and the deepest level are those of the last rebuild, the new set is
    // the last one changed only where the boxes moved: starting at the walk root, a child relevant under both centres
    // is descended into unless its whole cube lies inside the smallest box any node of its subtree explores with, under
    // both centres (then every node below it was and stays in the view: every child of a node inside its box is
    // relevant); a child relevant under only the new centre joins with its new subtree, one relevant under only the
    // old centre leaves with its old subtree. The result is the set a full rebuild makes (tests/test_streaming.py
    // compares them after every move); the walk costs the shell of nodes near the moving box faces.
    struct ViewWalk {
        bool valid = false;
        std::vector<size_t> path;  // root .. walk root
        Cube nb{};
        uint32_t mip = 0, min_mip = 0;
        F3 vc{}, center{};  // the clamped and the given centre of the last rebuild
        float dist = 0.f;
        int mip1_internal = -1;  // an Internal node at MIP level 1 exists (explores with B_1): -1 unknown
        uint64_t edit_seq = 0;   // the tree's edit_seq the walk (and mip1_internal) was made on
    } view_walk;
    uint64_t rebuilds_full = 0, rebuilds_incremental = 0;
    uint64_t dbg_shell = 0, dbg_ins = 0, dbg_era = 0;
    // whether any Internal node sits at MIP level 1 (children of the size of a brick); then subtrees explore down to
    // B_1, otherwise down to B_2
    bool mip1_internal() {
        if (view_walk.mip1_internal >= 0) return view_walk.mip1_internal != 0;
        bool found = false;
        std::vector<std::pair<size_t, uint32_t>> st{{0, max_mip_level()}};
        while (!st.empty() && !found) {
            const auto [k, m] = st.back();
            st.pop_back();
            if (!key_valid(k) || node(k).content != Content::Internal || m == 0) continue;
            if (m == 1) {
                found = true;
                break;
            }
            for (uint8_t c = 0; c < kChildren; ++c) {
                size_t ck;
                if (valid_child(k, c, ck)) st.push_back({ck, m - 1});
            }
        }
        view_walk.mip1_internal = found ? 1 : 0;
        return found;
    }
    static bool cube_in_box(const Cube &c, U3 lo, uint32_t size) {
        const float s = (float)size;
        return (float)lo.x <= c.min.x && (float)lo.y <= c.min.y && (float)lo.z <= c.min.z && c.min.x + c.size <= (float)lo.x + s &&
               c.min.y + c.size <= (float)lo.y + s && c.min.z + c.size <= (float)lo.z + s;
    }
    // relevant_sectants of a node depends on the box corner `lo` (edge I) only through, per axis, the node cell holding the
    // lower face (or "below the node" / "past it") and the number of node cells the upper face lo + I reaches into (see
    // relevant_sectants, boxtree.hpp: the samples start at max(lo, node min) and step by a cell; a cell is taken while
    // its lower edge lies below lo + I): boxes with equal keys give the same mask
    static uint32_t mask_key(const Cube &nb, U3 lo, uint32_t I) {
        const float cell = nb.size / 4.f, nx[3] = {nb.min.x, nb.min.y, nb.min.z};
        const uint32_t l[3] = {lo.x, lo.y, lo.z};
        uint32_t key = 0;
        for (int a = 0; a < 3; ++a) {
            const float lf = (float)l[a], end = lf + (float)I;
            int klo = lf > nx[a] + nb.size ? 5 : (lf < nx[a] ? -1 : std::min(4, (int)std::floor((lf - nx[a]) / cell)));
            int kend = (int)std::ceil((end - nx[a]) / cell);
            kend = kend < 0 ? 0 : (kend > 4 ? 4 : kend);
            key |= ((uint32_t)(klo + 1) | ((uint32_t)kend << 3)) << (6 * a);
        }
        return key;
    }
    static void include_box(F3 vc, float dist, uint32_t mip, U3 &lo, uint32_t &size) {  // view_children's box
        const float include = dist * std::pow(4.f, (float)mip - 1.f);
        const F3 c = sub(vc, unit(include / 2.f));
        lo = U3{round_u32(c.x), round_u32(c.y), round_u32(c.z)};
        size = as_u32(include);
    }
    uint64_t relevant_mask(const Cube &nb, U3 lo, uint32_t size) const {
        uint64_t m = 0;
        relevant_sectants(nb, lo, size, [&](U3, U3, uint8_t cs, const Cube &) { m |= 1ull << cs; });
        return m;
    }
    // the node's mask under box corner lo: its cached one when the keys agree, else computed
    uint64_t mask_at(const ViewItem &it, U3 lo, uint32_t size, uint32_t key) {
        const VMask &c = vmask[it.key];
        if (mask_key(it.nb, c.lo, size) == key) return c.m;
        return relevant_mask(it.nb, lo, size);
    }
    void view_subtree_apply(const ViewItem &it, F3 vc, float dist, uint32_t min_mip, bool insert) {
        std::vector<size_t> keys;
        view_subtree(it, vc, dist, min_mip, keys);
        for (size_t k : keys) insert ? nodes_to_see.insert(k) : nodes_to_see.erase(k);
    }
    static Cube child_cube(const Cube &nb, uint8_t cs) {  // relevant_sectants' tb (integer cubes: floor / ceil exact)
        Cube tb = child_bounds_for(nb, cs);
        return Cube{F3{std::floor(tb.min.x), std::floor(tb.min.y), std::floor(tb.min.z)}, std::ceil(tb.size)};
    }
    // the children of a node whose cubes lie inside the box [lo, lo + I] (all axes): per axis the node cells inside the
    // box's interval, combined into a sectant mask (bit x + 4y + 16z)
    static uint64_t inside_mask(const Cube &nb, U3 lo, uint32_t I) {
        const float cell = nb.size / 4.f, mn[3] = {nb.min.x, nb.min.y, nb.min.z};
        const uint32_t l[3] = {lo.x, lo.y, lo.z};
        uint32_t ax[3];
        for (int a = 0; a < 3; ++a) {
            ax[a] = 0;
            const float lf = (float)l[a], hf = lf + (float)I;
            for (uint32_t c = 0; c < 4; ++c)
                if (lf <= mn[a] + (float)c * cell && mn[a] + (float)(c + 1) * cell <= hf) ax[a] |= 1u << c;
        }
        uint64_t row = 0, m = 0;
        for (uint32_t y = 0; y < 4; ++y)
            if ((ax[1] >> y) & 1u) row |= (uint64_t)ax[0] << (4u * y);
        for (uint32_t z = 0; z < 4; ++z)
            if ((ax[2] >> z) & 1u) m |= row << (16u * z);
        return m;
    }
    // include boxes of the two centres per MIP level (shell walk)
    struct LevelBoxes {
        U3 lo0[32], lo1[32];
        uint32_t size[32];
    };
    void shell_walk(const ViewItem &it, const LevelBoxes &bx, F3 vc1, float dist, uint32_t min_mip, uint32_t jmin) {
        if (it.mip < min_mip || it.mip >= 32 || node(it.key).content != Content::Internal) return;  // explores in neither
        const U3 b0 = bx.lo0[it.mip], b1 = bx.lo1[it.mip];
        const uint32_t sz = bx.size[it.mip];
        const uint32_t k0 = mask_key(it.nb, b0, sz), k1 = mask_key(it.nb, b1, sz);
        const uint64_t m0 = mask_at(it, b0, sz, k0), m1 = k1 == k0 ? m0 : relevant_mask(it.nb, b1, sz);
        vmask[it.key] = VMask{m1, b1};
        // children relevant under both centres need a look only if their subtrees explore (level >= jmin) and their
        // cubes are not inside the smallest exploring box under both centres (then nothing below them changes)
        uint64_t look = m0 ^ m1;
        if (it.mip - 1 >= jmin)
            look |= (m0 & m1) & ~(inside_mask(it.nb, bx.lo0[jmin], bx.size[jmin]) &
                                  inside_mask(it.nb, bx.lo1[jmin], bx.size[jmin]));
        for (; look; look &= look - 1) {
            const uint8_t cs = (uint8_t)__builtin_ctzll(look);
            size_t ck;
            if (!valid_child(it.key, cs, ck)) continue;
            const ViewItem ch{ck, child_cube(it.nb, cs), it.mip - 1};
            const bool in0 = (m0 >> cs) & 1u, in1 = (m1 >> cs) & 1u;
            if (in1 && !in0) {
                nodes_to_see.insert(ck);
                view_subtree_apply(ch, vc1, dist, min_mip, true);  // records the masks of its explored nodes
            } else if (in0 && !in1) {
                std::vector<size_t> keys;
                view_subtree_cached(ch, min_mip, keys);  // the subtree as the view holds it
                for (size_t k : keys) nodes_to_see.erase(k);
                nodes_to_see.erase(ck);
            } else {
                shell_walk(ch, bx, vc1, dist, min_mip, jmin);
            }
        }
    }
    // the explored subtree below `it` as the last walks left it (cached masks: the old centre's, or equal to them)
    void view_subtree_cached(const ViewItem &it, uint32_t min_mip, std::vector<size_t> &out) const {
        if (it.mip < min_mip || node(it.key).content != Content::Internal) return;
        for (uint64_t m = vmask[it.key].m; m; m &= m - 1) {
            const uint8_t cs = (uint8_t)__builtin_ctzll(m);
            size_t ck;
            if (!valid_child(it.key, cs, ck)) continue;
            out.push_back(ck);
            view_subtree_cached(ViewItem{ck, child_cube(it.nb, cs), it.mip - 1}, min_mip, out);
        }
    }
    void rebuild(F3 center_, float dist) {  // upload_queue.rs:60-142
        // a walk made on an older tree is no base for an incremental rebuild: collect_frame runs a pending move's
        // rebuild before handle_tree_updates applies the same upload's queued edits, and the cached masks and levels
        // describe the tree before them
        if (view_walk.edit_seq != tree->edit_seq) {
            view_walk.valid = false;
            view_walk.mip1_internal = -1;
        }
        walk_started = false;
        last_cycle_work = UINT64_MAX;
        const float S = (float)tree->boxtree_size;
        const F3 vc = f3(clampf(center_.x, 0.f, S), clampf(center_.y, 0.f, S), clampf(center_.z, 0.f, S));
        const F3 bl_ = sub(center_, unit(dist / 2.f));
        const F3 bl = f3(clampf(bl_.x, 0.f, S), clampf(bl_.y, 0.f, S), clampf(bl_.z, 0.f, S));
        F3 tr = add(bl, unit(dist));
        tr = f3(clampf(tr.x, 0.f, S), clampf(tr.y, 0.f, S), clampf(tr.z, 0.f, S));
        uint32_t deepest = as_u32(std::ceil(length(sub(bl_, bl)) / dist));
        deepest = std::max(std::min(deepest, max_mip_level()), 1u);
        bool have_parent = false;
        size_t parent_key = 0;
        Cube parent_bounds{};
        uint32_t parent_mip = 0;
        Cube nb{f3(0.f, 0.f, 0.f), S};
        uint32_t mip = max_mip_level();
        size_t key = 0;
        // Deviation: the whole access path root -> center joins the view set. The reference marks only the center
        // node and its parent's relevant children, which leaves the root's slot 0 evictable and makes a center two
        // or more levels down unreachable for next_valid_node (it only descends into nodes of the view set).
        std::vector<size_t> path{0};
        for (;;) {
            const Content c = node(key).content;
            if (c != Content::Internal || (nb.size / 4.f) <= dist || !contains(nb, bl) || !contains(nb, tr)) break;
            const uint8_t cs = offset_sectant(sub(vc, nb.min), nb.size);  // Cube::sectant_for
            size_t ck;
            if (!valid_child(key, cs, ck)) break;
            have_parent = true;
            parent_key = key;
            parent_bounds = nb;
            parent_mip = mip;
            key = ck;
            path.push_back(ck);
            nb = child_bounds_for(nb, cs);
            mip -= 1;
        }
        path.push_back(key);
        const ViewItem wr = have_parent ? ViewItem{parent_key, parent_bounds, parent_mip} : ViewItem{key, nb, mip};
        ViewWalk &vw = view_walk;
        if (vmask.size() < tree->nodes.len()) {
            vmask.resize(tree->nodes.len(), VMask{0, U3{0, 0, 0}});
            vw.valid = false;  // nodes the cache does not know yet
        }
        if (vw.valid && vw.path == path && vw.dist == dist && vw.min_mip == deepest && vw.mip == wr.mip &&
            vw.nb.min.x == wr.nb.min.x && vw.nb.min.y == wr.nb.min.y && vw.nb.min.z == wr.nb.min.z &&
            vw.nb.size == wr.nb.size) {
            // the same walk root: change the set where the include boxes moved
            const uint32_t jmin = std::max(deepest, mip1_internal() ? 1u : 2u);
            LevelBoxes bx;
            for (uint32_t m = 1; m <= std::min(wr.mip, 31u); ++m) {
                include_box(vw.vc, dist, m, bx.lo0[m], bx.size[m]);
                include_box(vc, dist, m, bx.lo1[m], bx.size[m]);
            }
            shell_walk(wr, bx, vc, dist, deepest, jmin);
            ++rebuilds_incremental;
        } else {
            nodes_to_see.clear();
            for (size_t k : path) nodes_to_see.insert(k);
            add_children_nodes_to_upload_queue(wr.key, wr.nb, wr.mip, vc, dist, deepest);
            ++rebuilds_full;
        }
        vw.valid = true;
        vw.edit_seq = tree->edit_seq;
        vw.path = std::move(path);
        vw.nb = wr.nb;
        vw.mip = wr.mip;
        vw.min_mip = deepest;
        vw.vc = vc;
        vw.center = center_;
        vw.dist = dist;
    }
    // diagnostics (vhx_stream_view_set_check): the view set a full rebuild at the last rebuild's viewport makes, against
    // the one held (after incremental rebuilds); the stream's state is left as it was
    bool view_set_matches_full() {
        if (!view_walk.valid) return true;
        KeySet held = nodes_to_see;
        const ViewWalk vw = view_walk;
        const bool ws = walk_started;
        const uint64_t lcw = last_cycle_work, nf = rebuilds_full;
        view_walk.valid = false;
        rebuild(vw.center, vw.dist);
        std::vector<size_t> a(held.begin(), held.end()), b(nodes_to_see.begin(), nodes_to_see.end());
        std::sort(a.begin(), a.end());
        std::sort(b.begin(), b.end());
        nodes_to_see = std::move(held);
        view_walk = vw;
        walk_started = ws;
        last_cycle_work = lcw;
        rebuilds_full = nf;
        return a == b;
    }
    std::vector<StackItem> node_stack_init() const {  // streaming/mod.rs:553-559
        return {StackItem{0, (uint8_t)kChildren, Cube{f3(0.f, 0.f, 0.f), (float)tree->boxtree_size}}};
    }

    // -------------------------------------------------------------------------------------------- eviction
    std::vector<std::pair<size_t, uint64_t>> erase_node_child(size_t meta, size_t cs) {  // cache.rs:41-145
        std::vector<std::pair<size_t, uint64_t>> modified{{meta, 1ull << cs}};
        auto pk = key_by_meta.find(meta);
        if (pk == key_by_meta.end()) return modified;  // the reference unwraps (panics) here
        const size_t parent_key = pk->second;
        const size_t off = meta * kChildren + cs;
        const uint32_t desc = node_children[off];
        node_index_vs_parent.erase(desc);
        node_children[off] = kEmpty;
        const Content pc = node(parent_key).content;
        if (pc == Content::Internal) {
            // MIP connection of the erased child (MIP data is Empty in a tree without MIPs: nothing owned)
            if (desc < node_mips.size() && node_mips[desc] != kEmpty) set_mip(desc, kEmpty);
            modified.push_back({desc, 0});
        } else if (pc == Content::Leaf || pc == Content::UniformLeaf) {
            if (desc != kEmpty && !(desc & 0x80000000u)) owner_remove_index(desc & 0x7FFFFFFFu);
        }
        return modified;
    }
    bool first_available_node(size_t &idx, bool &has_parent, std::pair<size_t, uint8_t> &parent) {  // cache.rs:159-185
        size_t v = (victim_node + 1) % nodes_in_view;
        while (v != victim_node) {
            auto it = key_by_meta.find(v);
            if (it == key_by_meta.end() || !nodes_to_see.count(it->second)) {
                victim_node = v;
                idx = v;
                auto p = node_index_vs_parent.find(v);
                has_parent = p != node_index_vs_parent.end();
                if (has_parent) parent = p->second;
                return true;
            }
            v = (v + 1) % nodes_in_view;
        }
        return false;
    }
    bool outside_range(F3 b, float s) const {  // cache.rs:462-469
        const Cube &r = upload_range;
        return (b.x + s) < r.min.x || (r.min.x + r.size) < b.x || (b.y + s) < r.min.y || (r.min.y + r.size) < b.y ||
               (b.z + s) < r.min.z || (r.min.z + r.size) < b.z;
    }
    bool mip_children_all_empty(uint32_t node_key) const {
        auto it = meta_by_key.find(node_key);
        if (it == meta_by_key.end()) return true;
        const size_t m = it->second;
        for (size_t s = 0; s < kChildren; ++s)
            if (node_children[m * kChildren + s] != kEmpty) return false;
        return true;
    }
    bool first_available_brick(float brick_size, size_t &out) {  // cache.rs:460-573
        const size_t start = (size_t)std::max<long long>((long long)victim_brick -
                                                             (long long)brick_unload_search_perimeter / 2, 0);
        const size_t end = std::min(start + brick_unload_search_perimeter, bricks_in_view);
        bool have_priority = false, have_furthest = false;
        size_t priority = 0, furthest = 0;
        float furthest_d = 0.f;
        const F3 half = unit(upload_range.size / 2.f);
        for (size_t i = start; i < end; ++i) {
            auto it = brick_by_index.find(i);
            const Owned o = it == brick_by_index.end() ? Owned{} : it->second;
            if (o.kind == 0) {
                priority = i;
                have_priority = true;
                break;
            } else if (o.kind == 2) {
                if (!nodes_to_see.count(o.node) && mip_children_all_empty(o.node)) {
                    priority = i;
                    have_priority = true;
                    break;
                }
            } else {
                const float d = length(add(sub(o.bl, upload_range.min), half));
                if (outside_range(o.bl, brick_size) && (!have_furthest || d > furthest_d)) {
                    furthest_d = d;
                    furthest = i;
                    have_furthest = true;
                }
            }
        }
        if (have_priority || have_furthest) {
            out = have_priority ? priority : furthest;
            victim_brick = (out + 1) % bricks_in_view;
            return true;
        }
        for (int pass = 0; pass < 2; ++pass) {
            const size_t a = pass == 0 ? end : 0, b = pass == 0 ? bricks_in_view : start;
            for (size_t i = a; i < b; ++i) {
                auto it = brick_by_index.find(i);
                const Owned o = it == brick_by_index.end() ? Owned{} : it->second;
                const bool ok = o.kind == 0 || (o.kind == 2 && !nodes_to_see.count(o.node)) ||
                                (o.kind == 1 && outside_range(o.bl, brick_size));
                if (ok) {
                    victim_brick = (i + 1) % bricks_in_view;
                    out = i;
                    return true;
                }
            }
        }
        return false;
    }

    // ------------------------------------------------------------------------------------------ add_node
    bool add_node(size_t parent_key, uint8_t target_sectant, CacheUpdate &upd) {  // cache.rs:188-455
        const size_t key = target_sectant < kChildren ? child(parent_key, target_sectant) : 0;
        size_t idx = 0;
        bool robbed = false;
        std::pair<size_t, uint8_t> robbed_parent{0, 0};
        if (key == 0) {
            idx = 0;
        } else if (meta_by_key.count(key)) {
            idx = meta_by_key[key];
        } else {
            if (!first_available_node(idx, robbed, robbed_parent)) return false;
        }
        meta_insert(key, idx);
        if (robbed) {
            auto m = erase_node_child(robbed_parent.first, robbed_parent.second);
            upd.modified_nodes.insert(upd.modified_nodes.end(), m.begin(), m.end());
        }
        const Node &n = node(key);
        node_type[idx] = n.content == Content::Leaf          ? VHX_NODE_LEAF
                         : n.content == Content::UniformLeaf ? VHX_NODE_UNIFORM_LEAF
                         : n.content == Content::Internal    ? VHX_NODE_INTERNAL
                                                             : VHX_NODE_NOTHING;
        node_ocbits[idx] = n.occupied_bits;
        std::fill(node_children.begin() + (ptrdiff_t)(idx * kChildren),
                  node_children.begin() + (ptrdiff_t)((idx + 1) * kChildren), kEmpty);
        if (key != 0) {
            auto pmi = meta_by_key.find(parent_key);
            if (pmi == meta_by_key.end()) return false;  // parent not resident (the reference panics)
            const size_t pm = pmi->second;
            node_children[pm * kChildren + target_sectant] = (uint32_t)idx;
            node_index_vs_parent[idx] = {pm, target_sectant};
            upd.modified_nodes.push_back({pm, 1ull << target_sectant});
        }
        upd.modified_nodes.push_back({idx, ~0ull});
        const size_t first = idx * kChildren;
        auto brick_desc = [&](const Brick &b, uint8_t s) -> uint32_t {
            if (b.kind == BrickKind::Solid) return solid_descriptor(b.solid);
            if (b.kind == BrickKind::Empty) return kEmpty;
            Owned o;
            o.kind = 1;
            o.node = (uint32_t)key;
            o.sectant = s;
            auto it = brick_by_owner.find(o.key());
            return it == brick_by_owner.end() ? kEmpty : (0x7FFFFFFFu & (uint32_t)it->second);
        };
        if (n.content == Content::Internal) {
            for (uint8_t s = 0; s < kChildren; ++s) {
                size_t ck;
                if (valid_child(key, s, ck)) {
                    auto it = meta_by_key.find(ck);
                    node_children[first + s] = it == meta_by_key.end() ? kEmpty : (uint32_t)it->second;
                } else {
                    node_children[first + s] = kEmpty;
                }
            }
        } else if (n.content == Content::UniformLeaf) {
            node_children[first] = brick_desc(n.bricks[0], 0);
        } else if (n.content == Content::Leaf) {
            for (uint8_t s = 0; s < kChildren; ++s) node_children[first + s] = brick_desc(n.bricks[s], s);
        }
        set_mip(idx, mip_descriptor(key));  // cache.rs:435-453
        return true;
    }

    // ----------------------------------------------------------------------------------------- add_brick
    bool add_brick(const Owned &req, CacheUpdate &upd) {  // cache.rs:575-716
        size_t bi;
        if (!first_available_brick((float)tree->brick_dim, bi)) return false;
        auto prev = brick_by_index.find(bi);
        const Owned old = prev == brick_by_index.end() ? Owned{} : prev->second;
        if (old.kind == 1) {
            auto m = meta_by_key.find(old.node);
            if (m != meta_by_key.end()) {
                auto mod = erase_node_child(m->second, old.sectant);
                upd.modified_nodes.insert(upd.modified_nodes.end(), mod.begin(), mod.end());
            }
        } else if (old.kind == 2) {
            auto m = meta_by_key.find(old.node);
            if (m != meta_by_key.end()) {
                set_mip(m->second, kEmpty);
                upd.modified_nodes.push_back({m->second, 0});
            }
        }
        auto pmi = meta_by_key.find(req.node);
        if (pmi == meta_by_key.end()) return true;  // owner no longer resident: nothing to attach (reference panics)
        const size_t pm = pmi->second;
        if (req.kind == 1) {
            upd.modified_nodes.push_back({pm, 1ull << req.sectant});
            node_children[pm * kChildren + req.sectant] = 0x7FFFFFFFu & (uint32_t)bi;
        } else {
            upd.modified_nodes.push_back({pm, 0});
            owner_insert(bi, req);
            set_mip(pm, stream_mips() ? mip_descriptor(req.node) : (0x7FFFFFFFu & (uint32_t)bi));
            upd.brick_updates.push_back({bi, req});
            return true;
        }
        owner_insert(bi, req);
        upd.brick_updates.push_back({bi, req});
        return true;
    }

    // ----------------------------------------------------------------------------------------- process
    std::vector<Owned> process_node_child_bricks(size_t key, const Cube &nb, U3 vbl, float dist) const {
        std::vector<Owned> res;  // upload_queue.rs:406-476
        const Node &n = node(key);
        if (n.content == Content::UniformLeaf) {
            if (n.bricks[0].kind == BrickKind::Parted) {
                Owned o;
                o.kind = 1;
                o.node = (uint32_t)key;
                o.sectant = 0;
                o.bl = f3(std::round(nb.min.x), std::round(nb.min.y), std::round(nb.min.z));
                if (!owner_has(o)) res.push_back(o);
            }
        } else if (n.content == Content::Leaf) {
            relevant_sectants(nb, vbl, as_u32(dist), [&](U3, U3, uint8_t cs, const Cube &tb) {
                if (n.bricks[cs].kind != BrickKind::Parted) return;
                Owned o;
                o.kind = 1;
                o.node = (uint32_t)key;
                o.sectant = cs;
                o.bl = f3(std::round(tb.min.x), std::round(tb.min.y), std::round(tb.min.z));
                if (!owner_has(o)) res.push_back(o);
            });
        }
        return res;
    }
    bool next_valid_node(size_t &parent_out, uint8_t &sect_out, size_t &child_out, Cube &bounds_out) {
        if (target_node_stack.empty()) return false;  // upload_queue.rs:480-574
        auto &top = target_node_stack.back();
        const size_t cur = top.node;
        uint8_t ts = top.sectant;
        const Cube cb = top.bounds;
        // the root's cursor at 64 reads as "start": once the walk is through, it starts over from the root, so the
        // reference streams continuously (and picks up bricks that were evicted or not yet uploaded)
        if (cur == 0 && ts == kChildren) {
            if (walk_started) last_cycle_work = cycle_work;
            cycle_work = 0;
            walk_started = true;
            top.sectant = 0;
            parent_out = cur;
            sect_out = (uint8_t)kChildren;
            child_out = cur;
            bounds_out = cb;
            return true;
        }
        for (;;) {
            if (ts >= kChildren || !node(cur).has_children) {
                target_node_stack.pop_back();
                if (!target_node_stack.empty()) {
                    auto &p = target_node_stack.back();
                    p.sectant += 1;
                    parent_out = p.node;
                    sect_out = (uint8_t)(p.sectant - 1);
                    child_out = cur;
                    bounds_out = cb;
                    return true;
                }
                return false;
            }
            size_t ck = child(cur, ts);
            while (ts < kChildren && (!key_valid(ck) || !nodes_to_see.count(ck))) {
                ts += 1;
                if (ts < kChildren) ck = child(cur, ts);
            }
            if (ts >= kChildren) continue;
            if (!node(ck).has_children || node(ck).is_occluded()) {
                const uint8_t rs = ts;
                const size_t rc = ck;
                ts += 1;
                ck = ts < kChildren ? child(cur, ts) : SIZE_MAX;
                while (ts < kChildren && !key_valid(ck)) {
                    ts += 1;
                    if (ts < kChildren) ck = child(cur, ts);
                }
                target_node_stack.back().sectant = ts;
                parent_out = cur;
                sect_out = rs;
                child_out = rc;
                bounds_out = child_bounds_for(cb, rs);
                return true;
            }
            target_node_stack.back().sectant = ts;
            target_node_stack.push_back(StackItem{ck, 0, child_bounds_for(cb, ts)});
            parent_out = cur;
            sect_out = ts;
            child_out = ck;
            bounds_out = cb;
            return true;
        }
    }
    // returns false when the view ran out of capacity (re_evaluate_view_size was applied)
    bool process(std::vector<CacheUpdate> &updates) {  // upload_queue.rs:218-404
        if (reload) {
            rebuild_pending = false;  // superseded: the reload rebuilds at the current viewport
            rebuild(origin, view_distance);
            target_node_stack = node_stack_init();
            reload = false;
        }
        for (size_t k = 0; k < node_uploads_per_frame && !target_node_stack.empty(); ++k) {
            size_t parent, key;
            uint8_t ts;
            Cube nb;
            if (!next_valid_node(parent, ts, key, nb)) break;
            if (!meta_by_key.count(key)) {
                CacheUpdate u;
                if (!add_node(parent, ts, u)) return re_evaluate_view_size();
                updates.push_back(std::move(u));
                ++cycle_work;
            }
            {  // the MIP of every node takes a brick slot (empty MIPs upload no voxels)
                Owned mip;
                mip.kind = 2;
                mip.node = (uint32_t)key;
                CacheUpdate u;
                if (!add_brick(mip, u)) return re_evaluate_view_size();
                updates.push_back(std::move(u));
            }
            const F3 vbl_f = sub(origin, unit(view_distance / 2.f));
            const U3 vbl{round_u32(vbl_f.x), round_u32(vbl_f.y), round_u32(vbl_f.z)};
            auto more = process_node_child_bricks(key, nb, vbl, view_distance);
            cycle_work += more.size();
            bricks_to_upload.insert(bricks_to_upload.end(), more.begin(), more.end());
        }
        if (!bricks_to_upload.empty()) {
            const size_t take = std::min(brick_uploads_per_frame, bricks_to_upload.size());
            std::vector<Owned> reqs(bricks_to_upload.end() - (ptrdiff_t)take, bricks_to_upload.end());
            bricks_to_upload.resize(bricks_to_upload.size() - take);
            for (const Owned &r : reqs) {
                if (owner_has(r)) continue;
                CacheUpdate u;
                if (!add_brick(r, u)) return re_evaluate_view_size();
                updates.push_back(std::move(u));
            }
        }
        return true;
    }
    // handle_tree_updates, streaming/mod.rs:35-286: up to n queued tree changes, each re-uploading the root, the nodes
    // along the change's access stack (with their MIP slots) and the changed bricks of its bottom node. Returns false
    // when the view ran out of capacity (re_evaluate_view_size was applied; the updates so far are still written).
    bool handle_tree_updates(std::vector<CacheUpdate> &updates, size_t n) {
        for (size_t k = 0; k < n; ++k) {
            if (tree->changes.empty()) break;
            const BoxTree::Change ch = tree->changes.front();
            tree->changes.pop_front();
            if (ch.node_stack.empty()) continue;  // the reference asserts a root-first stack
            auto add_mip = [&](size_t key) -> bool {  // MIP slot of a node: re-upload when owned, else a new slot
                Owned mip;
                mip.kind = 2;
                mip.node = (uint32_t)key;
                auto own = brick_by_owner.find(mip.key());
                if (own != brick_by_owner.end()) {  // re-upload the (changed) MIP into its slot
                    auto m = meta_by_key.find(key);
                    if (m != meta_by_key.end()) set_mip(m->second, mip_descriptor(key));
                    CacheUpdate u;
                    u.brick_updates.push_back({own->second, mip});
                    updates.push_back(std::move(u));
                    return true;
                }
                CacheUpdate u;
                if (!add_brick(mip, u)) return false;
                updates.push_back(std::move(u));
                return true;
            };
            {
                CacheUpdate u;
                if (!add_node(0, (uint8_t)kChildren, u)) return re_evaluate_view_size();
                updates.push_back(std::move(u));
            }
            if (!add_mip(0)) return re_evaluate_view_size();
            const size_t parent_key = ch.node_stack.back().first;
            Cube node_bounds{f3(0.f, 0.f, 0.f), (float)tree->boxtree_size};
            for (const auto &e : ch.node_stack) nodes_to_see.insert(e.first);
            // the set now holds more than a walk's: the next rebuild is a full one; the tree changed: so may the
            // levels of its Internal nodes
            view_walk.valid = false;
            view_walk.mip1_internal = -1;
            for (const auto &e : ch.node_stack) {
                size_t ck;
                if (valid_child(e.first, e.second, ck)) {  // BoxTree::valid_child_for
                    CacheUpdate u;
                    if (!add_node(e.first, e.second, u)) return re_evaluate_view_size();
                    updates.push_back(std::move(u));
                    if (!add_mip(ck)) return re_evaluate_view_size();
                }
                node_bounds = child_bounds_for(node_bounds, e.second);
            }
            // the bottom node's bricks: re-upload the resident ones, request slots for the others. Deviation: a
            // sectant whose brick is not Parted (the reference only debug-asserts that it is) is skipped; add_node
            // above already wrote its Solid / Empty descriptor
            const Node &pn = node(parent_key);
            auto brick_owner = [&](uint8_t sec, const Cube &b) {
                Owned o;
                o.kind = 1;
                o.node = (uint32_t)parent_key;
                o.sectant = sec;
                o.bl = f3(std::round(b.min.x), std::round(b.min.y), std::round(b.min.z));
                return o;
            };
            std::vector<Owned> fresh;
            if (pn.content == Content::UniformLeaf && pn.bricks[0].kind == BrickKind::Parted) {
                const Owned o = brick_owner(0, node_bounds);
                auto it = brick_by_owner.find(o.key());
                if (it != brick_by_owner.end()) {
                    CacheUpdate u;
                    u.brick_updates.push_back({it->second, o});
                    updates.push_back(std::move(u));
                } else {
                    fresh.push_back(o);
                }
            } else if (pn.content == Content::Leaf) {
                for (uint8_t sec : ch.updated_sectants) {
                    if (sec >= kChildren || pn.bricks[sec].kind != BrickKind::Parted) continue;
                    const Owned o = brick_owner(sec, child_bounds_for(node_bounds, sec));
                    auto it = brick_by_owner.find(o.key());
                    if (it != brick_by_owner.end()) {
                        CacheUpdate u;
                        u.brick_updates.push_back({it->second, o});
                        updates.push_back(std::move(u));
                    } else {
                        fresh.push_back(o);
                    }
                }
            }
            for (const Owned &o : fresh) {
                CacheUpdate u;
                if (!add_brick(o, u)) return re_evaluate_view_size();
                updates.push_back(std::move(u));
            }
            if (tree->changes.empty()) {
                // Deviation: the reference only restarts the tree scan here; the view set is recomputed too, so
                // nodes an edit created off its access path (the 64 nodes of a leaf subdivided by an insert, a new
                // subtree's children) join the view and are uploaded by the scan, instead of staying missing until
                // the viewport moves
                rebuild(origin, view_distance);
                target_node_stack = node_stack_init();  // restart the tree scan
            }
        }
        return true;
    }
    bool re_evaluate_view_size() {  // streaming/mod.rs:292-340
        const size_t need_nodes = nodes_to_see.size();
        if (need_nodes > nodes_in_view) nodes_in_view = (size_t)((float)need_nodes * 1.2f);
        const size_t need_bricks = bricks_to_upload.size() + brick_by_index.size() + need_nodes;
        if (need_bricks > bricks_in_view) bricks_in_view = (size_t)((float)need_bricks * 1.2f);
        node_type.resize(nodes_in_view, VHX_NODE_NOTHING);
        node_ocbits.resize(nodes_in_view, 0);
        node_children.resize(nodes_in_view * kChildren, kEmpty);
        node_mips.resize(nodes_in_view, kEmpty);
        voxels.resize(bricks_in_view * (size_t)bd() * bd() * bd(), 0u);
        resize = true;
        return false;
    }

    // ------------------------------------------------------------------------------------------- device side
    vhx_tree_desc desc() const {
        vhx_tree_desc d{};
        d.boxtree_size = tree->boxtree_size;
        d.brick_dim = tree->brick_dim;
        d.node_count = (uint32_t)nodes_in_view;
        d.brick_count = (uint32_t)bricks_in_view;
        d.solid_count = (uint32_t)solid_capacity;
        d.color_count = kPaletteCapacity;
        d.data_count = kPaletteCapacity;
        d.node_type = node_type.data();
        d.node_ocbits = node_ocbits.data();
        d.node_children = node_children.data();
        d.voxels = voxels.data();
        return d;
    }
    int upload_all() {  // (re)creates the device view from the host mirror (view creation / view.resize)
        std::vector<uint32_t> solid(solid_capacity, 0u), color(kPaletteCapacity, 0u), data(kPaletteCapacity, 0u);
        std::copy(solid_values.begin(), solid_values.end(), solid.begin());
        std::copy(color_palette.begin(), color_palette.end(), color.begin());
        std::copy(data_palette.begin(), data_palette.end(), data.begin());
        vhx_tree_desc d = desc();
        d.solid_values = solid.data();
        d.color_palette = color.data();
        d.data_palette = data.data();
        int rc = ctx ? vhx_upload_tree(ctx, &d) : VHX_OK;  // ctx == NULL: host-only view (tests)
        if (rc) return rc;
        device_mips_on = false;  // a new upload switches them off on the device
        if ((rc = sync_device_mips(true))) return rc;
        uploaded_solid_size = solid_values.size();
        device_valid = true;
        resize = false;
        return VHX_OK;
    }
    // the frame's ranged writes, issued together by flush() as one vhx_update_ranges call (one staged host-to-device
    // copy and one scatter kernel per frame instead of one transfer per range); the sources are the host mirror's
    // arrays, unchanged until the flush
    std::vector<vhx_range> frame_writes;
    int write(int buf, size_t off, size_t n, const void *src) {
        if (n == 0) return VHX_OK;
        const size_t esz = buf == VHX_BUF_NODE_OCBITS ? 8 : 4;
        last_bytes += n * esz;
        vhx_range r{};
        r.buffer_id = buf;
        r.elem_offset = off;
        r.elem_count = n;
        r.src = src;
        frame_writes.push_back(r);
        return VHX_OK;
    }
    int flush() {
        const int rc = ctx && !frame_writes.empty()
                           ? vhx_update_ranges(ctx, frame_writes.data(), (uint32_t)frame_writes.size())
                           : VHX_OK;
        frame_writes.clear();
        return rc;
    }
    int upload_frame() {
        frame_writes.clear();
        const int rc = collect_frame();
        int frc = flush();  // also after a capacity stop: what was decided before it is written, as before
        if (!frc && device_valid) frc = sync_device_mips(false);
        return rc ? rc : frc;
    }
    // K frames of upload decisions (each exactly one upload_frame's: the reference's per-frame rates), written as ONE
    // vhx_update_ranges: one tree version for the K frames a renderer keeps in flight until the next call. A range's
    // source points into the host mirror, which a later frame of the batch may overwrite or reallocate (palettes are
    // reassigned, the solid table grows), so each frame's sources are copied when the frame is decided; the ranges
    // keep their order, so a later frame's write of the same elements wins, as in K separate calls.
    std::vector<std::vector<uint8_t>> batch_store;
    uint64_t batch_bytes = 0, batch_nodes = 0, batch_bricks = 0;
    int upload_frames(uint32_t K) {
        std::vector<vhx_range> all;
        batch_store.clear();
        batch_bytes = batch_nodes = batch_bricks = 0;
        int rc = VHX_OK;
        for (uint32_t k = 0; k < K && !rc; ++k) {
            frame_writes.clear();
            rc = collect_frame();
            batch_bytes += last_bytes;
            batch_nodes += last_nodes;
            batch_bricks += last_bricks;
            for (vhx_range r : frame_writes) {
                const size_t n = (size_t)r.elem_count * (r.buffer_id == VHX_BUF_NODE_OCBITS ? 8u : 4u);
                batch_store.emplace_back((const uint8_t *)r.src, (const uint8_t *)r.src + n);
                r.src = batch_store.back().data();
                all.push_back(r);
            }
        }
        frame_writes = std::move(all);
        int frc = flush();  // also after a capacity stop: the frames decided before it are written
        batch_store.clear();
        last_bytes = batch_bytes;
        last_nodes = batch_nodes;
        last_bricks = batch_bricks;
        if (!frc && device_valid) frc = sync_device_mips(false);
        return rc ? rc : frc;
    }
    int collect_frame() {  // streaming/mod.rs:420-635
        last_nodes = last_bricks = last_bytes = 0;
        if (resize) return VHX_E_CAPACITY;
        apply_pending_rebuild();
        std::vector<CacheUpdate> updates;
        // streaming::upload (streaming/mod.rs:446-457): a reloading view runs the upload queue; otherwise queued tree
        // changes go first, and the upload queue runs in a frame without any
        bool fits;
#ifdef VHX_STREAM_TIMING
        const auto t0 = std::chrono::steady_clock::now();
#endif
        if (reload) {
            fits = process(updates);
        } else {
            fits = handle_tree_updates(updates, node_uploads_per_frame);
            if (fits && updates.empty()) fits = process(updates);
        }
#ifdef VHX_STREAM_TIMING
        fprintf(stderr, "[stream] process %.3f ms\n",
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
#endif
        int rc = VHX_OK;
        // palettes: deltas of the host tree's palettes (capacity kPaletteCapacity entries on the device)
        if (tree->color_palette.size() > kPaletteCapacity || tree->data_palette.size() > kPaletteCapacity)
            return VHX_E_CAPACITY;
        if (tree->color_palette.size() > uploaded_color_palette_size) {
            color_palette = tree->color_palette;
            rc = write(VHX_BUF_COLOR_PALETTE, uploaded_color_palette_size,
                       color_palette.size() - uploaded_color_palette_size, color_palette.data() + uploaded_color_palette_size);
            if (rc) return rc;
            uploaded_color_palette_size = color_palette.size();
        }
        if (tree->data_palette.size() > uploaded_data_palette_size) {
            data_palette = tree->data_palette;
            rc = write(VHX_BUF_DATA_PALETTE, uploaded_data_palette_size,
                       data_palette.size() - uploaded_data_palette_size, data_palette.data() + uploaded_data_palette_size);
            if (rc) return rc;
            uploaded_data_palette_size = data_palette.size();
        }
        // voxel data of the uploaded bricks (Parted only; MIP slots only with MIPs on), before the nodes point at them
        const size_t n3 = (size_t)bd() * bd() * bd();
        for (const auto &u : updates)
            for (const auto &bu : u.brick_updates) {
                const Owned &o = bu.second;
                if (o.kind != 1 && !(o.kind == 2 && stream_mips())) continue;
                const Node &n = node(o.node);
                const Brick &b = o.kind == 2 ? n.mip : n.content == Content::UniformLeaf ? n.bricks[0] : n.bricks[o.sectant];
                if (b.kind != BrickKind::Parted) continue;
                std::copy(b.parted.begin(), b.parted.end(), voxels.begin() + (ptrdiff_t)(bu.first * n3));
                rc = write(VHX_BUF_VOXELS, bu.first * n3, n3, voxels.data() + bu.first * n3);
                if (rc) return rc;
                ++last_bricks;
            }
        if (solid_values.size() > solid_capacity) {  // grow the solid table: re-create the view
            while (solid_capacity < solid_values.size()) solid_capacity *= 2;
            resize = true;
            return VHX_E_CAPACITY;
        }
        if (solid_values.size() > uploaded_solid_size) {
            rc = write(VHX_BUF_SOLID_VALUES, uploaded_solid_size, solid_values.size() - uploaded_solid_size,
                       solid_values.data() + uploaded_solid_size);
            if (rc) return rc;
            uploaded_solid_size = solid_values.size();
        }
        size_t meta_lo = SIZE_MAX, meta_hi = 0, ch_lo = SIZE_MAX, ch_hi = 0;
        for (const auto &u : updates)
            for (const auto &mn : u.modified_nodes) {
                const size_t i = mn.first;
                if (i >= nodes_in_view) continue;
                meta_lo = std::min(meta_lo, i);
                meta_hi = std::max(meta_hi, i + 1);
                for (size_t s = 0; s < kChildren; ++s)
                    if (mn.second & (1ull << s)) {
                        ch_lo = std::min(ch_lo, i * kChildren + s);
                        ch_hi = std::max(ch_hi, i * kChildren + s + 1);
                    }
            }
        for (const auto &u : updates)
            for (const auto &mn : u.modified_nodes) last_nodes += mn.second == ~0ull ? 1 : 0;  // nodes (re)written
        if (meta_lo < meta_hi) {
            rc = write(VHX_BUF_NODE_TYPE, meta_lo, meta_hi - meta_lo, node_type.data() + meta_lo);
            if (!rc) rc = write(VHX_BUF_NODE_OCBITS, meta_lo, meta_hi - meta_lo, node_ocbits.data() + meta_lo);
            if (rc) return rc;
        }
        if (ch_lo < ch_hi) {
            rc = write(VHX_BUF_NODE_CHILDREN, ch_lo, ch_hi - ch_lo, node_children.data() + ch_lo);
            if (rc) return rc;
        }
        return fits ? VHX_OK : VHX_E_CAPACITY;
    }
};

extern "C" {

int vhx_stream_create(const vhx_boxtree *tree, vhx_ctx *ctx, const float origin[3], float view_distance,
                      vhx_stream **out) {
    if (!tree || !origin || !out || !(view_distance > 0.f)) return VHX_E_INVALID_ARG;
    *out = nullptr;
    auto s = std::make_unique<vhx_stream>();
    s->tree = tree->tree;
    s->tree->track_changes += 1;  // the tree queues its changes for the stream (BoxTreeGPUHost::new's trigger)
    s->ctx = ctx;
    s->nodes_to_see.resident = &s->resident_key;
    s->origin = f3(origin[0], origin[1], origin[2]);
    s->view_distance = view_distance;
    s->upload_range = Cube{sub(s->origin, unit(view_distance / 2.f)), view_distance};
    s->size_view();
    s->alloc_mirror();
    const int rc = s->upload_all();
    if (rc) return rc;
    *out = s.release();
    return VHX_OK;
}

void vhx_stream_destroy(vhx_stream *s) { delete s; }

int vhx_stream_set_rates(vhx_stream *s, uint32_t node_uploads_per_frame, uint32_t brick_uploads_per_frame,
                         uint32_t brick_unload_search_perimeter) {
    if (!s || node_uploads_per_frame == 0 || brick_uploads_per_frame == 0) return VHX_E_INVALID_ARG;
    s->node_uploads_per_frame = node_uploads_per_frame;
    s->brick_uploads_per_frame = brick_uploads_per_frame;
    s->brick_unload_search_perimeter = brick_unload_search_perimeter;
    return VHX_OK;
}

int vhx_stream_set_viewport(vhx_stream *s, const float origin[3], float view_distance) {
    if (!s || !origin || !(view_distance > 0.f)) return VHX_E_INVALID_ARG;
    const F3 o = f3(origin[0], origin[1], origin[2]);
    s->origin = o;
    const bool moved = !s->brick_slot_set || !contains(s->brick_slot, o) || view_distance != s->view_distance;
    s->view_distance = view_distance;
    if (moved) {  // bevy/mod.rs:110-155: a rebuild only when the origin leaves its brick slot
        s->upload_range = Cube{sub(o, unit(view_distance / 2.f)), view_distance};
        s->rebuild_pending = true;  // run by the next upload (apply_pending_rebuild)
        s->pending_origin = o;
        s->pending_distance = view_distance;
        const float bd = (float)s->tree->brick_dim;  // Cube::brick_slot_for, spatial/raytracing/mod.rs:65-70
        s->brick_slot = Cube{f3(o.x - std::fabs(std::fmod(o.x, bd)), o.y - std::fabs(std::fmod(o.y, bd)),
                                o.z - std::fabs(std::fmod(o.z, bd))),
                             bd};
        s->brick_slot_set = true;
    }
    return VHX_OK;
}

int vhx_stream_upload(vhx_stream *s, vhx_stream_stats *stats) { return vhx_stream_upload_frames(s, 1, stats); }

int vhx_stream_upload_frames(vhx_stream *s, uint32_t frames, vhx_stream_stats *stats) {
    if (!s || frames == 0) return VHX_E_INVALID_ARG;
    const int rc = frames == 1 ? s->upload_frame() : s->upload_frames(frames);
    if (stats) {
        stats->bytes_written = s->last_bytes;
        stats->nodes_written = s->last_nodes;
        stats->bricks_written = s->last_bricks;
        stats->nodes_resident = s->meta_by_key.size();
        stats->bricks_resident = s->brick_by_index.size();
        stats->nodes_in_view = s->nodes_in_view;
        stats->bricks_in_view = s->bricks_in_view;
        stats->nodes_to_see = s->nodes_to_see.size();
        const uint64_t missing = s->nodes_to_see.size() - s->nodes_to_see.n_resident;
        stats->pending = missing + s->bricks_to_upload.size() + s->tree->changes.size() +
                         (s->last_cycle_work == 0 ? 0u : 1u);
    }
    return rc;
}

int vhx_stream_view_set_check(vhx_stream *s, uint64_t *full_rebuilds, uint64_t *incremental_rebuilds) {
    if (!s) return VHX_E_INVALID_ARG;
    if (full_rebuilds) *full_rebuilds = s->rebuilds_full;
    if (incremental_rebuilds) *incremental_rebuilds = s->rebuilds_incremental;
    size_t res = 0;  // the set's resident count, kept incrementally, against a count over the set
    for (size_t k : s->nodes_to_see) res += s->is_resident(k) ? 1u : 0u;
    return s->view_set_matches_full() && res == s->nodes_to_see.n_resident ? VHX_OK : VHX_E_STATE;
}

int vhx_stream_resize(vhx_stream *s) {
    if (!s) return VHX_E_INVALID_ARG;
    return s->upload_all();
}

int vhx_stream_reload(vhx_stream *s) {
    if (!s) return VHX_E_INVALID_ARG;
    s->reset_targets();
    return VHX_OK;
}

int vhx_stream_node_mips(const vhx_stream *s, const uint32_t **node_mips, uint32_t *count) {
    if (!s || !node_mips || !count) return VHX_E_INVALID_ARG;
    *node_mips = s->node_mips.data();
    *count = (uint32_t)s->node_mips.size();
    return VHX_OK;
}

int vhx_stream_view(const vhx_stream *s, vhx_tree_desc *out) {
    if (!s || !out) return VHX_E_INVALID_ARG;
    *out = s->desc();
    out->solid_count = (uint32_t)s->solid_values.size();
    out->solid_values = s->solid_values.data();
    out->color_count = (uint32_t)s->color_palette.size();
    out->color_palette = s->color_palette.data();
    out->data_count = (uint32_t)s->data_palette.size();
    out->data_palette = s->data_palette.data();
    return VHX_OK;
}

}  // extern "C"
