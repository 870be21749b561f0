/*
 * vhx_boxtree.h — C ABI of the host-side BoxTree (libvhx.so, host code only, no GPU needed).
 *
 * The reference keeps the voxel tree in Rust (`BoxTree<T>`); its toolchain is not available to this build, so the
 * host side of the raytracing drop-in is restated in C++ behind this ABI:
 *
 *   vhx_boxtree_new            <- BoxTree::new            (src/boxtree/mod.rs:188-219)
 *   vhx_boxtree_insert         <- BoxTree::insert         (src/boxtree/update/insert.rs:21-30)
 *   vhx_boxtree_insert_at_lod  <- BoxTree::insert_at_lod  (src/boxtree/update/insert.rs:37-47)
 *   vhx_boxtree_update         <- BoxTree::update         (src/boxtree/update/insert.rs:53-62)
 *   vhx_boxtree_get            <- BoxTree::get            (src/boxtree/mod.rs:223-233)
 *   vhx_boxtree_simplify       <- BoxTree::simplify(ROOT, recursive) (src/boxtree/update/mod.rs:617-867)
 *   vhx_boxtree_flatten        <- BoxTreeGPUDataHandler::add_node/add_brick with every node resident
 *                                 (src/raytracing/bevy/streaming/cache.rs:226-455, 608-716)
 *   vhx_boxtree_load_vox       <- BoxTree::load_vox_file  (src/convert/magicavoxel.rs:234-374)
 *   vhx_boxtree_switch_mips    <- StrategyUpdater::switch_albedo_mip_maps (src/boxtree/mipmap.rs:588-609)
 *   vhx_boxtree_set_mip_method <- StrategyUpdater::set_method_at (mipmap.rs:414-431, 505-513)
 *   vhx_boxtree_set_mip_color_threshold <- StrategyUpdater::set_color_similarity_thr_at (mipmap.rs:365-379, 482-488)
 *   vhx_boxtree_recalculate_mips <- StrategyUpdater::recalculate_mips (mipmap.rs:536-586)
 *   vhx_boxtree_sample_root_mip <- StrategyUpdater::sample_root_mip (mipmap.rs:635-668, a test helper there)
 *   vhx_boxtree_flatten_lod    <- the streamed view with every node above a depth resident and the rest not: node_mips
 *                                 (src/raytracing/bevy/types.rs:245-247) stand in for the missing children
 *   vhx_scene_build            <- bulk builder producing exactly the flattened tree that inserting a procedural
 *                                 scene voxel by voxel (x, then y, then z loops) would produce
 *
 * Tree type parameter: T = u32 (the reference default, BoxTree<T = u32>, src/boxtree/types.rs:219).
 */
#ifndef VHX_BOXTREE_H
#define VHX_BOXTREE_H

#include "vhx.h"

#ifdef __cplusplus
extern "C" {
#endif

/* OctreeError (src/boxtree/types.rs:9-21) */
#define VHX_E_TREE_INVALID_SIZE (-10)
#define VHX_E_TREE_INVALID_BRICK_DIMENSION (-11)
#define VHX_E_TREE_INVALID_STRUCTURE (-12)
#define VHX_E_TREE_INVALID_POSITION (-13)
/* .vox import */
#define VHX_E_VOX_FORMAT (-14) /* not a .vox file the importer supports (see vhx_boxtree_load_vox) */
#define VHX_E_VOX_IO (-15)     /* the file could not be read */

/* BoxTreeEntry kinds (src/boxtree/types.rs:25-37) */
#define VHX_ENTRY_EMPTY 0u
#define VHX_ENTRY_VISUAL 1u      /* albedo only  */
#define VHX_ENTRY_INFORMATIVE 2u /* data only    */
#define VHX_ENTRY_COMPLEX 3u     /* albedo+data  */

/* Procedural scenes for vhx_scene_build / vhx_scene_insert */
#define VHX_SCENE_LATTICE_CUBE 1u /* examples/gpu_render.rs:57-82: lattice where any coord < S/4 + cube >= S/2, axis-plane colours */
#define VHX_SCENE_BENCH_REGION 2u /* benches/performance.rs:11-27: [0,100)^3 slab where x|y|z < S/4 or all >= S/2, 0x00ABCDEF */
#define VHX_SCENE_LATTICE 3u      /* src/raytracing/tests.rs:777-789 (context_bleed): lattice only, colour 255*c/S            */
#define VHX_SCENE_CUBE 4u         /* src/raytracing/tests.rs:736-748 (cube_flaps): cube >= S/2, colour 255*c/S                 */
#define VHX_SCENE_BOUNDARY 5u     /* src/raytracing/tests.rs:692-703 (brick_boundary): lattice+cube, colour 255*(c%6)/6         */
#define VHX_SCENE_HEIGHTFIELD 6u  /* seeded value-noise terrain (no reference equivalent; SURVEY.md 8d config 3 secondary)   */

typedef struct vhx_boxtree vhx_boxtree;
typedef struct vhx_flat vhx_flat;

int vhx_boxtree_new(uint32_t size, uint32_t brick_dim, vhx_boxtree **out);
void vhx_boxtree_free(vhx_boxtree *tree);
int vhx_boxtree_set_auto_simplify(vhx_boxtree *tree, int enabled);
/* albedo packed r | g<<8 | b<<16 | a<<24 */
int vhx_boxtree_insert(vhx_boxtree *tree, uint32_t x, uint32_t y, uint32_t z, uint32_t kind, uint32_t albedo,
                       uint32_t data);
int vhx_boxtree_insert_at_lod(vhx_boxtree *tree, uint32_t x, uint32_t y, uint32_t z, uint32_t insert_size,
                              uint32_t kind, uint32_t albedo, uint32_t data);
int vhx_boxtree_update(vhx_boxtree *tree, uint32_t x, uint32_t y, uint32_t z, uint32_t kind, uint32_t albedo,
                       uint32_t data);
int vhx_boxtree_get(const vhx_boxtree *tree, uint32_t x, uint32_t y, uint32_t z, uint32_t *kind, uint32_t *albedo,
                    uint32_t *data);
int vhx_boxtree_simplify(vhx_boxtree *tree, int recursive);
/* The deepest node containing a position (BoxTree::get_node_internal from the root, src/boxtree/iterate.rs:293-343):
 * its pool key, content (0 Nothing, 1 Internal, 2 Leaf, 3 UniformLeaf), occupied bits and occlusion bits. */
int vhx_boxtree_node_info(const vhx_boxtree *tree, float x, float y, float z, uint64_t *key, uint32_t *content,
                          uint64_t *occupied_bits, uint32_t *occlusion_bits);
/* size, brick_dim, node count (pool length), color and data palette sizes */
int vhx_boxtree_info(const vhx_boxtree *tree, uint32_t info[5]);
/* Runs the reference insert loop (x outer, z inner) of a procedural scene on `tree` (for cross-checking the bulk
 * builder at small sizes; O(size^3) inserts). */
int vhx_scene_insert(vhx_boxtree *tree, uint32_t scene, uint64_t seed);

/* Flattened trees ------------------------------------------------------------------------------------------- */
/* Nodes are renumbered breadth-first from the root; bricks and solid values are numbered in that node order. */
int vhx_boxtree_flatten(const vhx_boxtree *tree, vhx_flat **out);
int vhx_scene_build(uint32_t scene, uint32_t size, uint32_t brick_dim, uint64_t seed, int threads, vhx_flat **out);
/* MIP maps (src/boxtree/mipmap.rs): off by default (MIPMapStrategy::default, mipmap.rs:341-354: level 1 Posterize(0.05),
 * levels 2-4 BoxFilter, colour-matching thresholds {2: 0.1, 3: 0.05, 4: 0.02}). Once switched on, every insert updates
 * the MIPs of the nodes on its path (insert.rs:494); switching on recalculates all of them. A node's MIP level is
 * log2(node edge / brick_dim). Methods (MIPResamplingMethods, src/boxtree/types.rs:113-149): */
#define VHX_MIP_BOX_FILTER 0u      /* gamma-2 average of the cell's colours                                     */
#define VHX_MIP_POINT_FILTER 1u    /* most frequent colour                                                      */
#define VHX_MIP_POINT_FILTER_BD 2u /* most frequent colour, sampled from the voxels instead of the child MIPs    */
#define VHX_MIP_POSTERIZE 3u       /* average of the largest group of colours within threshold*255              */
#define VHX_MIP_POSTERIZE_BD 4u    /* as POSTERIZE (the reference samples it like POSTERIZE too, mipmap.rs:51-55) */
int vhx_boxtree_switch_mips(vhx_boxtree *tree, int enabled);
int vhx_boxtree_set_mip_method(vhx_boxtree *tree, uint32_t level, uint32_t method, float threshold);
int vhx_boxtree_set_mip_color_threshold(vhx_boxtree *tree, uint32_t level, float threshold);
int vhx_boxtree_recalculate_mips(vhx_boxtree *tree);
/* Process-wide options of the MIP generation (no reference counterpart; results never depend on them): direct = 1 runs
 * the direct restatement (get_internal per sample, full palette scans) instead of the exact shortcuts (tests compare the
 * two); threads caps the leaf-resampling workers (0 = up to 16). */
int vhx_boxtree_set_mip_options(int direct, int threads);
/* The root's MIP (sectant 64) or its child's (sectant < 64) at cell (x, y, z) of the brick, as an entry. */
int vhx_boxtree_sample_root_mip(const vhx_boxtree *tree, uint32_t sectant, uint32_t x, uint32_t y, uint32_t z,
                                uint32_t *kind, uint32_t *albedo, uint32_t *data);
/* Flattened tree with node MIPs: nodes deeper than max_depth (root = 0) are left out (their parents' child entries
 * are VHX_EMPTY, occupancy kept); every node's MIP brick is appended to the bricks / solid values and its descriptor
 * stored in node_mips (VHX_EMPTY where the node has no MIP). vhx_boxtree_flatten does the same with every node
 * included when the tree's MIPs are enabled, and leaves node_mips empty otherwise. */
int vhx_boxtree_flatten_lod(const vhx_boxtree *tree, uint32_t max_depth, vhx_flat **out);
/* vhx_scene_build, then the tree's MIP maps switched on with the default strategy and the LOD image of
 * vhx_boxtree_flatten_lod: the same buffers as vhx_scene_insert + vhx_boxtree_switch_mips(1) + vhx_boxtree_flatten_lod
 * without the voxel-by-voxel insert loop (minutes at 1024^3). */
int vhx_scene_build_lod(uint32_t scene, uint32_t size, uint32_t brick_dim, uint64_t seed, int threads,
                        uint32_t max_depth, vhx_flat **out);
/* The host BoxTree of vhx_scene_build's image without the voxel-by-voxel insert loop (a 1024^3 tree in seconds instead
 * of minutes): nodes (pool key = breadth-first index), bricks, occupancy and palettes as vhx_scene_insert builds them,
 * so vhx_boxtree_flatten gives vhx_scene_build's buffers. Not restored: occlusion bits (they record which siblings
 * existed when a node became full, an insert-history fact; all clear here, so a stream's upload walk may descend into
 * nodes the reference would skip) and MIP maps (off; vhx_boxtree_switch_mips builds them). */
int vhx_scene_build_tree(uint32_t scene, uint32_t size, uint32_t brick_dim, uint64_t seed, int threads,
                         vhx_boxtree **out);
int vhx_flat_node_mips(const vhx_flat *flat, const uint32_t **node_mips, uint32_t *count);
/* Fills *desc with pointers into the flat object (valid until vhx_flat_free). */
int vhx_flat_desc(const vhx_flat *flat, vhx_tree_desc *desc);
void vhx_flat_free(vhx_flat *flat);

/* MagicaVoxel .vox import — BoxTree::<u32>::load_vox_file(filename, brick_dimension) (src/convert/magicavoxel.rs:
 * 234-374): walks the scene graph at frame 0 (translations "_t", rotations "_r" composed like the reference, which
 * resets to identity where "_r" is absent), sizes the tree with model_size_to_tree_size (magicavoxel.rs:55-60),
 * converts Rz-up to Ly-up and inserts every voxel as BoxTreeEntry::Visual(palette colour), then simplifies the tree
 * recursively when auto-simplify is on (the default). The .vox reader is restated from the file format (the
 * reference's dot_vox 5.1.1 is not vendored): files without an RGBA palette or without a scene graph are rejected
 * with VHX_E_VOX_FORMAT. Voxels landing outside the tree return VHX_E_TREE_INVALID_POSITION (the reference panics). */
int vhx_boxtree_load_vox(const char *path, uint32_t brick_dim, vhx_boxtree **out);
int vhx_boxtree_load_vox_memory(const uint8_t *data, uint64_t size, uint32_t brick_dim, vhx_boxtree **out);
/* helpers of the import, exported for tests: model_size_to_tree_size and parse_rotation_matrix (row-major m[9]) */
uint32_t vhx_vox_tree_size(int32_t sx, int32_t sy, int32_t sz, uint32_t brick_dim);
int vhx_vox_rotation(uint8_t b, int32_t m[9]);

#ifdef __cplusplus
}
#endif
#endif /* VHX_BOXTREE_H */
