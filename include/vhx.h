/*
 * vhx.h — C ABI of the MI355X primary-ray voxel-brick raytracer (libvhx.so).
 *
 * This is the drop-in boundary for VoxelHex's `src/raytracing` module. Each entry point names the
 * reference interface it replaces (paths relative to the VoxelHex repository root):
 *
 *   vhx_tree_desc        <- BoxTreeRenderData + BoxTreeMetaData, the flattened node/brick/palette buffers
 *                           (src/raytracing/bevy/types.rs:27-57, 203-256) that the Bevy host builds in
 *                           BoxTreeGPUDataHandler::add_node / add_brick (src/raytracing/bevy/streaming/cache.rs:226-455,
 *                           608-716) and binds in create_tree_bind_group (src/raytracing/bevy/pipeline/bind_groups.rs:366-482)
 *   vhx_create/destroy   <- BoxTreeGPUHost::new / create_new_view (src/raytracing/bevy/mod.rs:164-180,
 *                           src/raytracing/bevy/view.rs:36-137): owns the device copy of the tree
 *   vhx_upload_tree      <- prepare_bind_groups full-buffer writes (src/raytracing/bevy/pipeline/mod.rs:242-402)
 *   vhx_update_range     <- write_range_to_buffer (src/raytracing/bevy/streaming/mod.rs:344-370)
 *   vhx_update_ranges    <- the write_range_to_buffer calls of one streaming::upload frame (streaming/mod.rs:420-635)
 *   vhx_trace_primary    <- VhxRenderNode::run main dispatch (src/raytracing/bevy/pipeline/mod.rs:96-155) running the
 *                           per-pixel kernel, with the semantics of the reference CPU raytracer
 *                           BoxTree::get_by_ray (src/raytracing/cpu.rs:296-458) and the CPU frame of
 *                           examples/gpu_render.rs:196-257 / benches/performance.rs:29-66
 *   vhx_trace_rays       <- BoxTree::get_by_ray (src/raytracing/cpu.rs:296) over an explicit batch of rays
 *   vhx_last_error       <- the Result<_, ()> / expect() error paths of the plugin (src/raytracing/bevy/streaming/mod.rs:63-73)
 *
 * Conventions: every function returns 0 on success or a negative VHX_E_* code; a message is kept per context
 * (vhx_last_error). Host pointers are only read during the call. A context is single-threaded and all work is
 * ordered on its HIP stream. Nothing in this header uses HIP, torch or C++ types.
 */
#ifndef VHX_H
#define VHX_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VHX_ABI_VERSION 6u

/* ---- error codes ------------------------------------------------------------------------------------------ */
#define VHX_OK 0
#define VHX_E_INVALID_ARG (-1) /* bad pointer / size / layout                                                 */
#define VHX_E_HIP (-2)         /* a HIP runtime call failed (message in vhx_last_error)                         */
#define VHX_E_CAPACITY (-3)    /* update_range outside the uploaded capacity: grow and re-upload, mirroring
                                  view.resize / re_evaluate_view_size (src/raytracing/bevy/streaming/mod.rs:292-340) */
#define VHX_E_NO_DEVICE (-4)   /* no HIP device available                                                       */
#define VHX_E_STATE (-5)       /* call order violated (e.g. trace before upload)                                */
#define VHX_E_RCCL (-6)        /* RCCL missing or an RCCL call failed (message in vhx_last_error)               */

/* ---- node types (NodeContent, src/boxtree/types.rs:57-73) ------------------------------------------------- */
#define VHX_NODE_NOTHING 0u
#define VHX_NODE_INTERNAL 1u
#define VHX_NODE_LEAF 2u
#define VHX_NODE_UNIFORM_LEAF 3u

/* ---- child / brick descriptors in node_children -----------------------------------------------------------
 * Internal node : node_children[64*n + s] = child node index, or VHX_EMPTY (NodeChildren, types.rs:75-80)
 * Leaf node     : node_children[64*n + s] = brick descriptor of sectant s (BrickData, types.rs:41-54)
 * UniformLeaf   : node_children[64*n + 0] = brick descriptor of the whole node, slots 1..63 = VHX_EMPTY
 * brick descriptor: VHX_EMPTY = BrickData::Empty;
 *                   bit31 set  = BrickData::Solid, low 31 bits index solid_values[] (exact 32-bit voxel value);
 *                   bit31 clear= BrickData::Parted, brick index into voxels[] (brick_dim^3 values per brick).
 * (The WGSL host ORs the solid voxel into bit 31 directly, cache.rs:391; that loses the data-palette index of
 *  PaletteIndexValues >= 0x80000000, so this ABI keeps solid values in their own table.)                        */
#define VHX_EMPTY 0xFFFFFFFFu
#define VHX_SOLID_BIT 0x80000000u

/* Flattened BoxTree<u32> (full residency). Node 0 is the root (ROOT_NODE_KEY, src/boxtree/detail.rs:140).
 * Voxel values are PaletteIndexValues (src/boxtree/types.rs:111): color index in bits 0-15, data index in
 * bits 16-31, 0xFFFF = none in either half (src/boxtree/node.rs:260-309).                                    */
typedef struct vhx_tree_desc {
    uint32_t boxtree_size;   /* BoxTree::boxtree_size (edge length of the root cube)                          */
    uint32_t brick_dim;      /* BoxTree::brick_dim                                                            */
    uint32_t node_count;
    uint32_t brick_count;    /* number of Parted bricks in voxels[]                                           */
    uint32_t solid_count;    /* entries of solid_values[]                                                     */
    uint32_t color_count;    /* entries of color_palette[]                                                    */
    uint32_t data_count;     /* entries of data_palette[]                                                     */
    uint32_t reserved0;
    const uint32_t *node_type;     /* [node_count]      VHX_NODE_*                                            */
    const uint64_t *node_ocbits;   /* [node_count]      NodeData::occupied_bits                               */
    const uint32_t *node_children; /* [node_count*64]   see above                                             */
    const uint32_t *voxels;        /* [brick_count*brick_dim^3] flat index x + y*bd + z*bd*bd                  */
    const uint32_t *solid_values;  /* [solid_count]                                                           */
    const uint32_t *color_palette; /* [color_count] Albedo packed r | g<<8 | b<<16 | a<<24                     */
    const uint32_t *data_palette;  /* [data_count]  user data T=u32 (empty <=> 0, src/boxtree/detail.rs:18-24)  */
} vhx_tree_desc;

/* ---- ray generation ---------------------------------------------------------------------------------------- */
#define VHX_RAY_INVERSE_VP 0u /* examples/gpu_render.rs:203-224: NDC -> world via inverse view-projection, glam op order */
#define VHX_RAY_GLASS 1u      /* benches/performance.rs:32-61: pinhole "glass" plane, V3c op order                    */

typedef struct vhx_camera {
    uint32_t ray_model;      /* VHX_RAY_*                                                                    */
    uint32_t width, height;  /* full frame resolution in pixels                                              */
    uint32_t reserved0;
    float origin[3];         /* ray origin for every pixel (Viewport::origin / viewport.origin)              */
    /* VHX_RAY_GLASS: glass_point = bottom_left + right*x*pixel_width + up*y*pixel_height                    */
    float glass_bottom_left[3];
    float glass_right[3];
    float glass_up[3];
    float pixel_width, pixel_height;
    /* VHX_RAY_INVERSE_VP: column-major 4x4 (glam Mat4 layout), Viewport::inverse_view_projection_matrix     */
    float inv_view_proj[16];
} vhx_camera;

/* Output layout of vhx_trace_primary */
#define VHX_LAYOUT_FRAMEBUFFER 0u /* ray (x,y) -> index y*width + x                                               */
#define VHX_LAYOUT_TILES 1u       /* tile-major: k-th traced tile owns indices [k*T*T, (k+1)*T*T), row-major inside */

/* Per-ray hit records, structure of arrays; any pointer may be NULL to skip that field.
 * Device pointers when passed to vhx_trace_primary/vhx_trace_rays with on_device=1, host pointers otherwise.
 *   value  : PaletteIndexValues of the hit voxel; VHX_EMPTY = no hit (get_by_ray returned None)
 *   cell   : flat index of the hit cell inside its Parted brick (cpu.rs:136-144); VHX_EMPTY for Solid/miss
 *   voxel  : 3 u32 per ray, integer min corner of the hit cube (the cell for Parted hits, the brick/node bounds
 *            for Solid hits); VHX_EMPTY x3 on miss
 *   impact : 3 f32 per ray, impact point (cpu.rs:257, 284);   miss: 0,0,0
 *   normal : 3 f32 per ray, cube_impact_normal (spatial/raytracing/mod.rs:97-125); miss: 0,0,0
 *   depth  : |impact - origin| (V3c::length);                   miss: +inf
 *   rgba   : r | g<<8 | b<<16 | a<<24 shaded as examples/gpu_render.rs:236-249 (miss 128,128,128,255;
 *            a hit without albedo - where the example would unwrap() None - is 0,0,0,255)
 *   bytes  : algorithmic bytes touched by this ray (instrumentation; definition in DESIGN.md)
 *   shadowed : with a shadow light set (vhx_set_shadow_light): 1 where the hit's hard-shadow ray hits a voxel (rgba
 *            then darkened, rgb >> 1), 0 elsewhere (misses included)                                          */
typedef struct vhx_hits {
    uint32_t *value;
    uint32_t *cell;
    uint32_t *voxel;
    float *impact;
    float *normal;
    float *depth;
    uint32_t *rgba;
    uint32_t *bytes;
    uint32_t *shadowed; /* ABI 6 */
} vhx_hits;

typedef struct vhx_ctx vhx_ctx;

/* Library / device ------------------------------------------------------------------------------------------ */
uint32_t vhx_abi_version(void);
/* The number of HIP devices visible to the process (0 on a host without a GPU). VHX_E_HIP when the HIP runtime fails
 * to answer for another reason; vhx_device_error() then names the hipError_t (thread-local text, "" after a success). */
int vhx_device_count(int *count);
const char *vhx_device_error(void);
int vhx_create(int hip_device, vhx_ctx **out);
/* A further context on the owner's device that traces the owner's uploaded tree (no second copy in HBM): one context
 * per frame in flight. Each context has its own stream, ray queues and outputs, so frame k+1's trace runs while frame
 * k's long-ray tail still occupies a few SIMDs (the frames of a renderer are independent of each other). Uploads and updates go through the owner (a shared context returns
 * VHX_E_STATE for them) and are ordered against the frames in flight by libvhx, on the device, without host waits: a
 * write of the tree (vhx_upload_tree, vhx_update_range(s), vhx_set_node_mips, vhx_upload_tree_device) first waits on
 * its stream for the last trace submitted on every other context of the tree, and the next trace of every context
 * waits on its own stream for that write. So a frame sees the tree as of its submission: every write submitted
 * before it and none submitted after it. The tree lives until its last context is destroyed, in any order. */
int vhx_create_shared(const vhx_ctx *owner, vhx_ctx **out);
void vhx_destroy(vhx_ctx *ctx);
const char *vhx_last_error(const vhx_ctx *ctx);
/* Use an external HIP stream (hipStream_t passed as void*; NULL = the context's own stream). */
int vhx_set_stream(vhx_ctx *ctx, void *hip_stream);
/* The context's stream (hipStream_t as void*): the one set by vhx_set_stream, else the context's own, created at its
 * first use (a context given a stream before its first call creates none: streams share the device's few hardware
 * queues round-robin, so frames in flight want one stream each and no idle ones). */
int vhx_get_stream(vhx_ctx *ctx, void **hip_stream);
/* Wait for all work of the context; optionally return the device time of the last trace in milliseconds. */
int vhx_sync(vhx_ctx *ctx, float *last_trace_ms);
/* Ray scheduling (no reference counterpart; results do not depend on it). A trace runs n+1 passes: pass i abandons
 * rays that need more than budgets[i] loop steps (saving their traversal state) and the next pass resumes them, 64
 * such rays per wave; the last pass is unbounded. n = 0 is a single pass. Budgets strictly increasing,
 * 0 < b < 2^22, n <= VHX_MAX_BUDGETS.
 * By default the schedule is adaptive: a trace submitted while another context of the same tree (vhx_create_shared)
 * has a frame in flight on another stream runs the frames-in-flight schedule {32, 128, 768} (shadow traces {24, 72, 216, 648}); otherwise (one frame
 * at a time, or frames serialised on one stream) the lone-frame schedule {64}. vhx_set_pass_budgets fixes the
 * budgets (and ends the adaptive choice; vhx_set_adaptive_schedule(ctx, 1) restores it). vhx_set_adaptive_schedule(ctx,
 * 0) fixes the frames-in-flight schedule whatever the last trace ran. */
#define VHX_MAX_BUDGETS 6
int vhx_set_pass_budgets(vhx_ctx *ctx, const uint32_t *budgets, uint32_t n);
int vhx_set_adaptive_schedule(vhx_ctx *ctx, int on);
/* The budgets of the context's last trace (or the fixed ones before any), n of them (budgets: VHX_MAX_BUDGETS entries,
 * may be NULL); *schedule (may be NULL) = 1 the frames-in-flight schedule, 0 the lone-frame one, -1 fixed. */
int vhx_get_pass_budgets(const vhx_ctx *ctx, uint32_t *budgets, uint32_t *n, int *schedule);
/* Scheduling knobs (no reference counterpart; results never depend on them -- experiments and probes): `spec` is
 * "key=value[;key=value...]" with keys budgets (list, fixes the schedule), adaptive (0/1), rpw (list: rays per wave of
 * queue passes 1.., 0 = adaptive), tw, xcdg, resume (0/1), qstate (0/1: states in queue order), save_from, qblock
 *  (64/128/256), tlists (0/1: tile sets list pass 0), qwaves (fixes the schedule),
 * qwavesm, qwaves0, qxcd, qxcd_all (0/1), sparse (list, fixes the schedule), qorder ("[m]N[z|r]" or 0), qsort (0 or
 * 256..2048: segment node sort of the queue passes, docs/DESIGN_LOG.md §15.3), qsortp (pass mask), qsortb (workgroups),
 * qwpc_idle / qwpc_busy (queue waves per CU of one schedule, which stays adaptive), stage_slots (1..4: batch staging
 * ring), finter (0/1: batch pass 0 frame-major / frames interleaved block by block), sbudget (fused shadows: a shadow
 * ray's steps in its primary ray's pass), tail / tail_min / tail_rpw /
 * tail_cap / tail_prio (the early tail of lone frames, vhx_tail_info). The
 * library reads no environment variable for any of them (docs/DESIGN_LOG.md §15). Unknown keys or malformed values:
 * VHX_E_INVALID_ARG and nothing is changed. */
int vhx_set_tuning(vhx_ctx *ctx, const char *spec);

/* Tree upload ----------------------------------------------------------------------------------------------- */
/* Copies the flattened tree to HBM (full residency) and builds the device-side layout. */
int vhx_upload_tree(vhx_ctx *ctx, const vhx_tree_desc *tree);
/* Same, from buffers already in device memory (the 7 array pointers of `tree` are device pointers: a tree produced on
 * the GPU, or another device's copy where peer access is enabled): device-to-device copies on the context's stream,
 * then the derived layout. The receive half of vhx_mgpu_broadcast_tree, which fills the same buffers by ncclBroadcast. */
int vhx_upload_tree_device(vhx_ctx *ctx, const vhx_tree_desc *tree);
#define VHX_BUF_NODE_TYPE 0
#define VHX_BUF_NODE_OCBITS 1
#define VHX_BUF_NODE_CHILDREN 2
#define VHX_BUF_VOXELS 3
#define VHX_BUF_SOLID_VALUES 4
#define VHX_BUF_COLOR_PALETTE 5
#define VHX_BUF_DATA_PALETTE 6
/* Overwrites elements [elem_offset, elem_offset+elem_count) of one uploaded buffer (element = one entry of the
 * corresponding vhx_tree_desc array) and refreshes the derived device state. VHX_E_CAPACITY past the end.
 * Stream-ordered: the source is copied into pinned staging before the call returns (the caller may reuse it at once),
 * and the device writes, like the derived-state refresh, run on the context's stream ahead of its next trace; no host
 * synchronisation. Same as vhx_update_ranges with one range. */
int vhx_update_range(vhx_ctx *ctx, int buffer_id, uint64_t elem_offset, uint64_t elem_count, const void *src);
/* One ranged write of vhx_update_ranges. */
typedef struct vhx_range {
    int32_t buffer_id;   /* VHX_BUF_* */
    uint32_t reserved0;
    uint64_t elem_offset;
    uint64_t elem_count;
    const void *src;     /* host memory, elem_count elements */
} vhx_range;
/* A frame's ranged writes in one call (the reference issues one write_range_to_buffer per range,
 * streaming/mod.rs:420-635): the sources are packed into pinned staging, moved to HBM by ONE host-to-device copy and
 * scattered to their buffers by one kernel; the derived state (node headers, brick bitmaps, and the child records of
 * the written nodes and of the nodes holding written bricks) is refreshed on the device, all stream-ordered without
 * host synchronisation. All ranges are validated before anything is written. */
int vhx_update_ranges(vhx_ctx *ctx, const vhx_range *ranges, uint32_t n);
/* Diagnostics: copies elements of a derived device buffer to host memory (for tests).
 * VHX_DERIVED_NODE_HDR: 16-byte {occ_lo, occ_hi, type, 0} per node; VHX_DERIVED_BRICK_OCC: u64 words, brick_dim^3
 * bits per brick (max(1, brick_dim^3/64) words), bit = flat cell index, set = cell not empty. */
#define VHX_DERIVED_NODE_HDR 0
#define VHX_DERIVED_BRICK_OCC 1
int vhx_read_derived(vhx_ctx *ctx, int which, uint64_t elem_offset, uint64_t elem_count, void *dst);
/* Device bytes held by the uploaded tree. */
int vhx_tree_device_bytes(const vhx_ctx *ctx, uint64_t *bytes);

/* Tracing --------------------------------------------------------------------------------------------------- */
/* Traces primary rays for every pixel of the square tiles k = tile_start, tile_start+tile_stride, ... (raster order
 * of ceil(W/T) x ceil(H/T) tiles, T = tile_size). tile_size 0 with layout FRAMEBUFFER traces the whole frame.
 * In the TILES layout, entries of pixels past the frame edge are not written (device outputs) or read back as 0
 * (host outputs). */
int vhx_trace_primary(vhx_ctx *ctx, const vhx_camera *cam, uint32_t tile_size, uint32_t tile_start,
                      uint32_t tile_stride, uint32_t layout, const vhx_hits *out, int on_device);
/* A batch of n whole frames (framebuffer layout, device outputs) traced as ONE pass ladder on the context's stream: pass
 * 0 over every pixel of every frame in one launch, one compaction over the union of their abandoned rays, and queue
 * passes shared by all frames (the frames-in-flight schedule), so a renderer gets frames-in-flight throughput from one
 * stream and one hardware queue (no GPU_MAX_HW_QUEUES setting; the per-frame dispatch of VhxRenderNode::run,
 * src/raytracing/bevy/pipeline/mod.rs:96-155, batched). Frame k is cams[k] (every camera the same width x height)
 * into outs[k] (device pointers, any subset of fields; byte counting and node MIPs are refused); results equal n
 * vhx_trace_primary calls bit for bit. The depth-prepass mode does not apply (the batch traces the exact path).
 * At most 2^31 rays per batch; output arrays of different frames (or fields) must not overlap: VHX_E_INVALID_ARG.
 * Stream-ordered like vhx_trace_primary; vhx_sync reports the batch's device time. The cameras and output pointers
 * are staged in pinned memory: by default the call waits until the context's previous batch has started on the GPU
 * (its staging copy ran), so one batch queues behind the running one -- the GPU stays fed, and three contexts
 * round-robin measured 3.5-4 % faster than with the host running further ahead. vhx_set_tuning "stage_slots=N"
 * (N <= 4) stages through a ring of N slots, so N batches queue back to back on one context before the call waits.
 * Batches on one context run one after another on its stream; for batches that overlap on the GPU, round-robin over
 * shared contexts. */
int vhx_trace_primary_batch(vhx_ctx *ctx, const vhx_camera *cams, uint32_t n, const vhx_hits *outs);
/* The same for tile sets (the rank's share of a multi-GPU frame, vhx_mgpu_render_batch): frame k is the TILES-layout
 * trace of cams[k] over tiles tile_starts[k], tile_starts[k] + tile_stride, ... (tile_size T), into outs[k] exactly as
 * vhx_trace_primary(ctx, &cams[k], T, tile_starts[k], tile_stride, VHX_LAYOUT_TILES, &outs[k], 1) writes it (entries
 * past the frame edge are not written); one pass ladder for all n frames. Frames may hold different tile counts
 * (a start past the last tile: no entries). Results equal n vhx_trace_primary calls bit for bit. */
int vhx_trace_tiles_batch(vhx_ctx *ctx, const vhx_camera *cams, uint32_t n, uint32_t tile_size,
                          const uint32_t *tile_starts, uint32_t tile_stride, const vhx_hits *outs);
/* Depth-prepass fast mode (opt-in; NOT the reference's CPU semantics, so outside the parity bar; the WGSL path's
 * prepass, src/raytracing/bevy/viewport_render.wgsl:702-726). When enabled, a vhx_trace_primary of a whole frame in
 * the FRAMEBUFFER layout without byte counting first traces a half-resolution depth frame (texel (X, Y) through the
 * centre of full pixels 2X..2X+1, 2Y..2Y+1), then starts every full-resolution ray at the minimum of depth texels
 * (x/2, y/2), (x/2+1, y/2), (x/2, y/2+1), (x/2+1, y/2+1) minus `margin` (distance units; 0 = the WGSL's choice), and
 * reports a miss where all four texels missed. Thin or grazing geometry that none of the four texel rays hits first can
 * be skipped: the pixels that differ from the exact path are measured in tests/test_gpu_fast.py and docs/DESIGN_LOG.md §10.
 * Other traces (tiles, ray batches, shadows, byte counting) stay exact. Default off. */
int vhx_set_depth_prepass(vhx_ctx *ctx, int enable, float margin);
/* Fused hard shadows (BASELINE config 5; shadow semantics of vhx_trace_shadows): with a light set, vhx_trace_primary,
 * vhx_trace_primary_batch and vhx_trace_tiles_batch also trace every hit's hard-shadow ray and write `shadowed` (and
 * darken `rgba`) of their outputs, which then need value, impact, normal and shadowed. Under the frames-in-flight /
 * batch schedule (pass 0 lists its rays) the shadow ray continues in the lane and pass that finished its primary ray,
 * while the nodes of its descent are still in that CU's caches; otherwise (a lone frame's schedule) the frame's shadow
 * rays are traced after its primary rays, as vhx_trace_shadows does. Results equal vhx_trace_primary followed by
 * vhx_trace_shadows bit for bit. light = NULL turns it off (the default). No byte counting, depth prepass or node
 * MIPs with a light set. */
int vhx_set_shadow_light(vhx_ctx *ctx, const float *light);
/* MIP stand-ins for absent children (the WGSL path's probe_MIP, src/raytracing/bevy/viewport_render.wgsl:328-364,
 * 438-454, enabled by tree_properties bit 16, streaming/mod.rs:288-290): node_mips[i] is node i's MIP brick descriptor
 * (same encoding as a leaf's child entry, VHX_EMPTY = none; the bricks live in voxels / solid_values like any other,
 * e.g. vhx_boxtree_flatten_lod). While set, a node iteration of an Internal or Leaf node whose target sectant is
 * occupied (occupancy bit set) but whose child entry is VHX_EMPTY (not resident) first traces the node's MIP brick
 * over the node's cube; a MIP hit ends the ray there, a miss leaves the ray where it was and ADVANCEs past the
 * sectant (where the reference CPU path would push into the child, which does not exist). Without MIPs (the default)
 * such a push ends the ray as a miss, as before. A tree whose children are all present traces identically either way.
 * NULL disables; count must equal the uploaded tree's node_count; a new vhx_upload_tree disables them. Like an update,
 * it goes through the owner of a shared tree and is ordered against frames in flight (vhx_create_shared); shared
 * contexts trace with them. */
int vhx_set_node_mips(vhx_ctx *ctx, const uint32_t *node_mips, uint32_t count);
/* Diagnostics of a VHX_PROF build (scripts/probes/probe_blocks.py; a regular build returns VHX_E_STATE): per pass
 * slot (5: budgets <= 24, <= 96, <= 256, larger, the unbounded pass) and traversal block (16), the wave executions
 * and the lanes active in them, as out[2 * (pass * 16 + block)] and out[2 * (pass * 16 + block) + 1], accumulated
 * over every trace since the last reset. */
int vhx_profile_counters(vhx_ctx *ctx, uint64_t *out, uint32_t n, int reset);
/* Diagnostics of a VHX_CHAIN build (libvhx_chain.so, scripts/chain_profile.py; a regular build returns VHX_E_STATE):
 * the primary rays of the n pixels (index y * width + x of `cam`'s frame, host array) each traced alone in a wave of
 * its own, its dependent chain stamped per node iteration; out (host, n x 64 words): [0] cycles of the traversal,
 * [1] node-load waits, [2] leaf probes, [3] POP / PUSH bookkeeping, [4] ADVANCE walks, [5] loop overhead, [6] node
 * iterations, [7] probes, [8] ADVANCE walks, [9] steps, [10] hit value, [16..63] node-load wait histogram in 64-cycle
 * buckets (the last one open). Shader cycles (s_memtime). */
int vhx_chain_profile(vhx_ctx *ctx, const vhx_camera *cam, const uint32_t *pixels, uint32_t n, uint64_t *out);
/* Early tail of lone frames (scheduling only; off by default: vhx_set_tuning "tail=1" turns it on, "tail_min",
 * "tail_rpw", "tail_cap", "tail_prio" tune it): a lone vhx_trace_primary of a whole framebuffer records the pixels whose rays took >= tail_min steps, and
 * the context's next lone frame of the same size traces them from its start on a second stream while the rest of the
 * frame takes the pass ladder -- the longest rays' chains no longer start last. Results are bit-identical either way.
 * Diagnostics: *listed = the pixels the next lone frame would trace early (0: none recorded, or tail off), *width /
 * *height = the frame size they were recorded for (either may be null); synchronises the context's stream. */
int vhx_tail_info(vhx_ctx *ctx, uint32_t *listed, uint32_t *width, uint32_t *height);
/* Traces n explicit rays; rays = 6 f32 per ray (origin xyz, direction xyz), host or device per on_device. */
int vhx_trace_rays(vhx_ctx *ctx, const float *rays, uint64_t n, const vhx_hits *out, int on_device);
/* Hard shadows (BASELINE config 5; the reference has no shadow rays — semantics defined in docs/DESIGN_LOG.md §9): for
 * every ray i < n of a previous trace with a hit (value[i] != VHX_EMPTY), one shadow ray from
 * impact[i] + normal[i] * 1e-3 toward `light` (e.g. the reference's ambient_light_position = (size, size, size),
 * src/raytracing/bevy/view.rs:81-85) is traced with get_by_ray semantics; shadowed[i] = 1 if it hits a voxel, else 0
 * (0 for primary misses). rgba (optional) is darkened in place (rgb >> 1) where shadowed; bytes (optional) receives
 * the algorithmic bytes of each shadow ray. All pointers are device memory (the on_device output of
 * vhx_trace_primary / vhx_trace_rays); hit pixels are compacted first so waves trace only shadow rays. The outputs
 * (shadowed, rgba, bytes) must not overlap the hit records (value, impact, normal) or each other: VHX_E_INVALID_ARG. */
int vhx_trace_shadows(vhx_ctx *ctx, const float light[3], uint64_t n, const uint32_t *value, const float *impact,
                      const float *normal, uint32_t *shadowed, uint32_t *rgba, uint32_t *bytes);
/* One frame of a shadow batch (vhx_trace_shadows_batch): a primary frame's hit records (value, impact, normal: n, 3n,
 * 3n entries) and its outputs (shadowed: n; rgba: n, optional, darkened in place), all device memory. */
typedef struct vhx_shadow_frame {
    const uint32_t *value;
    const float *impact;
    const float *normal;
    uint32_t *shadowed;
    uint32_t *rgba;
} vhx_shadow_frame;
/* Hard shadows of n_frames frames (n records each) as ONE pass ladder on the context's stream: the hit records of
 * every frame compacted together, shared queue passes (vhx_trace_primary_batch's shape for BASELINE config 5, e.g.
 * right after it on the same context). Results equal n_frames vhx_trace_shadows calls bit for bit; no byte counting
 * and no node MIPs; at most 2^31 records per batch; outputs must not overlap any frame's hit records or each other. */
int vhx_trace_shadows_batch(vhx_ctx *ctx, const float light[3], uint32_t n_frames, uint64_t n,
                            const vhx_shadow_frame *frames);

/* Scatters tile-major RGBA buffers gathered from `ranks` ranks (rank r traced tiles r, r+ranks, ...; each rank's
 * buffer holds tiles_per_rank*T*T pixels, concatenated by rank) into a width x height framebuffer.       */
int vhx_untile_rgba(vhx_ctx *ctx, const uint32_t *gathered, uint32_t ranks, uint32_t tiles_per_rank,
                    uint32_t tile_size, uint32_t width, uint32_t height, uint32_t *framebuffer, int on_device);

/* Scatters rank-gathered tile buffers into device framebuffers (the general form of vhx_untile_rgba). Rank r's part
 * of `gathered` (rank-major) holds `planes` planes of tiles_per_rank*T*T 32-bit words each — plane 0 the RGBA8 of its
 * tiles, plane 1 (planes = 2) their f32 depth — in the VHX_LAYOUT_TILES order of tiles r, r+ranks, ... Either
 * framebuffer may be NULL to skip its plane (fb_depth must be NULL when planes = 1). Device pointers only.           */
int vhx_untile_frame(vhx_ctx *ctx, const void *gathered, uint32_t planes, uint32_t ranks, uint32_t tiles_per_rank,
                     uint32_t tile_size, uint32_t width, uint32_t height, uint32_t *fb_rgba, float *fb_depth);

/* ---- multi-GPU: screen-tile split over RCCL ------------------------------------------------------
 * One context per GPU and process (the reference renders one view per Bevy render world, VhxRenderNode::run,
 * src/raytracing/bevy/pipeline/mod.rs:96-155; these calls spread that view over the GPUs of a node). The frame is cut
 * into tile_size^2 screen tiles dealt round-robin over V = R + N - 1 slots, rank 0 owning slots 0..R-1 and rank
 * r >= 1 slot R + r - 1 (R = 1, the default: rank r traces tiles r, r+N, ...); each frame every rank traces its slots
 * into contiguous RGBA8 + f32-depth parts, point-to-point RCCL transfers over xGMI bring the other ranks' parts to
 * rank 0, and rank 0 untiles them into its framebuffers. The tree is replicated: vhx_mgpu_broadcast_tree
 * uploads it on rank 0 and ncclBroadcasts the device buffers to the other ranks (no host copy of the tree there).
 * RCCL is loaded at run time (dlopen of librccl.so.1, or the path in VHX_RCCL_LIB), so libvhx itself has no link-time
 * RCCL dependency; without it these calls return VHX_E_RCCL. Errors are reported through vhx_last_error(ctx).      */
#define VHX_MGPU_ID_BYTES 128 /* = NCCL_UNIQUE_ID_BYTES */
typedef struct vhx_mgpu vhx_mgpu;
/* Rank 0 creates the communicator id; the caller sends its bytes to every rank out of band (e.g. a TCP store). */
int vhx_mgpu_unique_id(uint8_t id[VHX_MGPU_ID_BYTES]);
/* Collective over the N ranks (ncclCommInitRank): joins the communicator `id` as `rank` of `nranks`. */
int vhx_mgpu_create(vhx_ctx *ctx, const uint8_t id[VHX_MGPU_ID_BYTES], int nranks, int rank, uint32_t tile_size,
                    vhx_mgpu **out);
/* Same on a communicator the caller already owns (an ncclComm_t passed as void*; borrowed, never destroyed). */
int vhx_mgpu_create_from_comm(vhx_ctx *ctx, void *nccl_comm, uint32_t tile_size, vhx_mgpu **out);
/* Collective: rank 0 passes the tree (uploaded to its context like vhx_upload_tree), every other rank NULL; returns
 * once every rank holds the tree and its derived device layout. */
int vhx_mgpu_broadcast_tree(vhx_mgpu *m, const vhx_tree_desc *tree);
/* overlap = 1 (default): frame k's gather and untile run on a communication stream while frame k+1 is traced (two
 * tile buffers alternate); 0: each render completes its gather and untile in the context's stream order. */
int vhx_mgpu_set_overlap(vhx_mgpu *m, int overlap);
/* Collective: renders one frame. On rank 0, fb_rgba (width*height u32, RGBA8) and fb_depth (width*height f32, may be
 * NULL) are device framebuffers receiving the whole frame; other ranks pass NULL. Outputs are complete after
 * vhx_mgpu_sync. */
int vhx_mgpu_render(vhx_mgpu *m, const vhx_camera *cam, uint32_t *fb_rgba, float *fb_depth);
/* Collective: renders n frames (1..VHX_MGPU_MAX_INFLIGHT, every camera the same width x height) as one batch: each rank
 * traces its tile slots of all n frames with ONE vhx_trace_tiles_batch (the per-frame pass ladder's fixed costs paid
 * once per batch), then the n frames' transfers to rank 0 run as one RCCL group and rank 0 untiles frame k into
 * fb_rgba[k] / fb_depth[k] (arrays of n device pointers on rank 0; fb_depth may be NULL; other ranks pass NULL).
 * Successive batches are traced by the vhx_mgpu_set_frames_in_flight contexts in turn. Results equal n
 * vhx_mgpu_render calls bit for bit; complete after vhx_mgpu_sync. */
int vhx_mgpu_render_batch(vhx_mgpu *m, const vhx_camera *cams, uint32_t n, uint32_t *const *fb_rgba,
                          float *const *fb_depth);
/* Waits for every frame submitted on this rank (trace, gather and untile); optionally returns the device time of the
 * last frame's trace on this rank in milliseconds. */
int vhx_mgpu_sync(vhx_mgpu *m, float *last_trace_ms);
/* Frames in flight on this rank (1..VHX_MGPU_MAX_INFLIGHT, default 1): frame k is traced by the k % F-th of F contexts
 * sharing the tree (vhx_create_shared), each on its own stream, so frame k+1's trace overlaps frame k's long-ray tail;
 * gathers stay in frame order on the communication stream. Waits for the frames in flight before it changes them. */
#define VHX_MGPU_MAX_INFLIGHT 16
int vhx_mgpu_set_frames_in_flight(vhx_mgpu *m, uint32_t frames);
/* Collective, between frames: rank 0's share of the tiles, R of the R + N - 1 slots (1..VHX_MGPU_MAX_ROOT_SLOTS; every
 * rank must pass the same R). R > 1 suits a link-bound split: rank 0's own parts cross no link. */
#define VHX_MGPU_MAX_ROOT_SLOTS 4
int vhx_mgpu_set_root_slots(vhx_mgpu *m, uint32_t root_slots);
/* Collective: renders `frames` + 1 frames of `cam` one at a time with R = 1, takes on rank 0 the median device time of
 * its trace and of the transfers into it, and sets on every rank the R that minimises the modelled frame period
 * (N / (R + N - 1)) * max(R * trace, transfer) (a larger R must win by 3 %). Returns R and rank 0's two figures (ms);
 * any output pointer may be NULL. */
int vhx_mgpu_balance(vhx_mgpu *m, const vhx_camera *cam, uint32_t frames, uint32_t *root_slots, float *trace_ms,
                     float *transfer_ms);
/* Collective: planes each rank sends to rank 0 (waits for the frames in flight; the ranks agree on the value over the
 * communicator, and when they passed different values every rank fails with VHX_E_INVALID_ARG and keeps its old
 * count): 2 (default)
 * = RGBA8 + f32 depth, 1 = RGBA8 only -- the reference's display output is the rgba8unorm view texture
 * (src/raytracing/bevy/view.rs:269-289), so a renderer that needs no depth halves rank 0's intake over xGMI. With one
 * plane rank 0 passes fb_depth = NULL to vhx_mgpu_render. */
int vhx_mgpu_set_planes(vhx_mgpu *m, uint32_t planes);
/* Bytes rank 0 receives over xGMI per width x height frame at the current split and plane count. */
int vhx_mgpu_frame_bytes(const vhx_mgpu *m, uint32_t width, uint32_t height, uint64_t *into_root);
/* nranks, rank, and the rays this rank traces for a width x height frame (any pointer may be NULL). */
int vhx_mgpu_info(const vhx_mgpu *m, uint32_t width, uint32_t height, int *nranks, int *rank, uint64_t *rays);
/* The tile plan of the split, as vhx_mgpu_render deals it (a pure function: no device, no communicator). For N ranks,
 * rank 0 owning R slots, tile size T and a width x height frame: tiles = ceil(W/T) * ceil(H/T) raster-order tiles,
 * slots = R + N - 1, slot s traces tiles s, s + slots, ... (tiles_per_slot = ceil(tiles / slots) entries each, the last
 * ones padded), `rank` owns slots first_slot .. first_slot + slot_count - 1 and sends them to rank 0, whose
 * slot-major gather buffer holds slot s's part at s * tiles_per_slot * T * T words per plane. */
typedef struct vhx_tile_plan {
    uint32_t tiles_x, tiles_y, tiles, slots, tiles_per_slot, first_slot, slot_count, reserved;
} vhx_tile_plan;
int vhx_mgpu_tile_plan(uint32_t nranks, uint32_t root_slots, uint32_t tile_size, uint32_t width, uint32_t height,
                       uint32_t rank, vhx_tile_plan *plan);
/* Collective: renders `frames` + 1 frames of `cam` one at a time at the current split and returns THIS rank's median
 * device time of its trace and of its transfers (rank 0: its receives of the other ranks' parts; other ranks: the send), in ms
 * (the first frame is a warm-up). Diagnostics for the scaling model of DESIGN.md §7; any output may be NULL. */
int vhx_mgpu_measure(vhx_mgpu *m, const vhx_camera *cam, uint32_t frames, float *trace_ms, float *transfer_ms);
void vhx_mgpu_destroy(vhx_mgpu *m);

#ifdef __cplusplus
}
#endif
#endif /* VHX_H */
