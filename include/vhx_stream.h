/*
 * vhx_stream.h — streaming producer: a bounded device-resident view of a BoxTree around a viewport, kept up to date
 * with ranged writes. Restates the reference's BoxTreeGPUDataHandler and upload queue
 * (src/raytracing/bevy/streaming/{cache,upload_queue,mod}.rs, view sizing src/raytracing/bevy/view.rs:50-69) on top of
 * vhx_upload_tree / vhx_update_range; see voxelhex_amd/csrc/stream.cpp for the line-level mapping.
 *
 * Device view layout = vhx_tree_desc with node_count = nodes_in_view, brick_count = bricks_in_view: node slot 0 is
 * the root, a child that is not resident is VHX_EMPTY (traced as empty space, like the reference's empty_marker).
 * After every vhx_stream_upload the context traces the view (vhx_trace_primary / vhx_trace_rays).
 *
 *   vhx_stream_create       <- BoxTreeGPUHost::create_new_view (view.rs:36-137): sizes the view, uploads it empty
 *   vhx_stream_set_viewport <- viewport change handling (bevy/mod.rs:110-155): rebuild when the origin leaves its
 *                              brick slot (Cube::brick_slot_for) or the view distance changes
 *   vhx_stream_upload       <- streaming::upload (streaming/mod.rs:420-635): one frame of node + brick uploads
 *                              (node_uploads_per_frame / brick_uploads_per_frame); VHX_E_CAPACITY = the view is too
 *                              small (re_evaluate_view_size grew it): call vhx_stream_resize, then upload again
 *   vhx_stream_resize       <- view.resize (pipeline/mod.rs:293-353): re-creates the device view at the new capacity
 *   vhx_stream_reload       <- BoxTreeGPUView::reload (view.rs:141-145)
 *   vhx_stream_view         host mirror of the device view (for checking; pointers valid until the next call)
 *
 * Tree changes: inserts and updates of the tree (vhx_boxtree_insert / _insert_at_lod / _update) made while a stream
 * exists are queued by the tree (the update trigger of BoxTreeGPUHost::new, src/raytracing/bevy/mod.rs:164-173) and
 * re-uploaded by the next vhx_stream_upload calls (handle_tree_updates, streaming/mod.rs:35-286: up to
 * node_uploads_per_frame changes per frame, ahead of the upload queue). One stream per tree receives them, like the
 * reference's single changes buffer. The tree and the context must outlive the stream; ctx = NULL keeps the view on
 * the host only (vhx_stream_view), which is how the producer is tested without a GPU. Every frame's ranged writes go
 * to the device as one vhx_update_ranges call (stream-ordered, no host synchronisation).
 */
#ifndef VHX_STREAM_H
#define VHX_STREAM_H

#include "vhx.h"
#include "vhx_boxtree.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct vhx_stream vhx_stream;

typedef struct vhx_stream_stats {
    uint64_t bytes_written;   /* bytes written to the device by the last upload */
    uint64_t bricks_written;  /* bricks whose voxels were written by the last upload */
    uint64_t nodes_written;   /* nodes (re)written by the last upload */
    uint64_t nodes_resident;  /* nodes currently mapped to a slot */
    uint64_t bricks_resident; /* brick slots currently owned (incl. MIP slots) */
    uint64_t nodes_in_view;   /* node capacity */
    uint64_t bricks_in_view;  /* brick capacity */
    uint64_t nodes_to_see;    /* nodes the viewport needs */
    uint64_t pending;         /* work left: nodes to see that are not resident + queued brick requests + queued tree
                                 changes, + 1 until a
                                 complete walk cycle found nothing new (the node walk restarts from the root whenever
                                 it finishes, as in the reference, so a lost brick is requested on the next cycle) */
} vhx_stream_stats;

int vhx_stream_create(const vhx_boxtree *tree, vhx_ctx *ctx, const float origin[3], float view_distance,
                      vhx_stream **out);
void vhx_stream_destroy(vhx_stream *stream);
/* BoxTreeGPUDataHandler::{node_uploads_per_frame, brick_uploads_per_frame, brick_unload_search_perimeter};
 * defaults 25, 50, 10 as in view.rs:109-111 */
int vhx_stream_set_rates(vhx_stream *stream, uint32_t node_uploads_per_frame, uint32_t brick_uploads_per_frame,
                         uint32_t brick_unload_search_perimeter);
int vhx_stream_set_viewport(vhx_stream *stream, const float origin[3], float view_distance);
int vhx_stream_upload(vhx_stream *stream, vhx_stream_stats *stats);
/* `frames` frames of vhx_stream_upload's decisions (each frame at the reference's per-frame rates, tree changes
 * first), written to the device as ONE vhx_update_ranges call: one tree version for the `frames` frames a renderer
 * keeps in flight until its next call (with frames in flight, a write every frame serialises them: every write waits
 * for the frames before it and every frame for the write). The view after the call equals the view after `frames`
 * vhx_stream_upload calls; stats sum the frames. frames = 1 is vhx_stream_upload. */
int vhx_stream_upload_frames(vhx_stream *stream, uint32_t frames, vhx_stream_stats *stats);
int vhx_stream_resize(vhx_stream *stream);
int vhx_stream_reload(vhx_stream *stream);
/* Diagnostics: after a viewport move the view set (upload_queue.rs:60-148 rebuild) is updated incrementally where the
 * walk root stays the same; this recomputes it in full at the last rebuild's viewport and compares (VHX_OK: equal,
 * VHX_E_STATE: different), leaving the stream unchanged, and reports how many rebuilds ran in full / incrementally. */
int vhx_stream_view_set_check(vhx_stream *stream, uint64_t *full_rebuilds, uint64_t *incremental_rebuilds);
int vhx_stream_view(const vhx_stream *stream, vhx_tree_desc *out);
/* the view's node MIP descriptors (host mirror, nodes_in_view entries; all VHX_EMPTY unless the tree's MIP maps are
 * enabled, in which case the stream also writes the MIP bricks and hands the descriptors to vhx_set_node_mips) */
int vhx_stream_node_mips(const vhx_stream *stream, const uint32_t **node_mips, uint32_t *count);

#ifdef __cplusplus
}
#endif

#endif /* VHX_STREAM_H */
