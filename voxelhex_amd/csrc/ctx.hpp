// Internal context of libvhx (shared by the translation units of the device side: vhx_device.hip, vhx_mgpu.hip).
// Not part of the ABI: callers see vhx_ctx only as an opaque pointer (include/vhx.h).
#pragma once
#include <hip/hip_runtime.h>

#include <condition_variable>
#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/vhx.h"

struct DevBuf {
    void *ptr = nullptr;
    uint64_t bytes = 0;
};

// The device copy of a tree and its derived layout. Held by every context that traces it (vhx_create_shared gives
// further contexts — one per frame in flight — the same store), freed with the last of them.
struct TreeStore {
    int device = 0;
    bool uploaded = false;
    vhx_tree_desc desc{};  // counts of the uploaded tree (pointers unused)
    DevBuf raw[7];         // VHX_BUF_* raw copies
    DevBuf hdr, brick_occ;
    DevBuf child_rec;      // brick_dim <= 4: DevTree::child_rec, rebuilt before a trace when stale
    bool child_rec_stale = false;
    uint32_t occ_words = 1;
    // node_mips (src/raytracing/bevy/types.rs:245-247): one MIP brick descriptor per node; while set, a node
    // iteration whose target child is occupied but absent probes the node's MIP (vhx_set_node_mips)
    DevBuf mips;
    bool mips_on = false;
    // Ordering of tree writes against frames in flight (any context of the tree, any stream; no host waits): a write
    // (upload, ranged update, node MIPs) first makes its stream wait for the last submitted trace of every other
    // context (their use_ev), and records write_ev after it; a context's next trace waits for write_ev once per write
    // (write_seq against its seen_write). Contexts register in `users` at creation and leave at destruction.
    std::mutex mu;
    std::condition_variable cv;  // tracing / writing changed
    uint32_t tracing = 0;        // traces between trace_begin and trace_end (any thread)
    uint32_t writing = 0;        // writes between write_begin and write_end
    uint32_t writers_waiting = 0;  // writes blocked in write_begin (new traces wait for them: no writer starvation)
    std::vector<struct vhx_ctx *> users;
    hipEvent_t write_ev = nullptr;
    hipStream_t write_stream = nullptr;
    uint64_t write_seq = 0;
    ~TreeStore();
};

// default pass-0 queue orders of the two schedules (vhx_ctx::qorder encoding)
// Frames in flight: 64x64 tiles row-major, Morton order inside ("64z"): the bench frame at eight in flight 0.516-0.525
// ms against 0.564-0.567 in output-index (row-major) order, queue passes at 20.3 instead of 17.4 lanes per VALU
// instruction; 32r 0.515-0.523, 64 / 64r 0.524-0.530, 128r 0.536-0.539, Morton orders of tiles 0.509-0.540 from box to
// box (profiles/r03/qorder/). A lone frame keeps output-index order: 1.21-1.24 ms against 1.33-1.42 with tile orders
// (its critical path is its slowest chunk, and 2-D clusters gather the longest rays into fewer, longer chunks).
#define VHX_QORDER_BUSY 38u
#define VHX_QORDER_IDLE 0u
// Queue passes of the frames-in-flight schedule: every segment of VHX_QSORT_BUSY consecutive queue entries sorted by the
// node each ray's saved state stands at (k_sort_segments in vhx_device.hip; docs/DESIGN_LOG.md §15.3), so that a wave's rays start
// at the same node; 0 = off. Off by default: 2-7 % fewer VALU instructions per frame, but no faster (0.527-0.564 against
// 0.526-0.536 ms per bench frame over five sort variants, profiles/r04/qsort/); tune "qsort=N" turns it on
#ifndef VHX_QSORT_BUSY
#define VHX_QSORT_BUSY 0u
#endif
// ... and of the lone-frame schedule's unbounded pass: segments of 256 (the lone bench frame 1.19 against 1.22 ms in two
// runs, the orbiting lone frame unchanged; 512 / 1024 / 2048 no faster or slower: profiles/r04/final_check/lone_qsort*.log)
#ifndef VHX_QSORT_IDLE
#define VHX_QSORT_IDLE 256u
#endif
#define VHX_QSORT_MAX 2048u

struct vhx_ctx {
    int device = 0;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    bool timed = false;
    std::string err;
    std::shared_ptr<TreeStore> tree;  // shared by the contexts of one tree
    bool shared = false;              // made by vhx_create_shared: traces only (uploads and updates go to the owner)
    hipEvent_t use_ev = nullptr;      // recorded after every trace submitted on this context (TreeStore ordering)
    hipStream_t use_stream = nullptr;  // the stream use_ev was last recorded on
    bool use_recorded = false;
    uint64_t seen_write = 0;          // the TreeStore write_seq this context's stream already waits for
    DevBuf scratch, rays;
    DevBuf queue[2];  // multi-pass ray queues (ping-pong), output indices of abandoned rays in increasing order
    DevBuf qctl;      // QCTL_WORDS: [0..7] queue lengths after pass p (7: shadow hit list), [16 + 16p ..] counters
    DevBuf tmp;       // chunk-local lists of abandoned rays (a block's or a queue chunk's, in lane order)
    DevBuf counts;    // rays listed per chunk
    DevBuf offsets;   // exclusive scan of counts
    DevBuf scan_part; // scans of more than scan_multi segments: the segments' sums, then their exclusive scan
    DevBuf flags;     // primary pass 0: abandoned flag per output index
    DevBuf qargs;     // QueueArgs of the queue passes: slot 0 primary rays / ray batches, slot 1 shadow rays
    std::vector<uint8_t> qargs_host[2];  // the QueueArgs last written to each slot (skips the upload when unchanged)
    void *qargs_host_ptr[2] = {nullptr, nullptr};  // qargs.ptr they were written to
    DevBuf state;     // saved traversal state (64 B) of rays abandoned at a budget: per output index, or per list slot
    DevBuf stateq;    // queue-state mode: the states moved into the next pass's queue order by the compaction
    // ranged writes (vhx_update_ranges): two pinned host staging slots, alternating, each reusable once the
    // host-to-device copy that read it has completed (event), and the device staging buffer the scatter kernel reads
    struct Pinned {
        void *ptr = nullptr;
        uint64_t bytes = 0;
        hipEvent_t done = nullptr;
        bool used = false;
    } pinned[2];
    uint32_t pinned_next = 0;
    // vhx_trace_primary_batch: the batch's cameras and outputs (a ring of pinned staging slots, and their device
    // copy). A slot is rewritten only once the copy that read it has run; with N slots in use a caller can queue N
    // batches on one context before the host waits (the device copy itself is stream-ordered)
    static constexpr uint32_t VHX_STAGE_SLOTS = 4;
    Pinned batch_pinned[VHX_STAGE_SLOTS];
    uint32_t batch_next = 0;
    // slots in use (tune "stage_slots"). 1: a batch waits on the host until the context's previous batch started on
    // the GPU. Measured (profiles/r06/stage_slots/): the bench default (batches of 7 on 3 contexts) 0.483-0.487 ms
    // per frame at 1 slot against 0.500-0.507 at 4 and 0.501-0.502 at 2; 2 contexts 0.517-0.518 against 0.525-0.531;
    // one context equal (0.654-0.662). Letting the host run further ahead only slows the contexts' interleaving
    uint32_t stage_slots = 1;
    DevBuf batch_args;
    // vhx_trace_shadows_batch: the frames' ShD records and hit-value pointers (pinned staging ring, device copy)
    Pinned shadow_pinned[VHX_STAGE_SLOTS];
    uint32_t shadow_next = 0;
    DevBuf shadow_args;
    DevBuf upd;
    hipStream_t upd_stream = nullptr;  // the stream of the last scatter (reads upd)
    // depth-prepass mode (vhx_set_depth_prepass; opt-in, not the reference path)
    bool prepass = false, in_prepass = false;
    // fused hard shadows (vhx_set_shadow_light): each hit's shadow ray traced in the lane that finished its primary ray
    bool shadow_on = false;
    float shadow_light[3] = {0.f, 0.f, 0.f};
    bool keep_ev0 = false;  // the shadow rays of a frame traced after it: its time runs from the primary trace's ev0
    uint32_t shadow_budget = 0;  // fused shadows: a shadow ray's steps in its primary ray's budgeted pass (tune "sbudget")
    // Early tail (lone frames; tune "tail=1" turns it on, off by default until it pays): a lone frame's time is its
    // longest rays' serial chains, which the pass ladder starts last. Each lone frame records the pixels whose rays
    // took >= tail_min steps (tail_list, at most tail_cap; word 0 the count, entries from word 64); the next lone
    // frame of the same size traces those pixels from its start, tail_rpw to a wave, on a second stream of high
    // priority (k_trace_tail) while its other pixels go through the usual passes (pass 0 skips the listed ones,
    // tail_mask). Scheduling only: every pixel is traced once, completely, by the same get_by_ray, so the frame is
    // bit-identical whatever the list holds.
    bool tail_on = false;
    uint32_t tail_min = 512, tail_cap = 4096, tail_rpw = 4, tail_prio = 0;
    DevBuf tail_list[2], tail_mask;
    uint32_t tail_cur = 0, tail_w = 0, tail_h = 0;  // tail_list[tail_cur]: the last recorded list, of a tail_w x tail_h frame
    bool tail_valid = false;
    uint32_t *tail_rec = nullptr;  // during a recording trace: the list its final pass appends to
    hipStream_t tail_stream = nullptr;
    hipEvent_t tail_fork = nullptr, tail_join = nullptr;
    float prepass_margin = 0.0f;
    DevBuf prepass_depth;  // the half-resolution depth frame
    // Ray schedule of a trace: step budgets of the passes before the final (unbounded) one, the sparse-wave thresholds
    // of the budgeted passes and the waves of a queue pass. Results never depend on it (bit-identical for any
    // schedule); the frame time does, and what is best depends on whether the frame shares the GPU with other frames.
    struct Sched {
        uint32_t budgets[VHX_MAX_BUDGETS];
        uint32_t npass;                      // passes including the final one (1 = single pass)
        uint32_t sparse[VHX_MAX_BUDGETS];    // abandon a wave's rays once fewer lanes still trace (0 = off)
        uint32_t queue_waves_per_cu;         // waves of a queue pass per CU
        uint32_t qorder;                     // order of a primary frame's pass-0 queue (vhx_ctx::qorder below)
        uint32_t qsort;                      // queue passes: segments of this many queue entries sorted by saved node
        uint32_t queue_waves0_per_cu;        // waves of a first queue pass over fresh rays (the shadow rays) per CU
        uint32_t shadow_budgets[VHX_MAX_BUDGETS];  // the ladder of a shadow trace (vhx_trace_shadows / _batch)
        uint32_t shadow_npass;
    };
    // Adaptive scheduling (default; vhx_set_pass_budgets or a tuning key fixes the schedule instead): at each
    // trace the context looks at the other contexts of its tree (vhx_create_shared) and picks
    //  * `busy` when any of them still has a frame in flight on another stream, or a batch: {32, 128, 768} since round 6
    //    -- with batches of 7 on 3 contexts 0.4761-0.4770 ms per frame over 100 frames against 0.4867-0.4873 for
    //    {24, 72, 216, 648}, and in the driver's 20-frame window 0.487-0.496 against 0.500-0.514 ms (four alternating
    //    runs; {40, 160, 640} and {32, 128, 512} within noise of it, {24, 96, 768} between; profiles/r06/ladder/).
    //    Rounds 3-5: {24, 72, 216, 648} with 4 queue waves per CU -- the bench frame at eight frames in flight 0.561-0.567 ms against 0.593-0.598 for round 2's {24, 96, 768}
    //    at 8 waves per CU (profiles/r03/sched_r03.log, ladder_r03b.log; 4 against 8 queue waves per CU is within noise
    //    at eight frames in flight, 0.562-0.566 against 0.563-0.565 ms, qwaves_r03.log): the queue passes are most of
    //    the frame period (pass_share_r03.log); a finer ladder re-packs the surviving rays into full waves more often,
    //    and fewer queue waves leave the SIMDs to the other frames' first passes; 3 queue waves per CU since the bench
    //    runs sixteen frames in flight (0.478 against 0.484 ms for 4 and 0.489-0.491 for 6, two rounds,
    //    profiles/r03/inflight/);
    //  * `idle` otherwise (one frame at a time, or frames serialised on one stream): {64} without sparse-wave
    //    abandonment at 8 queue waves per CU -- 1.22 ms for the lone bench frame against 1.54 ms for the busy schedule
    //    run alone (profiles/r03/isolated_r03.log, reentry_r03c/isolated.log; {64, 1024}, {64, 512}, {48, 768} and
    //    three-budget ladders 1.31-1.51 ms, fewer rays per wave in a last pass no better): every extra pass lengthens a
    //    lone frame's critical path.
    bool adaptive = true;
    // first queue pass (shadow pass 0, 82 % memory waits): 4 waves per CU with frames in flight -- config 5 at twenty
    // contexts 0.993-1.000 ms per frame against 1.110-1.128 at 32 per CU, 1.029-1.034 at 8 and 0.995-1.000 at 3
    // (profiles/r06/shadows/) -- and 32 alone (the lone shadow frame 2.83 against 3.09-3.27 ms at 4)
    // shadow traces keep {24, 72, 216, 648} with frames in flight: config 5 at twenty contexts 1.007-1.016 ms per frame
    // in the driver's window against 1.029-1.033 with {32, 128, 768} (profiles/r06/ladder/)
    Sched sched_busy = {{32u, 128u, 768u}, 4u, {12u}, 3u, VHX_QORDER_BUSY, VHX_QSORT_BUSY, 4u, {24u, 72u, 216u, 648u}, 5u};
    Sched sched_idle = {{64u}, 2u, {0u}, 8u, VHX_QORDER_IDLE, VHX_QSORT_IDLE, 32u, {64u}, 2u};
    int last_sched = -1;  // the schedule of the last trace: 1 busy, 0 idle, -1 fixed (vhx_get_pass_budgets)
    // the schedule in force (the selected one, or the fixed one)
    uint32_t budgets[VHX_MAX_BUDGETS] = {32u, 128u, 768u};
    uint32_t npass = 4;
    uint32_t rpw[VHX_MAX_BUDGETS + 1] = {64u, 64u, 64u, 64u, 64u, 64u, 64u};  // rays per wave of each pass (tune "rpw=64,16" style override; 0 = adaptive)
    uint32_t tw = 1024;            // adaptive rays per wave: target waves per queue pass (tune "tw")
    uint32_t scan_multi = 8;       // chunk scans of more segments (SCAN_SEG counts) run on one workgroup per segment
    bool p0lists = true;           // pass 0 lists its abandoned rays in the queue order (ListOrder; tune "p0lists")
    bool resume = true;            // abandoned rays continue from saved state (tune "resume=0": re-traced from scratch)
    // queue-state mode (tune "qstate=1"; off by default): where a pass lists its abandoned rays per wave or chunk (the
    // listed pass 0 of the frames-in-flight and batch schedules, every queue pass), it saves their states at their list
    // slots, the compaction moves them into the next queue's order, and the next pass reads a ray's state at its queue
    // position -- coalesced, and in the same load round as the ray's output index instead of after it. Measured slower:
    // the bench frame 0.520-0.522 against 0.504 ms per frame (profiles/r06/qstate/): the compaction's chunk copies
    // gain a dependent 64 B state load per ray on the path between two passes
    bool qstate = false;
    // a tile set (VHX_LAYOUT_TILES) under the frames-in-flight schedule: pass 0 lists its rays (ListOrder::tl; tune
    // "tlists=0" falls back to flags compacted in output-index order)
    bool tile_lists = true;
    // batch pass 0: the frames' blocks interleaved (block b of frame 0, of frame 1, ...) instead of frame-major (tune
    // "finter"): the frames' rays through one screen region run together and share the caches (the XCD placement of
    // those workgroups measured indifferent) -- the headline in the driver's window 0.5115-0.5147 against 0.5200-0.5366 ms per frame (four alternating
    // runs), 100 frames 0.4914 against 0.5041-0.5085, config 4 1.786-1.794 against 1.863-1.879, the moving camera
    // 0.721-0.723 against 0.737-0.740 (profiles/r06/finter/)
    bool frame_interleave = true;
    // passes before save_from keep no state: the rays they abandon are traced again from scratch by pass save_from,
    // which saves (tune "save_from"; 0 = every budgeted pass saves)
    uint32_t save_from = 0;
    uint32_t xcd_group = 16;       // pass-0 XCD-aware block runs (tune "xcdg"; 0 = dispatch order)
    uint32_t qblock = 256;         // threads per workgroup of a queue pass (tune "qblock=64": one wave per workgroup)
    uint32_t queue_blocks = 2048;  // workgroups of a queue pass (CUs x resident workgroups)
    // waves of a queue pass (tune "qwaves"; the schedule's per-CU figure times the CUs). One frame at a time, 8 per CU:
    // round 1's tail pass (148 k rays, 2316 chunks of 64) took 1.55 ms/frame at 2048 waves against 1.62 at 8192 and
    // 1.82 at 1024 (fewer busy waves per CU at the start of the pass, while every chunk still starts at once); with
    // frames in flight 4 per CU (equal within noise there; profiles/r03/qwaves_r03.log)
    uint32_t queue_waves = 1024;
    uint32_t cus = 256;            // compute units of the device (the adaptive schedules' queue waves are per CU)
    uint32_t queue_waves0 = 8192;  // waves of a first queue pass over fresh rays (the schedule's per-CU figure x CUs)
    uint32_t queue_waves0_force = 0;  // tune "qwaves0": a fixed figure in every schedule (0 = the schedule's)
    uint32_t queue_waves_mid = 0;  // waves of a budgeted queue pass after the first (tune "qwavesm"; 0 = queue_waves)
    uint32_t qxcd = 16;            // queue passes: XCD-dealt chunk runs (tune "qxcd" = run length, 0 = one counter)
    bool qxcd_all = false;         // deal every queue pass, not only the last (tune "qxcd_all=1", diagnostics)
    // pass-0 queue of a framebuffer frame (the schedule's, or tune "qorder=[m]N[z|r]"): 0 output-index order; else
    // log2 of the tile size (bits 0-3), bit 4 Morton order of the tiles, bit 5 Morton order of the pixels inside a tile
    // (FlagOrder in vhx_device.hip)
    uint32_t qorder = VHX_QORDER_BUSY;
    uint32_t last_fb_w = 0, last_fb_h = 0;  // the last primary framebuffer frame traced on this context
    // budgeted passes: a wave abandons its rays once fewer than sparse[p] lanes still trace (tune "sparse=8,4,4").
    // Pass 0 at 12 under frames in flight: eight frames 0.645-0.651 ms per bench frame against 0.665-0.670 (8:
    // 0.651-0.661, 16: 0.646-0.657, 24 and 32 slower); the later budgeted passes gained nothing (profiles/r02/sparse*.log)
    uint32_t sparse[VHX_MAX_BUDGETS] = {12u};
    // segment node sort of the queue passes (Sched::qsort): in force for this trace; tune "qsort=N" forces it (-1: not)
    uint32_t qsort = 0;
    int qsort_force = -1;
    uint32_t qsort_passes = 0xFEu;   // bit p: the queue of pass p is sorted (tune "qsortp")
    uint32_t qsort_blocks = 2048u;   // workgroups of a sort launch, striding over the segments (tune "qsortb")
};

#define VHX_HIP(ctx, call)                                                                                         \
    do {                                                                                                           \
        hipError_t e_ = (call);                                                                                    \
        if (e_ != hipSuccess) {                                                                                    \
            (ctx)->err = std::string(#call) + ": " + hipGetErrorString(e_);                                        \
            return VHX_E_HIP;                                                                                      \
        }                                                                                                          \
    } while (0)

// The context's stream: the caller's (vhx_set_stream), else its own, created at first use. A context given a stream
// before its first call never creates one: the device has few hardware queues (GPU_MAX_HW_QUEUES, 4 by default) and
// streams share them round-robin in creation order, so an unused stream per context made frames in flight share
// queues (bench frame, four frames in flight: 0.91 against 0.70 ms per frame).
#define VHX_STREAM(ctx)                                                                                            \
    do {                                                                                                           \
        if (!(ctx)->stream) {                                                                                      \
            if (!(ctx)->own_stream) VHX_HIP(ctx, hipStreamCreateWithFlags(&(ctx)->own_stream, hipStreamNonBlocking)); \
            (ctx)->stream = (ctx)->own_stream;                                                                     \
        }                                                                                                          \
    } while (0)

static inline int fail(vhx_ctx *ctx, int code, const char *msg) {
    if (ctx) ctx->err = msg;
    return code;
}
static inline int fail(vhx_ctx *ctx, int code, const std::string &msg) { return fail(ctx, code, msg.c_str()); }

namespace vhx {
// device buffer of at least `bytes` (contents not kept when it grows)
int ensure(vhx_ctx *c, DevBuf &b, uint64_t bytes);
// element size / count of the VHX_BUF_* raw buffers of a tree
uint64_t elem_size(int id);
uint64_t elem_count(const vhx_tree_desc &d, int id);
// allocates the raw buffers for the counts of *t (t's pointers unused) and records the counts
int alloc_tree(vhx_ctx *c, const vhx_tree_desc *t);
// derives the device-side layout (node headers, brick bitmaps, child records) from the raw buffers, synchronously
int finish_upload(vhx_ctx *c);
// k_untile_planes on `stream` (arguments as vhx_untile_frame, already validated)
int launch_untile(vhx_ctx *c, hipStream_t stream, const void *gathered, uint32_t planes, uint32_t ranks,
                  uint32_t tiles_per_rank, uint32_t T, uint32_t width, uint32_t height, uint32_t *fb_rgba,
                  float *fb_depth);
// tree-write ordering (TreeStore): before a write of the tree on c's stream, wait for every other context's last
// submitted trace; after it, record the write
int write_begin(vhx_ctx *c);
int write_end(vhx_ctx *c);
// before a trace on c's stream: wait for the tree's last write (once per write); after it: record c's use
int trace_begin(vhx_ctx *c);
int trace_end(vhx_ctx *c);
// trace_begin .. trace_end (write_begin .. write_end) as a scope: the end runs on every exit once the begin succeeded,
// so an error return after the first launch still records the trace's use (or the write) for the ordering
// nested = true: a trace issued from inside an open scope of the same context and thread (the depth prepass's inner
// frame) joins the enclosing scope instead of opening a second one -- a second trace_begin would wait for a writer
// queued behind the enclosing trace, which in turn waits for that trace to end (a deadlock)
struct TraceScope {
    vhx_ctx *c;
    int rc;
    bool open;
    explicit TraceScope(vhx_ctx *ctx, bool nested = false)
        : c(ctx), rc(nested ? VHX_OK : trace_begin(ctx)), open(!nested) {}
    int end() {
        if (!open) return VHX_OK;
        open = false;
        return trace_end(c);
    }
    ~TraceScope() {
        if (open) (void)trace_end(c);
    }
    TraceScope(const TraceScope &) = delete;
    TraceScope &operator=(const TraceScope &) = delete;
};
struct WriteScope {
    vhx_ctx *c;
    int rc;
    bool open;
    explicit WriteScope(vhx_ctx *ctx) : c(ctx), rc(write_begin(ctx)), open(true) {}
    int end() {
        if (!open) return VHX_OK;
        open = false;
        return write_end(c);
    }
    ~WriteScope() {
        if (open) (void)write_end(c);
    }
    WriteScope(const WriteScope &) = delete;
    WriteScope &operator=(const WriteScope &) = delete;
};
// the tree counts as 8 u32 (the message of a device-side tree transfer) and back
void pack_counts(const vhx_tree_desc &d, uint32_t counts[8]);
vhx_tree_desc unpack_counts(const uint32_t counts[8]);
// A tree whose raw buffers arrive device-side (ncclBroadcast from rank 0, a peer copy): allocates the raw buffers for
// `counts`, calls fill(id, dst, bytes) for each of the 7 buffers (it enqueues the transfer on c's stream), then
// derives the device layout (synchronises). Ordered against the traces of every context of the tree.
int receive_tree(vhx_ctx *c, const vhx_tree_desc &counts,
                 int (*fill)(void *arg, void *const dst[7], const uint64_t bytes[7]), void *arg);
// the scheduling settings (pass budgets, rays per wave, queue shapes, sparse thresholds, depth prepass) of src
void copy_sched(vhx_ctx *dst, const vhx_ctx *src);
}  // namespace vhx

