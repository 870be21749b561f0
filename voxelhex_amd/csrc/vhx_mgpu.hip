// libvhx multi-GPU: the screen-tile split of a frame over the GPUs of one node, with RCCL over xGMI (SURVEY.md 8e,
// include/vhx.h vhx_mgpu_*).
//
// Tiles are dealt round-robin over V = R + N - 1 slots: rank 0 owns slots 0..R-1, rank r >= 1 slot R + r - 1 (R = 1:
// rank r traces tiles r, r+N, ...). Per frame and rank: trace the rank's slots, each into a contiguous [RGBA8 plane |
// f32 depth plane] part on the context's stream -- rank 0 straight into its gather buffer, the others into a send
// buffer; one group of point-to-point sends / receives brings the other ranks' parts to rank 0 (xGMI: each part crosses
// one link); rank 0 scatters the slot-major gathered buffer into its framebuffers (k_untile_planes). The transfers and
// the untile run on a communication stream, so frame k's transfer overlaps the next frames' traces; events order the
// reuse of a buffer after its transfer. R > 1 moves work to rank 0, whose own parts cross no link: when the transfers
// into rank 0 take longer than a slot's trace, the frame is link-bound and a larger share on rank 0 shortens it
// (vhx_mgpu_balance measures both and picks R). The tree is replicated on every GPU (3 GB against
// 288 GB of HBM): rank 0 uploads it from the host, ncclBroadcast copies the device buffers to the other ranks.
//
// RCCL is resolved at run time (dlopen + dlsym) so that the library loads on a host without it and binds to the RCCL
// instance already in the process when there is one (torch's librccl.so.1 has the same soname).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>  // types only: every RCCL function is called through the pointers below

#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "ctx.hpp"

using namespace vhx;

namespace {

struct Rccl {
    bool ok = false;
    std::string err;
    decltype(&ncclGetUniqueId) GetUniqueId = nullptr;
    decltype(&ncclCommInitRank) CommInitRank = nullptr;
    decltype(&ncclCommDestroy) CommDestroy = nullptr;
    decltype(&ncclCommCount) CommCount = nullptr;
    decltype(&ncclCommUserRank) CommUserRank = nullptr;
    decltype(&ncclBroadcast) Broadcast = nullptr;
    decltype(&ncclSend) Send = nullptr;
    decltype(&ncclRecv) Recv = nullptr;
    decltype(&ncclGroupStart) GroupStart = nullptr;
    decltype(&ncclGroupEnd) GroupEnd = nullptr;
    decltype(&ncclGetErrorString) GetErrorString = nullptr;
};

const Rccl &rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        const char *env = getenv("VHX_RCCL_LIB");
        const char *names[] = {env, "librccl.so.1", "/opt/rocm/lib/librccl.so.1", "librccl.so"};
        void *h = nullptr;
        for (const char *n : names)
            if (n && (h = dlopen(n, RTLD_NOW | RTLD_LOCAL))) break;
        if (!h) {
            r.err = "RCCL not found (dlopen librccl.so.1; set VHX_RCCL_LIB)";
            return;
        }
        bool all = true;
        auto sym = [&](auto &fp, const char *name) {
            fp = reinterpret_cast<std::remove_reference_t<decltype(fp)>>(dlsym(h, name));
            all = all && fp != nullptr;
        };
        sym(r.GetUniqueId, "ncclGetUniqueId");
        sym(r.CommInitRank, "ncclCommInitRank");
        sym(r.CommDestroy, "ncclCommDestroy");
        sym(r.CommCount, "ncclCommCount");
        sym(r.CommUserRank, "ncclCommUserRank");
        sym(r.Broadcast, "ncclBroadcast");
        sym(r.Send, "ncclSend");
        sym(r.Recv, "ncclRecv");
        sym(r.GroupStart, "ncclGroupStart");
        sym(r.GroupEnd, "ncclGroupEnd");
        sym(r.GetErrorString, "ncclGetErrorString");
        if (!all) {
            r.err = "the loaded RCCL lacks a symbol libvhx needs";
            return;
        }
        r.ok = true;
    });
    return r;
}

}  // namespace

struct vhx_mgpu {
    vhx_ctx *ctx = nullptr;
    ncclComm_t comm = nullptr;
    bool own_comm = false;
    int nranks = 1, rank = 0;
    uint32_t T = 64;
    uint32_t R = 1;  // slots of rank 0 (the others own one each)
    // planes of a slot's part: 2 = [RGBA8 | f32 depth], 1 = RGBA8 only (the reference's display output is the rgba8unorm
    // view texture, src/raytracing/bevy/view.rs:269-289; depth is optional), equal on every rank (vhx_mgpu_set_planes)
    uint32_t planes = 2;
    bool overlap = true;
    bool timing = false;  // vhx_mgpu_balance: time rank 0's trace and the transfers of each frame
    hipEvent_t tev[4] = {};  // trace start / end (tracing stream), transfer start / end (communication stream)
    hipStream_t cstream = nullptr;     // gather + untile
    // frames in flight: frame k is traced by context k % F (ctx, then the shared contexts extra[0..F-2], each on its
    // own stream) into the tile buffers of slot k % S, S = max(2, F)
    uint32_t F = 1, S = 2;
    vhx_ctx *extra[VHX_MGPU_MAX_INFLIGHT - 1] = {};
    hipEvent_t ready[VHX_MGPU_MAX_INFLIGHT] = {}, free_[VHX_MGPU_MAX_INFLIGHT] = {};  // slot traced / slot gathered
    bool used[VHX_MGPU_MAX_INFLIGHT] = {};
    DevBuf send[VHX_MGPU_MAX_INFLIGHT], gathered[VHX_MGPU_MAX_INFLIGHT];
    vhx_ctx *last = nullptr;  // the context of the last frame submitted
    DevBuf hdr;  // tree counts during the broadcast
    uint64_t k = 0;   // frames submitted
    uint64_t kb = 0;  // batches submitted (vhx_mgpu_render_batch: batch b is traced by context b % F)
};

#define VHX_NCCL(m, call)                                                                                          \
    do {                                                                                                           \
        ncclResult_t r_ = (call);                                                                                  \
        if (r_ != ncclSuccess) {                                                                                   \
            (m)->ctx->err = std::string(#call) + ": " + rccl().GetErrorString(r_);                                 \
            return VHX_E_RCCL;                                                                                     \
        }                                                                                                          \
    } while (0)

static int mgpu_init(vhx_mgpu *m) {
    vhx_ctx *c = m->ctx;
    VHX_HIP(c, hipSetDevice(c->device));
    VHX_HIP(c, hipStreamCreateWithFlags(&m->cstream, hipStreamNonBlocking));
    for (int s = 0; s < VHX_MGPU_MAX_INFLIGHT; ++s) {
        VHX_HIP(c, hipEventCreateWithFlags(&m->ready[s], hipEventDisableTiming));
        VHX_HIP(c, hipEventCreateWithFlags(&m->free_[s], hipEventDisableTiming));
    }
    for (hipEvent_t &e : m->tev) VHX_HIP(c, hipEventCreate(&e));
    return VHX_OK;
}

// The tile plan (vhx_mgpu_tile_plan, exported for the host tests): V = R + N - 1 slots, slot s traces tiles s, s + V, ...
// (per = tiles per slot; the last slots may hold fewer, their parts are padded); rank 0 owns slots 0..R-1, rank r >= 1
// slot R + r - 1
static vhx_tile_plan plan_of(uint32_t N, uint32_t R, uint32_t T, uint32_t W, uint32_t H, uint32_t rank) {
    vhx_tile_plan p{};
    p.tiles_x = (W + T - 1) / T;
    p.tiles_y = (H + T - 1) / T;
    p.tiles = p.tiles_x * p.tiles_y;
    p.slots = R + N - 1u;
    p.tiles_per_slot = (p.tiles + p.slots - 1) / p.slots;
    p.first_slot = rank == 0 ? 0u : R + rank - 1u;
    p.slot_count = rank == 0 ? R : 1u;
    return p;
}
static uint32_t slots_of(const vhx_mgpu *m) { return m->R + (uint32_t)m->nranks - 1u; }
static void tiles_of(const vhx_mgpu *m, uint32_t W, uint32_t H, uint32_t &ntiles, uint32_t &per_slot) {
    const vhx_tile_plan p = plan_of((uint32_t)m->nranks, m->R, m->T, W, H, 0);
    ntiles = p.tiles;
    per_slot = p.tiles_per_slot;
}
// the slots of a rank: first and count
static void rank_slots(const vhx_mgpu *m, int rank, uint32_t &first, uint32_t &count) {
    const vhx_tile_plan p = plan_of((uint32_t)m->nranks, m->R, m->T, 1, 1, (uint32_t)rank);
    first = p.first_slot;
    count = p.slot_count;
}

// a failed RCCL call inside a group still closes the group, so this rank's later collectives are not swallowed by it
#define VHX_NCCL_GROUP(m, call)                                                                                    \
    do {                                                                                                           \
        ncclResult_t r_ = (call);                                                                                  \
        if (r_ != ncclSuccess) {                                                                                   \
            rccl().GroupEnd();                                                                                     \
            (m)->ctx->err = std::string(#call) + ": " + rccl().GetErrorString(r_);                                 \
            return VHX_E_RCCL;                                                                                     \
        }                                                                                                          \
    } while (0)

extern "C" {

int vhx_mgpu_unique_id(uint8_t id[VHX_MGPU_ID_BYTES]) {
    if (!id) return VHX_E_INVALID_ARG;
    const Rccl &r = rccl();
    if (!r.ok) return VHX_E_RCCL;
    ncclUniqueId u;
    if (r.GetUniqueId(&u) != ncclSuccess) return VHX_E_RCCL;
    static_assert(sizeof(u) == VHX_MGPU_ID_BYTES, "ncclUniqueId size");
    std::memcpy(id, &u, sizeof(u));
    return VHX_OK;
}

int vhx_mgpu_create(vhx_ctx *c, const uint8_t id[VHX_MGPU_ID_BYTES], int nranks, int rank, uint32_t T,
                    vhx_mgpu **out) {
    if (!c || !id || !out || nranks < 1 || rank < 0 || rank >= nranks || T == 0 || T > 4096)
        return fail(c, VHX_E_INVALID_ARG, "vhx_mgpu_create: bad arguments");
    *out = nullptr;
    const Rccl &r = rccl();
    if (!r.ok) return fail(c, VHX_E_RCCL, r.err.c_str());
    vhx_mgpu *m = new vhx_mgpu();
    m->ctx = c;
    m->nranks = nranks;
    m->rank = rank;
    m->T = T;
    int rc = mgpu_init(m);
    if (!rc) {
        ncclUniqueId u;
        std::memcpy(&u, id, sizeof(u));
        const ncclResult_t e = r.CommInitRank(&m->comm, nranks, u, rank);
        if (e != ncclSuccess) {
            c->err = std::string("ncclCommInitRank: ") + r.GetErrorString(e);
            rc = VHX_E_RCCL;
        } else {
            m->own_comm = true;
        }
    }
    if (rc) {
        vhx_mgpu_destroy(m);
        return rc;
    }
    *out = m;
    return VHX_OK;
}

int vhx_mgpu_create_from_comm(vhx_ctx *c, void *comm, uint32_t T, vhx_mgpu **out) {
    if (!c || !comm || !out || T == 0 || T > 4096) return fail(c, VHX_E_INVALID_ARG, "vhx_mgpu_create_from_comm");
    *out = nullptr;
    const Rccl &r = rccl();
    if (!r.ok) return fail(c, VHX_E_RCCL, r.err.c_str());
    vhx_mgpu *m = new vhx_mgpu();
    m->ctx = c;
    m->comm = (ncclComm_t)comm;
    m->T = T;
    int rc = mgpu_init(m);
    if (!rc && (r.CommCount(m->comm, &m->nranks) != ncclSuccess || r.CommUserRank(m->comm, &m->rank) != ncclSuccess))
        rc = fail(c, VHX_E_RCCL, "vhx_mgpu_create_from_comm: not a valid communicator");
    if (rc) {
        vhx_mgpu_destroy(m);
        return rc;
    }
    *out = m;
    return VHX_OK;
}

void vhx_mgpu_destroy(vhx_mgpu *m) {
    if (!m) return;
    vhx_ctx *c = m->ctx;
    (void)hipSetDevice(c->device);
    if (m->cstream) (void)hipStreamSynchronize(m->cstream);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    for (vhx_ctx *x : m->extra) vhx_destroy(x);
    if (m->comm && m->own_comm) rccl().CommDestroy(m->comm);
    for (int s = 0; s < VHX_MGPU_MAX_INFLIGHT; ++s)
        for (DevBuf *b : {&m->send[s], &m->gathered[s]})
            if (b->ptr) (void)hipFree(b->ptr);
    if (m->hdr.ptr) (void)hipFree(m->hdr.ptr);
    for (int s = 0; s < VHX_MGPU_MAX_INFLIGHT; ++s) {
        if (m->ready[s]) (void)hipEventDestroy(m->ready[s]);
        if (m->free_[s]) (void)hipEventDestroy(m->free_[s]);
    }
    for (hipEvent_t e : m->tev)
        if (e) (void)hipEventDestroy(e);
    if (m->cstream) (void)hipStreamDestroy(m->cstream);
    delete m;
}

int vhx_mgpu_set_overlap(vhx_mgpu *m, int on) {
    if (!m) return VHX_E_INVALID_ARG;
    m->overlap = on != 0;
    return VHX_OK;
}

int vhx_mgpu_set_frames_in_flight(vhx_mgpu *m, uint32_t frames) {
    if (!m) return VHX_E_INVALID_ARG;
    vhx_ctx *c = m->ctx;
    if (frames < 1 || frames > VHX_MGPU_MAX_INFLIGHT)
        return fail(c, VHX_E_INVALID_ARG, "vhx_mgpu_set_frames_in_flight: 1..VHX_MGPU_MAX_INFLIGHT");
    int rc = vhx_mgpu_sync(m, nullptr);  // no frame may be in flight while the slots change
    if (rc) return rc;
    for (uint32_t i = 0; i + 1 < VHX_MGPU_MAX_INFLIGHT; ++i) {
        const bool want = i + 1 < frames;
        if (want && !m->extra[i] && (rc = vhx_create_shared(c, &m->extra[i]))) return fail(c, rc, "vhx_create_shared");
        if (!want && m->extra[i]) {
            vhx_destroy(m->extra[i]);
            m->extra[i] = nullptr;
        }
    }
    m->F = frames;
    m->S = frames < 2 ? 2u : frames;
    m->k = 0;
    m->kb = 0;
    for (bool &u : m->used) u = false;
    return VHX_OK;
}

int vhx_mgpu_info(const vhx_mgpu *m, uint32_t W, uint32_t H, int *nranks, int *rank, uint64_t *rays) {
    if (!m) return VHX_E_INVALID_ARG;
    if (nranks) *nranks = m->nranks;
    if (rank) *rank = m->rank;
    if (rays) {
        uint32_t ntiles, per, first, count;
        tiles_of(m, W, H, ntiles, per);
        rank_slots(m, m->rank, first, count);
        const uint32_t tx = (W + m->T - 1) / m->T;
        uint64_t n = 0;
        for (uint32_t s = first; s < first + count; ++s)
            for (uint32_t t = s; t < ntiles; t += slots_of(m)) {
                const uint32_t x0 = (t % tx) * m->T, y0 = (t / tx) * m->T;
                n += (uint64_t)std::min(m->T, W - x0) * std::min(m->T, H - y0);
            }
        *rays = n;
    }
    return VHX_OK;
}

// The raw tree buffers, device to device over xGMI from rank 0 (the root sends, the others receive in place), in
// chunks of at most 1 GiB per call, one RCCL group: the fill step of receive_tree on ranks >= 1, and the send on rank 0
static int broadcast_raw(void *arg, void *const dst[7], const uint64_t bytes[7]) {
    vhx_mgpu *m = (vhx_mgpu *)arg;
    vhx_ctx *c = m->ctx;
    const Rccl &r = rccl();
    VHX_NCCL(m, r.GroupStart());
    for (int id = 0; id < 7; ++id)
        for (uint64_t off = 0; off < bytes[id]; off += 1ull << 30) {
            const uint64_t n = std::min<uint64_t>(1ull << 30, bytes[id] - off);
            char *p = (char *)dst[id] + off;
            VHX_NCCL_GROUP(m, r.Broadcast(p, p, n, ncclUint8, 0, m->comm, c->stream));
        }
    VHX_NCCL(m, r.GroupEnd());
    return VHX_OK;
}

int vhx_mgpu_broadcast_tree(vhx_mgpu *m, const vhx_tree_desc *t) {
    if (!m) return VHX_E_INVALID_ARG;
    vhx_ctx *c = m->ctx;
    if ((m->rank == 0) != (t != nullptr)) return fail(c, VHX_E_INVALID_ARG, "vhx_mgpu_broadcast_tree: rank 0 passes the tree, the others NULL");
    const Rccl &r = rccl();
    VHX_HIP(c, hipSetDevice(c->device));
    if (c->shared) return fail(c, VHX_E_STATE, "vhx_mgpu_broadcast_tree on a shared context");
    // no frame of this renderer may still be in flight on the buffers about to be replaced (its gathers included)
    int rc = vhx_mgpu_sync(m, nullptr);
    if (rc) return rc;
    VHX_STREAM(c);
    if (m->rank == 0) {
        rc = vhx_upload_tree(c, t);  // host -> HBM of rank 0, derived layout included
        if (rc) return rc;
    }
    // the counts first (8 u32), so the other ranks can size their buffers
    if ((rc = ensure(c, m->hdr, 64))) return rc;
    uint32_t counts[8] = {0};
    if (m->rank == 0) {
        pack_counts(c->tree->desc, counts);
        VHX_HIP(c, hipMemcpyAsync(m->hdr.ptr, counts, sizeof(counts), hipMemcpyHostToDevice, c->stream));
    }
    VHX_NCCL(m, r.Broadcast(m->hdr.ptr, m->hdr.ptr, 8, ncclUint32, 0, m->comm, c->stream));
    VHX_HIP(c, hipMemcpyAsync(counts, m->hdr.ptr, sizeof(counts), hipMemcpyDeviceToHost, c->stream));
    VHX_HIP(c, hipStreamSynchronize(c->stream));
    if (m->rank != 0) return receive_tree(c, unpack_counts(counts), broadcast_raw, m);  // alloc, receive, derive
    void *src[7];
    uint64_t bytes[7];
    for (int id = 0; id < 7; ++id) {
        src[id] = c->tree->raw[id].ptr;
        bytes[id] = elem_count(c->tree->desc, id) * elem_size(id);
    }
    if ((rc = broadcast_raw(m, src, bytes))) return rc;
    VHX_HIP(c, hipStreamSynchronize(c->stream));
    return VHX_OK;
}

int vhx_mgpu_render(vhx_mgpu *m, const vhx_camera *cam, uint32_t *fb_rgba, float *fb_depth) {
    if (!m || !cam) return VHX_E_INVALID_ARG;
    vhx_ctx *c = m->ctx;
    if (m->rank == 0 && !fb_rgba && !fb_depth) return fail(c, VHX_E_INVALID_ARG, "vhx_mgpu_render: rank 0 needs a framebuffer");
    if (m->rank == 0 && m->planes == 1 && (fb_depth || !fb_rgba))
        return fail(c, VHX_E_INVALID_ARG, "vhx_mgpu_render: one plane (vhx_mgpu_set_planes) carries RGBA only: fb_rgba "
                                          "and no fb_depth");
    if (!c->tree->uploaded) return fail(c, VHX_E_STATE, "vhx_mgpu_render before the tree is uploaded");
    if (cam->width == 0 || cam->height == 0) return fail(c, VHX_E_INVALID_ARG, "vhx_mgpu_render: empty frame");
    const Rccl &r = rccl();
    VHX_HIP(c, hipSetDevice(c->device));
    uint32_t ntiles, per, first, count;
    tiles_of(m, cam->width, cam->height, ntiles, per);
    rank_slots(m, m->rank, first, count);
    const uint32_t V = slots_of(m);
    const uint64_t n_out = (uint64_t)per * m->T * m->T;  // words per plane of one slot's part
    const uint32_t P = m->planes;
    const uint32_t slot = (uint32_t)(m->k % m->S);
    vhx_ctx *tc = m->k % m->F == 0 ? c : m->extra[m->k % m->F - 1];  // the context tracing this frame
    if (tc != c) copy_sched(tc, c);  // the caller's settings (vhx_set_pass_budgets, ...) go to the owner context
    VHX_STREAM(tc);
    // a slot's buffers are rewritten only after the transfer that read them (stream order on the tracing stream)
    if (m->used[slot]) VHX_HIP(c, hipStreamWaitEvent(tc->stream, m->free_[slot], 0));
    DevBuf &buf = m->rank == 0 ? m->gathered[slot] : m->send[slot];
    const uint64_t need = n_out * 4 * P * (m->rank == 0 ? (uint64_t)V : 1u);
    if (buf.bytes < need) {
        int rc = vhx_mgpu_sync(m, nullptr);  // (re)allocation: no frame may still use the old buffers
        if (rc) return rc;
        if ((rc = ensure(c, buf, need))) return rc;
    }
    uint32_t *parts = (uint32_t *)buf.ptr;  // this rank's parts first (rank 0: the whole slot-major buffer)
    if (m->timing) VHX_HIP(c, hipEventRecord(m->tev[0], tc->stream));
    for (uint32_t s = first; s < first + count && s < ntiles; ++s) {
        vhx_hits h{};
        h.rgba = parts + P * n_out * (s - first);
        h.depth = P == 2 ? (float *)(h.rgba + n_out) : nullptr;
        const int rc = vhx_trace_primary(tc, cam, m->T, s, V, VHX_LAYOUT_TILES, &h, 1);
        if (rc) return tc == c ? rc : fail(c, rc, tc->err.c_str());
    }
    if (m->timing) VHX_HIP(c, hipEventRecord(m->tev[1], tc->stream));
    m->last = tc;
    VHX_HIP(c, hipEventRecord(m->ready[slot], tc->stream));
    VHX_HIP(c, hipStreamWaitEvent(m->cstream, m->ready[slot], 0));
    if (m->timing) VHX_HIP(c, hipEventRecord(m->tev[2], m->cstream));
    if (m->nranks > 1) {
        // every other rank's part to its place in rank 0's slot-major buffer (same counts on every rank: V and per
        // follow from the frame, the tile size and R, which vhx_mgpu_set_root_slots / _balance keep equal on all ranks)
        VHX_NCCL(m, r.GroupStart());
        if (m->rank == 0) {
            for (int q = 1; q < m->nranks; ++q) {
                uint32_t qf, qc;
                rank_slots(m, q, qf, qc);
                VHX_NCCL_GROUP(m, r.Recv(parts + P * n_out * qf, P * n_out, ncclUint32, q, m->comm, m->cstream));
            }
        } else {
            VHX_NCCL_GROUP(m, r.Send(parts, P * n_out, ncclUint32, 0, m->comm, m->cstream));
        }
        VHX_NCCL(m, r.GroupEnd());
    }
    if (m->timing) VHX_HIP(c, hipEventRecord(m->tev[3], m->cstream));
    if (m->rank == 0) {
        const int rc = launch_untile(c, m->cstream, parts, P, V, per, m->T, cam->width, cam->height, fb_rgba, fb_depth);
        if (rc) return rc;
    }
    VHX_HIP(c, hipEventRecord(m->free_[slot], m->cstream));
    m->used[slot] = true;
    ++m->k;
    if (!m->overlap) VHX_HIP(c, hipStreamWaitEvent(tc->stream, m->free_[slot], 0));
    return VHX_OK;
}

// K frames as one batch (vhx_mgpu_render_batch): every frame's slot parts traced by ONE vhx_trace_tiles_batch (K x the
// rank's slots entries) on the batch's context, then the K frames' transfers in one RCCL group on the communication
// stream and rank 0's K untiles. Frame k of the batch uses ring slot (frames submitted + k) % VHX_MGPU_MAX_INFLIGHT;
// a slot is rewritten only after the transfer that read it (events, as vhx_mgpu_render).
int vhx_mgpu_render_batch(vhx_mgpu *m, const vhx_camera *cams, uint32_t K, uint32_t *const *fb_rgba,
                          float *const *fb_depth) {
    if (!m || !cams || K == 0 || K > VHX_MGPU_MAX_INFLIGHT) return VHX_E_INVALID_ARG;
    vhx_ctx *c = m->ctx;
    const uint32_t W = cams[0].width, H = cams[0].height;
    for (uint32_t k = 0; k < K; ++k)
        if (cams[k].width != W || cams[k].height != H || W == 0 || H == 0)
            return fail(c, VHX_E_INVALID_ARG, "vhx_mgpu_render_batch: every frame needs the same non-empty width x height");
    if (m->rank == 0) {
        if (!fb_rgba) return fail(c, VHX_E_INVALID_ARG, "vhx_mgpu_render_batch: rank 0 needs framebuffers");
        for (uint32_t k = 0; k < K; ++k)
            if (!fb_rgba[k] || (m->planes == 1 && fb_depth && fb_depth[k]))
                return fail(c, VHX_E_INVALID_ARG, "vhx_mgpu_render_batch: rank 0 needs an RGBA framebuffer per frame (and "
                                                  "no depth with one plane)");
    }
    if (!c->tree->uploaded) return fail(c, VHX_E_STATE, "vhx_mgpu_render_batch before the tree is uploaded");
    const Rccl &r = rccl();
    VHX_HIP(c, hipSetDevice(c->device));
    uint32_t ntiles, per, first, count;
    tiles_of(m, W, H, ntiles, per);
    rank_slots(m, m->rank, first, count);
    const uint32_t V = slots_of(m);
    const uint64_t n_out = (uint64_t)per * m->T * m->T;
    const uint32_t P = m->planes;
    const uint32_t NS = VHX_MGPU_MAX_INFLIGHT;
    vhx_ctx *tc = m->kb % m->F == 0 ? c : m->extra[m->kb % m->F - 1];  // the context tracing this batch
    if (tc != c) copy_sched(tc, c);
    VHX_STREAM(tc);
    std::vector<uint32_t> slots(K);
    std::vector<vhx_camera> bc;
    std::vector<uint32_t> bstart;
    std::vector<vhx_hits> bh;
    for (uint32_t k = 0; k < K; ++k) {
        const uint32_t slot = (uint32_t)((m->k + k) % NS);
        slots[k] = slot;
        if (m->used[slot]) VHX_HIP(c, hipStreamWaitEvent(tc->stream, m->free_[slot], 0));
        DevBuf &buf = m->rank == 0 ? m->gathered[slot] : m->send[slot];
        const uint64_t need = n_out * 4 * P * (m->rank == 0 ? (uint64_t)V : 1u);
        if (buf.bytes < need) {
            int rc = vhx_mgpu_sync(m, nullptr);  // (re)allocation: no frame may still use the old buffers
            if (rc) return rc;
            if ((rc = ensure(c, buf, need))) return rc;
        }
        uint32_t *parts = (uint32_t *)buf.ptr;
        for (uint32_t s = first; s < first + count && s < ntiles; ++s) {
            vhx_hits h{};
            h.rgba = parts + P * n_out * (s - first);
            h.depth = P == 2 ? (float *)(h.rgba + n_out) : nullptr;
            bc.push_back(cams[k]);
            bstart.push_back(s);
            bh.push_back(h);
        }
    }
    if (!bc.empty()) {
        const int rc = vhx_trace_tiles_batch(tc, bc.data(), (uint32_t)bc.size(), m->T, bstart.data(), V, bh.data());
        if (rc) return tc == c ? rc : fail(c, rc, tc->err.c_str());
    }
    m->last = tc;
    VHX_HIP(c, hipEventRecord(m->ready[slots[0]], tc->stream));
    VHX_HIP(c, hipStreamWaitEvent(m->cstream, m->ready[slots[0]], 0));
    if (m->nranks > 1) {
        VHX_NCCL(m, r.GroupStart());
        for (uint32_t k = 0; k < K; ++k) {
            uint32_t *parts = (uint32_t *)(m->rank == 0 ? m->gathered[slots[k]] : m->send[slots[k]]).ptr;
            if (m->rank == 0) {
                for (int q = 1; q < m->nranks; ++q) {
                    uint32_t qf, qc;
                    rank_slots(m, q, qf, qc);
                    VHX_NCCL_GROUP(m, r.Recv(parts + P * n_out * qf, P * n_out, ncclUint32, q, m->comm, m->cstream));
                }
            } else {
                VHX_NCCL_GROUP(m, r.Send(parts, P * n_out, ncclUint32, 0, m->comm, m->cstream));
            }
        }
        VHX_NCCL(m, r.GroupEnd());
    }
    for (uint32_t k = 0; k < K; ++k) {
        if (m->rank == 0) {
            const uint32_t *parts = (const uint32_t *)m->gathered[slots[k]].ptr;
            const int rc = launch_untile(c, m->cstream, parts, P, V, per, m->T, W, H, fb_rgba[k],
                                         fb_depth ? fb_depth[k] : nullptr);
            if (rc) return rc;
        }
        VHX_HIP(c, hipEventRecord(m->free_[slots[k]], m->cstream));
        m->used[slots[k]] = true;
    }
    m->k += K;
    ++m->kb;
    if (!m->overlap) VHX_HIP(c, hipStreamWaitEvent(tc->stream, m->free_[slots[K - 1]], 0));
    return VHX_OK;
}

// Collective agreement on one word: every rank sends `value` to rank 0 (point to point), rank 0 broadcasts it back if
// all ranks sent the same, else VHX_MGPU_DISAGREE, so every rank sees the same outcome.
#define VHX_MGPU_DISAGREE 0xFFFFFFFFu
static int agree_u32(vhx_mgpu *m, uint32_t value, uint32_t &agreed) {
    agreed = value;
    if (m->nranks < 2) return VHX_OK;
    vhx_ctx *c = m->ctx;
    int rc = ensure(c, m->hdr, 64 + 4u * (uint32_t)m->nranks);
    if (rc) return rc;
    VHX_STREAM(c);
    uint32_t *w = (uint32_t *)m->hdr.ptr + 16;
    const Rccl &r = rccl();
    VHX_HIP(c, hipMemcpyAsync(w + m->rank, &value, 4, hipMemcpyHostToDevice, c->stream));
    VHX_NCCL(m, r.GroupStart());
    if (m->rank == 0) {
        for (int q = 1; q < m->nranks; ++q) VHX_NCCL_GROUP(m, r.Recv(w + q, 1, ncclUint32, q, m->comm, c->stream));
    } else {
        VHX_NCCL_GROUP(m, r.Send(w + m->rank, 1, ncclUint32, 0, m->comm, c->stream));
    }
    VHX_NCCL(m, r.GroupEnd());
    uint32_t out = value;
    if (m->rank == 0) {
        std::vector<uint32_t> all((size_t)m->nranks, 0u);
        VHX_HIP(c, hipMemcpyAsync(all.data(), w, 4u * (uint32_t)m->nranks, hipMemcpyDeviceToHost, c->stream));
        VHX_HIP(c, hipStreamSynchronize(c->stream));
        for (int q = 1; q < m->nranks; ++q)
            if (all[(size_t)q] != value) out = VHX_MGPU_DISAGREE;
        VHX_HIP(c, hipMemcpyAsync(m->hdr.ptr, &out, 4, hipMemcpyHostToDevice, c->stream));
    }
    VHX_NCCL(m, r.Broadcast(m->hdr.ptr, m->hdr.ptr, 1, ncclUint32, 0, m->comm, c->stream));
    VHX_HIP(c, hipMemcpyAsync(&out, m->hdr.ptr, 4, hipMemcpyDeviceToHost, c->stream));
    VHX_HIP(c, hipStreamSynchronize(c->stream));
    agreed = out;
    return VHX_OK;
}

int vhx_mgpu_set_planes(vhx_mgpu *m, uint32_t planes) {
    if (!m) return VHX_E_INVALID_ARG;
    // an out-of-range value still joins the agreement (as a disagreement), so that no rank is left waiting in it
    const bool ok = planes >= 1 && planes <= 2;
    int rc = vhx_mgpu_sync(m, nullptr);  // no frame may be in flight while the part layout changes
    if (rc) return rc;
    uint32_t agreed = 0;
    if ((rc = agree_u32(m, ok ? planes : VHX_MGPU_DISAGREE, agreed))) return rc;
    if (!ok) return fail(m->ctx, VHX_E_INVALID_ARG, "vhx_mgpu_set_planes: 1 (RGBA) or 2 (RGBA + depth)");
    if (agreed != planes)
        return fail(m->ctx, VHX_E_INVALID_ARG, "vhx_mgpu_set_planes: the ranks passed different plane counts");
    m->planes = planes;
    return VHX_OK;
}

int vhx_mgpu_frame_bytes(const vhx_mgpu *m, uint32_t W, uint32_t H, uint64_t *into_root) {
    if (!m || !into_root || W == 0 || H == 0) return VHX_E_INVALID_ARG;
    uint32_t ntiles, per;
    tiles_of(m, W, H, ntiles, per);
    // every rank >= 1 sends its one slot's part: planes x tiles per slot x T^2 words
    *into_root = (uint64_t)(m->nranks - 1) * m->planes * per * m->T * m->T * 4u;
    return VHX_OK;
}

int vhx_mgpu_set_root_slots(vhx_mgpu *m, uint32_t slots) {
    if (!m) return VHX_E_INVALID_ARG;
    if (slots < 1 || slots > VHX_MGPU_MAX_ROOT_SLOTS)
        return fail(m->ctx, VHX_E_INVALID_ARG, "vhx_mgpu_set_root_slots: 1..VHX_MGPU_MAX_ROOT_SLOTS");
    const int rc = vhx_mgpu_sync(m, nullptr);  // no frame may be in flight while the split changes
    if (rc) return rc;
    m->R = slots;
    return VHX_OK;
}

// Renders frames + 1 frames of cam one at a time (no overlap) at the current split with the trace / transfer events on,
// and returns this rank's medians of the last `frames` (device ms). Restores the overlap mode and frees its buffers on
// every exit. Collective (every rank renders the same frames).
static int measure_frames(vhx_mgpu *m, const vhx_camera *cam, uint32_t frames, float &trace_ms, float &xfer_ms) {
    vhx_ctx *c = m->ctx;
    const bool overlap = m->overlap;
    m->overlap = false;
    m->timing = true;
    DevBuf fb, fbd;
    int rc = VHX_OK;
    if (m->rank == 0) {
        rc = ensure(c, fb, (uint64_t)cam->width * cam->height * 4);
        if (!rc && m->planes == 2) rc = ensure(c, fbd, (uint64_t)cam->width * cam->height * 4);
    }
    std::vector<float> tr, tx;
    for (uint32_t i = 0; i < frames + 1 && !rc; ++i) {
        rc = vhx_mgpu_render(m, cam, (uint32_t *)fb.ptr, (float *)fbd.ptr);
        if (!rc) rc = vhx_mgpu_sync(m, nullptr);
        float a = 0, b = 0;
        if (!rc && i > 0 && hipEventElapsedTime(&a, m->tev[0], m->tev[1]) == hipSuccess &&
            hipEventElapsedTime(&b, m->tev[2], m->tev[3]) == hipSuccess) {
            tr.push_back(a);
            tx.push_back(b);
        }
    }
    m->timing = false;
    m->overlap = overlap;
    if (fb.ptr) (void)hipFree(fb.ptr);
    if (fbd.ptr) (void)hipFree(fbd.ptr);
    trace_ms = xfer_ms = 0.0f;
    if (!rc && !tr.empty()) {
        std::sort(tr.begin(), tr.end());
        std::sort(tx.begin(), tx.end());
        trace_ms = tr[tr.size() / 2];
        xfer_ms = tx[tx.size() / 2];
    }
    return rc;
}

int vhx_mgpu_measure(vhx_mgpu *m, const vhx_camera *cam, uint32_t frames, float *trace_ms, float *transfer_ms) {
    if (!m || !cam || frames == 0) return VHX_E_INVALID_ARG;
    if (!m->ctx->tree->uploaded) return fail(m->ctx, VHX_E_STATE, "vhx_mgpu_measure before the tree is uploaded");
    float a = 0, g = 0;
    const int rc = measure_frames(m, cam, frames, a, g);
    if (rc) return rc;
    if (trace_ms) *trace_ms = a;
    if (transfer_ms) *transfer_ms = g;
    return VHX_OK;
}

int vhx_mgpu_tile_plan(uint32_t nranks, uint32_t root_slots, uint32_t T, uint32_t W, uint32_t H, uint32_t rank,
                       vhx_tile_plan *plan) {
    if (!plan || nranks < 1 || rank >= nranks || root_slots < 1 || root_slots > VHX_MGPU_MAX_ROOT_SLOTS || T == 0 ||
        T > 4096 || W == 0 || H == 0)
        return VHX_E_INVALID_ARG;
    const uint64_t tiles = (uint64_t)((W + T - 1) / T) * ((H + T - 1) / T);
    if (tiles > 0xFFFFFFFFull) return VHX_E_INVALID_ARG;
    *plan = plan_of(nranks, root_slots, T, W, H, rank);
    return VHX_OK;
}

int vhx_mgpu_balance(vhx_mgpu *m, const vhx_camera *cam, uint32_t frames, uint32_t *root_slots, float *trace_ms,
                     float *transfer_ms) {
    if (!m || !cam || frames == 0) return VHX_E_INVALID_ARG;
    vhx_ctx *c = m->ctx;
    // measure with one slot per rank, frames one after the other (no overlap), the last frames' medians
    int rc = vhx_mgpu_set_root_slots(m, 1);
    if (rc) return rc;
    float a = 0.0f, g = 0.0f;
    const int mrc = measure_frames(m, cam, frames, a, g);
    // every rank's measurement status to rank 0 (one word per rank, point to point), so that a failure on any rank
    // makes rank 0 send R = 0 below and every rank fails together
    if ((rc = ensure(c, m->hdr, 64 + 4u * (uint32_t)m->nranks))) return rc;
    VHX_STREAM(c);
    bool all_ok = mrc == VHX_OK;
    if (m->nranks > 1) {
        uint32_t *st = (uint32_t *)m->hdr.ptr + 16;
        const Rccl &r = rccl();
        if (m->rank != 0) {
            const uint32_t mine = mrc ? 1u : 0u;
            VHX_HIP(c, hipMemcpyAsync(st, &mine, 4, hipMemcpyHostToDevice, c->stream));
        }
        VHX_NCCL(m, r.GroupStart());
        if (m->rank == 0) {
            for (int q = 1; q < m->nranks; ++q) VHX_NCCL_GROUP(m, r.Recv(st + q, 1, ncclUint32, q, m->comm, c->stream));
        } else {
            VHX_NCCL_GROUP(m, r.Send(st, 1, ncclUint32, 0, m->comm, c->stream));
        }
        VHX_NCCL(m, r.GroupEnd());
        if (m->rank == 0) {
            std::vector<uint32_t> all((size_t)m->nranks, 0u);
            VHX_HIP(c, hipMemcpyAsync(all.data() + 1, st + 1, 4u * (uint32_t)(m->nranks - 1), hipMemcpyDeviceToHost,
                                      c->stream));
            VHX_HIP(c, hipStreamSynchronize(c->stream));
            for (int q = 1; q < m->nranks; ++q) all_ok = all_ok && all[(size_t)q] == 0u;
        }
    }
    // rank 0 picks R: with V = R + N - 1 slots a slot's trace and transfer scale by N / V, the frame period is bounded by
    // rank 0's R slots and by the transfers into rank 0 (one slot part per link, concurrent), so it is about
    // N / V * max(R * trace, transfer) with the one-slot figures; the other ranks' single slot never exceeds rank 0's R.
    // A rank whose measurement failed still joins the closing broadcast (rank 0 then sends R = 0: every rank fails)
    uint32_t best = all_ok ? 1u : 0u;
    if (m->rank == 0 && all_ok) {
        const double N = (double)m->nranks;
        double best_t = 0;
        for (uint32_t R = 1; R <= VHX_MGPU_MAX_ROOT_SLOTS; ++R) {
            const double t = N / (R + N - 1.0) * std::max(R * (double)a, (double)g);
            if (R == 1 || t < best_t * 0.97) {  // a larger share must win by 3 %
                best = R;
                best_t = t;
            }
        }
    }
    // every rank takes rank 0's choice (and its two figures)
    uint32_t msg[3] = {best, 0, 0};
    std::memcpy(&msg[1], &a, 4);
    std::memcpy(&msg[2], &g, 4);
    VHX_HIP(c, hipMemcpyAsync(m->hdr.ptr, msg, sizeof(msg), hipMemcpyHostToDevice, c->stream));
    VHX_NCCL(m, rccl().Broadcast(m->hdr.ptr, m->hdr.ptr, 3, ncclUint32, 0, m->comm, c->stream));
    VHX_HIP(c, hipMemcpyAsync(msg, m->hdr.ptr, sizeof(msg), hipMemcpyDeviceToHost, c->stream));
    VHX_HIP(c, hipStreamSynchronize(c->stream));
    if (mrc) return mrc;
    if (msg[0] < 1 || msg[0] > VHX_MGPU_MAX_ROOT_SLOTS)
        return fail(c, VHX_E_RCCL, "vhx_mgpu_balance: the measurement failed on another rank");
    if ((rc = vhx_mgpu_set_root_slots(m, msg[0]))) return rc;
    if (root_slots) *root_slots = msg[0];
    if (trace_ms) std::memcpy(trace_ms, &msg[1], 4);
    if (transfer_ms) std::memcpy(transfer_ms, &msg[2], 4);
    return VHX_OK;
}

int vhx_mgpu_sync(vhx_mgpu *m, float *ms) {
    if (!m) return VHX_E_INVALID_ARG;
    vhx_ctx *c = m->ctx;
    VHX_HIP(c, hipSetDevice(c->device));
    VHX_HIP(c, hipStreamSynchronize(m->cstream));
    for (vhx_ctx *x : m->extra)
        if (x && x->stream) VHX_HIP(c, hipStreamSynchronize(x->stream));
    int rc = vhx_sync(c, ms);
    if (!rc && ms && m->last && m->last != c) rc = vhx_sync(m->last, ms);
    return rc;
}

}  // extern "C"
