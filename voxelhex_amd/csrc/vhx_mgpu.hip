// libvhx multi-GPU: the screen-tile split of a frame over the GPUs of one node, with RCCL over xGMI (SURVEY.md 8e,
// include/vhx.h vhx_mgpu_*).
//
// Per frame and rank: trace this rank's tiles (r, r+N, ...) into a contiguous send buffer [RGBA8 plane | f32 depth
// plane] on the context's stream; one ncclGather of the send buffers to rank 0 (xGMI point-to-point: each rank's
// buffer crosses one link); rank 0 scatters the gathered buffer into its framebuffers (k_untile_planes). The gather and
// the untile run on a communication stream, so with two alternating send buffers frame k's transfer overlaps frame
// k+1's trace; events order the reuse of a buffer after its gather. The tree is replicated on every GPU (3 GB against
// 288 GB of HBM): rank 0 uploads it from the host, ncclBroadcast copies the device buffers to the other ranks.
//
// RCCL is resolved at run time (dlopen + dlsym) so that the library loads on a host without it and binds to the RCCL
// instance already in the process when there is one (torch's librccl.so.1 has the same soname).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>  // types only: every RCCL function is called through the pointers below

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>

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
    decltype(&ncclGather) Gather = nullptr;
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
        sym(r.Gather, "ncclGather");
        sym(r.GroupStart, "ncclGroupStart");
        sym(r.GroupEnd, "ncclGroupEnd");
        sym(r.GetErrorString, "ncclGetErrorString");
        if (!all) {
            r.err = "the loaded RCCL lacks a symbol libvhx needs (ncclGather needs RCCL >= 2.18)";
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
    bool overlap = true;
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
    uint64_t k = 0;  // frames submitted
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
    return VHX_OK;
}

static void tiles_of(const vhx_mgpu *m, uint32_t W, uint32_t H, uint32_t &ntiles, uint32_t &per_rank) {
    const uint32_t tx = (W + m->T - 1) / m->T, ty = (H + m->T - 1) / m->T;
    ntiles = tx * ty;
    per_rank = (ntiles + (uint32_t)m->nranks - 1) / (uint32_t)m->nranks;
}

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
    for (bool &u : m->used) u = false;
    return VHX_OK;
}

int vhx_mgpu_info(const vhx_mgpu *m, uint32_t W, uint32_t H, int *nranks, int *rank, uint64_t *rays) {
    if (!m) return VHX_E_INVALID_ARG;
    if (nranks) *nranks = m->nranks;
    if (rank) *rank = m->rank;
    if (rays) {
        uint32_t ntiles, per;
        tiles_of(m, W, H, ntiles, per);
        const uint32_t tx = (W + m->T - 1) / m->T;
        uint64_t n = 0;
        for (uint32_t t = (uint32_t)m->rank; t < ntiles; t += (uint32_t)m->nranks) {
            const uint32_t x0 = (t % tx) * m->T, y0 = (t / tx) * m->T;
            n += (uint64_t)std::min(m->T, W - x0) * std::min(m->T, H - y0);
        }
        *rays = n;
    }
    return VHX_OK;
}

int vhx_mgpu_broadcast_tree(vhx_mgpu *m, const vhx_tree_desc *t) {
    if (!m) return VHX_E_INVALID_ARG;
    vhx_ctx *c = m->ctx;
    if ((m->rank == 0) != (t != nullptr)) return fail(c, VHX_E_INVALID_ARG, "vhx_mgpu_broadcast_tree: rank 0 passes the tree, the others NULL");
    const Rccl &r = rccl();
    VHX_HIP(c, hipSetDevice(c->device));
    if (c->shared) return fail(c, VHX_E_STATE, "vhx_mgpu_broadcast_tree on a shared context");
    VHX_STREAM(c);
    if (m->rank == 0) {
        int rc = vhx_upload_tree(c, t);  // host -> HBM of rank 0, derived layout included
        if (rc) return rc;
    }
    // the counts first (8 u32), so the other ranks can size their buffers
    int rc = ensure(c, m->hdr, 64);
    if (rc) return rc;
    uint32_t counts[8] = {0};
    if (m->rank == 0) {
        const vhx_tree_desc &d = c->tree->desc;
        const uint32_t v[8] = {d.boxtree_size, d.brick_dim, d.node_count, d.brick_count,
                               d.solid_count, d.color_count, d.data_count, 0};
        std::memcpy(counts, v, sizeof(v));
        VHX_HIP(c, hipMemcpyAsync(m->hdr.ptr, counts, sizeof(counts), hipMemcpyHostToDevice, c->stream));
    }
    VHX_NCCL(m, r.Broadcast(m->hdr.ptr, m->hdr.ptr, 8, ncclUint32, 0, m->comm, c->stream));
    VHX_HIP(c, hipMemcpyAsync(counts, m->hdr.ptr, sizeof(counts), hipMemcpyDeviceToHost, c->stream));
    VHX_HIP(c, hipStreamSynchronize(c->stream));
    if (m->rank != 0) {
        vhx_tree_desc d{};
        d.boxtree_size = counts[0];
        d.brick_dim = counts[1];
        d.node_count = counts[2];
        d.brick_count = counts[3];
        d.solid_count = counts[4];
        d.color_count = counts[5];
        d.data_count = counts[6];
        if ((rc = alloc_tree(c, &d))) return rc;
    }
    // the raw buffers, device to device over xGMI, in chunks of at most 1 GiB per call
    VHX_NCCL(m, r.GroupStart());
    for (int id = 0; id < 7; ++id) {
        const uint64_t bytes = elem_count(c->tree->desc, id) * elem_size(id);
        for (uint64_t off = 0; off < bytes; off += 1ull << 30) {
            const uint64_t n = std::min<uint64_t>(1ull << 30, bytes - off);
            char *p = (char *)c->tree->raw[id].ptr + off;
            const ncclResult_t e = r.Broadcast(p, p, n, ncclUint8, 0, m->comm, c->stream);
            if (e != ncclSuccess) {
                r.GroupEnd();
                c->err = std::string("ncclBroadcast (tree): ") + r.GetErrorString(e);
                return VHX_E_RCCL;
            }
        }
    }
    VHX_NCCL(m, r.GroupEnd());
    if (m->rank != 0) return finish_upload(c);  // derived layout from the received buffers (synchronises)
    VHX_HIP(c, hipStreamSynchronize(c->stream));
    return VHX_OK;
}

int vhx_mgpu_render(vhx_mgpu *m, const vhx_camera *cam, uint32_t *fb_rgba, float *fb_depth) {
    if (!m || !cam) return VHX_E_INVALID_ARG;
    vhx_ctx *c = m->ctx;
    if (m->rank == 0 && !fb_rgba && !fb_depth) return fail(c, VHX_E_INVALID_ARG, "vhx_mgpu_render: rank 0 needs a framebuffer");
    if (!c->tree->uploaded) return fail(c, VHX_E_STATE, "vhx_mgpu_render before the tree is uploaded");
    if (cam->width == 0 || cam->height == 0) return fail(c, VHX_E_INVALID_ARG, "vhx_mgpu_render: empty frame");
    const Rccl &r = rccl();
    VHX_HIP(c, hipSetDevice(c->device));
    uint32_t ntiles, per;
    tiles_of(m, cam->width, cam->height, ntiles, per);
    const uint64_t n_out = (uint64_t)per * m->T * m->T;  // words per plane of one rank
    const uint32_t slot = (uint32_t)(m->k % m->S);
    vhx_ctx *tc = m->k % m->F == 0 ? c : m->extra[m->k % m->F - 1];  // the context tracing this frame
    VHX_STREAM(tc);
    // a slot's buffers are rewritten only after the gather that read them (stream order on the tracing stream)
    if (m->used[slot]) VHX_HIP(c, hipStreamWaitEvent(tc->stream, m->free_[slot], 0));
    if (m->send[slot].bytes < n_out * 8 || (m->rank == 0 && m->gathered[slot].bytes < n_out * 8 * m->nranks)) {
        // (re)allocation: no frame may still use the old buffers
        int rc = vhx_mgpu_sync(m, nullptr);
        if (rc) return rc;
    }
    int rc = ensure(c, m->send[slot], n_out * 8);
    if (!rc && m->rank == 0) rc = ensure(c, m->gathered[slot], n_out * 8 * (uint64_t)m->nranks);
    if (rc) return rc;
    uint32_t *send = (uint32_t *)m->send[slot].ptr;
    vhx_hits h{};
    h.rgba = send;
    h.depth = (float *)(send + n_out);
    if ((uint32_t)m->rank < ntiles) {
        rc = vhx_trace_primary(tc, cam, m->T, (uint32_t)m->rank, (uint32_t)m->nranks, VHX_LAYOUT_TILES, &h, 1);
        if (rc) return tc == c ? rc : fail(c, rc, tc->err.c_str());
    }
    m->last = tc;
    VHX_HIP(c, hipEventRecord(m->ready[slot], tc->stream));
    VHX_HIP(c, hipStreamWaitEvent(m->cstream, m->ready[slot], 0));
    void *recv = m->rank == 0 ? m->gathered[slot].ptr : nullptr;
    VHX_NCCL(m, r.Gather(send, recv, n_out * 2, ncclUint32, 0, m->comm, m->cstream));  // a local copy at N = 1
    if (m->rank == 0)
        if ((rc = launch_untile(c, m->cstream, recv, 2, (uint32_t)m->nranks, per, m->T, cam->width, cam->height,
                                fb_rgba, fb_depth)))
            return rc;
    VHX_HIP(c, hipEventRecord(m->free_[slot], m->cstream));
    m->used[slot] = true;
    ++m->k;
    if (!m->overlap) VHX_HIP(c, hipStreamWaitEvent(tc->stream, m->free_[slot], 0));
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
