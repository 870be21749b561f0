// TEST INFRASTRUCTURE, not part of libvhx: an in-process loopback communicator with RCCL's C ABI, so that the
// multi-rank code of vhx_mgpu (voxelhex_amd/csrc/vhx_mgpu.hip) runs on one GPU box. libvhx resolves RCCL at run time
// (dlopen, VHX_RCCL_LIB overrides the library), and tests/abi_c/mgpu_ranks.c points it here: every rank is a thread
// of one process with its own vhx_ctx on the same device, and the transfers are device-to-device copies instead of
// xGMI links. What it keeps of RCCL's semantics is what vhx_mgpu relies on:
//  * ncclCommInitRank blocks until all ranks of the unique id have joined;
//  * the calls between ncclGroupStart and ncclGroupEnd (or a single call outside a group) form one step that every
//    rank enters with the same sequence of collectives; broadcasts match by their order in the step, a receive from
//    rank q matches q's k-th send to the receiver;
//  * everything is stream-ordered: a copy starts after the work its source stream had queued when the step was
//    posted (an event), and the source's stream continues only after the copy (so the sender may reuse its buffer
//    in stream order, as with RCCL); the host does not wait for the device.
// A rank that does not arrive within VHX_LOOPBACK_TIMEOUT_S seconds (default 120) fails the step with
// ncclSystemError and poisons the communicator, so a broken test ends instead of hanging.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <random>
#include <string>
#include <vector>

namespace {

enum Kind { BCAST, SEND, RECV };
struct Op {
    Kind kind;
    const void *src;
    void *dst;
    size_t bytes;
    int peer;  // SEND / RECV: the other rank; BCAST: the root
    hipStream_t stream;
    hipEvent_t ready = nullptr;  // the stream's position when the step was posted
    hipEvent_t done = nullptr;   // receiver side: its copy has been queued up to here
};

struct World {
    int n = 0;
    int joined = 0;
    int users = 0;
    bool broken = false;
    std::mutex mu;
    std::condition_variable cv;
    // barrier
    int arrived = 0;
    uint64_t gen = 0;
    std::vector<std::vector<Op> *> posted;  // per rank, during a step
    std::vector<hipEvent_t> garbage;         // events of finished steps (destroyed with the communicator)
};

std::mutex g_mu;
std::map<std::string, World *> g_worlds;

double timeout_s() {
    const char *e = getenv("VHX_LOOPBACK_TIMEOUT_S");
    return e && atof(e) > 0 ? atof(e) : 120.0;
}

// all ranks of w reach this point (or the wait times out: false, and the world is broken for good)
bool barrier(World *w) {
    std::unique_lock<std::mutex> lk(w->mu);
    if (w->broken) return false;
    const uint64_t g = w->gen;
    if (++w->arrived == w->n) {
        w->arrived = 0;
        ++w->gen;
        w->cv.notify_all();
        return true;
    }
    const bool ok = w->cv.wait_for(lk, std::chrono::duration<double>(timeout_s()),
                                   [&] { return w->gen != g || w->broken; });
    if (!ok || w->broken) {
        w->broken = true;
        w->cv.notify_all();
        return false;
    }
    return true;
}

size_t type_size(ncclDataType_t t) {
    switch (t) {
        case ncclInt8:
        case ncclUint8:
            return 1;
        case ncclFloat16:
        case ncclBfloat16:
            return 2;
        case ncclInt32:
        case ncclUint32:
        case ncclFloat32:
            return 4;
        case ncclInt64:
        case ncclUint64:
        case ncclFloat64:
            return 8;
        default:
            return 0;
    }
}

}  // namespace

struct ncclComm {
    World *w;
    int rank;
};

namespace {

thread_local int t_depth = 0;
thread_local ncclComm *t_comm = nullptr;
thread_local std::vector<Op> t_ops;

#define LB_HIP(call)                                                                                              \
    do {                                                                                                          \
        if ((call) != hipSuccess) return ncclUnhandledCudaError;                                                  \
    } while (0)

// one step: post this rank's ops, queue the copies this rank receives, then order the sources after them
ncclResult_t run_step(ncclComm *c, std::vector<Op> &ops) {
    World *w = c->w;
    const int me = c->rank;
    for (Op &o : ops) {
        LB_HIP(hipEventCreateWithFlags(&o.ready, hipEventDisableTiming));
        LB_HIP(hipEventCreateWithFlags(&o.done, hipEventDisableTiming));
        LB_HIP(hipEventRecord(o.ready, o.stream));
    }
    {
        std::lock_guard<std::mutex> lk(w->mu);
        w->posted[me] = &ops;
    }
    if (!barrier(w)) return ncclSystemError;
    ncclResult_t rc = ncclSuccess;
    // phase 1: receiving side (RECV, non-root BCAST) and a root's own copy
    {
        std::map<int, int> nrecv;  // RECVs from peer q seen so far
        int nb = 0;                // BCASTs seen so far
        for (Op &o : ops) {
            const Op *src = nullptr;
            if (o.kind == RECV) {
                int k = nrecv[o.peer]++;
                for (const Op &s : *w->posted[o.peer])
                    if (s.kind == SEND && s.peer == me && k-- == 0) {
                        src = &s;
                        break;
                    }
            } else if (o.kind == BCAST) {
                int k = nb++;
                for (const Op &s : *w->posted[o.peer])
                    if (s.kind == BCAST && k-- == 0) {
                        src = &s;
                        break;
                    }
                if (src && src->peer != o.peer) src = nullptr;  // the ranks disagree on the root
                if (src && o.peer == me) {  // the root: its own copy (in place: nothing to do)
                    if (o.dst != o.src && o.bytes && hipMemcpyAsync(o.dst, o.src, o.bytes, hipMemcpyDeviceToDevice,
                                                                    o.stream) != hipSuccess)
                        rc = ncclUnhandledCudaError;
                    src = nullptr;
                    continue;
                }
            } else {
                continue;
            }
            if (!src || src->bytes != o.bytes) {
                rc = ncclInvalidUsage;
                continue;
            }
            if (hipStreamWaitEvent(o.stream, src->ready, 0) != hipSuccess ||
                (o.bytes && hipMemcpyAsync(o.dst, src->src, o.bytes, hipMemcpyDeviceToDevice, o.stream) != hipSuccess) ||
                hipEventRecord(o.done, o.stream) != hipSuccess)
                rc = ncclUnhandledCudaError;
        }
    }
    if (!barrier(w)) return ncclSystemError;
    // phase 2: sending side waits for the copies that read its buffers
    {
        std::map<int, int> nsend;
        int nb = 0;
        for (Op &o : ops) {
            if (o.kind == SEND) {
                int k = nsend[o.peer]++;
                for (const Op &r : *w->posted[o.peer])
                    if (r.kind == RECV && r.peer == me && k-- == 0) {
                        if (hipStreamWaitEvent(o.stream, r.done, 0) != hipSuccess) rc = ncclUnhandledCudaError;
                        break;
                    }
            } else if (o.kind == BCAST) {
                const int k = nb++;
                if (o.peer != me) continue;
                for (int q = 0; q < w->n; ++q) {
                    if (q == me) continue;
                    int kk = k;
                    for (const Op &r : *w->posted[q])
                        if (r.kind == BCAST && kk-- == 0) {
                            if (hipStreamWaitEvent(o.stream, r.done, 0) != hipSuccess) rc = ncclUnhandledCudaError;
                            break;
                        }
                }
            }
        }
    }
    // phase 3: nobody reads another rank's op list after this
    if (!barrier(w)) return ncclSystemError;
    {
        std::lock_guard<std::mutex> lk(w->mu);
        w->posted[me] = nullptr;
        for (Op &o : ops) {
            w->garbage.push_back(o.ready);
            w->garbage.push_back(o.done);
        }
    }
    return rc;
}

ncclResult_t enqueue(ncclComm *c, Op o) {
    if (!c || !c->w) return ncclInvalidArgument;
    if (t_depth > 0) {
        if (t_comm && t_comm != c) return ncclInvalidUsage;  // one communicator per group (all vhx_mgpu needs)
        t_comm = c;
        t_ops.push_back(o);
        return ncclSuccess;
    }
    std::vector<Op> ops{o};
    return run_step(c, ops);
}

}  // namespace

extern "C" {

ncclResult_t ncclGetUniqueId(ncclUniqueId *id) {
    if (!id) return ncclInvalidArgument;
    std::memset(id->internal, 0, sizeof(id->internal));
    std::memcpy(id->internal, "vhx-loopback", 12);
    std::random_device rd;
    for (int i = 16; i < 48; ++i) id->internal[i] = (char)(rd() & 0xFF);
    return ncclSuccess;
}

ncclResult_t ncclCommInitRank(ncclComm_t *comm, int nranks, ncclUniqueId id, int rank) {
    if (!comm || nranks < 1 || rank < 0 || rank >= nranks) return ncclInvalidArgument;
    const std::string key(id.internal, sizeof(id.internal));
    World *w;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        World *&slot = g_worlds[key];
        if (!slot) {
            slot = new World();
            slot->n = nranks;
            slot->posted.assign(nranks, nullptr);
        }
        w = slot;
        ++w->users;
    }
    if (w->n != nranks) return ncclInvalidUsage;
    {
        std::unique_lock<std::mutex> lk(w->mu);
        ++w->joined;
        w->cv.notify_all();
        if (!w->cv.wait_for(lk, std::chrono::duration<double>(timeout_s()), [&] { return w->joined >= w->n; })) {
            w->broken = true;
            return ncclSystemError;
        }
    }
    *comm = new ncclComm{w, rank};
    return ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm_t comm) {
    if (!comm) return ncclInvalidArgument;
    World *w = comm->w;
    delete comm;
    std::lock_guard<std::mutex> lk(g_mu);
    if (--w->users == 0) {
        (void)hipDeviceSynchronize();
        for (hipEvent_t e : w->garbage) (void)hipEventDestroy(e);
        for (auto it = g_worlds.begin(); it != g_worlds.end(); ++it)
            if (it->second == w) {
                g_worlds.erase(it);
                break;
            }
        delete w;
    }
    return ncclSuccess;
}

ncclResult_t ncclCommCount(const ncclComm_t comm, int *count) {
    if (!comm || !count) return ncclInvalidArgument;
    *count = comm->w->n;
    return ncclSuccess;
}

ncclResult_t ncclCommUserRank(const ncclComm_t comm, int *rank) {
    if (!comm || !rank) return ncclInvalidArgument;
    *rank = comm->rank;
    return ncclSuccess;
}

ncclResult_t ncclBroadcast(const void *sendbuff, void *recvbuff, size_t count, ncclDataType_t datatype, int root,
                           ncclComm_t comm, hipStream_t stream) {
    const size_t ts = type_size(datatype);
    if (!comm || !ts || root < 0 || root >= comm->w->n) return ncclInvalidArgument;
    return enqueue(comm, Op{BCAST, sendbuff, recvbuff, count * ts, root, stream});
}

ncclResult_t ncclSend(const void *sendbuff, size_t count, ncclDataType_t datatype, int peer, ncclComm_t comm,
                      hipStream_t stream) {
    const size_t ts = type_size(datatype);
    if (!comm || !ts || peer < 0 || peer >= comm->w->n || peer == comm->rank) return ncclInvalidArgument;
    return enqueue(comm, Op{SEND, sendbuff, nullptr, count * ts, peer, stream});
}

ncclResult_t ncclRecv(void *recvbuff, size_t count, ncclDataType_t datatype, int peer, ncclComm_t comm,
                      hipStream_t stream) {
    const size_t ts = type_size(datatype);
    if (!comm || !ts || peer < 0 || peer >= comm->w->n || peer == comm->rank) return ncclInvalidArgument;
    return enqueue(comm, Op{RECV, nullptr, recvbuff, count * ts, peer, stream});
}

ncclResult_t ncclGroupStart() {
    ++t_depth;
    return ncclSuccess;
}

ncclResult_t ncclGroupEnd() {
    if (t_depth == 0) return ncclInvalidUsage;
    if (--t_depth > 0) return ncclSuccess;
    ncclComm *c = t_comm;
    std::vector<Op> ops;
    ops.swap(t_ops);
    t_comm = nullptr;
    if (!c) return ncclSuccess;
    return run_step(c, ops);
}

const char *ncclGetErrorString(ncclResult_t r) {
    switch (r) {
        case ncclSuccess:
            return "no error (loopback)";
        case ncclUnhandledCudaError:
            return "a HIP call failed (loopback)";
        case ncclSystemError:
            return "a rank did not arrive in time (loopback)";
        case ncclInvalidArgument:
            return "invalid argument (loopback)";
        case ncclInvalidUsage:
            return "invalid usage: ranks disagree on the step (loopback)";
        default:
            return "error (loopback)";
    }
}

}  // extern "C"
