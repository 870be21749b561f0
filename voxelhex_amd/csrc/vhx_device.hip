// libvhx device side: HIP kernels for gfx950 and the C ABI of include/vhx.h.
//
// Kernels
//   k_trace_primary  per-pixel primary rays (examples/gpu_render.rs:196-257, benches/performance.rs:29-66) traced with
//                    get_by_ray semantics (src/raytracing/cpu.rs:296-458); replaces the WGSL `update` kernel dispatched
//                    by VhxRenderNode::run (src/raytracing/bevy/pipeline/mod.rs:96-155)
//   k_trace_rays     explicit ray batch (BoxTree::get_by_ray over many rays)
//   k_brick_occ_*    upload-time brick occupancy bitmaps from pix_points_to_empty (src/boxtree/node.rs:311-333)
//   k_pack_hdr       node type + occupied_bits -> one 16-byte record per node
//   k_untile_rgba    scatters rank-gathered tile buffers into the framebuffer (multi-GPU screen-tile split)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/vhx.h"
#include "trace.hpp"

namespace vhx {
__constant__ uint8_t c_step_lut[64 * 27];
}

using namespace vhx;

#include "ctx.hpp"

// SECTANT_STEP_RESULT_LUT generator (src/bin/sectant_step_result_lut.rs:48-114), host side
static void make_step_lut(uint8_t *lut) {
    for (int s = 0; s < 64; ++s)
        for (int x = -1; x <= 1; ++x)
            for (int y = -1; y <= 1; ++y)
                for (int z = -1; z <= 1; ++z) {
                    float off[3] = {(float)(s % 4) / 4.f, (float)((s / 4) % 4) / 4.f, (float)(s / 16) / 4.f};
                    float st[3] = {(float)x, (float)y, (float)z};
                    float after[3];
                    bool out = false;
                    for (int k = 0; k < 3; ++k) {
                        after[k] = (off[k] + 0.25f / 2.f) + 0.25f * st[k];
                        out |= after[k] < 0.f || after[k] > 1.f;
                    }
                    int base = 0;
                    if (out) {
                        for (int k = 0; k < 3; ++k) {
                            after[k] = std::fmod(after[k], 1.f);
                            if (after[k] < 0.f) after[k] += 1.f;
                        }
                        base = 64;
                    }
                    int ix = (int)std::floor(after[0] * 4.f), iy = (int)std::floor(after[1] * 4.f),
                        iz = (int)std::floor(after[2] * 4.f);
                    lut[s * 27 + (x + 1) * 9 + (y + 1) * 3 + (z + 1)] = (uint8_t)(base + ix + iy * 4 + iz * 16);
                }
}

// ------------------------------------------------------------------------------------------------ upload kernels
__device__ __forceinline__ bool cell_empty(uint32_t v, const uint32_t *color, uint32_t ncolor, const uint32_t *data,
                                           uint32_t ndata) {
    const uint32_t ci = v & 0xFFFFu, di = v >> 16;
    const bool cn = ci == 0xFFFFu || ci >= ncolor || ((color[ci] >> 24) & 0xFFu) == 0;
    const bool dn = di == 0xFFFFu || di >= ndata || data[di] == 0;
    return cn && dn;
}

// bd^3 >= 64: one lane per cell, the wave's ballot is one 64-bit occupancy word
__global__ void __launch_bounds__(256) k_brick_occ_ballot(const uint32_t *__restrict__ vox, uint64_t ncells,
                                                          uint64_t cell0, const uint32_t *__restrict__ color,
                                                          uint32_t ncolor, const uint32_t *__restrict__ data,
                                                          uint32_t ndata, uint64_t *__restrict__ words) {
    const uint64_t i = cell0 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool in = i < cell0 + ncells;
    const bool full = in && !cell_empty(vox[in ? i : cell0], color, ncolor, data, ndata);
    const uint64_t m = __ballot(full);
    if ((threadIdx.x & 63u) == 0 && in) words[i >> 6] = m;
}

// bd^3 < 64 (bd = 1, 2): one lane per brick
__global__ void __launch_bounds__(256) k_brick_occ_small(const uint32_t *__restrict__ vox, uint32_t nbricks,
                                                         uint32_t brick0, uint32_t n3,
                                                         const uint32_t *__restrict__ color, uint32_t ncolor,
                                                         const uint32_t *__restrict__ data, uint32_t ndata,
                                                         uint64_t *__restrict__ words) {
    const uint32_t b = brick0 + blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= brick0 + nbricks) return;
    uint64_t m = 0;
    for (uint32_t c = 0; c < n3; ++c)
        if (!cell_empty(vox[(uint64_t)b * n3 + c], color, ncolor, data, ndata)) m |= 1ull << c;
    words[b] = m;
}

// DevTree::child_rec for brick_dim <= 4: one record per child entry. Entries [e0, e1) are visited; with sel, only the
// entries of nodes [node_lo, node_hi) and those holding a Parted brick in [brick_lo, brick_hi) are rewritten (a ranged
// update: the records of written nodes and of the nodes whose bricks were written)
struct RecSel {
    uint32_t sel, node_lo, node_hi, brick_lo, brick_hi;
};
__global__ void __launch_bounds__(256) k_child_rec(const uint32_t *__restrict__ type,
                                                   const uint32_t *__restrict__ children,
                                                   const uint64_t *__restrict__ words, uint32_t brick_count,
                                                   uint64_t e0, uint64_t e1, RecSel s, uint4 *__restrict__ rec) {
    const uint64_t i = e0 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= e1) return;
    const uint32_t node = (uint32_t)(i >> 6);
    const uint32_t ty = type[node];
    const bool uniform = ty == VHX_NODE_UNIFORM_LEAF;
    const uint32_t v = children[uniform ? (i & ~63ull) : i];
    const bool parted = (uniform || ty == VHX_NODE_LEAF) && v != VHX_EMPTY && (v & VHX_SOLID_BIT) == 0 && v < brick_count;
    if (s.sel && !(node >= s.node_lo && node < s.node_hi) && !(parted && v >= s.brick_lo && v < s.brick_hi)) return;
    const uint64_t o = parted ? words[v] : 0ull;
    rec[i] = make_uint4(v, (uint32_t)o, (uint32_t)(o >> 32), 0u);
}

// Ranged writes: job j copies `words` 32-bit words from the staging buffer at src_off to the device address dst (a
// range cut into pieces of at most 16 KiB, one workgroup per piece)
struct UpdJob {
    uint64_t dst, src_off;
    uint32_t words, pad0;
    uint64_t pad1;
};
#define UPD_PIECE_BYTES 16384u
__global__ void __launch_bounds__(256) k_scatter_ranges(const uint8_t *__restrict__ stage, uint32_t j0, uint32_t j1) {
    const UpdJob *jobs = (const UpdJob *)stage;
    for (uint32_t j = j0 + blockIdx.x; j < j1; j += gridDim.x) {
        const UpdJob jb = jobs[j];
        const uint32_t *src = (const uint32_t *)(stage + jb.src_off);
        uint32_t *dst = (uint32_t *)jb.dst;
        for (uint32_t w = threadIdx.x; w < jb.words; w += blockDim.x) dst[w] = src[w];
    }
}

__global__ void __launch_bounds__(256) k_pack_hdr(const uint32_t *__restrict__ type, const uint64_t *__restrict__ occ,
                                                  uint32_t n0, uint32_t n, uint4 *__restrict__ hdr) {
    const uint32_t i = n0 + blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n0 + n) return;
    const uint64_t o = occ[i];
    hdr[i] = make_uint4((uint32_t)o, (uint32_t)(o >> 32), type[i], 0u);
}

// ------------------------------------------------------------------------------------------------ trace kernels
struct CamD {
    uint32_t model, width, height;
    float ox, oy, oz;
    float blx, bly, blz, rx, ry, rz, ux, uy, uz, pw, ph;
    float m[16];
};

struct OutD {
    uint32_t *value, *cell, *voxel, *rgba, *bytes;
    float *impact, *normal, *depth;
    uint32_t *shadowed;  // fused hard shadows (vhx_set_shadow_light)
};

// examples/gpu_render.rs:199, 236-251
__device__ __forceinline__ uint32_t shade(const DevTree &t, const HitOut &h) {
    if (!h.hit) return 128u | (128u << 8) | (128u << 16) | (255u << 24);
    const uint32_t ci = h.value & 0xFFFFu;
    if (ci == 0xFFFFu || ci >= t.color_count) return 255u << 24;
    const uint32_t c = t.color[ci];
    const F3d L = vnorm(mk(0.0f, -1.0f, 1.0f));
    const float dot = (h.nx * L.x + h.ny * L.y) + h.nz * L.z;
    const float s = 1.0f - (dot / 2.0f + 0.5f);
    const uint32_t r = ras_u8((float)(c & 0xFFu) * s), g = ras_u8((float)((c >> 8) & 0xFFu) * s),
                   b = ras_u8((float)((c >> 16) & 0xFFu) * s);
    return r | (g << 8) | (b << 16) | (255u << 24);
}

__device__ __forceinline__ void store(const DevTree &t, const OutD &o, uint64_t i, F3d org, const HitOut &h) {
    if (o.value) o.value[i] = h.hit ? h.value : VHX_EMPTY;
    if (o.cell) o.cell[i] = h.hit ? h.cell : VHX_EMPTY;
    if (o.voxel) {
        o.voxel[3 * i] = h.hit ? h.vx : VHX_EMPTY;
        o.voxel[3 * i + 1] = h.hit ? h.vy : VHX_EMPTY;
        o.voxel[3 * i + 2] = h.hit ? h.vz : VHX_EMPTY;
    }
    if (o.impact) {
        o.impact[3 * i] = h.hit ? h.ix : 0.0f;
        o.impact[3 * i + 1] = h.hit ? h.iy : 0.0f;
        o.impact[3 * i + 2] = h.hit ? h.iz : 0.0f;
    }
    if (o.normal) {
        o.normal[3 * i] = h.hit ? h.nx : 0.0f;
        o.normal[3 * i + 1] = h.hit ? h.ny : 0.0f;
        o.normal[3 * i + 2] = h.hit ? h.nz : 0.0f;
    }
    if (o.depth) o.depth[i] = h.hit ? vlen(vsub(mk(h.ix, h.iy, h.iz), org)) : __builtin_huge_valf();
    if (o.rgba) o.rgba[i] = shade(t, h);
    if (o.bytes) o.bytes[i] = h.bytes;
}

// benches/performance.rs:54-61 (glass) and examples/gpu_render.rs:203-224 (inverse VP, glam op order)
__device__ __forceinline__ void primary_ray(const CamD &c, uint32_t px, uint32_t py, F3d &o, F3d &d) {
    const uint32_t x = px, y = c.height - 1u - py;
    o = mk(c.ox, c.oy, c.oz);
    if (c.model == VHX_RAY_GLASS) {
        const F3d gp = vadd(vadd(mk(c.blx, c.bly, c.blz), vmul(vmul(mk(c.rx, c.ry, c.rz), (float)x), c.pw)),
                            vmul(vmul(mk(c.ux, c.uy, c.uz), (float)y), c.ph));
        d = vnorm(vsub(gp, o));
    } else {
        const float nx = ((float)x + 0.5f) / (float)c.width * 2.0f - 1.0f;
        const float ny = ((float)y + 0.5f) / (float)c.height * 2.0f - 1.0f;
        float nr[4], fr[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            nr[k] = ((c.m[k] * nx + c.m[4 + k] * ny) + c.m[8 + k] * -1.0f) + c.m[12 + k] * 1.0f;
            fr[k] = ((c.m[k] * nx + c.m[4 + k] * ny) + c.m[8 + k] * 1.0f) + c.m[12 + k] * 1.0f;
        }
        const F3d np = mk(nr[0] / nr[3], nr[1] / nr[3], nr[2] / nr[3]);
        const F3d fp = mk(fr[0] / fr[3], fr[1] / fr[3], fr[2] / fr[3]);
        const F3d dd = vsub(fp, np);
        const float rcp = 1.0f / __builtin_sqrtf((dd.x * dd.x + dd.y * dd.y) + dd.z * dd.z);
        d = vmul(dd, rcp);
    }
}

// A glass-camera ray that misses the root cube by a clear margin (the sky around the tree: two thirds of the bench
// frame's pass-0 waves hold no ray that enters it) ends as the miss record whatever its exact direction, so the exact
// setup -- normalising the direction (3 divisions, a square root) and the root slab test (6 divisions; cpu.rs:302-313,
// spatial/raytracing/mod.rs:33-62) -- is skipped. The test runs on the unnormalised direction v = gp - o with
// approximate reciprocals: t'_k = (bound - o_k) * rcp(v_k) and the exact t_k = (bound - o_k) / (v_k / |v|) agree up to
// the common factor |v| within a few roundings (6 ulp, 4e-7 relative), so tmax' < -m or tmin' - tmax' > m with
// m = 1e-5 * max(|tmin'|, |tmax'|) implies the exact test's miss (tmax < 0 or tmin > tmax). A zero, tiny or non-finite
// component, or anything closer, takes the exact path.
__device__ __forceinline__ bool glass_clear_miss(const CamD &c, uint32_t px, uint32_t py, float tsize) {
    if (c.model != VHX_RAY_GLASS) return false;
    const uint32_t x = px, y = c.height - 1u - py;
    const F3d o = mk(c.ox, c.oy, c.oz);
    const F3d gp = vadd(vadd(mk(c.blx, c.bly, c.blz), vmul(vmul(mk(c.rx, c.ry, c.rz), (float)x), c.pw)),
                        vmul(vmul(mk(c.ux, c.uy, c.uz), (float)y), c.ph));
    const F3d v = vsub(gp, o);
    const float vk[3] = {v.x, v.y, v.z}, ok[3] = {o.x, o.y, o.z};
    float tmin = -__builtin_huge_valf(), tmax = __builtin_huge_valf();
    bool safe = true;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        safe = safe && __builtin_fabsf(vk[k]) > 1e-20f;  // false for NaN too
        const float r = __builtin_amdgcn_rcpf(vk[k]);
        const float t1 = (0.0f - ok[k]) * r, t2 = (tsize - ok[k]) * r;
        tmin = __builtin_fmaxf(tmin, __builtin_fminf(t1, t2));
        tmax = __builtin_fminf(tmax, __builtin_fmaxf(t1, t2));
    }
    if (!safe || !__builtin_isfinite(tmin) || !__builtin_isfinite(tmax)) return false;
    const float m = 1e-5f * __builtin_fmaxf(__builtin_fabsf(tmin), __builtin_fabsf(tmax));
    return tmax < -m || tmin - tmax > m;
}

// ------------------------------------------------------------------------------------------- multi-pass scheduling
// Per-ray work is heavy-tailed (bench frame: mean 14 steps, p99 311, max 2160), and a wave64 runs as long as its
// longest lane. Pass 0 traces every ray with a small step budget; the rays that exhaust it are listed per chunk (a
// workgroup's 16x16 pixel block, or a queue pass's chunk) in lane order, a scan over the chunk counts and a gather
// turn the lists into the next pass's queue, and the next pass traces them again from scratch, 64 long rays per
// wave, with a larger budget; the last pass is unbounded (VHX_MAX_ITERS). Keeping the queue in spatial order keeps
// neighbouring rays together in a wave: the bench frame's long rays take 1.17 ms in frame order and 1.48 ms in
// completion (atomic-append) order. Every ray's result comes from one uninterrupted, deterministic traversal, so the
// output is bit-identical to a single pass.
struct PassQ {
    uint32_t budget;   // VHX_MAX_ITERS on the final pass
    uint32_t rpw;      // queue passes: rays per wave (lanes >= rpw idle); 0 = adaptive (pass_rpw)
    uint32_t tw;       // adaptive rays per wave: the pass spreads its rays over about this many waves
    uint32_t resume;   // queue passes: the input rays continue from their saved state (else traced from scratch)
    uint32_t *tmp;     // chunk-local lists of abandoned rays (null on the final pass)
    uint32_t *counts;  // per chunk
    uint8_t *flags;    // primary pass 0: abandoned flag per output index (every entry written, no clearing needed)
    uint4 *state;      // per output index, 4 x uint4: saved traversal state of an abandoned ray (null: re-trace); in the
                       // queue-state mode per slot of this pass's chunk lists instead
    const uint4 *sin;  // queue-state mode: the input rays' states in queue order (k_gather_chunks moved them there)
    uint32_t qmode;    // 1: queue-state mode (states saved by list slot, resumed by queue position), 0: by output index
    uint32_t xcd_group;  // pass 0: XCD-aware block runs (xcd_block), 0 = dispatch order
    uint32_t qxcd;       // queue passes: runs of this many chunks dealt over the 8 XCDs, one counter each (0 = off)
    uint32_t sparse;     // budgeted passes with saved state: abandon a wave's rays once fewer lanes trace (0 = off)
    uint32_t *zero;      // pass 0 with block lists: the queue passes' work counters, zeroed by workgroup 0
    float lx, ly, lz;    // fused hard shadows (the FUSE kernels): the light
    uint32_t sbud;       // fused: a shadow ray's steps in the budgeted pass its primary ray finished (0 = the rest)
    // early tail (vhx_ctx::tail_*): pass 0 skips the pixels set in `skip` (the early tail traces them); the final pass
    // appends the pixels of rays that took >= tail_min steps to tail_out (count at word 0, entries from word 64)
    const uint32_t *skip;
    uint32_t *tail_out;
    uint32_t tail_min, tail_cap;
    uint32_t finter;  // batch pass 0: frames interleaved block by block (vhx_ctx::frame_interleave)
};

// one more pixel of the early-tail list (at most cap; the count keeps growing past it, the entries stop)
__device__ __forceinline__ void tail_record(uint32_t *list, uint32_t cap, uint32_t idx) {
    const uint32_t k = atomicAdd(list, 1u);
    if (k < cap) list[64u + k] = idx;
}

// Rays per wave of a queue pass over n rays: fixed, or (rpw == 0) as many as spread the pass over about `tw` waves.
// Long rays traced 64 per wave pay for their divergence (the bench frame's 256 longest: 1.05 ms at 64 per wave,
// 0.56 ms at one per wave and one wave per workgroup); short queues are better spread thin.
__device__ __forceinline__ uint32_t pass_rpw(uint32_t rpw, uint32_t tw, uint32_t n) {
    if (rpw) return rpw;
    const uint32_t k = (n + tw - 1) / tw;
    return k < 1u ? 1u : (k > 64u ? 64u : k);
}

// Block-level ordered append (all 256 threads of the workgroup call it): the workgroup's rays with push set are
// listed at tmp[pos * 256 ...] in thread order, their number at counts[pos] (pos: the workgroup's chunk position).
__device__ __forceinline__ void block_append(bool push, uint32_t idx, uint32_t *tmp, uint32_t *counts,
                                             uint32_t pos) {
    __shared__ uint32_t s_cnt[4];
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    const uint64_t m = __ballot(push);
    if (lane == 0) s_cnt[wave] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t before = 0;
    for (uint32_t w = 0; w < wave; ++w) before += s_cnt[w];
    if (push) tmp[(uint64_t)pos * 256u + before + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = idx;
    if (threadIdx.x == 0) counts[pos] = s_cnt[0] + s_cnt[1] + s_cnt[2] + s_cnt[3];
}

// Exclusive scan of the chunk counts in one workgroup of SCAN_THREADS threads; nchunks = ceil(*n_in / per_chunk) when
// n_in is given (a queue pass: its input length is only known on the device), else nchunks_host. Writes *total.
// Each wave scans 1024 consecutive counts per segment as 16 coalesced rows of 64 (a wave-wide scan per row), the
// waves' totals are combined through LDS. Four waves, not sixteen: with other frames in flight the GPU is full, and a
// 1024-thread workgroup waited up to 0.25 ms for a CU with room for it (kernel trace of three frames in flight).
#define SCAN_THREADS 256u
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, uint32_t lane) {
    for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint32_t x = __shfl_up(v, d);
        if (lane >= d) v += x;
    }
    return v;
}
#define SCAN_SEG (SCAN_THREADS * 16u)  // counts per segment
__device__ __forceinline__ uint32_t scan_nchunks(uint32_t nchunks_host, const uint32_t *n_in, uint32_t per_chunk,
                                                 uint32_t tw) {
    if (!n_in) return nchunks_host;
    const uint32_t pc = pass_rpw(per_chunk, tw, *n_in);
    return (*n_in + pc - 1) / pc;
}
// seg_base == null: one workgroup walks every segment and writes *total. seg_base != null (a large scan, launch_scan):
// workgroup b scans segment b only, starting from seg_base[b] (the exclusive scan of the segments' sums).
__global__ void __launch_bounds__(SCAN_THREADS) k_scan_counts(const uint32_t *__restrict__ counts,
                                                              uint32_t nchunks_host, const uint32_t *n_in,
                                                              uint32_t per_chunk, uint32_t tw,
                                                              uint32_t *__restrict__ offsets, uint32_t *total,
                                                              const uint32_t *__restrict__ seg_base = nullptr) {
    constexpr uint32_t NW = SCAN_THREADS / 64u;
    __shared__ uint32_t s_wave[NW];
    __shared__ uint32_t s_carry;
    const uint32_t nchunks = scan_nchunks(nchunks_host, n_in, per_chunk, tw);
    const uint32_t t = threadIdx.x, lane = t & 63u, wave = t >> 6;
    constexpr uint32_t K = 16;  // rows of 64 per wave per segment; loads issued together
    uint32_t seg0 = 0, seg_end = nchunks;
    if (seg_base) {
        seg0 = blockIdx.x * SCAN_SEG;
        if (seg0 >= nchunks) return;  // the whole workgroup
        seg_end = seg0 + 1u;
    }
    if (t == 0) s_carry = seg_base ? seg_base[blockIdx.x] : 0u;
    __syncthreads();
    for (uint32_t seg = seg0; seg < seg_end; seg += SCAN_THREADS * K) {
        const uint32_t b = seg + wave * (64u * K) + lane;
        uint32_t v[K];
#pragma unroll
        for (uint32_t k = 0; k < K; ++k) v[k] = b + 64u * k < nchunks ? counts[b + 64u * k] : 0u;
        uint32_t run = 0;  // the wave's sum of the rows before row k
#pragma unroll
        for (uint32_t k = 0; k < K; ++k) {
            const uint32_t inc = wave_incl_scan(v[k], lane);
            const uint32_t row = __shfl(inc, 63);
            v[k] = run + inc - v[k];  // exclusive within the wave's 1024 counts
            run += row;
        }
        if (lane == 0) s_wave[wave] = run;
        __syncthreads();
        uint32_t before = s_carry;
        for (uint32_t w = 0; w < wave; ++w) before += s_wave[w];
#pragma unroll
        for (uint32_t k = 0; k < K; ++k)
            if (b + 64u * k < nchunks) offsets[b + 64u * k] = before + v[k];
        __syncthreads();
        if (t == 0) {
            uint32_t sum = s_carry;
            for (uint32_t w = 0; w < NW; ++w) sum += s_wave[w];
            s_carry = sum;
        }
        __syncthreads();
    }
    if (t == 0 && !seg_base) *total = s_carry;
}
// sums[b] = the sum of segment b's counts (0 past the end)
__global__ void __launch_bounds__(SCAN_THREADS) k_scan_sums(const uint32_t *__restrict__ counts, uint32_t nchunks_host,
                                                            const uint32_t *n_in, uint32_t per_chunk, uint32_t tw,
                                                            uint32_t *__restrict__ sums) {
    __shared__ uint32_t s_wave[SCAN_THREADS / 64u];
    const uint32_t nchunks = scan_nchunks(nchunks_host, n_in, per_chunk, tw);
    const uint32_t t = threadIdx.x, base = blockIdx.x * SCAN_SEG;
    uint32_t v = 0;
#pragma unroll
    for (uint32_t k = 0; k < 16u; ++k) {
        const uint32_t i = base + k * SCAN_THREADS + t;
        v += base < nchunks && i < nchunks ? counts[i] : 0u;
    }
    for (uint32_t d = 32; d > 0; d >>= 1) v += __shfl_down(v, d);
    if ((t & 63u) == 0) s_wave[t >> 6] = v;
    __syncthreads();
    if (t == 0) {
        uint32_t sum = 0;
        for (uint32_t w = 0; w < SCAN_THREADS / 64u; ++w) sum += s_wave[w];
        sums[blockIdx.x] = sum;
    }
}

// Flag compaction in output-index order, 1024 entries per workgroup, 4 per thread. The flag of entry i is flags[i]
// (primary pass 0: the ray was abandoned) or, with HITS, value[i] != VHX_EMPTY (the hit pixels a shadow pass starts
// from).
template <bool HITS>
__device__ __forceinline__ uint32_t flag_bits(const void *src, uint64_t i, uint64_t n) {
    uint32_t bits = 0;  // bit k: flag of entry i + k
    if (i + 3 < n) {
        if (HITS) {
            const uint32_t *v = (const uint32_t *)src + i;  // the caller's array: no alignment beyond 4 B assumed
            bits = (v[0] != VHX_EMPTY ? 1u : 0u) | (v[1] != VHX_EMPTY ? 2u : 0u) | (v[2] != VHX_EMPTY ? 4u : 0u) |
                   (v[3] != VHX_EMPTY ? 8u : 0u);
        } else {
            const uint32_t w = *(const uint32_t *)((const uint8_t *)src + i);
            bits = (w & 1u) | ((w >> 7) & 2u) | ((w >> 14) & 4u) | ((w >> 21) & 8u);
        }
    } else {
        for (uint64_t k = i; k < n && k < i + 4; ++k) {
            const bool f = HITS ? ((const uint32_t *)src)[k] != VHX_EMPTY : (((const uint8_t *)src)[k] & 1u) != 0;
            if (f) bits |= 1u << (k - i);
        }
    }
    return bits;
}

// qctl: [0..7] queue lengths written after pass p (7: shadow hit list), [16 + QCTL_PASS_WORDS p ..] pass p's work
// counters: the single counter, then the 8 XCD counters, each on a 256-byte line of its own (with the XCD counters in
// one line, the drain of a budgeted pass over many short chunks, every wave probing every exhausted counter, took 2.5 -
// 3.6 times as long as with one counter: DESIGN.md §3)
#define QCTL_PASS_WORDS (9u * 64u)
#define QCTL_WORDS (16u + QCTL_PASS_WORDS * (VHX_MAX_BUDGETS + 1u))
// Order of the pass-0 queue of a primary frame (vhx_ctx::qorder): W = 0 keeps output-index order (row-major in the
// framebuffer layout); W > 0 lists the rays tile by tile -- TS x TS pixel tiles (TS = 1 << tsl >= 8), the tiles
// row-major over the frame (tx per row) or, with mdim > 0, in Morton order over a 2^mdim x 2^mdim grid (tiles outside
// the frame hold no rays), and inside a tile either its 8x8 sub-tiles row-major with their pixels row-major (a pass-0
// wave's footprint), or (zin 1) every pixel in Morton order, or (zin 2) the tile's rows. 2-D neighbourhoods instead
// of frame rows: a queue wave's 64 rays are neighbours in both directions. Only the order of the queue changes, never
// a result.
struct FlagOrder {
    uint32_t W, H, tx, ty, tsl, mdim, zin;
    // a batch of frames (vhx_trace_primary_batch): positions [f * fpos, (f + 1) * fpos) are frame f's, in the order
    // above, and its pixels are output indices [f * fpix, (f + 1) * fpix); fpos = 0: one frame
    uint64_t fpos, fpix;
    // a shadow batch (vhx_trace_shadows_batch): frame f's hit values are the array at fvals[f] (entry i of the batch
    // is fvals[i / fpix][i % fpix]), not one array
    const uint64_t *fvals;
};
__device__ __forceinline__ bool frame_hit(const FlagOrder &o, uint64_t i) {
    const uint64_t f = i / o.fpix;
    return ((const uint32_t *)o.fvals[f])[i - f * o.fpix] != VHX_EMPTY;
}
__device__ __forceinline__ uint32_t compact_bits(uint32_t v) {  // even bits of v -> low half
    v &= 0x55555555u;
    v = (v | (v >> 1)) & 0x33333333u;
    v = (v | (v >> 2)) & 0x0F0F0F0Fu;
    v = (v | (v >> 4)) & 0x00FF00FFu;
    return (v | (v >> 8)) & 0x0000FFFFu;
}
// pixel of position k; false if it lies outside the frame
__device__ __forceinline__ bool order_pixel(const FlagOrder &o, uint64_t k, uint32_t &px, uint32_t &py) {
    const uint32_t t = (uint32_t)(k >> (2u * o.tsl)), r = (uint32_t)k & ((1u << (2u * o.tsl)) - 1u);
    uint32_t gx, gy;
    if (o.mdim) {
        gx = compact_bits(t);
        gy = compact_bits(t >> 1);
    } else {
        gx = t % o.tx;
        gy = t / o.tx;
    }
    uint32_t ix, iy;
    if (o.zin == 2u) {  // rows of the tile
        ix = r & ((1u << o.tsl) - 1u);
        iy = r >> o.tsl;
    } else if (o.zin) {
        ix = compact_bits(r);
        iy = compact_bits(r >> 1);
    } else {
        const uint32_t spr = 1u << (o.tsl - 3u), sub = r >> 6, u = r & 63u;
        ix = (sub % spr) * 8u + (u & 7u);
        iy = (sub / spr) * 8u + (u >> 3);
    }
    px = (gx << o.tsl) + ix;
    py = (gy << o.tsl) + iy;
    return gx < o.tx && gy < o.ty && px < o.W && py < o.H;
}
// output index of position k; false if it names no pixel
__device__ __forceinline__ bool order_index(const FlagOrder &o, uint64_t k, uint64_t &i) {
    uint64_t base = 0;
    if (o.fpos) {
        const uint64_t f = k / o.fpos;
        k -= f * o.fpos;
        base = f * o.fpix;
    }
    uint32_t px, py;
    if (!order_pixel(o, k, px, py)) return false;
    i = base + (uint64_t)py * o.W + px;
    return true;
}
// flags of positions k..k+3 (bit j: position k + j): a pass-0 flag byte, or with HITS a hit value != VHX_EMPTY
template <bool HITS>
__device__ __forceinline__ uint32_t order_bits(const void *src, const FlagOrder &o, uint64_t k) {
    uint32_t bits = 0;
    for (uint32_t j = 0; j < 4u; ++j) {
        uint64_t i;
        if (!order_index(o, k + j, i)) continue;
        // a pass-0 flag byte: 1 = abandoned
        const bool hit = HITS && o.fvals ? frame_hit(o, i) : ((const uint32_t *)src)[i] != VHX_EMPTY;
        if (HITS ? hit : (((const uint8_t *)src)[i] & 1u) != 0) bits |= 1u << j;
    }
    return bits;
}

// hit flags of entries i..i+3 of a shadow batch in output-index order (FlagOrder::fvals)
__device__ __forceinline__ uint32_t frame_bits(const FlagOrder &o, uint64_t i, uint64_t n) {
    uint32_t bits = 0;
    for (uint64_t k = i; k < n && k < i + 4; ++k)
        if (frame_hit(o, k)) bits |= 1u << (k - i);
    return bits;
}

// k_count_flags: the number of set flags per 1024 positions. zero: the queue passes' work counters (qctl[16..79]),
// zeroed here instead of by a separate memset launch; clear (optional, nclear entries): an output array zeroed
// alongside (the shadow flags of a shadow frame)
template <bool HITS>
__global__ void __launch_bounds__(256) k_count_flags(const void *__restrict__ src, uint64_t n,
                                                     uint32_t *__restrict__ counts, uint32_t *zero,
                                                     uint32_t *__restrict__ clear = nullptr, FlagOrder ord = {},
                                                     uint64_t nclear = 0) {
    __shared__ uint32_t s_cnt[4];
    if (blockIdx.x == 0)
        for (uint32_t w = threadIdx.x; w < QCTL_WORDS - 16u; w += blockDim.x) zero[w] = 0u;
    const uint64_t i = ((uint64_t)blockIdx.x * 256u + threadIdx.x) * 4u;
    if (clear)
        for (uint64_t k = i; k < nclear && k < i + 4u; ++k) clear[k] = 0u;
    uint32_t c = __popc(ord.W ? (i < n ? order_bits<HITS>(src, ord, i) : 0u)
                              : (HITS && ord.fvals ? frame_bits(ord, i, n) : flag_bits<HITS>(src, i, n)));
    for (uint32_t d = 32; d > 0; d >>= 1) c += __shfl_down(c, d);
    if ((threadIdx.x & 63u) == 0) s_cnt[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) counts[blockIdx.x] = s_cnt[0] + s_cnt[1] + s_cnt[2] + s_cnt[3];
}

template <bool HITS>
__global__ void __launch_bounds__(256) k_emit_flags(const void *__restrict__ src, uint64_t n,
                                                    const uint32_t *__restrict__ offsets, uint32_t *__restrict__ out,
                                                    FlagOrder ord = {}) {
    __shared__ uint32_t s_wave[4];
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint64_t i = ((uint64_t)blockIdx.x * 256u + threadIdx.x) * 4u;
    const uint32_t bits = ord.W ? (i < n ? order_bits<HITS>(src, ord, i) : 0u)
                                : (HITS && ord.fvals ? frame_bits(ord, i, n) : flag_bits<HITS>(src, i, n));
    const uint32_t c = __popc(bits);
    uint32_t inc = c;
    for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint32_t x = __shfl_up(inc, d);
        if (lane >= d) inc += x;
    }
    if (lane == 63) s_wave[wave] = inc;
    __syncthreads();
    uint32_t o = offsets[blockIdx.x] + inc - c;
    for (uint32_t w = 0; w < wave; ++w) o += s_wave[w];
    for (uint32_t k = 0; k < 4; ++k)
        if (bits & (1u << k)) {
            uint64_t ix = i + k;
            if (ord.W) order_index(ord, i + k, ix);
            out[o++] = (uint32_t)ix;
        }
}

// One wave per chunk: copies the chunk's list to the queue at its offset; in the queue-state mode (st_q) the listed
// rays' saved states too, from their list slots to their queue positions (64 B each, coalesced both ways), so that the
// next pass reads a ray's state at its queue position, in the same load round as its output index.
__global__ void __launch_bounds__(256) k_gather_chunks(const uint32_t *__restrict__ tmp, uint32_t stride,
                                                       const uint32_t *__restrict__ counts,
                                                       const uint32_t *__restrict__ offsets, uint32_t nchunks_host,
                                                       const uint32_t *n_in, uint32_t per_chunk, uint32_t tw,
                                                       uint32_t *__restrict__ out,
                                                       const uint4 *__restrict__ st_slot = nullptr,
                                                       uint4 *__restrict__ st_q = nullptr) {
    const uint32_t pc = n_in ? pass_rpw(per_chunk, tw, *n_in) : per_chunk;
    const uint32_t nchunks = n_in ? (*n_in + pc - 1) / pc : nchunks_host;
    if (n_in) stride = pc;  // a queue pass lists its chunk c at tmp[c * rays per wave]
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t waves = gridDim.x * 4u;
    for (uint32_t c = blockIdx.x * 4u + (threadIdx.x >> 6); c < nchunks; c += waves) {
        const uint32_t n = counts[c], o = offsets[c];
        for (uint32_t k = lane; k < n; k += 64u) out[o + k] = tmp[(uint64_t)c * stride + k];
        if (st_q)
            for (uint32_t k = lane; k < n; k += 64u) {
                const uint4 *src = st_slot + 4ull * ((uint64_t)c * stride + k);
                uint4 *dst = st_q + 4ull * ((uint64_t)o + k);
                const uint4 a = src[0], b = src[1], e = src[2], f = src[3];
                dst[0] = a;
                dst[1] = b;
                dst[2] = e;
                dst[3] = f;
            }
    }
}

// Segment node sort of a queue pass's input (docs/DESIGN_LOG.md §15.3): every segment of `seg` consecutive entries (a power of two
// <= VHX_QSORT_MAX) is reordered by the node each ray's saved state stands at (the NodeStack top, state word 12), ties
// in queue order, so that a wave's 64 rays start their first node iteration together and at the same node loads, while
// the segments keep the queue's 2-D order. Bitonic sort of {node, position} keys in LDS; the queue length is read on the
// device, and the workgroups stride over its segments. Only the order of the queue changes, never a result.
#define QSORT_THREADS 256u
__global__ void __launch_bounds__(QSORT_THREADS) k_sort_segments(uint32_t *__restrict__ q, const uint32_t *n_ptr,
                                                                 const uint32_t *__restrict__ state, uint32_t seg) {
    __shared__ unsigned long long key[VHX_QSORT_MAX];
    __shared__ uint32_t val[VHX_QSORT_MAX];
    const uint32_t n = *n_ptr, t = threadIdx.x;
    for (uint64_t base = (uint64_t)blockIdx.x * seg; base < n; base += (uint64_t)gridDim.x * seg) {
        const uint32_t cnt = (uint32_t)min<uint64_t>(seg, n - base);
        for (uint32_t i = t; i < seg; i += QSORT_THREADS) {
            uint32_t v = 0;
            unsigned long long k = ~0ull;  // past the queue's end: sorts last, never written back
            if (i < cnt) {
                v = q[base + i];
                k = ((unsigned long long)state[16ull * v + 12u] << 32) | i;
            }
            key[i] = k;
            val[i] = v;
        }
        __syncthreads();
        for (uint32_t k = 2; k <= seg; k <<= 1)
            for (uint32_t j = k >> 1; j > 0; j >>= 1) {
                for (uint32_t i = t; i < seg; i += QSORT_THREADS) {
                    const uint32_t l = i ^ j;
                    if (l > i) {
                        const unsigned long long a = key[i], b = key[l];
                        if ((a > b) == ((i & k) == 0u)) {
                            key[i] = b;
                            key[l] = a;
                        }
                    }
                }
                __syncthreads();
            }
        for (uint32_t i = t; i < cnt; i += QSORT_THREADS) q[base + i] = val[(uint32_t)key[i]];
        __syncthreads();
    }
}

// One frame of a shadow batch on the device (vhx_shadow_frame)
struct ShD {
    const uint32_t *value;
    const float *impact, *normal;
    uint32_t *shadowed, *rgba;
};

// Where a queued output index comes from: a primary-ray frame (framebuffer or tile layout) or an explicit ray batch.
struct RaySrc {
    uint32_t kind;  // 0 framebuffer, 1 tiles, 2 explicit rays, 3 shadow rays from hit records, 4 a batch of frames,
                    // 5 a batch of shadow frames
    uint32_t T, tiles_x, tile_start, tile_stride;
    const float *rays;
    const float *impact, *normal;  // kind 3
    float lx, ly, lz;               // kind 3: light position
    // kind 4 (vhx_trace_primary_batch): frame f = idx / npix of the batch has camera cams[f] and outputs outs[f]
    // (framebuffer layout, index idx - f * npix); device arrays of the batch
    const CamD *cams;
    const OutD *outs;
    uint32_t npix;
    const ShD *shs;  // kind 5: frame f = idx / npix is shs[f], entry idx - f * npix
    // kind 4 with T > 0 (vhx_trace_tiles_batch): frame f is the tile set starts[f], starts[f] + tile_stride, ... of
    // T x T tiles (tiles_x per row) in the tile layout; npix = the per-frame index stride (the largest set's entries)
    const uint32_t *starts;
};

// Hard-shadow ray of hit record idx (BASELINE config 5; semantics in docs/DESIGN_LOG.md §9): from impact + normal * 1e-3
// toward the light, direction normalised like V3c::normalized (src/spatial/math/vector.rs).
__device__ __forceinline__ void shadow_ray(const RaySrc &src, uint32_t idx, F3d &o, F3d &d) {
    const float *ip, *np;
    if (src.kind == 5u) {  // a shadow batch: frame f's records
        const uint32_t f = idx / src.npix, local = idx - f * src.npix;
        ip = src.shs[f].impact + 3ull * local;
        np = src.shs[f].normal + 3ull * local;
    } else {
        ip = src.impact + 3ull * idx;
        np = src.normal + 3ull * idx;
    }
    o = mk(ip[0] + np[0] * 1e-3f, ip[1] + np[1] * 1e-3f, ip[2] + np[2] * 1e-3f);
    d = vnorm(mk(src.lx - o.x, src.ly - o.y, src.lz - o.z));
}

__device__ __forceinline__ void ray_of(const CamD &cam, const RaySrc &src, uint32_t idx, F3d &o, F3d &d) {
    if (src.kind == 3u || src.kind == 5u) {
        shadow_ray(src, idx, o, d);
        return;
    }
    if (src.kind == 2u) {
        o = mk(src.rays[6ull * idx], src.rays[6ull * idx + 1], src.rays[6ull * idx + 2]);
        d = mk(src.rays[6ull * idx + 3], src.rays[6ull * idx + 4], src.rays[6ull * idx + 5]);
        return;
    }
    if (src.kind == 4u) {  // a batch: the frame's camera, read where the ray is set up
        const uint32_t f = idx / src.npix, local = idx - f * src.npix;
        const CamD *cf = src.cams + f;
        if (src.T) {  // a batch of tile sets: entry local of frame f's set in the tile layout
            const uint32_t tt = src.T * src.T, j = local / tt, l = local - j * tt;
            const uint32_t tile = src.starts[f] + j * src.tile_stride;
            primary_ray(*cf, (tile % src.tiles_x) * src.T + l % src.T, (tile / src.tiles_x) * src.T + l / src.T, o, d);
            return;
        }
        const uint32_t W = cf->width, py = local / W;
        primary_ray(*cf, local - py * W, py, o, d);
        return;
    }
    uint32_t px, py;
    if (src.kind == 0u) {
        py = idx / cam.width;
        px = idx - py * cam.width;
    } else {
        const uint32_t tt = src.T * src.T;
        const uint32_t j = idx / tt, local = idx - j * tt;
        const uint32_t tile = src.tile_start + j * src.tile_stride;
        px = (tile % src.tiles_x) * src.T + local % src.T;
        py = (tile / src.tiles_x) * src.T + local / src.T;
    }
    primary_ray(cam, px, py, o, d);
}

// XCD-aware block order: the dispatcher deals workgroups round-robin over the 8 XCDs (blockIdx % 8 share one XCD and
// its L2; MI355X_MICROARCH.md, workgroup dispatch), so with G > 0 each XCD's blocks are taken in runs of G
// consecutive frame blocks (neighbouring pixels walk the same nodes and bricks). A bijection on [0, n) for any n (the
// last n mod 8G blocks keep their order); only the speed depends on the placement. G = 0: dispatch order.
__device__ __forceinline__ uint32_t xcd_block(uint32_t bid, uint32_t n, uint32_t G) {
    if (G == 0u) return bid;
    const uint32_t full = n / (8u * G) * (8u * G);
    if (bid >= full) return bid;
    const uint32_t x = bid & 7u, k = bid >> 3;
    return ((k / G) * 8u + x) * G + k % G;
}

// occupancy of the queue kernel (waves per SIMD the register allocation must allow): the queue kernel of brick_dim 1
// and 4 fits 96 VGPRs (5 waves per SIMD instead of 4, no spills under the iterative-ilp scheduler of _build.py);
// brick_dim 2 would spill 4 VGPRs and 8..32 16, so they keep 4 waves (the minimum of 4 compiles to the same code as no
// attribute)
#define VHX_QUEUE_ATTR __attribute__((amdgpu_waves_per_eu(!COUNT && (BD == 1 || BD == 4) ? 5 : 4)))

// One workgroup = 256 lanes = a 16x16 pixel block made of four 8x8 wave tiles (wave64-coherent ray bundles, the
// 8x8 footprint of the reference's @workgroup_size(8, 8, 1)). Blocks are dealt tile by tile.
// Depth-prepass mode (opt-in, not the reference path; SURVEY.md 8f #4, viewport_render.wgsl:702-726): a half-resolution
// depth frame traced first; a full-resolution ray starts at the minimum of the 4 depth texels (x/2, y/2) .. (x/2 + 1,
// y/2 + 1) (clamped at the edge) minus `margin`, and misses outright where that minimum is +inf (all four missed)
struct FastD {
    const float *depth;
    uint32_t w, h;
    float margin;
};
__device__ __forceinline__ float prepass_start(const FastD &f, uint32_t px, uint32_t py) {
    const uint32_t x0 = px >> 1, y0 = py >> 1;
    const uint32_t x1 = x0 + 1 < f.w ? x0 + 1 : f.w - 1, y1 = y0 + 1 < f.h ? y0 + 1 : f.h - 1;
    const float m = __builtin_fminf(__builtin_fminf(f.depth[(uint64_t)y0 * f.w + x0], f.depth[(uint64_t)y1 * f.w + x0]),
                                    __builtin_fminf(f.depth[(uint64_t)y0 * f.w + x1], f.depth[(uint64_t)y1 * f.w + x1]));
    return m - f.margin;
}

// Pass 0's abandoned rays listed per workgroup in the order of the pass-1 queue (ListOrder, lo.tx > 0; the
// framebuffer layout): workgroup position b is block (bx, by) of a tile of 2^tbl x 2^tbl blocks, the tiles row-major
// (tx per row), the blocks of a tile and the pixels of a block in Morton order -- the 16x16 block's four 8x8 waves are
// its Morton quadrants, and lane l is pixel (even bits of l, odd bits of l) of its wave's 8x8 -- so the lists in
// position order are the frame's abandoned rays in the FlagOrder of 2^(tbl+4)-pixel tiles with Morton inside (zin 1),
// without a flag per pixel and the compaction kernels over every pixel. A wave holds the same 64 pixels either way.
struct ListOrder {
    uint32_t tx, tbl;
    // tl = 1: the tile layout (a rank's tile set, vhx_mgpu) lists its abandoned rays too, in its own block order --
    // tile by tile, 16x16 blocks row-major inside a tile, a block's four 8x8 waves, each wave's 64 pixels row-major:
    // the queue order of its flags (output-index order) up to the order of the waves inside a 16x16 block
    uint32_t tl;
};
__device__ __forceinline__ void list_block(const ListOrder &lo, uint32_t b, uint32_t &bx, uint32_t &by) {
    const uint32_t tb = b >> (2u * lo.tbl), m = b & ((1u << (2u * lo.tbl)) - 1u);
    bx = ((tb % lo.tx) << lo.tbl) + compact_bits(m);
    by = ((tb / lo.tx) << lo.tbl) + compact_bits(m >> 1);
}
// Wave-level ordered append (no barrier: a wave that finishes early leaves at once): the wave's rays with push set are
// listed at tmp[pos * 64 ...] in lane order, their number at counts[pos].
__device__ __forceinline__ void wave_append(bool push, uint32_t idx, uint32_t *tmp, uint32_t *counts, uint32_t pos) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t m = __ballot(push);
    if (push) tmp[(uint64_t)pos * 64u + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = idx;
    if (lane == 0) counts[pos] = (uint32_t)__popcll(m);
}
__device__ __forceinline__ void zero_ctl(uint32_t *zero) {
    if (zero && blockIdx.x == 0)
        for (uint32_t w = threadIdx.x; w < QCTL_WORDS - 16u; w += blockDim.x) zero[w] = 0u;
}

// Fused hard shadows (vhx_set_shadow_light; the FUSE instantiations, BASELINE config 5): a lane whose primary ray
// finished goes on, in the same pass, with the hit's shadow ray -- the shadow semantics of vhx_trace_shadows (from
// impact + normal * 1e-3 toward the light) -- while the nodes of the hit's descent are still in this
// CU's caches. A shadow ray abandoned at the pass budget saves its state at its pixel's index (the primary ray's is
// done by then) and is listed with VHX_QSHADOW; a queue pass recomputes its ray from the stored hit record.
#define VHX_QSHADOW 0x80000000u
__device__ __forceinline__ void hit_shadow_ray(const PassQ &q, float ix, float iy, float iz, float nx, float ny,
                                               float nz, F3d &o, F3d &d) {
    o = mk(ix + nx * 1e-3f, iy + ny * 1e-3f, iz + nz * 1e-3f);  // shadow_ray's op order
    d = vnorm(mk(q.lx - o.x, q.ly - o.y, q.lz - o.z));
}
__device__ __forceinline__ void store_fused_shadow(const OutD &o, uint64_t i, bool shadowed) {
    o.shadowed[i] = shadowed ? 1u : 0u;  // store_shadow's darkening
    if (shadowed && o.rgba) o.rgba[i] = ((o.rgba[i] >> 1) & 0x007F7F7Fu) | (o.rgba[i] & 0xFF000000u);
}
// the steps a pass's budget leaves a shadow ray started after a primary ray that used `used` of them (at least 1;
// any split is bit-identical, the traversal being deterministic)
__device__ __forceinline__ uint32_t rest_budget(uint32_t budget, uint32_t used) {
    return budget >= VHX_MAX_ITERS ? budget : (budget > used + 1u ? budget - used : 1u);
}
// the shadow continuation of a finished primary ray h (output entry li of o, state index sidx); false: abandoned
template <int BD>
__device__ __forceinline__ bool fused_shadow(const DevTree &t, const uint64_t *occ_tab, const PassQ &q, const OutD &o,
                                             uint64_t li, const HitOut &h, uint32_t sidx) {
    if (!h.hit) {
        o.shadowed[li] = 0u;
        return true;
    }
    F3d so, sd;
    hit_shadow_ray(q, h.ix, h.iy, h.iz, h.nx, h.ny, h.nz, so, sd);
    HitOut hs;
    hs.bytes = 0;
    const bool fin =
        get_by_ray<false, BD>(t, occ_tab, so, sd, hs,
                              q.sbud && q.budget < VHX_MAX_ITERS ? q.sbud : rest_budget(q.budget, h.iters), q.state,
                              sidx, false, 0.0f, q.sparse);
    if (fin) store_fused_shadow(o, li, hs.hit);
    return fin;
}

template <bool COUNT, int BD, bool FAST = false, bool MIP = false, bool FUSE = false>
__global__ void __launch_bounds__(256) k_trace_primary(DevTree t, CamD cam, OutD out, uint32_t T, uint32_t tiles_x,
                                                       uint32_t tile_start, uint32_t tile_stride, uint32_t layout,
                                                       uint32_t blocks_per_tile_x, uint32_t blocks_per_tile,
                                                       PassQ q, FastD fast = FastD{}, ListOrder lo = ListOrder{}) {
    __shared__ uint64_t occ_tab[OCC_TAB_WORDS];
    fill_occ_tab(occ_tab);
    zero_ctl(q.zero);
    __syncthreads();
    const uint32_t bid = xcd_block(blockIdx.x, gridDim.x, q.xcd_group);
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    uint32_t lx, ly, px, py;
    if (lo.tx) {  // framebuffer layout (T = 16: a tile per block), workgroups in list order
        uint32_t bx, by;
        list_block(lo, bid, bx, by);
        lx = (wave & 1u) * 8u + compact_bits(lane);
        ly = (wave >> 1) * 8u + compact_bits(lane >> 1);
        px = bx * 16u + lx;
        py = by * 16u + ly;
    } else {
        const uint32_t j = bid / blocks_per_tile;  // j-th tile of this rank
        const uint32_t sb = bid - j * blocks_per_tile;
        const uint32_t tile = tile_start + j * tile_stride;
        // 8x8 pixels per wave, four waves per 16x16 block
        lx = (sb % blocks_per_tile_x) * 16u + (wave & 1u) * 8u + (lane & 7u);
        ly = (sb / blocks_per_tile_x) * 16u + (wave >> 1) * 8u + (lane >> 3);
        px = (tile % tiles_x) * T + lx;
        py = (tile / tiles_x) * T + ly;
    }
    const uint32_t j = lo.tx ? 0u : bid / blocks_per_tile;
    const bool valid = lx < T && ly < T && px < cam.width && py < cam.height;
    const uint64_t idx = layout == VHX_LAYOUT_FRAMEBUFFER ? (uint64_t)py * cam.width + px
                                                          : (uint64_t)j * T * T + (uint64_t)ly * T + lx;
    bool done = true;
    uint32_t tag = 0u;  // FUSE: VHX_QSHADOW when the ray left over is the hit's shadow ray
    // the early tail traces the pixels in q.skip (its kernel stores them): done here, no store, no flag
    const bool skipped = valid && q.skip && ((q.skip[idx >> 5] >> (idx & 31u)) & 1u) != 0u;
    if (valid && !skipped) {
        F3d o, d;
        HitOut h;
        h.bytes = 0;
        if (glass_clear_miss(cam, px, py, (float)t.size)) {  // the miss record, as get_by_ray's root test gives it
            o = mk(cam.ox, cam.oy, cam.oz);
            h.hit = false;
            h.iters = 0;
        } else {
            primary_ray(cam, px, py, o, d);
            const float start = FAST ? prepass_start(fast, px, py) : 0.0f;
            // queue-state mode (listed pass 0 only): this wave's abandoned rays take the slots of its list
            done = get_by_ray<COUNT, BD, FAST, MIP>(t, occ_tab, o, d, h, q.budget, q.state,
                                                    q.qmode ? (bid * 4u + wave) * 64u : (uint32_t)idx, false, start,
                                                    q.sparse, nullptr, 0, q.qmode != 0);
        }
        if (done) {
            store(t, out, idx, o, h);
            if (FUSE && !fused_shadow<BD>(t, occ_tab, q, out, idx, h, (uint32_t)idx)) {
                done = false;
                tag = VHX_QSHADOW;
            }
        } else if (COUNT && q.state) {
            out.bytes[idx] = h.bytes;  // the running count, continued by the pass that resumes the ray
        }
    }
    // every entry of the output gets its flag, so the flags need no clearing between frames: in the tile layout
    // every in-tile entry (frame padding included, done = true there); in the framebuffer layout only pixels of the
    // frame (a lane past the frame edge has no entry of its own: its idx aliases the next row or runs past the end)
    if (q.flags && (layout == VHX_LAYOUT_FRAMEBUFFER ? valid : (lx < T && ly < T)))
        q.flags[idx] = done ? 0 : 1;
    if ((lo.tx || lo.tl) && q.tmp) wave_append(!done, (uint32_t)idx | tag, q.tmp, q.counts, bid * 4u + wave);
}

// Pass 0 of a batch of frames (vhx_trace_primary_batch): frame f's 16x16 pixel blocks are blocks [f * nblocks_frame,
// (f + 1) * nblocks_frame) of one launch (XCD-dealt like k_trace_primary), with the frame's camera and outputs read from
// the batch arrays (block-uniform: scalar loads). Framebuffer layout; output index f * npix + y * width + x.
// A batch of tile sets (vhx_trace_tiles_batch; tb.T > 0): frame f's blocks cover the T x T tiles starts[f] +
// j * stride, j < the largest set's tile count, 16x16 blocks row-major inside a tile (k_trace_primary's tile layout);
// output index f * npix + j * T * T + y * T + x inside the tile.
struct TileB {
    uint32_t T, tiles_x, ntiles, stride, bpx, bpt;
    const uint32_t *starts;
};
// VHX_BATCH_WAVES (a variant build): waves per SIMD the batch pass 0 must allow (0: the compiler's choice, 72 VGPRs
// for brick_dim 4 = 7 waves)
#ifndef VHX_BATCH_WAVES
#define VHX_BATCH_WAVES 0
#endif
#if VHX_BATCH_WAVES
#define VHX_BATCH_ATTR __attribute__((amdgpu_waves_per_eu(VHX_BATCH_WAVES)))
#else
#define VHX_BATCH_ATTR
#endif
template <int BD, bool FUSE = false>
__global__ void __launch_bounds__(256) VHX_BATCH_ATTR k_trace_primary_batch(DevTree t, const CamD *__restrict__ cams,
                                                             const OutD *__restrict__ outs, uint32_t nblocks_frame,
                                                             uint32_t blocks_x, uint32_t npix, PassQ q,
                                                             ListOrder lo = ListOrder{}, TileB tb = TileB{}) {
    __shared__ uint64_t occ_tab[OCC_TAB_WORDS];
    fill_occ_tab(occ_tab);
    zero_ctl(q.zero);
    __syncthreads();
    const uint32_t bid = xcd_block(blockIdx.x, gridDim.x, q.xcd_group);
    // frame-major (all of frame 0's blocks, then frame 1's, ...) or interleaved (block sb of every frame in turn: the
    // frames' rays through one screen region run together and share the caches)
    const uint32_t nfr = gridDim.x / nblocks_frame;
    const uint32_t f = q.finter ? bid % nfr : bid / nblocks_frame;
    const uint32_t sb = q.finter ? bid / nfr : bid - f * nblocks_frame;
    const CamD cam = cams[f];
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    uint32_t px, py, local;
    bool valid, entry;  // entry: the position has an output entry (its flag is written)
    if (tb.T) {
        const uint32_t j = sb / tb.bpt, sbb = sb - j * tb.bpt;
        const uint32_t lx = (sbb % tb.bpx) * 16u + (wave & 1u) * 8u + (lane & 7u);
        const uint32_t ly = (sbb / tb.bpx) * 16u + (wave >> 1) * 8u + (lane >> 3);
        const uint32_t tile = tb.starts[f] + j * tb.stride;
        px = (tile % tb.tiles_x) * tb.T + lx;
        py = (tile / tb.tiles_x) * tb.T + ly;
        entry = lx < tb.T && ly < tb.T;
        valid = entry && tile < tb.ntiles && px < cam.width && py < cam.height;
        local = (j * tb.T + ly) * tb.T + lx;
    } else {
        if (lo.tx) {  // this frame's blocks in list order (k_trace_primary)
            uint32_t bx, by;
            list_block(lo, sb, bx, by);
            px = bx * 16u + (wave & 1u) * 8u + compact_bits(lane);
            py = by * 16u + (wave >> 1) * 8u + compact_bits(lane >> 1);
        } else {
            px = (sb % blocks_x) * 16u + (wave & 1u) * 8u + (lane & 7u);
            py = (sb / blocks_x) * 16u + (wave >> 1) * 8u + (lane >> 3);
        }
        valid = entry = px < cam.width && py < cam.height;
        local = py * cam.width + px;
    }
    const uint64_t idx = (uint64_t)f * npix + local;
    bool done = true;
    uint32_t tag = 0u;  // FUSE: VHX_QSHADOW when the ray left over is the hit's shadow ray
    if (valid) {
        F3d o, d;
        HitOut h;
        h.bytes = 0;
        if (glass_clear_miss(cam, px, py, (float)t.size)) {  // k_trace_primary
            o = mk(cam.ox, cam.oy, cam.oz);
            h.hit = false;
            h.iters = 0;
        } else {
            primary_ray(cam, px, py, o, d);
            done = get_by_ray<false, BD>(t, occ_tab, o, d, h, q.budget, q.state,
                                         q.qmode ? (bid * 4u + wave) * 64u : (uint32_t)idx, false, 0.0f, q.sparse,
                                         nullptr, 0, q.qmode != 0);
        }
        if (done) {
            store(t, outs[f], local, o, h);
            if (FUSE && !fused_shadow<BD>(t, occ_tab, q, outs[f], local, h, (uint32_t)idx)) {
                done = false;
                tag = VHX_QSHADOW;
            }
        }
    }
    // every entry gets its flag (a tile set's entries past the frame edge or past a smaller set's tiles: 0)
    if (q.flags && entry) q.flags[idx] = done ? 0 : 1;
    if ((lo.tx || lo.tl) && q.tmp) wave_append(!done, (uint32_t)idx | tag, q.tmp, q.counts, bid * 4u + wave);
}

template <bool COUNT, int BD, bool MIP = false>
__global__ void __launch_bounds__(256) k_trace_rays(DevTree t, const float *__restrict__ rays, uint64_t n, OutD out,
                                                    PassQ q) {
    __shared__ uint64_t occ_tab[OCC_TAB_WORDS];
    fill_occ_tab(occ_tab);
    __syncthreads();
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool done = true;
    if (i < n) {
        const F3d o = mk(rays[6 * i], rays[6 * i + 1], rays[6 * i + 2]);
        const F3d d = mk(rays[6 * i + 3], rays[6 * i + 4], rays[6 * i + 5]);
        HitOut h;
        h.bytes = 0;
        done = get_by_ray<COUNT, BD, false, MIP>(t, occ_tab, o, d, h, q.budget, q.state, (uint32_t)i);
        if (done)
            store(t, out, i, o, h);
        else if (COUNT && q.state)
            out.bytes[i] = h.bytes;
    }
    if (q.tmp) block_append(!done, (uint32_t)i, q.tmp, q.counts, blockIdx.x);
}


#if VHX_CHAIN
// One ray per wave (lane 0; a workgroup of one wave per ray), traced whole with the chain stamps (trace.hpp,
// VHX_CHAIN): per ray VHX_CHAIN_WORDS words -- [0] cycles of the traversal, [1] node-load waits, [2] probes, [3] POP /
// PUSH bookkeeping, [4] ADVANCE walks, [5] loop overhead, [6] node iterations, [7] probes, [8] ADVANCE walks,
// [9] steps, [10] hit value, [16..16+VHX_CHAIN_HIST) node-load wait histogram (64-cycle buckets)
#define VHX_CHAIN_WORDS 64u
template <int BD>
__global__ void __launch_bounds__(64) k_chain(DevTree t, CamD cam, const uint32_t *__restrict__ pix, uint32_t n,
                                              unsigned long long *__restrict__ out) {
    __shared__ uint64_t occ_tab[OCC_TAB_WORDS];
    fill_occ_tab(occ_tab);
    __syncthreads();
    if (threadIdx.x != 0 || blockIdx.x >= n) return;
    const uint32_t idx = pix[blockIdx.x], py = idx / cam.width, px = idx - py * cam.width;
    F3d o, d;
    primary_ray(cam, px, py, o, d);
    HitOut h;
    h.bytes = 0;
    h.chain = ChainAcc{};
    const unsigned long long t0 = chain_stamp();
    get_by_ray<false, BD>(t, occ_tab, o, d, h, VHX_MAX_ITERS);
    const unsigned long long t1 = chain_stamp();
    unsigned long long *w = out + (uint64_t)blockIdx.x * VHX_CHAIN_WORDS;
    const unsigned long long v[11] = {t1 - t0,        h.chain.load,   h.chain.probe, h.chain.move,
                                      h.chain.adv,    h.chain.other,  h.chain.nload, h.chain.nprobe,
                                      h.chain.nadv,   h.iters,        h.hit ? h.value : VHX_EMPTY};
    for (uint32_t k = 0; k < 11u; ++k) w[k] = v[k];
    for (uint32_t k = 0; k < VHX_CHAIN_HIST; ++k) w[16 + k] = h.chain.hist[k];
}
#endif

// Queue pass: each wave takes 64 consecutive queue entries at a time from a shared counter until the queue written
// by the previous pass is drained (its length is read on the device; the host never synchronises between passes).
// Store of a shadow ray's result: shadowed flag (in out.value), rgb halved in place when shadowed, byte count.
__device__ __forceinline__ void store_shadow(const OutD &o, uint64_t i, const HitOut &h) {
    o.value[i] = h.hit ? 1u : 0u;
    if (o.rgba && h.hit) o.rgba[i] = ((o.rgba[i] >> 1) & 0x007F7F7Fu) | (o.rgba[i] & 0xFF000000u);
    if (o.bytes) o.bytes[i] = h.bytes;
}

// Camera, ray source and outputs of a queue pass: read through a pointer where a wave picks up or stores a ray, so
// they do not occupy scalar registers across the traversal (as kernel arguments they did, and spilled ~100 SGPRs)
struct QueueArgs {
    CamD cam;
    RaySrc src;
    OutD out;
};
__global__ void k_put_queue_args(QueueArgs a, QueueArgs *dst) {
    if (threadIdx.x == 0) *dst = a;
}

// QM: the queue-state mode (PassQ::qmode) as a separate instantiation: carried as a run-time flag, its state pointers
// and slot indices cost the default kernel 2 VGPRs and 4 spilled ones
template <bool COUNT, int BD, bool MIP = false, bool FUSE = false, bool QM = false>
__global__ void __launch_bounds__(256) VHX_QUEUE_ATTR k_trace_queue(DevTree t, const QueueArgs *qa, const uint32_t *__restrict__ in,
                                                     const uint32_t *in_n, uint32_t *grab, PassQ q) {
    __shared__ uint64_t occ_tab[OCC_TAB_WORDS];
    fill_occ_tab(occ_tab);
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t n = *in_n;
    const uint32_t rpw = pass_rpw(q.rpw, q.tw, n);
    // q.qxcd = G > 0: chunk runs of G are dealt round-robin over the XCDs (blockIdx % 8 runs on one XCD and shares
    // its L2), each XCD's waves take its runs in order from their own counter (grab[64 (x + 1)]) and move on to the next
    // XCD's runs once theirs are taken
    uint32_t xcd = blockIdx.x & 7u, tries = 0;
    // only a queue with more chunks than waves is dealt over the XCDs (a smaller one starts every chunk at once
    // anyway and measured slower dealt)
    const uint32_t qxcd = (n + rpw - 1) / rpw > gridDim.x * (blockDim.x / 64u) ? q.qxcd : 0u;
    for (;;) {
        uint32_t base = 0;
        if (qxcd == 0u) {
            if (lane == 0) base = atomicAdd(grab, rpw);
            base = __shfl(base, 0);
            if (base >= n) break;  // wave-uniform
        } else {
            const uint32_t G = qxcd;
            const uint32_t nch = (n + rpw - 1) / rpw, nfull = nch / G, rem = nch % G;
            uint32_t chunk = 0xFFFFFFFFu;
            while (tries < 8u) {
                // XCD xcd owns runs xcd, xcd + 8, ...: kmax of its takes are valid (the last run may be partial); an
                // exhausted counter is recognised by a plain load, so finished waves do not queue atomics on it
                const uint32_t kmax = (nfull > xcd ? (nfull - xcd + 7u) / 8u : 0u) * G +
                                      (rem > 0u && nfull % 8u == xcd ? rem : 0u);
                uint32_t k = 0xFFFFFFFFu;
                uint32_t *ctr = grab + 64u * (xcd + 1u);
                if (lane == 0 && __atomic_load_n(ctr, __ATOMIC_RELAXED) < kmax) k = atomicAdd(ctr, 1u);
                k = __builtin_amdgcn_readfirstlane(__shfl(k, 0));
                if (k < kmax) {
                    chunk = ((k / G) * 8u + xcd) * G + k % G;
                    break;
                }
                xcd = (xcd + 1u) & 7u;
                ++tries;
            }
            if (chunk == 0xFFFFFFFFu) break;
            base = chunk * rpw;
        }
        const uint32_t i = base + lane;
        bool push = false;
        uint32_t idx = 0, tag = 0;
        if (lane < rpw && i < n) {
            idx = in[i];
            F3d o, d;
            const QueueArgs *a = qa;
            asm volatile("" : "+s"(a));  // loads through `a` stay here (not hoisted into live registers)
            // FUSE: the entry's frame outputs (a batch's frame, or the frame's); a shadow entry's ray from its hit record
            bool sh = false;
            OutD fo{};
            uint64_t li = 0;
            if (FUSE) {
                sh = (idx & VHX_QSHADOW) != 0u;
                idx &= ~VHX_QSHADOW;
                if (a->src.kind == 4u) {
                    const uint32_t f = idx / a->src.npix;
                    fo = a->src.outs[f];
                    li = idx - f * a->src.npix;
                } else {
                    fo = a->out;
                    li = idx;
                }
            }
            if (FUSE && sh)
                hit_shadow_ray(q, fo.impact[3 * li], fo.impact[3 * li + 1], fo.impact[3 * li + 2], fo.normal[3 * li],
                               fo.normal[3 * li + 1], fo.normal[3 * li + 2], o, d);
            else
                ray_of(a->cam, a->src, idx, o, d);
            HitOut h;
            h.bytes = COUNT && q.resume ? a->out.bytes[idx] : 0u;
            // queue-state mode: resumed from queue position i, abandoned into this chunk's list slots (base = chunk *
            // rays per wave, the chunk's list position)
            const bool fin = get_by_ray<COUNT, BD, false, MIP>(
                t, occ_tab, o, d, h, q.budget, q.state, QM ? base : idx, q.resume != 0, 0.0f, q.sparse,
                QM ? q.sin : nullptr, QM ? i : 0u, QM && q.tmp);
            const QueueArgs *b = qa;
            asm volatile("" : "+s"(b));
            if (!fin) {
                push = true;
                tag = FUSE && sh ? VHX_QSHADOW : 0u;
                if (COUNT && q.state) b->out.bytes[idx] = h.bytes;
            } else if (FUSE) {
                if (sh) {
                    store_fused_shadow(fo, li, h.hit);
                } else {  // a primary ray finished here: its shadow ray goes on in this lane
                    store(t, fo, li, o, h);
                    if (!fused_shadow<BD>(t, occ_tab, q, fo, li, h, idx)) {
                        push = true;
                        tag = VHX_QSHADOW;
                    }
                }
            } else if (b->src.kind == 3u) {
                store_shadow(b->out, idx, h);
            } else if (b->src.kind == 5u) {
                const uint32_t f = idx / b->src.npix;
                OutD so{};
                so.value = b->src.shs[f].shadowed;
                so.rgba = b->src.shs[f].rgba;
                store_shadow(so, idx - f * b->src.npix, h);
            } else if (b->src.kind == 4u) {
                const uint32_t f = idx / b->src.npix;
                store(t, b->src.outs[f], idx - f * b->src.npix, o, h);
            } else {
                store(t, b->out, idx, o, h);
                if (q.tail_out && h.iters >= q.tail_min) tail_record(q.tail_out, q.tail_cap, idx);
            }
        }
        if (q.tmp) {  // this chunk's abandoned rays, in lane order
            const uint32_t chunk = base / rpw;
            const uint64_t m = __ballot(push);
            if (push) q.tmp[(uint64_t)chunk * rpw + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = idx | tag;
            if (lane == 0) q.counts[chunk] = (uint32_t)__popcll(m);
        }
    }
}

// Early tail (vhx_ctx::tail_*): the pixels of a recorded list as bits of the frame's skip mask (cleared before)
__global__ void k_tail_mask(const uint32_t *__restrict__ list, uint32_t cap, uint32_t npix, uint32_t *mask) {
    const uint32_t n = min(list[0], cap);
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint32_t idx = list[64u + i];
        if (idx < npix) atomicOr(mask + (idx >> 5), 1u << (idx & 31u));
    }
}

// Early tail: the listed pixels of a framebuffer frame traced to the end from the start of the frame, rpw to a wave
// (entry i of the list in wave i / rpw), on the context's second stream while pass 0 skips them; each still-long ray
// is listed again for the next lone frame. Same ray, traversal and store as k_trace_primary + the queue passes.
template <int BD>
__global__ void __launch_bounds__(256) k_trace_tail(DevTree t, CamD cam, OutD out, const uint32_t *__restrict__ list,
                                                    uint32_t *next, uint32_t cap, uint32_t tail_min, uint32_t rpw,
                                                    uint32_t prio) {
    __shared__ uint64_t occ_tab[OCC_TAB_WORDS];
    fill_occ_tab(occ_tab);
    __syncthreads();
    // issue priority of these waves over the frame's other waves on their SIMD (a serial chain is what they carry)
    if (prio == 3u) __builtin_amdgcn_s_setprio(3);
    else if (prio == 2u) __builtin_amdgcn_s_setprio(2);
    else if (prio == 1u) __builtin_amdgcn_s_setprio(1);
    const uint32_t n = min(list[0], cap);
    const uint32_t lane = threadIdx.x & 63u, wave = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const uint32_t i = wave * rpw + lane;
    if (lane >= rpw || i >= n) return;
    const uint32_t idx = list[64u + i];
    if (idx >= cam.width * cam.height) return;
    const uint32_t px = idx % cam.width, py = idx / cam.width;
    F3d o, d;
    HitOut h;
    h.bytes = 0;
    if (glass_clear_miss(cam, px, py, (float)t.size)) {
        o = mk(cam.ox, cam.oy, cam.oz);
        h.hit = false;
        h.iters = 0;
    } else {
        primary_ray(cam, px, py, o, d);
        get_by_ray<false, BD>(t, occ_tab, o, d, h, VHX_MAX_ITERS, nullptr, 0u, false, 0.0f, 0u);
    }
    store(t, out, idx, o, h);
    if (h.iters >= tail_min) tail_record(next, cap, idx);
}

// Scatters rank-gathered tile buffers into framebuffers. Rank r's part of `gathered` holds `planes` planes of
// tiles_per_rank*T*T words each (plane 0 RGBA8, plane 1 f32 depth bits), rank r traced tiles r, r + ranks, ...
__global__ void __launch_bounds__(256) k_untile_planes(const uint32_t *__restrict__ gathered, uint32_t planes,
                                                       uint32_t ranks, uint32_t tiles_per_rank, uint32_t T,
                                                       uint32_t tiles_x, uint32_t ntiles, uint32_t width,
                                                       uint32_t height, uint32_t *__restrict__ fb0,
                                                       uint32_t *__restrict__ fb1) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t per_plane = (uint64_t)tiles_per_rank * T * T, per_rank = per_plane * planes;
    if (i >= per_rank * ranks) return;
    const uint32_t r = (uint32_t)(i / per_rank);
    const uint64_t w = i - (uint64_t)r * per_rank;
    const uint32_t plane = (uint32_t)(w / per_plane);
    const uint64_t k = w - (uint64_t)plane * per_plane;
    uint32_t *fb = plane ? fb1 : fb0;
    if (!fb) return;
    const uint32_t j = (uint32_t)(k / ((uint64_t)T * T));
    const uint32_t local = (uint32_t)(k - (uint64_t)j * T * T);
    const uint32_t tile = r + j * ranks;
    if (tile >= ntiles) return;
    const uint32_t px = (tile % tiles_x) * T + local % T, py = (tile / tiles_x) * T + local / T;
    if (px >= width || py >= height) return;
    fb[(uint64_t)py * width + px] = gathered[i];
}

// ------------------------------------------------------------------------------------------------ host helpers
template <int V>
struct BdTag {
    static constexpr int value = V;
};
// brick_dim is a template parameter of the traversal kernels (exact / brick_dim as a constant multiply)
template <class F>
static bool dispatch_bd(uint32_t bd, F &&f) {
    switch (bd) {
        case 1: f(BdTag<1>{}); return true;
        case 2: f(BdTag<2>{}); return true;
        case 4: f(BdTag<4>{}); return true;
        case 8: f(BdTag<8>{}); return true;
        case 16: f(BdTag<16>{}); return true;
        case 32: f(BdTag<32>{}); return true;
        default: return false;
    }
}
static DevTree dev_tree(const vhx_ctx *c) {
    DevTree t;
    t.hdr = (const uint4 *)c->tree->hdr.ptr;
    t.children = (const uint32_t *)c->tree->raw[VHX_BUF_NODE_CHILDREN].ptr;
    t.voxels = (const uint32_t *)c->tree->raw[VHX_BUF_VOXELS].ptr;
    t.brick_occ = (const uint64_t *)c->tree->brick_occ.ptr;
    t.child_rec = (const uint4 *)c->tree->child_rec.ptr;
    t.solid = (const uint32_t *)c->tree->raw[VHX_BUF_SOLID_VALUES].ptr;
    t.color = (const uint32_t *)c->tree->raw[VHX_BUF_COLOR_PALETTE].ptr;
    t.color_count = c->tree->desc.color_count;
    t.node_count = c->tree->desc.node_count;
    t.size = c->tree->desc.boxtree_size;
    t.bd = c->tree->desc.brick_dim;
    t.occ_words = c->tree->occ_words;
    t.mips = c->tree->mips_on ? (const uint32_t *)c->tree->mips.ptr : nullptr;
    return t;
}

TreeStore::~TreeStore() {
    (void)hipSetDevice(device);
    if (write_ev) (void)hipEventDestroy(write_ev);
    for (auto &b : raw)
        if (b.ptr) (void)hipFree(b.ptr);
    for (DevBuf *b : {&hdr, &brick_occ, &child_rec, &mips})
        if (b->ptr) (void)hipFree(b->ptr);
}

int vhx::ensure(vhx_ctx *c, DevBuf &b, uint64_t bytes) {
    if (b.bytes >= bytes && b.ptr) return VHX_OK;
    if (b.ptr) VHX_HIP(c, hipFree(b.ptr));
    b.ptr = nullptr;
    b.bytes = 0;
    if (bytes == 0) bytes = 16;
    VHX_HIP(c, hipMalloc(&b.ptr, bytes));
    b.bytes = bytes;
    return VHX_OK;
}

// ---- tree-write ordering (TreeStore): frames in flight on shared contexts and writes through the owner ----------
// VHX_UNORDERED_WRITES=1 (a diagnostic build only, never the shipped library: voxelhex_amd._build.build(defines=
// ("VHX_UNORDERED_WRITES=1",), lib=...)): no waits either way, the behaviour before round 3, to show that
// tests/test_gpu_ordering.py detects the missing ordering
#ifndef VHX_UNORDERED_WRITES
#define VHX_UNORDERED_WRITES 0
#endif
static constexpr bool unordered_writes() { return VHX_UNORDERED_WRITES != 0; }

// Writes and traces of one tree may come from several host threads (one per context): a write waits until no trace is
// between trace_begin and trace_end (a trace in submission is not yet visible in its use event), and a trace waits
// until no write is between write_begin and write_end, so every frame sees the tree as of its submission.
int vhx::write_begin(vhx_ctx *c) {
    TreeStore &ts = *c->tree;
    std::unique_lock<std::mutex> lock(ts.mu);
    // a waiting writer holds off traces that have not begun yet (trace_begin waits while writers_waiting > 0), so that
    // a stream of back-to-back traces from other threads cannot keep `tracing` above 0 forever
    ++ts.writers_waiting;
    ts.cv.wait(lock, [&] { return ts.tracing == 0 && ts.writing == 0; });
    --ts.writers_waiting;
    ++ts.writing;
    if (unordered_writes()) return VHX_OK;
    // every other context's last submitted trace, whatever stream it went to (waiting on an event of c's own stream is
    // a no-op, so no stream comparison: a context moved between streams by vhx_set_stream is still waited for)
    for (vhx_ctx *u : ts.users)
        if (u != c && u->use_recorded) VHX_HIP(c, hipStreamWaitEvent(c->stream, u->use_ev, 0));
    // a write on another stream than the previous write also follows it (writes are ordered among themselves)
    if (ts.write_seq && ts.write_stream != c->stream) VHX_HIP(c, hipStreamWaitEvent(c->stream, ts.write_ev, 0));
    return VHX_OK;
}

int vhx::write_end(vhx_ctx *c) {
    TreeStore &ts = *c->tree;
    std::lock_guard<std::mutex> lock(ts.mu);
    ts.writing = ts.writing > 0 ? ts.writing - 1 : 0;
    ts.cv.notify_all();
    // recorded on every exit (also after a failed write: the next traces wait for whatever it enqueued)
    if (!ts.write_ev) VHX_HIP(c, hipEventCreateWithFlags(&ts.write_ev, hipEventDisableTiming));
    VHX_HIP(c, hipEventRecord(ts.write_ev, c->stream));
    ts.write_stream = c->stream;
    ++ts.write_seq;
    c->seen_write = ts.write_seq;
    return VHX_OK;
}

int vhx::trace_begin(vhx_ctx *c) {
    TreeStore &ts = *c->tree;
    std::unique_lock<std::mutex> lock(ts.mu);
    ts.cv.wait(lock, [&] { return ts.writing == 0 && ts.writers_waiting == 0; });
    ++ts.tracing;
    if (unordered_writes()) return VHX_OK;
    if (c->seen_write != ts.write_seq) {
        if (ts.write_stream != c->stream) VHX_HIP(c, hipStreamWaitEvent(c->stream, ts.write_ev, 0));
        c->seen_write = ts.write_seq;
    }
    return VHX_OK;
}

int vhx::trace_end(vhx_ctx *c) {
    TreeStore &ts = *c->tree;
    std::lock_guard<std::mutex> lock(ts.mu);  // write_begin reads use_recorded / waits on use_ev
    ts.tracing = ts.tracing > 0 ? ts.tracing - 1 : 0;
    ts.cv.notify_all();
    if (!c->use_ev) VHX_HIP(c, hipEventCreateWithFlags(&c->use_ev, hipEventDisableTiming));
    VHX_HIP(c, hipEventRecord(c->use_ev, c->stream));
    c->use_stream = c->stream;
    c->use_recorded = true;
    return VHX_OK;
}

static void register_user(vhx_ctx *c) {
    std::lock_guard<std::mutex> lock(c->tree->mu);
    c->tree->users.push_back(c);
    c->seen_write = 0;  // the first trace waits for the tree's last write (if any, and on another stream)
}

static void unregister_user(vhx_ctx *c) {
    std::lock_guard<std::mutex> lock(c->tree->mu);
    auto &u = c->tree->users;
    u.erase(std::remove(u.begin(), u.end(), c), u.end());
}

void vhx::pack_counts(const vhx_tree_desc &d, uint32_t counts[8]) {
    const uint32_t v[8] = {d.boxtree_size, d.brick_dim, d.node_count, d.brick_count,
                           d.solid_count, d.color_count, d.data_count, 0};
    std::memcpy(counts, v, sizeof(v));
}

vhx_tree_desc vhx::unpack_counts(const uint32_t counts[8]) {
    vhx_tree_desc d{};
    d.boxtree_size = counts[0];
    d.brick_dim = counts[1];
    d.node_count = counts[2];
    d.brick_count = counts[3];
    d.solid_count = counts[4];
    d.color_count = counts[5];
    d.data_count = counts[6];
    return d;
}

uint64_t vhx::elem_size(int id) {
    switch (id) {
        case VHX_BUF_NODE_OCBITS: return 8;
        default: return 4;
    }
}
uint64_t vhx::elem_count(const vhx_tree_desc &d, int id) {
    const uint64_t n3 = (uint64_t)d.brick_dim * d.brick_dim * d.brick_dim;
    switch (id) {
        case VHX_BUF_NODE_TYPE: return d.node_count;
        case VHX_BUF_NODE_OCBITS: return d.node_count;
        case VHX_BUF_NODE_CHILDREN: return (uint64_t)d.node_count * 64;
        case VHX_BUF_VOXELS: return (uint64_t)d.brick_count * n3;
        case VHX_BUF_SOLID_VALUES: return d.solid_count;
        case VHX_BUF_COLOR_PALETTE: return d.color_count;
        case VHX_BUF_DATA_PALETTE: return d.data_count;
    }
    return 0;
}

static int rebuild_hdr(vhx_ctx *c, uint32_t n0, uint32_t n) {
    if (n == 0) return VHX_OK;
    k_pack_hdr<<<(n + 255) / 256, 256, 0, c->stream>>>((const uint32_t *)c->tree->raw[VHX_BUF_NODE_TYPE].ptr,
                                                       (const uint64_t *)c->tree->raw[VHX_BUF_NODE_OCBITS].ptr, n0, n,
                                                       (uint4 *)c->tree->hdr.ptr);
    VHX_HIP(c, hipGetLastError());
    return VHX_OK;
}

static bool has_child_rec(const vhx_ctx *c) {
    const uint32_t bd = c->tree->desc.brick_dim;
    return bd * bd * bd <= 64;
}

// DevTree::child_rec depends on node types, children and brick occupancy: updates mark it stale and the next trace
// rebuilds it whole (one pass over the child entries, ~n_nodes * 64 * 24 bytes)
static int refresh_child_rec(vhx_ctx *c) {
    if (!has_child_rec(c) || !c->tree->child_rec_stale) return VHX_OK;
    const uint64_t n = (uint64_t)c->tree->desc.node_count * 64;
    k_child_rec<<<(unsigned)((n + 255) / 256), 256, 0, c->stream>>>(
        (const uint32_t *)c->tree->raw[VHX_BUF_NODE_TYPE].ptr, (const uint32_t *)c->tree->raw[VHX_BUF_NODE_CHILDREN].ptr,
        (const uint64_t *)c->tree->brick_occ.ptr, c->tree->desc.brick_count, 0, n, RecSel{0, 0, 0, 0, 0},
        (uint4 *)c->tree->child_rec.ptr);
    VHX_HIP(c, hipGetLastError());
    c->tree->child_rec_stale = false;
    return VHX_OK;
}

// The child records of nodes [node_lo, node_hi) and of the nodes holding Parted bricks [brick_lo, brick_hi) (either
// range may be empty): a pass over the written nodes' entries, or over every child entry when bricks were written (the
// brick -> holder relation lives only in the children array; reading it is 256 B per node, the records are 1 KB).
static int refresh_child_rec_sel(vhx_ctx *c, uint32_t node_lo, uint32_t node_hi, uint32_t brick_lo, uint32_t brick_hi) {
    if (!has_child_rec(c) || c->tree->child_rec_stale) return VHX_OK;  // a stale buffer is rebuilt whole anyway
    const bool bricks = brick_lo < brick_hi, nodes = node_lo < node_hi;
    if (!bricks && !nodes) return VHX_OK;
    const uint64_t e0 = bricks ? 0 : (uint64_t)node_lo * 64, e1 = bricks ? (uint64_t)c->tree->desc.node_count * 64
                                                                           : (uint64_t)node_hi * 64;
    k_child_rec<<<(unsigned)((e1 - e0 + 255) / 256), 256, 0, c->stream>>>(
        (const uint32_t *)c->tree->raw[VHX_BUF_NODE_TYPE].ptr, (const uint32_t *)c->tree->raw[VHX_BUF_NODE_CHILDREN].ptr,
        (const uint64_t *)c->tree->brick_occ.ptr, c->tree->desc.brick_count, e0, e1,
        RecSel{1, node_lo, node_hi, brick_lo, brick_hi}, (uint4 *)c->tree->child_rec.ptr);
    VHX_HIP(c, hipGetLastError());
    return VHX_OK;
}

static int rebuild_occ(vhx_ctx *c, uint32_t brick0, uint32_t nbricks) {
    if (nbricks == 0) return VHX_OK;
    const uint32_t bd = c->tree->desc.brick_dim;
    const uint32_t n3 = bd * bd * bd;
    const uint32_t *vox = (const uint32_t *)c->tree->raw[VHX_BUF_VOXELS].ptr;
    const uint32_t *col = (const uint32_t *)c->tree->raw[VHX_BUF_COLOR_PALETTE].ptr;
    const uint32_t *dat = (const uint32_t *)c->tree->raw[VHX_BUF_DATA_PALETTE].ptr;
    if (n3 >= 64) {
        const uint64_t cell0 = (uint64_t)brick0 * n3, ncells = (uint64_t)nbricks * n3;
        // grid-stride chunks keep gridDim.x within range for multi-GB voxel buffers
        const uint64_t chunk = 1ull << 30;
        for (uint64_t s = 0; s < ncells; s += chunk) {
            const uint64_t n = std::min(chunk, ncells - s);
            k_brick_occ_ballot<<<(unsigned)((n + 255) / 256), 256, 0, c->stream>>>(
                vox, n, cell0 + s, col, c->tree->desc.color_count, dat, c->tree->desc.data_count, (uint64_t *)c->tree->brick_occ.ptr);
            VHX_HIP(c, hipGetLastError());
        }
    } else {
        k_brick_occ_small<<<(nbricks + 255) / 256, 256, 0, c->stream>>>(vox, nbricks, brick0, n3, col,
                                                                         c->tree->desc.color_count, dat, c->tree->desc.data_count,
                                                                         (uint64_t *)c->tree->brick_occ.ptr);
        VHX_HIP(c, hipGetLastError());
    }
    return VHX_OK;
}

struct HostOut {
    OutD dev{};
    std::vector<std::pair<void *, std::pair<void *, uint64_t>>> copies;  // (host dst, (dev src, bytes))
};

// Maps the caller's vhx_hits onto device pointers (scratch-backed when the caller passed host memory).
// zero_fill: staging is cleared first (tile layout: pixels past the frame edge are never written and read back as 0)
static int map_out(vhx_ctx *c, const vhx_hits *h, uint64_t n, int on_device, HostOut &ho, bool zero_fill = false) {
    struct F {
        void *user;
        uint64_t per;
        void **dst;
    } fields[] = {{h->value, 4, (void **)&ho.dev.value},   {h->cell, 4, (void **)&ho.dev.cell},
                  {h->voxel, 12, (void **)&ho.dev.voxel},  {h->impact, 12, (void **)&ho.dev.impact},
                  {h->normal, 12, (void **)&ho.dev.normal}, {h->depth, 4, (void **)&ho.dev.depth},
                  {h->rgba, 4, (void **)&ho.dev.rgba},     {h->bytes, 4, (void **)&ho.dev.bytes},
                  {h->shadowed, 4, (void **)&ho.dev.shadowed}};
    if (on_device) {
        for (auto &f : fields) *f.dst = f.user;
        return VHX_OK;
    }
    uint64_t total = 0;
    for (auto &f : fields)
        if (f.user) total += (f.per * n + 255) & ~255ull;
    int rc = ensure(c, c->scratch, total);
    if (rc) return rc;
    if (zero_fill && total) VHX_HIP(c, hipMemsetAsync(c->scratch.ptr, 0, total, c->stream));
    uint64_t off = 0;
    for (auto &f : fields) {
        if (!f.user) continue;
        void *p = (char *)c->scratch.ptr + off;
        *f.dst = p;
        ho.copies.push_back({f.user, {p, f.per * n}});
        off += (f.per * n + 255) & ~255ull;
    }
    return VHX_OK;
}

static int finish_out(vhx_ctx *c, HostOut &ho) {
    for (auto &cp : ho.copies)
        VHX_HIP(c, hipMemcpyAsync(cp.first, cp.second.first, cp.second.second, hipMemcpyDeviceToHost, c->stream));
    if (!ho.copies.empty()) VHX_HIP(c, hipStreamSynchronize(c->stream));
    return VHX_OK;
}

// Multi-pass plumbing: allocates queues, chunk lists and counters for `nout` rays whose pass 0 runs in `nblocks0`
// workgroups of 256 (may synchronise; called before the trace is timed). Returns the number of passes to run.
// Adaptive scheduling (ctx.hpp, Sched): the busy schedule while another context of the tree has a frame in flight on
// another stream (its last trace's use event not yet reached), else the idle one. A host-side query per other context;
// no waits.
static void select_schedule(vhx_ctx *c, bool batch = false, bool shadow = false) {
    if (!c->adaptive) {
        c->last_sched = -1;
        c->qsort = c->qsort_force >= 0 ? (uint32_t)c->qsort_force : c->sched_busy.qsort;  // a fixed schedule: the busy one's
        return;
    }
    // a batch of frames is a throughput job by itself: the frames-in-flight schedule (its passes re-pack the surviving
    // rays of every frame of the batch; the last pass's tail is shared by them all)
    bool busy = batch;
    if (!busy) {
        std::lock_guard<std::mutex> lock(c->tree->mu);
        for (vhx_ctx *u : c->tree->users)
            if (u != c && u->use_recorded && u->use_stream != c->stream && hipEventQuery(u->use_ev) == hipErrorNotReady) {
                busy = true;
                break;
            }
    }
    const vhx_ctx::Sched &s = busy ? c->sched_busy : c->sched_idle;
    std::memcpy(c->budgets, shadow ? s.shadow_budgets : s.budgets, sizeof(c->budgets));
    std::memcpy(c->sparse, s.sparse, sizeof(c->sparse));
    c->npass = shadow ? s.shadow_npass : s.npass;
    c->queue_waves = s.queue_waves_per_cu * c->cus;
    c->queue_waves0 = c->queue_waves0_force ? c->queue_waves0_force : s.queue_waves0_per_cu * c->cus;
    c->qorder = s.qorder;
    c->qsort = c->qsort_force >= 0 ? (uint32_t)c->qsort_force : s.qsort;
    c->last_sched = busy ? 1 : 0;
}

static int prepare_passes(vhx_ctx *c, uint64_t nout, uint64_t nblocks0, uint32_t &npass, bool shadow = false,
                          bool batch = false) {
    select_schedule(c, batch, shadow);
    npass = nout < 0x7FFFFFFFull ? c->npass : 1u;
    if (npass < 2 && !shadow) return VHX_OK;
    uint64_t chunks = std::max(nblocks0, (nout + 1023) / 1024), list = nblocks0 * 256;
    for (uint32_t p = 1; p < npass; ++p) {  // queue passes: chunk = one grab of rpw rays (adaptive: >= 1)
        const uint64_t r = c->rpw[p] ? c->rpw[p] : 1u;
        const uint64_t ch = (nout + r - 1) / r;
        chunks = std::max(chunks, ch);
        list = std::max(list, ch * r + 64u);
    }
    int rc = ensure(c, c->queue[0], nout * 4);
    if (!rc && (npass > 2 || shadow)) rc = ensure(c, c->queue[1], nout * 4);
    if (!rc) rc = ensure(c, c->qctl, QCTL_WORDS * sizeof(uint32_t));
    if (!rc) rc = ensure(c, c->qargs, 2 * sizeof(QueueArgs));
    if (!rc) rc = ensure(c, c->tmp, list * 4);
    if (!rc) rc = ensure(c, c->counts, chunks * 4);
    if (!rc) rc = ensure(c, c->offsets, chunks * 4);
    if (!rc) rc = ensure(c, c->scan_part, ((chunks + SCAN_SEG - 1) / SCAN_SEG) * 8);
    if (!rc) rc = ensure(c, c->flags, ((nout + 3) & ~3ull));
    if (!rc && c->resume && npass > 1) rc = ensure(c, c->state, std::max<uint64_t>(nout, c->qstate ? list : 0ull) * 64);
    if (!rc && c->resume && c->qstate && npass > 1) rc = ensure(c, c->stateq, nout * 64);
    return rc;
}

// Stream-ordered per-trace reset of the pass state (inside the timed region) for ray batches; primary and shadow
// frames zero the counters in their first compaction kernel instead.
static int reset_passes(vhx_ctx *c, uint32_t npass) {
    if (npass < 2) return VHX_OK;
    VHX_HIP(c, hipMemsetAsync(c->qctl.ptr, 0, QCTL_WORDS * sizeof(uint32_t), c->stream));
    return VHX_OK;
}

// Pass 0 traces fresh rays (the grid kernel of primary and explicit rays, or the shadow path's first queue pass);
// every later pass resumes the rays its predecessor abandoned.
static PassQ pass_q(const vhx_ctx *c, uint32_t p, uint32_t npass, bool qm = false) {
    PassQ q{};  // every field a kernel reads is set below or zero (q.zero, q.flags: null unless a caller sets them)
    const bool last = p + 1 >= npass;
    q.budget = last ? VHX_MAX_ITERS : c->budgets[p];
    q.rpw = c->rpw[p];
    q.tw = c->tw;
    q.xcd_group = c->xcd_group;
    // the unbounded last pass only: dealing the budgeted passes too measured the same (shadow frames 2.90 against
    // 2.87 ms, primary frames equal) once the XCD counters had cache lines of their own; tune "qxcd_all=1" deals every
    // queue pass (diagnostics)
    q.qxcd = last || c->qxcd_all ? c->qxcd : 0u;
    q.tmp = last ? nullptr : (uint32_t *)c->tmp.ptr;
    q.counts = (uint32_t *)c->counts.ptr;
    q.flags = nullptr;
    // the state buffer is written by every pass that can abandon rays and read by every pass after the first
    q.state = c->resume && npass > 1 && p >= c->save_from ? (uint4 *)c->state.ptr : nullptr;
    q.resume = c->resume && p > c->save_from ? 1u : 0u;
    q.sparse = last || !q.state ? 0u : c->sparse[p];
    q.qmode = qm && q.state ? 1u : 0u;
    q.sin = q.qmode ? (const uint4 *)c->stateq.ptr : nullptr;
    q.lx = c->shadow_light[0];
    q.ly = c->shadow_light[1];
    q.lz = c->shadow_light[2];
    q.sbud = c->shadow_budget;
    q.skip = nullptr;
    q.tail_out = last ? c->tail_rec : nullptr;
    q.tail_min = c->tail_min;
    q.tail_cap = c->tail_cap;
    q.finter = c->frame_interleave ? 1u : 0u;
    return q;
}

// Whether a trace runs in the queue-state mode (PassQ::qmode): its pass 0 lists its abandoned rays per wave or chunk
// (listed: the ordered primary pass 0; first_queue: pass 0 is itself a queue pass, the shadow path), every pass saves
// (save_from 0, resume on), and no queue is node-sorted (the sort reorders a queue by the states at output indices)
static bool queue_state_mode(const vhx_ctx *c, bool listed, bool first_queue, uint32_t npass) {
    // (fused shadows keep states at output indices: a pixel's primary and shadow ray are never pending together)
    // (and MIP frames: the queue kernel's queue-state instantiation is built for the exact path only)
    if (!c->qstate || !c->resume || c->save_from != 0 || npass < 2 || !(listed || first_queue) || c->shadow_on ||
        c->tree->mips_on)
        return false;
    if (!c->stateq.ptr) return false;
    for (uint32_t p = 1; p < npass && p < 32u; ++p)
        if (c->qsort && ((c->qsort_passes >> p) & 1u)) return false;
    return true;
}

// VHX_DEBUG_PASSES=1 (a diagnostic build only): synchronise after every pass step and print the queue counters
#ifndef VHX_DEBUG_PASSES
#define VHX_DEBUG_PASSES 0
#endif
static void debug_passes(vhx_ctx *c, const char *what) {
    if (!VHX_DEBUG_PASSES || !c->qctl.ptr) return;
    uint32_t v[16];
    (void)hipStreamSynchronize(c->stream);
    (void)hipMemcpy(v, c->qctl.ptr, sizeof(v), hipMemcpyDeviceToHost);
    fprintf(stderr, "[vhx passes] %-24s counts %u %u %u %u ... %u  grabs %u %u %u %u\n", what, v[0], v[1], v[2], v[3],
            v[7], v[8], v[9], v[10], v[11]);
}

// Exclusive scan of nchunks counts (nchunks_host, or derived on the device from *n_in) into offsets, their sum at
// *total. At most max_chunks counts: up to c->scan_multi segments one workgroup walks them (a frame's scans); a larger
// scan (a batch of frames: one workgroup took ~10 us per segment while the rest of the GPU waited) sums the segments,
// scans the sums and scans every segment from its base, one workgroup per segment.
static void launch_scan(vhx_ctx *c, const uint32_t *counts, uint32_t nchunks_host, const uint32_t *n_in,
                        uint32_t per_chunk, uint32_t *offsets, uint32_t *total, uint64_t max_chunks) {
    const uint64_t nseg = (max_chunks + SCAN_SEG - 1) / SCAN_SEG;
    if (nseg <= c->scan_multi || c->scan_multi == 0 || !c->scan_part.ptr || c->scan_part.bytes < nseg * 8) {
        k_scan_counts<<<1, SCAN_THREADS, 0, c->stream>>>(counts, nchunks_host, n_in, per_chunk, c->tw, offsets, total);
        return;
    }
    uint32_t *sums = (uint32_t *)c->scan_part.ptr, *base = sums + nseg;
    k_scan_sums<<<(unsigned)nseg, SCAN_THREADS, 0, c->stream>>>(counts, nchunks_host, n_in, per_chunk, c->tw, sums);
    k_scan_counts<<<1, SCAN_THREADS, 0, c->stream>>>(sums, (uint32_t)nseg, nullptr, 1, c->tw, base, total);
    k_scan_counts<<<(unsigned)nseg, SCAN_THREADS, 0, c->stream>>>(counts, nchunks_host, n_in, per_chunk, c->tw,
                                                                   offsets, nullptr, base);
}

// Chunk lists -> queue `out` with its length at *total: pass-0 style (nchunks_host workgroup chunks of stride 256) or
// queue-pass style (chunks of per_chunk rays, their number derived from the device-side input length n_in).
static int compact_chunks(vhx_ctx *c, uint32_t nchunks_host, const uint32_t *n_in, uint32_t per_chunk,
                          uint32_t stride, uint32_t *out, uint32_t *total, uint64_t max_chunks, bool move_state = false) {
    const uint32_t *counts = (const uint32_t *)c->counts.ptr;
    uint32_t *offsets = (uint32_t *)c->offsets.ptr;
    // adaptive rays per chunk (pass_rpw, per_chunk 0; max_chunks is then the ray count): ceil(n / ceil(n / tw)) <= tw
    // chunks, or ceil(n / 64) once a chunk holds 64 rays
    const uint64_t scan_max = n_in && per_chunk == 0u
                                  ? std::min<uint64_t>(max_chunks, std::max<uint64_t>(c->tw, (max_chunks + 63) / 64))
                                  : max_chunks;
    launch_scan(c, counts, nchunks_host, n_in, per_chunk, offsets, total, scan_max);
    const uint64_t want = (max_chunks + 3) / 4;
    const unsigned grid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(want, c->queue_blocks));
    k_gather_chunks<<<grid, 256, 0, c->stream>>>((const uint32_t *)c->tmp.ptr, stride, counts, offsets,
                                                 nchunks_host, n_in, per_chunk, c->tw, out,
                                                 move_state ? (const uint4 *)c->state.ptr : nullptr,
                                                 move_state ? (uint4 *)c->stateq.ptr : nullptr);
    VHX_HIP(c, hipGetLastError());
    debug_passes(c, "compacted");
    return VHX_OK;
}

// k_sort_segments over the queue of pass p (its length at *n_dev, at most nmax entries) when the schedule sorts and the
// rays of that pass resume from saved state (the node is read there)
static int sort_segments(vhx_ctx *c, uint32_t p, uint32_t npass, uint32_t *queue, const uint32_t *n_dev, uint64_t nmax) {
    const PassQ q = pass_q(c, p, npass);
    if (!c->qsort || !q.resume || !q.state || p >= 32u || !((c->qsort_passes >> p) & 1u)) return VHX_OK;
    const uint64_t segs = (nmax + c->qsort - 1) / c->qsort;
    const unsigned grid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(segs, c->qsort_blocks));
    k_sort_segments<<<grid, QSORT_THREADS, 0, c->stream>>>(queue, n_dev, (const uint32_t *)q.state, c->qsort);
    VHX_HIP(c, hipGetLastError());
    debug_passes(c, "sorted segments");
    return VHX_OK;
}

// The FlagOrder of code `qorder` for a W x H framebuffer frame (W = 0 or qorder = 0: output-index order) and the
// number of positions its compaction scans (npos: in / out)
static FlagOrder flag_order(uint32_t qorder, uint32_t W, uint32_t H, uint64_t &npos, uint32_t frames = 1) {
    FlagOrder ord{};
    if (!qorder || !W || !H) return ord;
    const uint32_t tsl = qorder & 15u, ts = 1u << tsl;
    ord = FlagOrder{W, H, (W + ts - 1u) / ts, (H + ts - 1u) / ts, tsl, 0u, (qorder & 64u) ? 2u : (qorder & 32u) ? 1u : 0u,
                    0u, 0u};
    if (qorder & 16u)  // Morton order over the smallest 2^m x 2^m grid of tiles covering the frame
        while ((1u << ord.mdim) < std::max(ord.tx, ord.ty)) ++ord.mdim;
    const uint64_t np = (ord.mdim ? 1ull << (2u * ord.mdim) : (uint64_t)ord.tx * ord.ty) << (2u * tsl);
    // the chunk counts are sized for ceil(pixels / 256) chunks, the compaction needs ceil(npos / 1024): a tile far
    // larger than the frame keeps output-index order
    if (np > 4ull * W * H) return FlagOrder{};
    npos = np * frames;
    if (frames > 1) {
        ord.fpos = np;
        ord.fpix = (uint64_t)W * H;
    }
    return ord;
}

// The ListOrder of code `qorder` for a W x H framebuffer frame, when pass 0 can list its rays in that order itself:
// tiles row-major (no Morton over the tiles), Morton inside, at least 16 pixels per side (the default, 38); nblocks =
// the workgroups of pass 0 over whole tiles. Else false (pass 0 writes flags, flag_order compacts them).
static bool list_order(uint32_t qorder, uint32_t W, uint32_t H, ListOrder &lo, uint64_t &nblocks) {
    const uint32_t tsl = qorder & 15u;
    if (!qorder || !W || !H || (qorder & (16u | 64u)) || !(qorder & 32u) || tsl < 4u) return false;
    const uint32_t ts = 1u << tsl, ty = (H + ts - 1u) / ts;
    lo = ListOrder{(W + ts - 1u) / ts, tsl - 4u};
    nblocks = ((uint64_t)lo.tx * ty) << (2u * lo.tbl);
    // flag_order keeps output-index order for tiles far larger than the frame
    return nblocks * 256u <= 4ull * W * H;
}

// Pass 0's workgroups over whole tiles of the list order: the buffers of its per-workgroup lists
static int ensure_lists(vhx_ctx *c, uint64_t nblocks) {
    int rc = ensure(c, c->tmp, nblocks * 256 * 4);
    // the queue-state mode saves pass 0's abandoned rays at their list slots (every slot of whole tiles)
    if (!rc && c->resume && c->qstate) rc = ensure(c, c->state, nblocks * 256 * 64);
    if (!rc) rc = ensure(c, c->counts, nblocks * 4 * 4);
    if (!rc) rc = ensure(c, c->offsets, nblocks * 4 * 4);
    if (!rc) rc = ensure(c, c->scan_part, ((nblocks * 4 + SCAN_SEG - 1) / SCAN_SEG) * 8);
    return rc;
}

// The QueueArgs slot of a frame (camera, ray source, outputs) on c's stream. They rarely change between frames: the
// device copy is rewritten only when they do.
static int put_qargs(vhx_ctx *c, const CamD &cam, const RaySrc &src, const OutD &o, QueueArgs *&qa) {
    const uint32_t slot = src.kind == 3u || src.kind == 5u ? 1u : 0u;  // a shadow frame alternates with its primary
    qa = (QueueArgs *)c->qargs.ptr + slot;
    QueueArgs a;
    std::memset(&a, 0, sizeof(a));  // padding included, for the comparison
    a.cam = cam;
    a.src = src;
    a.out = o;
    const uint8_t *ab = (const uint8_t *)&a;
    if (c->qargs_host_ptr[slot] != c->qargs.ptr || c->qargs_host[slot].size() != sizeof(a) ||
        std::memcmp(c->qargs_host[slot].data(), ab, sizeof(a)) != 0) {
        k_put_queue_args<<<1, 64, 0, c->stream>>>(a, qa);
        VHX_HIP(c, hipGetLastError());
        c->qargs_host[slot].assign(ab, ab + sizeof(a));
        c->qargs_host_ptr[slot] = c->qargs.ptr;
    }
    return VHX_OK;
}

// Queue passes first..npass-1: pass p re-traces the queue of pass p-1 (pass 0's queue, for first == 0, is the list
// in queue[1] with its length in qctl[7]); what exceeds its budget is listed per chunk and compacted into the next
// pass's queue. For first == 1, pass 0 (a grid kernel of nblocks0 workgroups) has just run and is compacted first:
// its per-workgroup lists (P0_LISTS, in workgroup order; P0_ORDERED, already in the queue order, ListOrder), or its
// per-ray flags in the queue order (P0_FLAGS).
enum { P0_LISTS = 0, P0_FLAGS = 1, P0_ORDERED = 2 };
template <bool COUNT, int BD, bool MIP = false, bool FUSE = false>
static int launch_queue_passes(vhx_ctx *c, const DevTree &t, const CamD &cam, const RaySrc &src, const OutD &o,
                               uint32_t first, uint32_t npass, uint64_t nout, uint64_t nblocks0,
                               int pass0 = P0_LISTS, uint32_t order_w = 0, uint32_t order_h = 0,
                               uint32_t frames = 1, bool qm = false) {
    uint32_t *ctl = (uint32_t *)c->qctl.ptr;
    int rc = VHX_OK;
    if (first > 0 && npass > 1) {
        if (pass0 == P0_FLAGS) {  // primary frames: per-ray flags compacted in output-index (frame) order
            // tile order (c->qorder, framebuffer layout only): positions over the frame's tiles
            uint64_t npos = nout;
            const FlagOrder ord = flag_order(c->qorder, order_w, order_h, npos, frames);
            const unsigned nb = (unsigned)((npos + 1023) / 1024);
            uint32_t *counts = (uint32_t *)c->counts.ptr, *offsets = (uint32_t *)c->offsets.ptr;
            const uint8_t *flags = (const uint8_t *)c->flags.ptr;
            k_count_flags<false><<<nb, 256, 0, c->stream>>>(flags, npos, counts, ctl + 16, nullptr, ord);
            launch_scan(c, counts, nb, nullptr, 1, offsets, ctl, nb);
            k_emit_flags<false><<<nb, 256, 0, c->stream>>>(flags, npos, offsets, (uint32_t *)c->queue[0].ptr, ord);
            VHX_HIP(c, hipGetLastError());
            debug_passes(c, "compacted flags");
            if ((rc = sort_segments(c, 1, npass, (uint32_t *)c->queue[0].ptr, ctl, nout))) return rc;
        } else if (pass0 == P0_ORDERED) {  // per-wave lists (wave_append): 4 chunks of 64 per workgroup
            rc = compact_chunks(c, (uint32_t)(nblocks0 * 4), nullptr, 64, 64, (uint32_t *)c->queue[0].ptr, ctl,
                                nblocks0 * 4, qm);
            if (!rc) rc = sort_segments(c, 1, npass, (uint32_t *)c->queue[0].ptr, ctl, nout);
        } else {
            rc = compact_chunks(c, (uint32_t)nblocks0, nullptr, 256, 256, (uint32_t *)c->queue[0].ptr, ctl, nblocks0);
        }
    }
    QueueArgs *qa = nullptr;
    if (first < npass && (rc = put_qargs(c, cam, src, o, qa))) return rc;
    for (uint32_t p = first; p < npass && !rc; ++p) {
        const uint32_t *in = (const uint32_t *)c->queue[(p - 1) & 1u].ptr;  // p = 0: queue[1]
        const uint32_t *in_n = p > 0 ? ctl + (p - 1) : ctl + 7;
        const PassQ q = pass_q(c, p, npass, qm);
        // a first pass over fresh rays (the shadow path) is throughput-bound like a grid launch: more waves
        uint32_t qwaves = p == 0 ? c->queue_waves0
                          : (p + 1 < npass && c->queue_waves_mid ? c->queue_waves_mid : c->queue_waves);
        // a batch of frames: the waves the same frames would bring as frames in flight (one frame's queue waves each),
        // up to the queue kernel's residency (5 waves per SIMD): its queue passes are memory-latency bound and need
        // the waves in flight
        if (frames > 1 && p > 0) qwaves = (uint32_t)std::min<uint64_t>((uint64_t)qwaves * frames, 20ull * c->cus);
        const unsigned qgrid = (qwaves * 64u + c->qblock - 1) / c->qblock;
        uint32_t *grab = ctl + 16u + QCTL_PASS_WORDS * p;
        if constexpr (!FUSE && !MIP) {  // (the queue-state mode excludes fused shadows; MIP frames never list pass 0)
            if (q.qmode)
                k_trace_queue<COUNT, BD, MIP, FUSE, true><<<qgrid, c->qblock, 0, c->stream>>>(t, qa, in, in_n, grab, q);
            else
                k_trace_queue<COUNT, BD, MIP, FUSE><<<qgrid, c->qblock, 0, c->stream>>>(t, qa, in, in_n, grab, q);
        } else {
            k_trace_queue<COUNT, BD, MIP, FUSE><<<qgrid, c->qblock, 0, c->stream>>>(t, qa, in, in_n, grab, q);
        }
        debug_passes(c, "queue pass");
        if (p + 1 < npass) {
            rc = compact_chunks(c, 0, in_n, q.rpw, q.rpw, (uint32_t *)c->queue[p & 1u].ptr, ctl + p,
                                q.rpw ? (nout + q.rpw - 1) / q.rpw : nout, qm);
            if (!rc) rc = sort_segments(c, p + 1, npass, (uint32_t *)c->queue[p & 1u].ptr, ctl + p, nout);
        }
    }
    return rc;
}

// ------------------------------------------------------------------------------------------------ C ABI
extern "C" {

uint32_t vhx_abi_version(void) { return VHX_ABI_VERSION; }

// The HIP runtime's answer, with its error: hipGetDeviceCount failing for any reason other than "no device" is
// VHX_E_HIP (count 0) and its text is kept for vhx_device_error (there is no context to hold it), instead of a silent
// count of 0 (a process that lost the device must say why)
static thread_local std::string g_device_err;
int vhx_device_count(int *count) {
    if (!count) return VHX_E_INVALID_ARG;
    int n = 0;
    const hipError_t e = hipGetDeviceCount(&n);
    if (e == hipErrorNoDevice) n = 0;  // no GPU visible: a count of 0, not an error (a CPU-only host)
    else if (e != hipSuccess) {
        g_device_err = std::string("hipGetDeviceCount: ") + hipGetErrorName(e) + ": " + hipGetErrorString(e);
        *count = 0;
        return VHX_E_HIP;
    }
    g_device_err.clear();
    *count = n;
    return VHX_OK;
}

const char *vhx_device_error(void) { return g_device_err.c_str(); }

int vhx_create(int hip_device, vhx_ctx **out) {
    if (!out) return VHX_E_INVALID_ARG;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return VHX_E_NO_DEVICE;
    if (hip_device < 0 || hip_device >= n) return VHX_E_INVALID_ARG;
    vhx_ctx *c = new vhx_ctx();
    c->device = hip_device;
    c->tree = std::make_shared<TreeStore>();
    c->tree->device = hip_device;
    register_user(c);
    auto bail = [&](const char *what, hipError_t e) {
        fprintf(stderr, "vhx_create: %s: %s\n", what, hipGetErrorString(e));
        delete c;
        return VHX_E_HIP;
    };
    hipError_t e;
    if ((e = hipSetDevice(hip_device)) != hipSuccess) return bail("hipSetDevice", e);
    // no stream yet: the caller's (vhx_set_stream) or the context's own, created at first use (VHX_STREAM). The
    // library reads no environment: the schedule is the adaptive default until vhx_set_pass_budgets / vhx_set_tuning.
    {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, hip_device) == hipSuccess && prop.multiProcessorCount > 0) {
            c->cus = (uint32_t)prop.multiProcessorCount;
            c->queue_blocks = c->cus * 8u;
            c->queue_waves = c->sched_busy.queue_waves_per_cu * c->cus;
        }
    }
    if ((e = hipEventCreate(&c->ev0)) != hipSuccess) return bail("hipEventCreate", e);
    if ((e = hipEventCreate(&c->ev1)) != hipSuccess) return bail("hipEventCreate", e);

    uint8_t lut[64 * 27];
    make_step_lut(lut);
    if ((e = hipMemcpyToSymbol(HIP_SYMBOL(vhx::c_step_lut), lut, sizeof(lut))) != hipSuccess)
        return bail("hipMemcpyToSymbol", e);
    *out = c;
    return VHX_OK;
}

int vhx_create_shared(const vhx_ctx *owner, vhx_ctx **out) {
    if (!owner || !out) return VHX_E_INVALID_ARG;
    *out = nullptr;
    vhx_ctx *c = nullptr;
    int rc = vhx_create(owner->device, &c);
    if (rc) return rc;
    c->tree = owner->tree;  // the same device tree (reference-counted); the context's fresh store goes with it
    register_user(c);
    c->shared = true;
    copy_sched(c, owner);  // the owner's scheduling settings (as of now; vhx_mgpu re-copies them per frame)
    *out = c;
    return VHX_OK;
}

void vhx_destroy(vhx_ctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    unregister_user(c);
    c->tree.reset();  // frees the device tree with its last context
    if (c->use_ev) (void)hipEventDestroy(c->use_ev);
    for (DevBuf *b : {&c->scratch, &c->rays, &c->queue[0], &c->queue[1], &c->qctl, &c->tmp, &c->counts, &c->offsets,
                      &c->flags, &c->qargs, &c->state, &c->stateq, &c->upd, &c->prepass_depth, &c->batch_args, &c->scan_part,
                      &c->shadow_args, &c->tail_list[0], &c->tail_list[1], &c->tail_mask})
        if (b->ptr) (void)hipFree(b->ptr);
    if (c->tail_stream) {
        (void)hipStreamSynchronize(c->tail_stream);
        (void)hipStreamDestroy(c->tail_stream);
    }
    if (c->tail_fork) (void)hipEventDestroy(c->tail_fork);
    if (c->tail_join) (void)hipEventDestroy(c->tail_join);
    std::vector<vhx_ctx::Pinned *> pins = {&c->pinned[0], &c->pinned[1]};
    for (auto &P : c->batch_pinned) pins.push_back(&P);
    for (auto &P : c->shadow_pinned) pins.push_back(&P);
    for (auto *P : pins) {
        if (P->ptr) (void)hipHostFree(P->ptr);
        if (P->done) (void)hipEventDestroy(P->done);
    }
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
    delete c;
}

int vhx_set_pass_budgets(vhx_ctx *c, const uint32_t *budgets, uint32_t n) {
    if (!c || n > VHX_MAX_BUDGETS || (n && !budgets)) return VHX_E_INVALID_ARG;
    for (uint32_t i = 0; i < n; ++i)
        if (budgets[i] == 0 || budgets[i] >= VHX_MAX_ITERS || (i && budgets[i] <= budgets[i - 1]))
            return fail(c, VHX_E_INVALID_ARG, "pass budgets must be increasing, > 0 and < 2^22");
    for (uint32_t i = 0; i < VHX_MAX_BUDGETS; ++i) c->budgets[i] = i < n ? budgets[i] : 0u;
    c->npass = n + 1;
    if (c->adaptive) {  // leaving the adaptive choice: the rest of the schedule is the busy one's
        std::memcpy(c->sparse, c->sched_busy.sparse, sizeof(c->sparse));
        c->queue_waves = c->sched_busy.queue_waves_per_cu * c->cus;
        c->queue_waves0 = c->queue_waves0_force ? c->queue_waves0_force : c->sched_busy.queue_waves0_per_cu * c->cus;
        c->qorder = c->sched_busy.qorder;
        c->adaptive = false;
    }
    c->last_sched = -1;
    return VHX_OK;
}

// vhx_set_tuning: the scheduling knobs of the probes (they used to be environment variables read at vhx_create; the
// library now reads none). Parsed into a copy of the context first, so a malformed spec changes nothing.
static bool parse_u32_list(const std::string &v, uint32_t *out, uint32_t cap, uint32_t &n) {
    n = 0;
    const char *q = v.c_str();
    if (!*q) return true;
    for (;;) {
        char *end = nullptr;
        const unsigned long x = strtoul(q, &end, 10);
        if (end == q || n >= cap || x > 0xFFFFFFFFul) return false;
        out[n++] = (uint32_t)x;
        if (*end == '\0') return true;
        if (*end != ',') return false;
        q = end + 1;
    }
}
static bool parse_u32(const std::string &v, uint32_t &out) {
    uint32_t n = 0, x[1];
    if (!parse_u32_list(v, x, 1, n) || n != 1) return false;
    out = x[0];
    return true;
}
static int apply_tuning(vhx_ctx *c, const std::string &key, const std::string &val) {
    uint32_t x = 0, n = 0, l[VHX_MAX_BUDGETS + 1];
    auto bad = [&]() { return fail(c, VHX_E_INVALID_ARG, ("vhx_set_tuning: bad value for " + key).c_str()); };
    if (key == "budgets") {  // "" or "0" = one pass
        if (!parse_u32_list(val, l, VHX_MAX_BUDGETS, n)) return bad();
        if (n == 1 && l[0] == 0) n = 0;
        return vhx_set_pass_budgets(c, l, n);
    } else if (key == "adaptive") {
        if (!parse_u32(val, x) || x > 1) return bad();
        return vhx_set_adaptive_schedule(c, (int)x);
    } else if (key == "rpw") {  // queue passes 1.., 0 = adaptive
        if (!parse_u32_list(val, l, VHX_MAX_BUDGETS, n)) return bad();
        for (uint32_t i = 0; i < n; ++i) {
            if (l[i] > 64) return bad();
            c->rpw[i + 1] = l[i];
        }
    } else if (key == "tw") {
        if (!parse_u32(val, x) || x == 0) return bad();
        c->tw = x;
    } else if (key == "xcdg") {
        if (!parse_u32(val, x)) return bad();
        c->xcd_group = x;
    } else if (key == "resume") {
        if (!parse_u32(val, x) || x > 1) return bad();
        c->resume = x != 0;
    } else if (key == "tlists") {
        if (!parse_u32(val, x) || x > 1) return bad();
        c->tile_lists = x != 0;
    } else if (key == "qstate") {
        if (!parse_u32(val, x) || x > 1) return bad();
        c->qstate = x != 0;
    } else if (key == "save_from") {
        if (!parse_u32(val, x)) return bad();
        c->save_from = x;
    } else if (key == "qblock") {
        if (!parse_u32(val, x) || (x != 64 && x != 128 && x != 256)) return bad();
        c->qblock = x;
    } else if (key == "qwaves") {  // fixes the schedule
        if (!parse_u32(val, x) || x == 0) return bad();
        if (c->adaptive) vhx_set_adaptive_schedule(c, 0);
        c->queue_waves = x;
    } else if (key == "qwpc_idle" || key == "qwpc_busy") {  // queue waves per CU of one schedule (stays adaptive)
        if (!parse_u32(val, x) || x == 0 || x > 64) return bad();
        (key == "qwpc_idle" ? c->sched_idle : c->sched_busy).queue_waves_per_cu = x;
    } else if (key == "qwavesm") {
        if (!parse_u32(val, x)) return bad();
        c->queue_waves_mid = x;
    } else if (key == "p0lists") {  // pass 0 of primary frames: 1 = lists in the queue order (ListOrder), 0 = flags
        if (!parse_u32(val, x) || x > 1) return bad();
        c->p0lists = x != 0;
    } else if (key == "scan_multi") {  // 0 = every scan on one workgroup
        if (!parse_u32(val, x)) return bad();
        c->scan_multi = x;
    } else if (key == "tail") {  // early tail of lone frames (vhx_ctx::tail_*): 1 on, 0 off
        if (!parse_u32(val, x) || x > 1) return bad();
        c->tail_on = x != 0;
    } else if (key == "tail_min") {  // steps from which a ray joins the next lone frame's early tail
        if (!parse_u32(val, x) || x == 0) return bad();
        c->tail_min = x;
    } else if (key == "tail_rpw") {  // early-tail rays per wave
        if (!parse_u32(val, x) || x == 0 || x > 64) return bad();
        c->tail_rpw = x;
    } else if (key == "tail_prio") {  // s_setprio of the early-tail waves (0-3)
        if (!parse_u32(val, x) || x > 3) return bad();
        c->tail_prio = x;
    } else if (key == "tail_cap") {  // longest list recorded
        if (!parse_u32(val, x) || x > (1u << 20)) return bad();
        c->tail_cap = x;
        c->tail_valid = false;  // (a list recorded under another cap may hold more entries)
    } else if (key == "finter") {  // batches: pass-0 blocks of the frames interleaved (1) or frame-major (0)
        if (!parse_u32(val, x) || x > 1) return bad();
        c->frame_interleave = x != 0;
    } else if (key == "stage_slots") {  // batch staging ring slots in use (1 = wait for the previous batch's copy)
        if (!parse_u32(val, x) || x == 0 || x > vhx_ctx::VHX_STAGE_SLOTS) return bad();
        c->stage_slots = x;
    } else if (key == "sbudget") {  // fused shadows: steps of a shadow ray in its primary ray's pass (0 = the rest)
        if (!parse_u32(val, x)) return bad();
        c->shadow_budget = x;
    } else if (key == "qwaves0") {
        if (!parse_u32(val, x) || x == 0) return bad();
        c->queue_waves0 = c->queue_waves0_force = x;
    } else if (key == "qxcd") {
        if (!parse_u32(val, x)) return bad();
        c->qxcd = x;
    } else if (key == "qxcd_all") {
        if (!parse_u32(val, x) || x > 1) return bad();
        c->qxcd_all = x != 0;
    } else if (key == "sparse") {  // per budgeted pass; fixes the schedule
        if (!parse_u32_list(val, l, VHX_MAX_BUDGETS, n)) return bad();
        for (uint32_t i = 0; i < n; ++i)
            if (l[i] > 64) return bad();
        if (c->adaptive) vhx_set_adaptive_schedule(c, 0);
        for (uint32_t i = 0; i < VHX_MAX_BUDGETS; ++i) c->sparse[i] = i < n ? l[i] : 0u;
    } else if (key == "qorder") {  // "[m]N[z|r]": NxN tiles, (m) Morton order of the tiles, (z) Morton / (r) rows inside
        const bool m = !val.empty() && val[0] == 'm';
        char *end = nullptr;
        const char *b = val.c_str() + (m ? 1 : 0);
        const long ts = strtol(b, &end, 10);
        if (end == b) return bad();
        const bool z = *end == 'z', rows = *end == 'r';
        if (*end && !((z || rows) && end[1] == '\0')) return bad();
        uint32_t lg = 0;
        while (lg < 12u && (1l << lg) < ts) ++lg;
        uint32_t code = 0;
        if (ts != 0) {
            if (ts < 8 || ts > 4096 || (1l << lg) != ts) return bad();
            code = lg | (m ? 16u : 0u) | (z ? 32u : 0u) | (rows ? 64u : 0u);
        }
        c->qorder = c->sched_busy.qorder = c->sched_idle.qorder = code;  // both schedules (the rest stays adaptive)
    } else if (key == "qsort") {  // segment length of the queue passes' node sort: 0 = off, else 256 .. VHX_QSORT_MAX
        if (!parse_u32(val, x) || (x && (x < 256 || x > VHX_QSORT_MAX || (x & (x - 1))))) return bad();
        c->qsort_force = (int)x;
    } else if (key == "qsortp") {  // bit mask of the queue passes whose input is sorted
        if (!parse_u32(val, x)) return bad();
        c->qsort_passes = x;
    } else if (key == "qsortb") {
        if (!parse_u32(val, x) || x == 0) return bad();
        c->qsort_blocks = x;
    } else {
        return fail(c, VHX_E_INVALID_ARG, ("vhx_set_tuning: unknown key " + key).c_str());
    }
    return VHX_OK;
}

int vhx_set_tuning(vhx_ctx *c, const char *spec) {
    if (!c || !spec) return VHX_E_INVALID_ARG;
    std::vector<std::pair<std::string, std::string>> kv;
    for (const char *q = spec; *q;) {
        const char *e = q;
        while (*e && *e != ';') ++e;
        const std::string item(q, e);
        q = *e ? e + 1 : e;
        if (item.empty()) continue;
        const size_t eq = item.find('=');
        if (eq == std::string::npos || eq == 0) return fail(c, VHX_E_INVALID_ARG, "vhx_set_tuning: expected key=value");
        kv.emplace_back(item.substr(0, eq), item.substr(eq + 1));
    }
    // a dry run on a scratch context first: a malformed spec leaves c unchanged
    {
        vhx_ctx dry;
        copy_sched(&dry, c);
        for (const auto &p : kv) {
            const int rc = apply_tuning(&dry, p.first, p.second);
            if (rc) {
                c->err = dry.err;
                return rc;
            }
        }
    }
    for (const auto &p : kv) {
        const int rc = apply_tuning(c, p.first, p.second);
        if (rc) return rc;
    }
    return VHX_OK;
}

int vhx_set_adaptive_schedule(vhx_ctx *c, int on) {
    if (!c) return VHX_E_INVALID_ARG;
    if (!on && c->adaptive) {  // leaving the adaptive choice: the frames-in-flight schedule, whatever the last trace ran
        const vhx_ctx::Sched &s = c->sched_busy;
        std::memcpy(c->budgets, s.budgets, sizeof(c->budgets));
        std::memcpy(c->sparse, s.sparse, sizeof(c->sparse));
        c->npass = s.npass;
        c->queue_waves = s.queue_waves_per_cu * c->cus;
        c->queue_waves0 = c->queue_waves0_force ? c->queue_waves0_force : s.queue_waves0_per_cu * c->cus;
        c->qorder = s.qorder;
        c->last_sched = -1;
    }
    c->adaptive = on != 0;
    return VHX_OK;
}

int vhx_get_pass_budgets(const vhx_ctx *c, uint32_t *budgets, uint32_t *n, int *sched) {
    if (!c || !n) return VHX_E_INVALID_ARG;
    *n = c->npass > 0 ? c->npass - 1 : 0;
    if (budgets)
        for (uint32_t i = 0; i < VHX_MAX_BUDGETS; ++i) budgets[i] = i < *n ? c->budgets[i] : 0u;
    if (sched) *sched = c->last_sched;
    return VHX_OK;
}

const char *vhx_last_error(const vhx_ctx *c) { return c ? c->err.c_str() : "null context"; }

int vhx_set_stream(vhx_ctx *c, void *s) {
    if (!c) return VHX_E_INVALID_ARG;
    c->stream = s ? (hipStream_t)s : c->own_stream;  // null own stream: created at the next use
    c->qargs_host_ptr[0] = c->qargs_host_ptr[1] = nullptr;  // written on the previous stream: rewrite them
    return VHX_OK;
}

int vhx_get_stream(vhx_ctx *c, void **s) {
    if (!c || !s) return VHX_E_INVALID_ARG;
    VHX_HIP(c, hipSetDevice(c->device));
    VHX_STREAM(c);
    *s = (void *)c->stream;
    return VHX_OK;
}

int vhx_sync(vhx_ctx *c, float *ms) {
    if (!c) return VHX_E_INVALID_ARG;
    VHX_HIP(c, hipSetDevice(c->device));
    if (c->stream) VHX_HIP(c, hipStreamSynchronize(c->stream));
    if (ms) {
        *ms = 0.f;
        if (c->timed) VHX_HIP(c, hipEventElapsedTime(ms, c->ev0, c->ev1));
    }
    return VHX_OK;
}

}  // extern "C"

int vhx::launch_untile(vhx_ctx *c, hipStream_t stream, const void *gathered, uint32_t planes, uint32_t ranks,
                       uint32_t tiles_per_rank, uint32_t T, uint32_t width, uint32_t height, uint32_t *fb_rgba,
                       float *fb_depth) {
    const uint32_t tiles_x = (width + T - 1) / T, tiles_y = (height + T - 1) / T;
    const uint64_t n = (uint64_t)ranks * planes * tiles_per_rank * T * T;
    if (n == 0) return VHX_OK;
    k_untile_planes<<<(unsigned)((n + 255) / 256), 256, 0, stream>>>((const uint32_t *)gathered, planes, ranks,
                                                                     tiles_per_rank, T, tiles_x, tiles_x * tiles_y,
                                                                     width, height, fb_rgba, (uint32_t *)fb_depth);
    VHX_HIP(c, hipGetLastError());
    return VHX_OK;
}

int vhx::alloc_tree(vhx_ctx *c, const vhx_tree_desc *t) {
    const uint32_t bd = t->brick_dim;
    if (t->node_count == 0 || bd == 0 || t->boxtree_size == 0 || (bd & (bd - 1)) != 0 || bd > 32 ||
        (t->boxtree_size & (t->boxtree_size - 1)) != 0 || t->boxtree_size > (1u << 24))
        return fail(c, VHX_E_INVALID_ARG, "vhx_upload_tree: invalid sizes");
    VHX_HIP(c, hipSetDevice(c->device));
    // a buffer that grows is freed and reallocated: the frames in flight on the tree's contexts (which c's stream
    // already waits for, write_begin) finish first
    bool grows = false;
    for (int id = 0; id < 7; ++id) grows |= c->tree->raw[id].bytes < elem_count(*t, id) * elem_size(id);
    if (grows && c->stream) VHX_HIP(c, hipStreamSynchronize(c->stream));
    c->tree->uploaded = false;
    c->tree->mips_on = false;  // a new tree has no MIPs until vhx_set_node_mips
    for (int id = 0; id < 7; ++id) {
        int rc = ensure(c, c->tree->raw[id], elem_count(*t, id) * elem_size(id));
        if (rc) return rc;
    }
    c->tree->desc = *t;
    for (const void **q : {(const void **)&c->tree->desc.node_type, (const void **)&c->tree->desc.node_ocbits,
                           (const void **)&c->tree->desc.node_children, (const void **)&c->tree->desc.voxels,
                           (const void **)&c->tree->desc.solid_values, (const void **)&c->tree->desc.color_palette,
                           (const void **)&c->tree->desc.data_palette})
        *q = nullptr;  // only the counts are kept
    return VHX_OK;
}

int vhx::finish_upload(vhx_ctx *c) {
    const vhx_tree_desc *t = &c->tree->desc;
    const uint64_t bd = t->brick_dim, n3 = bd * bd * bd;
    c->tree->occ_words = n3 >= 64 ? (uint32_t)(n3 / 64) : 1u;
    int rc = ensure(c, c->tree->hdr, (uint64_t)t->node_count * 16);
    if (rc) return rc;
    rc = ensure(c, c->tree->brick_occ, (uint64_t)t->brick_count * c->tree->occ_words * 8);
    if (rc) return rc;
    if ((rc = rebuild_hdr(c, 0, t->node_count))) return rc;
    if ((rc = rebuild_occ(c, 0, t->brick_count))) return rc;
    if (has_child_rec(c)) {
        if ((rc = ensure(c, c->tree->child_rec, (uint64_t)t->node_count * 64 * 16))) return rc;
        c->tree->child_rec_stale = true;
        if ((rc = refresh_child_rec(c))) return rc;
    }
    VHX_HIP(c, hipStreamSynchronize(c->stream));
    c->tree->uploaded = true;
    return VHX_OK;
}

extern "C" {

int vhx_upload_tree(vhx_ctx *c, const vhx_tree_desc *t) {
    if (!c || !t) return VHX_E_INVALID_ARG;
    if (c->shared) return fail(c, VHX_E_STATE, "vhx_upload_tree on a shared context: upload through the owner");
    const void *src[7] = {t->node_type, t->node_ocbits, t->node_children, t->voxels,
                          t->solid_values, t->color_palette, t->data_palette};
    for (int id = 0; id < 7; ++id)
        if (elem_count(*t, id) && !src[id])
            return fail(c, VHX_E_INVALID_ARG, "vhx_upload_tree: null array with non-zero count");
    VHX_HIP(c, hipSetDevice(c->device));
    VHX_STREAM(c);
    WriteScope ws(c);  // frames in flight on the tree's other contexts finish reading it first
    int rc = ws.rc;
    if (!rc) rc = alloc_tree(c, t);
    if (rc) return rc;
    for (int id = 0; id < 7; ++id) {
        const uint64_t bytes = elem_count(*t, id) * elem_size(id);
        if (bytes) VHX_HIP(c, hipMemcpyAsync(c->tree->raw[id].ptr, src[id], bytes, hipMemcpyHostToDevice, c->stream));
    }
    if ((rc = finish_upload(c))) return rc;
    return ws.end();
}

}  // extern "C"

int vhx::receive_tree(vhx_ctx *c, const vhx_tree_desc &counts,
                      int (*fill)(void *, void *const[7], const uint64_t[7]), void *arg) {
    VHX_HIP(c, hipSetDevice(c->device));
    VHX_STREAM(c);
    WriteScope ws(c);
    int rc = ws.rc;
    if (!rc) rc = alloc_tree(c, &counts);
    if (rc) return rc;
    void *dst[7];
    uint64_t bytes[7];
    for (int id = 0; id < 7; ++id) {
        dst[id] = c->tree->raw[id].ptr;
        bytes[id] = elem_count(c->tree->desc, id) * elem_size(id);
    }
    if ((rc = fill(arg, dst, bytes))) return rc;  // the transfers, enqueued on c's stream
    if ((rc = finish_upload(c))) return rc;       // derived layout from the received buffers (synchronises)
    return ws.end();
}

void vhx::copy_sched(vhx_ctx *c, const vhx_ctx *owner) {
    std::memcpy(c->budgets, owner->budgets, sizeof(c->budgets));
    std::memcpy(c->rpw, owner->rpw, sizeof(c->rpw));
    c->npass = owner->npass;
    c->tw = owner->tw;
    c->scan_multi = owner->scan_multi;
    c->p0lists = owner->p0lists;
    c->resume = owner->resume;
    c->qstate = owner->qstate;
    c->tile_lists = owner->tile_lists;
    c->save_from = owner->save_from;
    c->qorder = owner->qorder;
    c->adaptive = owner->adaptive;
    c->sched_busy = owner->sched_busy;
    c->sched_idle = owner->sched_idle;
    c->cus = owner->cus;
    c->xcd_group = owner->xcd_group;
    c->qblock = owner->qblock;
    c->queue_blocks = owner->queue_blocks;
    c->queue_waves = owner->queue_waves;
    c->queue_waves0 = owner->queue_waves0;
    c->queue_waves0_force = owner->queue_waves0_force;
    c->shadow_budget = owner->shadow_budget;
    c->stage_slots = owner->stage_slots;
    c->frame_interleave = owner->frame_interleave;
    c->tail_on = owner->tail_on;
    c->tail_min = owner->tail_min;
    c->tail_rpw = owner->tail_rpw;
    c->tail_prio = owner->tail_prio;
    if (c->tail_cap != owner->tail_cap) c->tail_valid = false;
    c->tail_cap = owner->tail_cap;
    c->queue_waves_mid = owner->queue_waves_mid;
    c->qxcd = owner->qxcd;
    c->qxcd_all = owner->qxcd_all;
    c->qsort_force = owner->qsort_force;
    c->qsort_passes = owner->qsort_passes;
    c->qsort_blocks = owner->qsort_blocks;
    std::memcpy(c->sparse, owner->sparse, sizeof(c->sparse));
    c->prepass = owner->prepass;
    c->prepass_margin = owner->prepass_margin;
    c->shadow_on = owner->shadow_on;
    std::memcpy(c->shadow_light, owner->shadow_light, sizeof(c->shadow_light));
}

extern "C" {

static int fill_device_copies(void *arg, void *const dst[7], const uint64_t bytes[7]) {
    const std::pair<vhx_ctx *, const vhx_tree_desc *> &a = *(const std::pair<vhx_ctx *, const vhx_tree_desc *> *)arg;
    vhx_ctx *c = a.first;
    const void *src[7] = {a.second->node_type,  a.second->node_ocbits,    a.second->node_children, a.second->voxels,
                          a.second->solid_values, a.second->color_palette, a.second->data_palette};
    for (int id = 0; id < 7; ++id)
        if (bytes[id]) VHX_HIP(c, hipMemcpyAsync(dst[id], src[id], bytes[id], hipMemcpyDefault, c->stream));
    return VHX_OK;
}

int vhx_upload_tree_device(vhx_ctx *c, const vhx_tree_desc *t) {
    if (!c || !t) return VHX_E_INVALID_ARG;
    if (c->shared) return fail(c, VHX_E_STATE, "vhx_upload_tree_device on a shared context: upload through the owner");
    const void *src[7] = {t->node_type, t->node_ocbits, t->node_children, t->voxels,
                          t->solid_values, t->color_palette, t->data_palette};
    for (int id = 0; id < 7; ++id)
        if (elem_count(*t, id) && !src[id])
            return fail(c, VHX_E_INVALID_ARG, "vhx_upload_tree_device: null array with non-zero count");
    std::pair<vhx_ctx *, const vhx_tree_desc *> arg{c, t};
    return receive_tree(c, *t, fill_device_copies, &arg);
}

int vhx_update_ranges(vhx_ctx *c, const vhx_range *r, uint32_t n) {
    if (!c || (n && !r)) return VHX_E_INVALID_ARG;
    if (c->shared) return fail(c, VHX_E_STATE, "vhx_update_range(s) on a shared context: update through the owner");
    if (!c->tree->uploaded) return fail(c, VHX_E_STATE, "vhx_update_range(s) before vhx_upload_tree");
    // validate every range first: a failing call writes nothing
    uint64_t data_bytes = 0, njobs = 0;
    for (uint32_t k = 0; k < n; ++k) {
        if (r[k].buffer_id < 0 || r[k].buffer_id > 6 || (!r[k].src && r[k].elem_count)) return VHX_E_INVALID_ARG;
        const uint64_t cap = elem_count(c->tree->desc, r[k].buffer_id);
        if (r[k].elem_offset > cap || r[k].elem_count > cap - r[k].elem_offset)
            return fail(c, VHX_E_CAPACITY, "vhx_update_range(s): range beyond the uploaded buffer");
        const uint64_t bytes = r[k].elem_count * elem_size(r[k].buffer_id);
        data_bytes += (bytes + 15) & ~15ull;
        njobs += (bytes + UPD_PIECE_BYTES - 1) / UPD_PIECE_BYTES;
    }
    if (data_bytes == 0) return VHX_OK;
    if (njobs > 0xFFFFFFFFull) return fail(c, VHX_E_INVALID_ARG, "vhx_update_ranges: too much data in one call");
    VHX_HIP(c, hipSetDevice(c->device));
    VHX_STREAM(c);
    // the scatter and the derived-state rebuilds write the tree: frames in flight on the other contexts first
    WriteScope ws(c);
    int rc = ws.rc;
    if (rc) return rc;
    // pinned staging slot (the one used two calls ago: its copy has normally long completed)
    vhx_ctx::Pinned &P = c->pinned[c->pinned_next];
    c->pinned_next ^= 1u;
    if (P.used) VHX_HIP(c, hipEventSynchronize(P.done));
    const uint64_t jobs_bytes = (njobs * sizeof(UpdJob) + 255) & ~255ull, total = jobs_bytes + data_bytes;
    if (P.bytes < total) {
        if (P.ptr) VHX_HIP(c, hipHostFree(P.ptr));
        P.ptr = nullptr;
        P.bytes = 0;
        const uint64_t want = std::max<uint64_t>(total + total / 4, 1ull << 20);
        VHX_HIP(c, hipHostMalloc(&P.ptr, want, hipHostMallocDefault));
        P.bytes = want;
    }
    if (!P.done) VHX_HIP(c, hipEventCreateWithFlags(&P.done, hipEventDisableTiming));
    // the device staging buffer: the previous batch's scatter may still read it (on this stream, or on the stream the
    // context used then), so a growth or a stream change waits for it
    if (c->upd_stream && (c->upd_stream != c->stream || c->upd.bytes < P.bytes))
        VHX_HIP(c, hipStreamSynchronize(c->upd_stream));
    rc = ensure(c, c->upd, P.bytes);
    if (rc) return rc;
    c->upd_stream = c->stream;
    // pack: the job table, then each range's data (16-byte aligned)
    UpdJob *jobs = (UpdJob *)P.ptr;
    uint64_t off = jobs_bytes, j = 0;
    // ranges of one scatter launch are written in no particular order, so a range that overlaps an earlier range of
    // the call starts a new launch (launches on a stream run in order: the later write wins, as in a sequence of
    // write_range_to_buffer calls)
    std::vector<uint32_t> group_start{0};
    std::vector<std::pair<uint64_t, uint64_t>> group_spans[7];  // byte spans of the current group, per buffer
    uint32_t node_lo = UINT32_MAX, node_hi = 0, hdr_lo = UINT32_MAX, hdr_hi = 0, brick_lo = UINT32_MAX, brick_hi = 0;
    bool palette = false;
    const uint64_t n3 = (uint64_t)c->tree->desc.brick_dim * c->tree->desc.brick_dim * c->tree->desc.brick_dim;
    for (uint32_t k = 0; k < n; ++k) {
        const int id = r[k].buffer_id;
        const uint64_t es = elem_size(id), bytes = r[k].elem_count * es;
        if (!bytes) continue;
        std::memcpy((uint8_t *)P.ptr + off, r[k].src, bytes);
        const uint64_t dst = (uint64_t)(uintptr_t)c->tree->raw[id].ptr + r[k].elem_offset * es;
        {
            const uint64_t b0 = r[k].elem_offset * es, b1 = b0 + bytes;
            bool overlaps = false;
            for (const auto &sp : group_spans[id]) overlaps |= b0 < sp.second && sp.first < b1;
            if (overlaps) {
                group_start.push_back((uint32_t)j);
                for (auto &g : group_spans) g.clear();
            }
            group_spans[id].push_back({b0, b1});
        }
        for (uint64_t p = 0; p < bytes; p += UPD_PIECE_BYTES) {
            UpdJob &jb = jobs[j++];
            jb.dst = dst + p;
            jb.src_off = off + p;
            jb.words = (uint32_t)(std::min<uint64_t>(UPD_PIECE_BYTES, bytes - p) / 4);
            jb.pad0 = 0;
            jb.pad1 = 0;
        }
        off += (bytes + 15) & ~15ull;
        const uint64_t e0 = r[k].elem_offset, e1 = e0 + r[k].elem_count;
        if (id == VHX_BUF_NODE_TYPE || id == VHX_BUF_NODE_OCBITS) {
            hdr_lo = std::min<uint32_t>(hdr_lo, (uint32_t)e0);
            hdr_hi = std::max<uint32_t>(hdr_hi, (uint32_t)e1);
        }
        if (id == VHX_BUF_NODE_TYPE) {
            node_lo = std::min<uint32_t>(node_lo, (uint32_t)e0);
            node_hi = std::max<uint32_t>(node_hi, (uint32_t)e1);
        } else if (id == VHX_BUF_NODE_CHILDREN) {
            node_lo = std::min<uint32_t>(node_lo, (uint32_t)(e0 / 64));
            node_hi = std::max<uint32_t>(node_hi, (uint32_t)((e1 + 63) / 64));
        } else if (id == VHX_BUF_VOXELS) {
            brick_lo = std::min<uint32_t>(brick_lo, (uint32_t)(e0 / n3));
            brick_hi = std::max<uint32_t>(brick_hi, (uint32_t)((e1 + n3 - 1) / n3));
        } else if (id == VHX_BUF_COLOR_PALETTE || id == VHX_BUF_DATA_PALETTE) {
            palette = true;
        }
    }
    // one host-to-device copy of the packed batch, one scatter kernel
    VHX_HIP(c, hipMemcpyAsync(c->upd.ptr, P.ptr, total, hipMemcpyHostToDevice, c->stream));
    VHX_HIP(c, hipEventRecord(P.done, c->stream));
    P.used = true;
    group_start.push_back((uint32_t)j);
    for (size_t g = 0; g + 1 < group_start.size(); ++g) {
        const uint32_t j0 = group_start[g], j1 = group_start[g + 1];
        if (j1 > j0)
            k_scatter_ranges<<<std::min<uint32_t>(j1 - j0, 8192u), 256, 0, c->stream>>>((const uint8_t *)c->upd.ptr,
                                                                                         j0, j1);
    }
    VHX_HIP(c, hipGetLastError());
    // derived state, stream-ordered
    if (hdr_lo < hdr_hi && (rc = rebuild_hdr(c, hdr_lo, hdr_hi - hdr_lo))) return rc;
    if (palette) {
        // emptiness of any cell may change: every bitmap and record
        if ((rc = rebuild_occ(c, 0, c->tree->desc.brick_count))) return rc;
        c->tree->child_rec_stale = true;
        rc = refresh_child_rec(c);
    } else {
        if (brick_lo < brick_hi && (rc = rebuild_occ(c, brick_lo, brick_hi - brick_lo))) return rc;
        rc = refresh_child_rec_sel(c, node_lo, node_hi, brick_lo, brick_hi);
    }
    if (rc) return rc;
    return ws.end();  // the next trace of every context of the tree waits for this write
}

int vhx_update_range(vhx_ctx *c, int id, uint64_t off, uint64_t count, const void *src) {
    if (!c || id < 0 || id > 6 || (!src && count)) return VHX_E_INVALID_ARG;
    vhx_range r{};
    r.buffer_id = id;
    r.elem_offset = off;
    r.elem_count = count;
    r.src = src;
    return vhx_update_ranges(c, &r, 1);
}

int vhx_read_derived(vhx_ctx *c, int which, uint64_t off, uint64_t count, void *dst) {
    if (!c || (!dst && count) || which < 0 || which > 1) return VHX_E_INVALID_ARG;
    if (!c->tree->uploaded) return fail(c, VHX_E_STATE, "vhx_read_derived before vhx_upload_tree");
    const uint64_t es = which == VHX_DERIVED_NODE_HDR ? 16 : 8;
    const uint64_t cap = which == VHX_DERIVED_NODE_HDR ? c->tree->desc.node_count
                                                       : (uint64_t)c->tree->desc.brick_count * c->tree->occ_words;
    if (off + count > cap) return fail(c, VHX_E_CAPACITY, "vhx_read_derived: range beyond the buffer");
    const DevBuf &b = which == VHX_DERIVED_NODE_HDR ? c->tree->hdr : c->tree->brick_occ;
    VHX_HIP(c, hipSetDevice(c->device));
    VHX_STREAM(c);
    TraceScope tscope(c);  // after the tree's last write
    if (tscope.rc) return tscope.rc;
    VHX_HIP(c, hipMemcpyAsync(dst, (const char *)b.ptr + off * es, count * es, hipMemcpyDeviceToHost, c->stream));
    VHX_HIP(c, hipStreamSynchronize(c->stream));
    return tscope.end();
}

int vhx_tree_device_bytes(const vhx_ctx *c, uint64_t *bytes) {
    if (!c || !bytes) return VHX_E_INVALID_ARG;
    uint64_t b = c->tree->hdr.bytes + c->tree->brick_occ.bytes + c->tree->child_rec.bytes;
    for (auto &r : c->tree->raw) b += r.bytes;
    *bytes = b;
    return VHX_OK;
}

static CamD cam_of(const vhx_camera *cam) {
    CamD d;
    d.model = cam->ray_model;
    d.width = cam->width;
    d.height = cam->height;
    d.ox = cam->origin[0];
    d.oy = cam->origin[1];
    d.oz = cam->origin[2];
    d.blx = cam->glass_bottom_left[0];
    d.bly = cam->glass_bottom_left[1];
    d.blz = cam->glass_bottom_left[2];
    d.rx = cam->glass_right[0];
    d.ry = cam->glass_right[1];
    d.rz = cam->glass_right[2];
    d.ux = cam->glass_up[0];
    d.uy = cam->glass_up[1];
    d.uz = cam->glass_up[2];
    d.pw = cam->pixel_width;
    d.ph = cam->pixel_height;
    std::memcpy(d.m, cam->inv_view_proj, sizeof(d.m));
    return d;
}

int vhx_trace_primary(vhx_ctx *c, const vhx_camera *cam, uint32_t T, uint32_t tile_start, uint32_t tile_stride,
                      uint32_t layout, const vhx_hits *out, int on_device) {
    if (!c || !cam || !out) return VHX_E_INVALID_ARG;
    if (!c->tree->uploaded) return fail(c, VHX_E_STATE, "vhx_trace_primary before vhx_upload_tree");
    if (cam->width == 0 || cam->height == 0 || cam->ray_model > VHX_RAY_GLASS || layout > VHX_LAYOUT_TILES)
        return fail(c, VHX_E_INVALID_ARG, "vhx_trace_primary: bad camera or layout");
    if (T == 0) {
        if (layout != VHX_LAYOUT_FRAMEBUFFER) return fail(c, VHX_E_INVALID_ARG, "tile_size 0 needs the framebuffer layout");
        T = 16;
        tile_start = 0;
        tile_stride = 1;
    }
    if (tile_stride == 0) return fail(c, VHX_E_INVALID_ARG, "tile_stride 0");
    const uint32_t tiles_x = (cam->width + T - 1) / T, tiles_y = (cam->height + T - 1) / T;
    const uint32_t ntiles = tiles_x * tiles_y;
    if (tile_start >= ntiles) return VHX_OK;
    const uint32_t my_tiles = (ntiles - tile_start + tile_stride - 1) / tile_stride;
    const uint32_t bpx = (T + 15) / 16, bpt = bpx * bpx;
    const uint64_t nblocks = (uint64_t)my_tiles * bpt;
    if (nblocks > 0x7FFFFFFFull) return fail(c, VHX_E_INVALID_ARG, "frame too large");
    const uint64_t nout = layout == VHX_LAYOUT_FRAMEBUFFER ? (uint64_t)cam->width * cam->height
                                                           : (uint64_t)my_tiles * T * T;
    VHX_HIP(c, hipSetDevice(c->device));
    VHX_STREAM(c);
    // after the tree's last write (an update through the owner, on its stream); the prepass's inner frame runs inside
    // the outer frame's scope
    TraceScope tscope(c, c->in_prepass);
    int rc = tscope.rc;
    if (rc) return rc;
    HostOut ho;
    rc = map_out(c, out, nout, on_device, ho, layout == VHX_LAYOUT_TILES);
    if (rc) return rc;
    if ((rc = refresh_child_rec(c))) return rc;
    const DevTree t = dev_tree(c);
    if (t.mips && (out->bytes || (c->prepass && !c->in_prepass)))
        return fail(c, VHX_E_INVALID_ARG, "vhx_trace_primary: byte counting and the depth prepass are not available "
                                          "with node MIPs (vhx_set_node_mips)");
    // fused hard shadows (vhx_set_shadow_light): the shadow rays start from the stored hit records
    const bool shadows = c->shadow_on && !c->in_prepass;
    if (shadows && (!out->value || !out->impact || !out->normal || !out->shadowed || out->bytes || t.mips || c->prepass))
        return fail(c, VHX_E_INVALID_ARG, "vhx_trace_primary with a shadow light: value, impact, normal and shadowed "
                                          "outputs needed; no byte counting, node MIPs or depth prepass");
    const CamD cd = cam_of(cam);
    uint32_t npass = 1;
    rc = prepare_passes(c, nout, nblocks, npass);
    if (rc) return rc;
    // pass 0's list buffers for either schedule's queue order: a context's first frames often run alone (the idle
    // schedule), and growing the buffers at its first frame among others would hipFree -- a device-wide
    // synchronisation that drains every frame in flight (measured: 0.61 against 0.54 ms per bench frame)
    if (c->p0lists && layout == VHX_LAYOUT_FRAMEBUFFER && T == 16 && tile_start == 0 && tile_stride == 1) {
        const uint32_t orders[2] = {c->sched_busy.qorder, c->qorder};
        for (uint32_t o : orders) {
            ListOrder l2{};
            uint64_t nb2 = 0;
            if (list_order(o, cam->width, cam->height, l2, nb2) && (rc = ensure_lists(c, nb2))) return rc;
        }
    }
    RaySrc src{};
    src.kind = layout == VHX_LAYOUT_FRAMEBUFFER ? 0u : 1u;
    src.T = T;
    src.tiles_x = tiles_x;
    src.tile_start = tile_start;
    src.tile_stride = tile_stride;
    if (!c->in_prepass) VHX_HIP(c, hipEventRecord(c->ev0, c->stream));
    // depth-prepass mode (vhx_set_depth_prepass): a whole framebuffer frame without byte counting first traces the
    // half-resolution depth frame (a nested call, same stream), then the full frame starts from it
    const bool fast = c->prepass && !c->in_prepass && layout == VHX_LAYOUT_FRAMEBUFFER && tile_start == 0 &&
                      tile_stride == 1 && !out->bytes;
    FastD fd{};
    if (fast) {
        vhx_camera hc = *cam;
        hc.width = (cam->width + 1) / 2;
        hc.height = (cam->height + 1) / 2;
        if (cam->ray_model == VHX_RAY_GLASS) {
            // texel (X, Y) looks through the centre of full pixels 2X..2X+1, 2Y..2Y+1 (y counted upward in the glass)
            const float ox = 0.5f * cam->pixel_width, oy = ((float)cam->height + 0.5f - 2.0f * (float)hc.height) * cam->pixel_height;
            for (int k = 0; k < 3; ++k)
                hc.glass_bottom_left[k] = cam->glass_bottom_left[k] + cam->glass_right[k] * ox + cam->glass_up[k] * oy;
            hc.pixel_width = 2.0f * cam->pixel_width;
            hc.pixel_height = 2.0f * cam->pixel_height;
        }
        int rc2 = ensure(c, c->prepass_depth, (uint64_t)hc.width * hc.height * 4);
        if (rc2) return rc2;
        vhx_hits dh{};
        dh.depth = (float *)c->prepass_depth.ptr;
        c->in_prepass = true;
        rc2 = vhx_trace_primary(c, &hc, 0, 0, 1, VHX_LAYOUT_FRAMEBUFFER, &dh, 1);
        c->in_prepass = false;
        if (rc2) return rc2;
        fd = FastD{(const float *)c->prepass_depth.ptr, hc.width, hc.height, c->prepass_margin};
    }
    // no reset_passes: the flag compaction after pass 0 zeroes the queue passes' counters.
    // A rank-sharded framebuffer (tile_start > 0 or tile_stride > 1) leaves the flags of other ranks' pixels unwritten,
    // while the compaction scans every pixel: they are cleared first (stale flags would queue foreign pixels)
    if (npass > 1 && layout == VHX_LAYOUT_FRAMEBUFFER && (tile_start > 0 || tile_stride > 1))
        VHX_HIP(c, hipMemsetAsync(c->flags.ptr, 0, nout, c->stream));

    const bool count = ho.dev.bytes != nullptr;
    int qrc = VHX_OK;
    // the queue order's frame (c->qorder): the framebuffer layout only. The tile layout's output index is already
    // tile-major with T-wide rows inside a tile (config 4 on one rank, 64x64 tiles: 2.019-2.025 ms per frame in that
    // order against 2.071-2.074 with the tiles re-ordered Morton inside, profiles/r03/qorder/mgpu1_*.log)
    const uint32_t ow = layout == VHX_LAYOUT_FRAMEBUFFER ? cam->width : 0u;
    const uint32_t oh = cam->height;
    // a whole framebuffer frame in the default queue order: pass 0 lists its rays in that order itself (ListOrder)
    ListOrder lo{};
    uint64_t nb0 = nblocks;
    bool listed = c->p0lists && npass > 1 && layout == VHX_LAYOUT_FRAMEBUFFER && T == 16 && tile_start == 0 &&
                  tile_stride == 1 && list_order(c->qorder, cam->width, cam->height, lo, nb0);
    if (!listed) lo = ListOrder{}, nb0 = nblocks;
    // a tile set (the rank's share of a multi-GPU frame) under the frames-in-flight schedule lists its rays in its own
    // block order: no flag per entry, no compaction over every entry, and the queue-state mode (ListOrder::tl)
    if (!listed && c->p0lists && c->tile_lists && npass > 1 && layout == VHX_LAYOUT_TILES && c->qorder != 0) {
        listed = true;
        lo.tl = 1;
    }
    if (listed && (rc = ensure_lists(c, nb0))) return rc;
    if ((listed ? nb0 * 4 : nb0) > 0x7FFFFFFFull) return fail(c, VHX_E_INVALID_ARG, "frame too large");
    const int p0 = listed ? P0_ORDERED : P0_FLAGS;
    const bool qm = queue_state_mode(c, listed, false, npass);
    // shadows fuse into the ladder where pass 0 lists its rays (the list entries carry the shadow tag); a single pass
    // or the lone frame's flag compaction traces them after the primary rays instead (below)
    const bool fuse = shadows && listed && npass > 1;
    // early tail (vhx_ctx::tail_*): a lone frame (the idle schedule) of a whole framebuffer on the exact path records
    // its longest rays; with a list recorded by this context's last such frame of the same size, they start now
    const bool tail = c->tail_on && !fast && !ho.dev.bytes && !t.mips && !shadows && !listed && npass > 1 &&
                      c->last_sched == 0 && layout == VHX_LAYOUT_FRAMEBUFFER && T == 16 && tile_start == 0 &&
                      tile_stride == 1 && c->tail_cap > 0;
    bool tail_use = false;
    const uint32_t tail_blocks = (c->tail_cap + c->tail_rpw * 4u - 1u) / (c->tail_rpw * 4u);
    if (tail) {
        const uint64_t lbytes = (64ull + c->tail_cap) * 4ull, mbytes = ((nout + 31) / 32) * 4;
        if ((rc = ensure(c, c->tail_list[0], lbytes)) || (rc = ensure(c, c->tail_list[1], lbytes)) ||
            (rc = ensure(c, c->tail_mask, mbytes)))
            return rc;
        if (!c->tail_stream) {
            int least = 0, greatest = 0;
            VHX_HIP(c, hipDeviceGetStreamPriorityRange(&least, &greatest));
            VHX_HIP(c, hipStreamCreateWithPriority(&c->tail_stream, hipStreamNonBlocking, greatest));
            VHX_HIP(c, hipEventCreateWithFlags(&c->tail_fork, hipEventDisableTiming));
            VHX_HIP(c, hipEventCreateWithFlags(&c->tail_join, hipEventDisableTiming));
        }
        uint32_t *next = (uint32_t *)c->tail_list[c->tail_cur ^ 1u].ptr;
        VHX_HIP(c, hipMemsetAsync(next, 0, 4, c->stream));
        tail_use = c->tail_valid && c->tail_w == cam->width && c->tail_h == cam->height;
        if (tail_use) {
            VHX_HIP(c, hipMemsetAsync(c->tail_mask.ptr, 0, mbytes, c->stream));
            k_tail_mask<<<16, 256, 0, c->stream>>>((const uint32_t *)c->tail_list[c->tail_cur].ptr, c->tail_cap,
                                                   (uint32_t)nout, (uint32_t *)c->tail_mask.ptr);
            VHX_HIP(c, hipEventRecord(c->tail_fork, c->stream));
            VHX_HIP(c, hipStreamWaitEvent(c->tail_stream, c->tail_fork, 0));
        }
        c->tail_rec = next;
    }
    auto launch = [&](auto bd_tag) {
        constexpr int BD = decltype(bd_tag)::value;
        PassQ q0 = pass_q(c, 0, npass, qm);
        if (listed)
            q0.zero = (uint32_t *)c->qctl.ptr + 16;
        else if (npass > 1)
            q0.flags = (uint8_t *)c->flags.ptr;
        const unsigned g0 = (unsigned)nb0;
        if (t.mips) {  // MIP stand-ins (no byte counting, no depth prepass: refused above)
            k_trace_primary<false, BD, false, true><<<g0, 256, 0, c->stream>>>(
                t, cd, ho.dev, T, tiles_x, tile_start, tile_stride, layout, bpx, bpt, q0, FastD{}, lo);
            qrc = launch_queue_passes<false, BD, true>(c, t, cd, src, ho.dev, 1, npass, nout, nb0, p0, ow, oh, 1, qm);
        } else if (count) {
            k_trace_primary<true, BD><<<g0, 256, 0, c->stream>>>(
                t, cd, ho.dev, T, tiles_x, tile_start, tile_stride, layout, bpx, bpt, q0, FastD{}, lo);
            qrc = launch_queue_passes<true, BD>(c, t, cd, src, ho.dev, 1, npass, nout, nb0, p0, ow, oh, 1, qm);
        } else if (fuse) {  // listed pass 0 and queue passes with the shadow continuations
            k_trace_primary<false, BD, false, false, true><<<g0, 256, 0, c->stream>>>(
                t, cd, ho.dev, T, tiles_x, tile_start, tile_stride, layout, bpx, bpt, q0, FastD{}, lo);
            qrc = launch_queue_passes<false, BD, false, true>(c, t, cd, src, ho.dev, 1, npass, nout, nb0, p0, ow, oh, 1,
                                                              qm);
        } else {
            if (tail_use) {  // the listed long rays first, on the second stream; pass 0 skips them
                k_trace_tail<BD><<<tail_blocks, 256, 0, c->tail_stream>>>(
                    t, cd, ho.dev, (const uint32_t *)c->tail_list[c->tail_cur].ptr, c->tail_rec, c->tail_cap,
                    c->tail_min, c->tail_rpw, c->tail_prio);
                q0.skip = (const uint32_t *)c->tail_mask.ptr;
            }
            if (fast)
                k_trace_primary<false, BD, true><<<g0, 256, 0, c->stream>>>(
                    t, cd, ho.dev, T, tiles_x, tile_start, tile_stride, layout, bpx, bpt, q0, fd, lo);
            else
                k_trace_primary<false, BD><<<g0, 256, 0, c->stream>>>(
                    t, cd, ho.dev, T, tiles_x, tile_start, tile_stride, layout, bpx, bpt, q0, FastD{}, lo);
            qrc = launch_queue_passes<false, BD>(c, t, cd, src, ho.dev, 1, npass, nout, nb0, p0, ow, oh, 1, qm);
        }
    };
    const bool bd_ok = dispatch_bd(c->tree->desc.brick_dim, launch);
    c->tail_rec = nullptr;
    if (tail) {
        // the frame ends with its early tail (joined before ev1 and the trace's use event); its record is next frame's
        // list (the list it traced stays valid: an error below still leaves two well-formed lists)
        if (tail_use) {
            VHX_HIP(c, hipEventRecord(c->tail_join, c->tail_stream));
            VHX_HIP(c, hipStreamWaitEvent(c->stream, c->tail_join, 0));
        }
        c->tail_cur ^= 1u;
        c->tail_valid = true;
        c->tail_w = cam->width;
        c->tail_h = cam->height;
    }
    if (!bd_ok) return fail(c, VHX_E_INVALID_ARG, "unsupported brick_dim");
    if (qrc) return qrc;
    VHX_HIP(c, hipGetLastError());
    if (c->in_prepass) return VHX_OK;  // the outer call records the end and copies its outputs
    // a shadow trace of this frame's hit records lists them in the same tile order (vhx_trace_shadows)
    c->last_fb_w = layout == VHX_LAYOUT_FRAMEBUFFER ? cam->width : 0u;
    c->last_fb_h = layout == VHX_LAYOUT_FRAMEBUFFER ? cam->height : 0u;
    VHX_HIP(c, hipEventRecord(c->ev1, c->stream));
    c->timed = true;
    if ((rc = tscope.end())) return rc;  // a later write of the tree waits for this frame
    if (shadows && !fuse) {
        // the frame's shadow rays after its primary rays (vhx_trace_shadows on the same stream); the frame's time then
        // spans both (ev0 of the primary trace, ev1 re-recorded by the shadow trace)
        c->keep_ev0 = true;
        rc = vhx_trace_shadows(c, c->shadow_light, nout, ho.dev.value, ho.dev.impact, ho.dev.normal, ho.dev.shadowed,
                               ho.dev.rgba, nullptr);
        c->keep_ev0 = false;
        if (rc) return rc;
    }
    return finish_out(c, ho);
}

// The next slot of a context's pinned staging ring, sized for `bytes`: the host waits only if that slot's previous copy
// (VHX_STAGE_SLOTS batches ago on this context) has not run yet
static int stage_slot(vhx_ctx *c, vhx_ctx::Pinned *ring, uint32_t &next, uint64_t bytes, vhx_ctx::Pinned *&out) {
    vhx_ctx::Pinned &P = ring[next];
    next = (next + 1) % std::max<uint32_t>(1u, std::min(c->stage_slots, vhx_ctx::VHX_STAGE_SLOTS));
    if (P.used) VHX_HIP(c, hipEventSynchronize(P.done));
    if (P.bytes < bytes) {
        if (P.ptr) VHX_HIP(c, hipHostFree(P.ptr));
        P.ptr = nullptr;
        P.bytes = 0;
        VHX_HIP(c, hipHostMalloc(&P.ptr, bytes, hipHostMallocDefault));
        P.bytes = bytes;
    }
    if (!P.done) VHX_HIP(c, hipEventCreateWithFlags(&P.done, hipEventDisableTiming));
    out = &P;
    return VHX_OK;
}

// A batch of whole frames (T == 0: vhx_trace_primary_batch) or of tile sets (T > 0: vhx_trace_tiles_batch; frame k is
// the tiles starts[k], starts[k] + stride, ... of its camera's T x T tile grid, in the tile layout) as one pass ladder.
static int trace_batch(vhx_ctx *c, const vhx_camera *cams, uint32_t n, const vhx_hits *outs, uint32_t T,
                       const uint32_t *starts, uint32_t stride, const char *fn) {
    if (!c || !cams || !outs || n == 0 || (T && (!starts || stride == 0 || T > 4096))) return VHX_E_INVALID_ARG;
    if (!c->tree->uploaded) return fail(c, VHX_E_STATE, std::string(fn) + " before vhx_upload_tree");
    const uint32_t W = cams[0].width, H = cams[0].height;
    for (uint32_t k = 0; k < n; ++k) {
        if (cams[k].width != W || cams[k].height != H || W == 0 || H == 0 || cams[k].ray_model > VHX_RAY_GLASS)
            return fail(c, VHX_E_INVALID_ARG, std::string(fn) + ": every frame needs one valid camera model and the "
                                              "same non-empty width x height");
        if (outs[k].bytes)
            return fail(c, VHX_E_INVALID_ARG, std::string(fn) + ": byte counting is a vhx_trace_primary option");
        if (c->shadow_on && (!outs[k].value || !outs[k].impact || !outs[k].normal || !outs[k].shadowed))
            return fail(c, VHX_E_INVALID_ARG, std::string(fn) + " with a shadow light: value, impact, normal and "
                                              "shadowed outputs needed");
    }
    // per frame: its output entries (a tile set: its tiles' entries), the index stride between frames (npix) and the
    // pass-0 workgroups (nbf)
    const uint32_t tiles_x = T ? (W + T - 1) / T : 0u, ntiles = T ? tiles_x * ((H + T - 1) / T) : 0u;
    const uint32_t bpx = T ? (T + 15) / 16 : 0u, bpt = bpx * bpx;
    auto set_tiles = [&](uint32_t k) -> uint64_t {
        return starts[k] >= ntiles ? 0ull : (uint64_t)(ntiles - starts[k] + stride - 1) / stride;
    };
    uint64_t max_tiles = 0;
    if (T)
        for (uint32_t k = 0; k < n; ++k) max_tiles = std::max(max_tiles, set_tiles(k));
    if (T && max_tiles == 0) return VHX_OK;  // no frame holds a tile
    const uint64_t npix = T ? max_tiles * T * T : (uint64_t)W * H, nout = npix * n;
    // the frames are traced concurrently: two frames writing one output range would leave a result that depends on the
    // schedule instead of equalling n single-frame calls
    {
        struct R {
            const char *p;
            uint64_t bytes;
        };
        std::vector<R> rs;
        for (uint32_t k = 0; k < n; ++k) {
            const vhx_hits &o = outs[k];
            const uint64_t ent = T ? set_tiles(k) * T * T : npix;
            const void *f[7] = {o.value, o.cell, o.rgba, o.depth, o.voxel, o.impact, o.normal};
            const uint64_t w[7] = {1, 1, 1, 1, 3, 3, 3};
            for (int j = 0; j < 7; ++j)
                if (f[j] && ent) rs.push_back({(const char *)f[j], ent * 4 * w[j]});
        }
        std::sort(rs.begin(), rs.end(), [](const R &a, const R &b) { return a.p < b.p; });
        for (size_t i = 1; i < rs.size(); ++i)
            if (rs[i].p < rs[i - 1].p + rs[i - 1].bytes)
                return fail(c, VHX_E_INVALID_ARG, std::string(fn) + ": output arrays overlap each other");
    }
    const uint32_t bx = (W + 15) / 16, by = (H + 15) / 16;
    const uint64_t nbf = T ? max_tiles * bpt : (uint64_t)bx * by, nblocks = nbf * n;
    if (nout > 0x7FFFFFFFull || nblocks > 0x7FFFFFFFull)
        return fail(c, VHX_E_INVALID_ARG, std::string(fn) + ": more than 2^31 rays in one batch");
    VHX_HIP(c, hipSetDevice(c->device));
    VHX_STREAM(c);
    TraceScope tscope(c);
    int rc = tscope.rc;
    if (rc) return rc;
    if ((rc = refresh_child_rec(c))) return rc;
    const DevTree t = dev_tree(c);
    if (t.mips) return fail(c, VHX_E_INVALID_ARG, std::string(fn) + ": not available with node MIPs");
    // the batch's cameras, outputs (and tile-set starts): packed into the next slot of the context's pinned staging ring,
    // one copy to the device ahead of the launches on the context's stream (stage_slot: back-to-back batches on one
    // context do not wait on the host until the ring wraps onto a copy that has not run)
    const uint64_t cam_bytes = ((uint64_t)n * sizeof(CamD) + 255) & ~255ull;
    const uint64_t out_bytes = ((uint64_t)n * sizeof(OutD) + 255) & ~255ull;
    const uint64_t args_bytes = cam_bytes + out_bytes + (T ? (uint64_t)n * 4 : 0ull);
    vhx_ctx::Pinned *PP = nullptr;
    if ((rc = stage_slot(c, c->batch_pinned, c->batch_next, args_bytes, PP))) return rc;
    vhx_ctx::Pinned &P = *PP;
    // the device copy is read by this context's earlier batches: a stream change waits for them
    if (c->use_recorded && c->use_stream != c->stream) VHX_HIP(c, hipStreamWaitEvent(c->stream, c->use_ev, 0));
    if ((rc = ensure(c, c->batch_args, args_bytes))) return rc;
    CamD *hc = (CamD *)P.ptr;
    OutD *ho = (OutD *)((uint8_t *)P.ptr + cam_bytes);
    for (uint32_t k = 0; k < n; ++k) {
        hc[k] = cam_of(&cams[k]);
        ho[k] = OutD{outs[k].value, outs[k].cell,   outs[k].voxel, outs[k].rgba,
                     nullptr,       outs[k].impact, outs[k].normal, outs[k].depth, outs[k].shadowed};
    }
    if (T) std::memcpy((uint8_t *)P.ptr + cam_bytes + out_bytes, starts, (size_t)n * 4);
    uint32_t npass = 1;
    if ((rc = prepare_passes(c, nout, nblocks, npass, false, n > 1))) return rc;
    VHX_HIP(c, hipEventRecord(c->ev0, c->stream));
    VHX_HIP(c, hipMemcpyAsync(c->batch_args.ptr, P.ptr, args_bytes, hipMemcpyHostToDevice, c->stream));
    VHX_HIP(c, hipEventRecord(P.done, c->stream));
    P.used = true;
    const CamD *dcams = (const CamD *)c->batch_args.ptr;
    const OutD *douts = (const OutD *)((const uint8_t *)c->batch_args.ptr + cam_bytes);
    const uint32_t *dstarts = T ? (const uint32_t *)((const uint8_t *)c->batch_args.ptr + cam_bytes + out_bytes) : nullptr;
    RaySrc src{};
    src.kind = 4u;
    src.cams = dcams;
    src.outs = douts;
    src.npix = (uint32_t)npix;
    src.T = T;
    src.tiles_x = tiles_x;
    src.tile_stride = stride;
    src.starts = dstarts;
    const TileB tb{T, tiles_x, ntiles, stride, bpx, bpt, dstarts};
    const CamD cd{};
    int qrc = VHX_OK;
    // the frames' blocks over whole tiles of the list order (k_trace_primary), or flags in the flag order; a batch of
    // tile sets lists its rays in its own block order (ListOrder::tl) or compacts flags in output-index order
    ListOrder lo{};
    uint64_t nbf0 = nbf;
    bool listed = !T && c->p0lists && npass > 1 && list_order(c->qorder, W, H, lo, nbf0) && nbf0 * n * 4 <= 0x7FFFFFFFull;
    if (!listed) lo = ListOrder{}, nbf0 = nbf;
    if (T && c->p0lists && c->tile_lists && npass > 1 && nbf * n * 4 <= 0x7FFFFFFFull) {
        listed = true;
        lo.tl = 1;
    }
    if (listed && (rc = ensure_lists(c, nbf0 * n))) return rc;
    const bool qm = queue_state_mode(c, listed, false, npass);
    const bool fuse = c->shadow_on && listed && npass > 1;  // vhx_trace_primary's rule
    auto launch = [&](auto bd_tag) {
        constexpr int BD = decltype(bd_tag)::value;
        PassQ q0 = pass_q(c, 0, npass, qm);
        if (listed)
            q0.zero = (uint32_t *)c->qctl.ptr + 16;
        else if (npass > 1)
            q0.flags = (uint8_t *)c->flags.ptr;
        if (fuse) {
            k_trace_primary_batch<BD, true><<<(unsigned)(nbf0 * n), 256, 0, c->stream>>>(
                t, dcams, douts, (uint32_t)nbf0, bx, (uint32_t)npix, q0, lo, tb);
            qrc = launch_queue_passes<false, BD, false, true>(c, t, cd, src, OutD{}, 1, npass, nout, nbf0 * n,
                                                              P0_ORDERED, T ? 0u : W, H, n, qm);
        } else {
            k_trace_primary_batch<BD><<<(unsigned)(nbf0 * n), 256, 0, c->stream>>>(t, dcams, douts, (uint32_t)nbf0, bx,
                                                                                   (uint32_t)npix, q0, lo, tb);
            qrc = launch_queue_passes<false, BD>(c, t, cd, src, OutD{}, 1, npass, nout, nbf0 * n,
                                                 listed ? P0_ORDERED : P0_FLAGS, T ? 0u : W, H, n, qm);
        }
    };
    if (!dispatch_bd(c->tree->desc.brick_dim, launch)) return fail(c, VHX_E_INVALID_ARG, "unsupported brick_dim");
    if (qrc) return qrc;
    VHX_HIP(c, hipGetLastError());
    // a shadow trace (or shadow batch) of these frames' hit records lists them in the same tile order
    c->last_fb_w = T ? 0u : W;
    c->last_fb_h = T ? 0u : H;
    VHX_HIP(c, hipEventRecord(c->ev1, c->stream));
    c->timed = true;
    if ((rc = tscope.end())) return rc;
    if (c->shadow_on && !fuse) {  // the frames' shadow rays after their primary rays (vhx_trace_primary's fallback)
        c->keep_ev0 = true;
        for (uint32_t k = 0; k < n && !rc; ++k) {
            const uint64_t ent = T ? set_tiles(k) * T * T : npix;
            if (ent)
                rc = vhx_trace_shadows(c, c->shadow_light, ent, outs[k].value, outs[k].impact, outs[k].normal,
                                       outs[k].shadowed, outs[k].rgba, nullptr);
        }
        c->keep_ev0 = false;
    }
    return rc;
}

int vhx_trace_primary_batch(vhx_ctx *c, const vhx_camera *cams, uint32_t n, const vhx_hits *outs) {
    return trace_batch(c, cams, n, outs, 0, nullptr, 1, "vhx_trace_primary_batch");
}

int vhx_trace_tiles_batch(vhx_ctx *c, const vhx_camera *cams, uint32_t n, uint32_t tile_size, const uint32_t *tile_starts,
                          uint32_t tile_stride, const vhx_hits *outs) {
    if (tile_size == 0) return c ? fail(c, VHX_E_INVALID_ARG, "vhx_trace_tiles_batch: tile_size 0") : VHX_E_INVALID_ARG;
    return trace_batch(c, cams, n, outs, tile_size, tile_starts, tile_stride, "vhx_trace_tiles_batch");
}

int vhx_tail_info(vhx_ctx *c, uint32_t *listed, uint32_t *width, uint32_t *height) {
    if (!c) return VHX_E_INVALID_ARG;
    uint32_t n = 0;
    if (c->tail_on && c->tail_valid && c->tail_list[c->tail_cur].ptr) {
        VHX_HIP(c, hipSetDevice(c->device));
        VHX_STREAM(c);
        VHX_HIP(c, hipMemcpyAsync(&n, c->tail_list[c->tail_cur].ptr, 4, hipMemcpyDeviceToHost, c->stream));
        VHX_HIP(c, hipStreamSynchronize(c->stream));
        n = std::min(n, c->tail_cap);
    }
    if (listed) *listed = n;
    if (width) *width = c->tail_valid ? c->tail_w : 0u;
    if (height) *height = c->tail_valid ? c->tail_h : 0u;
    return VHX_OK;
}

int vhx_chain_profile(vhx_ctx *c, const vhx_camera *cam, const uint32_t *pixels, uint32_t n, uint64_t *out) {
    if (!c || !cam || (n && (!pixels || !out))) return VHX_E_INVALID_ARG;
#if VHX_CHAIN
    if (!c->tree->uploaded) return fail(c, VHX_E_STATE, "vhx_chain_profile before vhx_upload_tree");
    if (n == 0) return VHX_OK;
    for (uint32_t k = 0; k < n; ++k)
        if (pixels[k] >= (uint64_t)cam->width * cam->height) return fail(c, VHX_E_INVALID_ARG, "vhx_chain_profile: pixel outside the frame");
    VHX_HIP(c, hipSetDevice(c->device));
    VHX_STREAM(c);
    TraceScope tscope(c);
    int rc = tscope.rc;
    if (rc) return rc;
    if ((rc = refresh_child_rec(c))) return rc;
    const DevTree t = dev_tree(c);
    if (t.mips) return fail(c, VHX_E_INVALID_ARG, "vhx_chain_profile: not with node MIPs");
    const uint64_t pbytes = ((uint64_t)n * 4 + 255) & ~255ull, obytes = (uint64_t)n * VHX_CHAIN_WORDS * 8;
    if ((rc = ensure(c, c->scratch, pbytes + obytes))) return rc;
    uint32_t *dpix = (uint32_t *)c->scratch.ptr;
    unsigned long long *dout = (unsigned long long *)((uint8_t *)c->scratch.ptr + pbytes);
    VHX_HIP(c, hipMemcpyAsync(dpix, pixels, (uint64_t)n * 4, hipMemcpyHostToDevice, c->stream));
    const CamD cd = cam_of(cam);
    auto launch = [&](auto bd_tag) {
        constexpr int BD = decltype(bd_tag)::value;
        k_chain<BD><<<n, 64, 0, c->stream>>>(t, cd, dpix, n, dout);
    };
    if (!dispatch_bd(c->tree->desc.brick_dim, launch)) return fail(c, VHX_E_INVALID_ARG, "unsupported brick_dim");
    VHX_HIP(c, hipGetLastError());
    VHX_HIP(c, hipMemcpyAsync(out, dout, obytes, hipMemcpyDeviceToHost, c->stream));
    VHX_HIP(c, hipStreamSynchronize(c->stream));
    return tscope.end();
#else
    return fail(c, VHX_E_STATE, "vhx_chain_profile: libvhx was built without VHX_CHAIN");
#endif
}

int vhx_profile_counters(vhx_ctx *c, uint64_t *out, uint32_t n, int reset) {
    if (!c || (n && !out)) return VHX_E_INVALID_ARG;
#if VHX_PROF
    uint64_t v[5 * 16 * 2];
    VHX_HIP(c, hipSetDevice(c->device));
    VHX_HIP(c, hipDeviceSynchronize());
    VHX_HIP(c, hipMemcpyFromSymbol(v, HIP_SYMBOL(vhx::g_prof), sizeof(v)));
    for (uint32_t i = 0; i < n && i < 5 * 16 * 2; ++i) out[i] = v[i];
    if (reset) {
        std::memset(v, 0, sizeof(v));
        VHX_HIP(c, hipMemcpyToSymbol(HIP_SYMBOL(vhx::g_prof), v, sizeof(v)));
    }
    return VHX_OK;
#else
    (void)reset;
    return fail(c, VHX_E_STATE, "vhx_profile_counters: libvhx was built without VHX_PROF");
#endif
}

int vhx_set_shadow_light(vhx_ctx *c, const float *light) {
    if (!c) return VHX_E_INVALID_ARG;
    if (light && !(std::isfinite(light[0]) && std::isfinite(light[1]) && std::isfinite(light[2])))
        return fail(c, VHX_E_INVALID_ARG, "vhx_set_shadow_light: a finite light position");
    c->shadow_on = light != nullptr;
    for (int k = 0; k < 3; ++k) c->shadow_light[k] = light ? light[k] : 0.0f;
    return VHX_OK;
}

int vhx_set_depth_prepass(vhx_ctx *c, int enable, float margin) {
    if (!c || !(margin >= 0.0f)) return VHX_E_INVALID_ARG;
    c->prepass = enable != 0;
    c->prepass_margin = margin;
    return VHX_OK;
}

int vhx_set_node_mips(vhx_ctx *c, const uint32_t *node_mips, uint32_t count) {
    if (!c) return VHX_E_INVALID_ARG;
    if (c->shared) return fail(c, VHX_E_STATE, "vhx_set_node_mips on a shared context: set them through the owner");
    if (!node_mips) {
        // switching MIPs off is a tree write too: frames in flight finish with the descriptors they started with, and
        // traces on other host threads see the switch in submission order (TreeStore ordering)
        VHX_HIP(c, hipSetDevice(c->device));
        VHX_STREAM(c);
        WriteScope ws(c);
        if (ws.rc) return ws.rc;
        c->tree->mips_on = false;
        return ws.end();
    }
    if (!c->tree->uploaded) return fail(c, VHX_E_STATE, "vhx_set_node_mips: no tree uploaded");
    const vhx_tree_desc &d = c->tree->desc;
    if (count != d.node_count) return fail(c, VHX_E_INVALID_ARG, "vhx_set_node_mips: count != node_count");
    for (uint32_t i = 0; i < count; ++i) {  // every descriptor must name an uploaded brick or solid value
        const uint32_t m = node_mips[i];
        if (m == VHX_EMPTY) continue;
        if ((m & VHX_SOLID_BIT) ? (m & 0x7FFFFFFFu) >= d.solid_count : m >= d.brick_count)
            return fail(c, VHX_E_INVALID_ARG, "vhx_set_node_mips: descriptor out of range");
    }
    VHX_HIP(c, hipSetDevice(c->device));
    VHX_STREAM(c);
    WriteScope ws(c);  // frames in flight may still read the previous descriptors
    int rc = ws.rc;
    if (!rc && c->tree->mips.bytes < (uint64_t)count * 4) VHX_HIP(c, hipStreamSynchronize(c->stream));  // regrowth
    if (!rc) rc = ensure(c, c->tree->mips, (uint64_t)count * 4);
    if (rc) return rc;
    VHX_HIP(c, hipMemcpyAsync(c->tree->mips.ptr, node_mips, (uint64_t)count * 4, hipMemcpyHostToDevice, c->stream));
    VHX_HIP(c, hipStreamSynchronize(c->stream));
    c->tree->mips_on = true;
    return ws.end();
}

int vhx_trace_rays(vhx_ctx *c, const float *rays, uint64_t n, const vhx_hits *out, int on_device) {
    if (!c || !out || (!rays && n)) return VHX_E_INVALID_ARG;
    if (!c->tree->uploaded) return fail(c, VHX_E_STATE, "vhx_trace_rays before vhx_upload_tree");
    if (n == 0) return VHX_OK;
    if ((n + 255) / 256 > 0x7FFFFFFFull) return fail(c, VHX_E_INVALID_ARG, "too many rays");
    VHX_HIP(c, hipSetDevice(c->device));
    VHX_STREAM(c);
    TraceScope tscope(c);
    int rc = tscope.rc;
    if (rc) return rc;
    HostOut ho;
    rc = map_out(c, out, n, on_device, ho);
    if (rc) return rc;
    const float *drays = rays;
    if (!on_device) {
        // context-owned staging buffer (a stream-ordered hipMallocAsync buffer here intermittently handed the
        // kernel stale ray data after a pageable host copy on ROCm 7.2)
        rc = ensure(c, c->rays, n * 24);
        if (rc) return rc;
        VHX_HIP(c, hipMemcpyAsync(c->rays.ptr, rays, n * 24, hipMemcpyHostToDevice, c->stream));
        drays = (const float *)c->rays.ptr;
    }
    if ((rc = refresh_child_rec(c))) return rc;
    const DevTree t = dev_tree(c);
    if (t.mips && out->bytes)
        return fail(c, VHX_E_INVALID_ARG, "vhx_trace_rays: byte counting is not available with node MIPs");
    uint32_t npass = 1;
    const uint64_t nb64 = (n + 255) / 256;
    rc = prepare_passes(c, n, nb64, npass);
    if (rc) return rc;
    RaySrc src{};
    src.kind = 2u;
    src.rays = drays;
    CamD cd{};
    VHX_HIP(c, hipEventRecord(c->ev0, c->stream));
    rc = reset_passes(c, npass);
    if (rc) return rc;
    const bool count = ho.dev.bytes != nullptr;
    const unsigned nb = (unsigned)((n + 255) / 256);
    int qrc = VHX_OK;
    auto launch = [&](auto bd_tag) {
        constexpr int BD = decltype(bd_tag)::value;
        const PassQ q0 = pass_q(c, 0, npass);
        if (t.mips) {
            k_trace_rays<false, BD, true><<<nb, 256, 0, c->stream>>>(t, drays, n, ho.dev, q0);
            qrc = launch_queue_passes<false, BD, true>(c, t, cd, src, ho.dev, 1, npass, n, nb64);
        } else if (count) {
            k_trace_rays<true, BD><<<nb, 256, 0, c->stream>>>(t, drays, n, ho.dev, q0);
            qrc = launch_queue_passes<true, BD>(c, t, cd, src, ho.dev, 1, npass, n, nb64);
        } else {
            k_trace_rays<false, BD><<<nb, 256, 0, c->stream>>>(t, drays, n, ho.dev, q0);
            qrc = launch_queue_passes<false, BD>(c, t, cd, src, ho.dev, 1, npass, n, nb64);
        }
    };
    if (!dispatch_bd(c->tree->desc.brick_dim, launch)) return fail(c, VHX_E_INVALID_ARG, "unsupported brick_dim");
    if (qrc) return qrc;
    VHX_HIP(c, hipGetLastError());
    VHX_HIP(c, hipEventRecord(c->ev1, c->stream));
    c->timed = true;
    if ((rc = tscope.end())) return rc;
    return finish_out(c, ho);
}

int vhx_trace_shadows(vhx_ctx *c, const float light[3], uint64_t n, const uint32_t *value, const float *impact,
                      const float *normal, uint32_t *shadowed, uint32_t *rgba, uint32_t *bytes) {
    if (!c || !light || (n && (!value || !impact || !normal || !shadowed))) return VHX_E_INVALID_ARG;
    if (!c->tree->uploaded) return fail(c, VHX_E_STATE, "vhx_trace_shadows before vhx_upload_tree");
    if (n == 0) return VHX_OK;
    if (n >= 0x7FFFFFFFull) return fail(c, VHX_E_INVALID_ARG, "too many rays");
    // the outputs are written while the hit records are still being read (the flags are cleared by the compaction
    // kernel that reads value[]): they must not overlap them or each other
    {
        struct R {
            const void *p;
            uint64_t bytes;
        } outs[] = {{shadowed, n * 4}, {rgba, n * 4}, {bytes, n * 4}},
          ins[] = {{value, n * 4}, {impact, n * 12}, {normal, n * 12}};
        auto overlap = [](const R &a, const R &b) {
            return a.p && b.p && (const char *)a.p < (const char *)b.p + b.bytes &&
                   (const char *)b.p < (const char *)a.p + a.bytes;
        };
        for (int i = 0; i < 3; ++i) {
            for (int j = 0; j < 3; ++j)
                if (overlap(outs[i], ins[j]))
                    return fail(c, VHX_E_INVALID_ARG, "vhx_trace_shadows: an output overlaps the hit records");
            for (int j = i + 1; j < 3; ++j)
                if (overlap(outs[i], outs[j]))
                    return fail(c, VHX_E_INVALID_ARG, "vhx_trace_shadows: outputs overlap each other");
        }
    }
    VHX_HIP(c, hipSetDevice(c->device));
    VHX_STREAM(c);
    TraceScope tscope(c);
    int rc = tscope.rc;
    if (rc) return rc;
    uint32_t npass = 1;
    const uint64_t nb64 = (n + 255) / 256;
    rc = prepare_passes(c, n, nb64, npass, true);
    if (rc) return rc;
    if ((rc = refresh_child_rec(c))) return rc;
    const DevTree t = dev_tree(c);
    if (t.mips && bytes)
        return fail(c, VHX_E_INVALID_ARG, "vhx_trace_shadows: byte counting is not available with node MIPs");
    RaySrc src{};
    src.kind = 3u;
    src.impact = impact;
    src.normal = normal;
    src.lx = light[0];
    src.ly = light[1];
    src.lz = light[2];
    OutD so{};
    so.value = shadowed;
    so.rgba = rgba;
    so.bytes = bytes;
    CamD cd{};
    if (!c->keep_ev0) VHX_HIP(c, hipEventRecord(c->ev0, c->stream));  // (a fused-shadow fallback keeps the primary's)
    // no reset_passes: the hit compaction (k_count_flags) zeroes the queue passes' counters
    if (bytes) VHX_HIP(c, hipMemsetAsync(bytes, 0, n * 4, c->stream));
    // wave-dense secondary rays: the hit pixels, in frame order, are pass 0's queue
    // (when n is the pixel count of this context's last framebuffer frame, in the tile order of c->qorder: any
    // order is a permutation of 0..n-1, so the records need not even be that frame's for the result to be exact)
    {
        uint64_t npos = n;
        const bool fb = c->last_fb_w && (uint64_t)c->last_fb_w * c->last_fb_h == n;
        const FlagOrder ord = flag_order(fb ? c->qorder : 0u, c->last_fb_w, c->last_fb_h, npos);
        const unsigned nb = (unsigned)((npos + 1023) / 1024);
        uint32_t *counts = (uint32_t *)c->counts.ptr, *offsets = (uint32_t *)c->offsets.ptr;
        k_count_flags<true><<<nb, 256, 0, c->stream>>>(value, npos, counts, (uint32_t *)c->qctl.ptr + 16, shadowed,
                                                       ord, n);
        launch_scan(c, counts, nb, nullptr, 1, offsets, (uint32_t *)c->qctl.ptr + 7, nb);
        k_emit_flags<true><<<nb, 256, 0, c->stream>>>(value, npos, offsets, (uint32_t *)c->queue[1].ptr, ord);
        VHX_HIP(c, hipGetLastError());
    }
    int qrc = VHX_OK;
    auto launch = [&](auto bd_tag) {
        constexpr int BD = decltype(bd_tag)::value;
        if (t.mips)
            qrc = launch_queue_passes<false, BD, true>(c, t, cd, src, so, 0, npass, n, nb64, P0_LISTS, 0, 0, 1,
                                                     queue_state_mode(c, false, true, npass));
        else if (bytes)
            qrc = launch_queue_passes<true, BD>(c, t, cd, src, so, 0, npass, n, nb64, P0_LISTS, 0, 0, 1,
                                                     queue_state_mode(c, false, true, npass));
        else
            qrc = launch_queue_passes<false, BD>(c, t, cd, src, so, 0, npass, n, nb64, P0_LISTS, 0, 0, 1,
                                                     queue_state_mode(c, false, true, npass));
    };
    if (!dispatch_bd(c->tree->desc.brick_dim, launch)) return fail(c, VHX_E_INVALID_ARG, "unsupported brick_dim");
    if (qrc) return qrc;
    VHX_HIP(c, hipGetLastError());
    VHX_HIP(c, hipEventRecord(c->ev1, c->stream));
    c->timed = true;
    return tscope.end();
}

int vhx_trace_shadows_batch(vhx_ctx *c, const float light[3], uint32_t nf, uint64_t n, const vhx_shadow_frame *frames) {
    if (!c || !light || nf == 0 || !frames) return VHX_E_INVALID_ARG;
    if (!c->tree->uploaded) return fail(c, VHX_E_STATE, "vhx_trace_shadows_batch before vhx_upload_tree");
    if (n == 0) return VHX_OK;
    // tested before the product is formed (a huge n would wrap n * nf)
    if (n >= 0x7FFFFFFFull / nf) return fail(c, VHX_E_INVALID_ARG, "vhx_trace_shadows_batch: more than 2^31 records");
    const uint64_t ntot = n * nf;
    // every frame's outputs are written while every frame's hit records are read: no overlaps anywhere in the batch
    {
        struct R {
            const void *p;
            uint64_t bytes;
        };
        std::vector<R> outs, ins;
        for (uint32_t k = 0; k < nf; ++k) {
            const vhx_shadow_frame &f = frames[k];
            if (!f.value || !f.impact || !f.normal || !f.shadowed)
                return fail(c, VHX_E_INVALID_ARG, "vhx_trace_shadows_batch: a frame lacks value, impact, normal or shadowed");
            outs.push_back({f.shadowed, n * 4});
            if (f.rgba) outs.push_back({f.rgba, n * 4});
            ins.push_back({f.value, n * 4});
            ins.push_back({f.impact, n * 12});
            ins.push_back({f.normal, n * 12});
        }
        auto overlap = [](const R &a, const R &b) {
            return (const char *)a.p < (const char *)b.p + b.bytes && (const char *)b.p < (const char *)a.p + a.bytes;
        };
        for (size_t i = 0; i < outs.size(); ++i) {
            for (const R &in : ins)
                if (overlap(outs[i], in))
                    return fail(c, VHX_E_INVALID_ARG, "vhx_trace_shadows_batch: an output overlaps the hit records");
            for (size_t j = i + 1; j < outs.size(); ++j)
                if (overlap(outs[i], outs[j]))
                    return fail(c, VHX_E_INVALID_ARG, "vhx_trace_shadows_batch: outputs overlap each other");
        }
    }
    VHX_HIP(c, hipSetDevice(c->device));
    VHX_STREAM(c);
    TraceScope tscope(c);
    int rc = tscope.rc;
    if (rc) return rc;
    if ((rc = refresh_child_rec(c))) return rc;
    const DevTree t = dev_tree(c);
    if (t.mips) return fail(c, VHX_E_INVALID_ARG, "vhx_trace_shadows_batch: not available with node MIPs");
    uint32_t npass = 1;
    const uint64_t nb64 = (ntot + 255) / 256;
    if ((rc = prepare_passes(c, ntot, nb64, npass, true, nf > 1))) return rc;
    // the frames' ShD records, then their value pointers (FlagOrder::fvals), staged like vhx_trace_primary_batch's
    const uint64_t sh_bytes = ((uint64_t)nf * sizeof(ShD) + 255) & ~255ull, args_bytes = sh_bytes + (uint64_t)nf * 8;
    vhx_ctx::Pinned *PP = nullptr;
    if ((rc = stage_slot(c, c->shadow_pinned, c->shadow_next, args_bytes, PP))) return rc;
    vhx_ctx::Pinned &P = *PP;
    if (c->use_recorded && c->use_stream != c->stream) VHX_HIP(c, hipStreamWaitEvent(c->stream, c->use_ev, 0));
    if ((rc = ensure(c, c->shadow_args, args_bytes))) return rc;
    ShD *hs = (ShD *)P.ptr;
    uint64_t *hv = (uint64_t *)((uint8_t *)P.ptr + sh_bytes);
    for (uint32_t k = 0; k < nf; ++k) {
        hs[k] = ShD{frames[k].value, frames[k].impact, frames[k].normal, frames[k].shadowed, frames[k].rgba};
        hv[k] = (uint64_t)(uintptr_t)frames[k].value;
    }
    VHX_HIP(c, hipEventRecord(c->ev0, c->stream));
    VHX_HIP(c, hipMemcpyAsync(c->shadow_args.ptr, P.ptr, args_bytes, hipMemcpyHostToDevice, c->stream));
    VHX_HIP(c, hipEventRecord(P.done, c->stream));
    P.used = true;
    // shadowed = 0 where no shadow ray is cast (vhx_trace_shadows clears inside its count kernel)
    for (uint32_t k = 0; k < nf; ++k) VHX_HIP(c, hipMemsetAsync(frames[k].shadowed, 0, n * 4, c->stream));
    RaySrc src{};
    src.kind = 5u;
    src.lx = light[0];
    src.ly = light[1];
    src.lz = light[2];
    src.npix = (uint32_t)n;
    src.shs = (const ShD *)c->shadow_args.ptr;
    {
        // every frame's hit records in the tile order of the frames they came from (c->last_fb_*), frame by frame
        uint64_t npos = ntot;
        const bool fb = c->last_fb_w && (uint64_t)c->last_fb_w * c->last_fb_h == n;
        FlagOrder ord = flag_order(fb ? c->qorder : 0u, c->last_fb_w, c->last_fb_h, npos, nf);
        if (!ord.W) npos = ntot;
        ord.fpix = n;
        ord.fvals = (const uint64_t *)((const uint8_t *)c->shadow_args.ptr + sh_bytes);
        const unsigned nb = (unsigned)((npos + 1023) / 1024);
        uint32_t *counts = (uint32_t *)c->counts.ptr, *offsets = (uint32_t *)c->offsets.ptr;
        if ((uint64_t)nb * 4 > c->counts.bytes || (uint64_t)nb * 4 > c->offsets.bytes) {
            if ((rc = ensure_lists(c, nb))) return rc;
            counts = (uint32_t *)c->counts.ptr;
            offsets = (uint32_t *)c->offsets.ptr;
        }
        k_count_flags<true><<<nb, 256, 0, c->stream>>>(nullptr, npos, counts, (uint32_t *)c->qctl.ptr + 16, nullptr, ord);
        launch_scan(c, counts, nb, nullptr, 1, offsets, (uint32_t *)c->qctl.ptr + 7, nb);
        k_emit_flags<true><<<nb, 256, 0, c->stream>>>(nullptr, npos, offsets, (uint32_t *)c->queue[1].ptr, ord);
        VHX_HIP(c, hipGetLastError());
    }
    int qrc = VHX_OK;
    const CamD cd{};
    auto launch = [&](auto bd_tag) {
        constexpr int BD = decltype(bd_tag)::value;
        qrc = launch_queue_passes<false, BD>(c, t, cd, src, OutD{}, 0, npass, ntot, nb64, P0_LISTS, 0, 0, nf,
                                             queue_state_mode(c, false, true, npass));
    };
    if (!dispatch_bd(c->tree->desc.brick_dim, launch)) return fail(c, VHX_E_INVALID_ARG, "unsupported brick_dim");
    if (qrc) return qrc;
    VHX_HIP(c, hipGetLastError());
    VHX_HIP(c, hipEventRecord(c->ev1, c->stream));
    c->timed = true;
    return tscope.end();
}

int vhx_untile_frame(vhx_ctx *c, const void *gathered, uint32_t planes, uint32_t ranks, uint32_t tiles_per_rank,
                     uint32_t T, uint32_t width, uint32_t height, uint32_t *fb_rgba, float *fb_depth) {
    if (!c || !gathered || (!fb_rgba && !fb_depth) || planes < 1 || planes > 2 || (planes == 1 && fb_depth) ||
        ranks == 0 || T == 0 || width == 0 || height == 0)
        return fail(c, VHX_E_INVALID_ARG, "vhx_untile_frame: bad arguments");
    const uint32_t tiles_x = (width + T - 1) / T, tiles_y = (height + T - 1) / T;
    const uint64_t ntiles = (uint64_t)tiles_x * tiles_y;
    if (ntiles > 0xFFFFFFFFull || (uint64_t)tiles_per_rank * ranks < ntiles)
        return fail(c, VHX_E_INVALID_ARG, "vhx_untile_frame: tiles_per_rank * ranks does not cover the frame");
    const uint64_t n = (uint64_t)ranks * planes * tiles_per_rank * T * T;
    if ((n + 255) / 256 > 0x7FFFFFFFull) return fail(c, VHX_E_INVALID_ARG, "too many pixels");
    VHX_HIP(c, hipSetDevice(c->device));
    VHX_STREAM(c);
    return launch_untile(c, c->stream, gathered, planes, ranks, tiles_per_rank, T, width, height, fb_rgba, fb_depth);
}

int vhx_untile_rgba(vhx_ctx *c, const uint32_t *gathered, uint32_t ranks, uint32_t tiles_per_rank, uint32_t T,
                    uint32_t width, uint32_t height, uint32_t *fb, int on_device) {
    if (!c || !gathered || !fb || ranks == 0 || T == 0 || width == 0 || height == 0) return VHX_E_INVALID_ARG;
    if (!on_device) return fail(c, VHX_E_INVALID_ARG, "vhx_untile_rgba works on device buffers");
    return vhx_untile_frame(c, gathered, 1, ranks, tiles_per_rank, T, width, height, fb, nullptr);
}

}  // extern "C"
