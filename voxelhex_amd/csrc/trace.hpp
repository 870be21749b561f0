// Device-side traversal of the flattened BoxTree for gfx950 — the per-ray state machine of the reference CPU
// raytracer BoxTree::get_by_ray (src/raytracing/cpu.rs:296-458), restated for one ray per lane of a wave64.
//
// Bit-exactness with the reference needs its float semantics: every f32 op that produces a value is issued in the
// reference order (the library is compiled with -ffp-contract=off, IEEE division and sqrt, f32 denormals kept),
// fminf/fmaxf ignore NaN like f32::min/max, signum(+-0) = +-1, and `as` casts saturate.
//
// Strength reductions that leave every result bit-identical:
//  * every cube size is a power of two (boxtree_size = brick_dim * 4^k, children are /4, cells /brick_dim, POP *4),
//    so x / size == x * (1/size) exactly; 1/size is formed from the exponent bits (rcp_pow2) and fmod by a size is
//    x - trunc(x / size) * size, exact by Sterbenz (fmod_pow2);
//  * brick_dim is a template parameter, so / brick_dim is a multiply by an exact constant;
//  * SECTANT_STEP_RESULT_LUT (src/spatial/lut.rs:27-92) and RAY_TO_NODE_OCCUPANCY_BITMASK_LUT (lut.rs:96-161) are
//    evaluated in closed form (both forms are checked against the reference tables in tests/test_oracle_spatial.py);
//  * a DDA step's float result is always (+-1 or 0) per axis, selected from signum(direction): the steps are carried
//    as a 3-bit axis mask, and the integer index updates use the precomputed `as i32` of the signs;
//  * node type + 64-bit occupancy are one 16-byte record per node (one global_load_dwordx4 per node visit);
//  * emptiness of brick cells comes from a per-brick occupancy bitmap (brick_dim^3 bits, built at upload from
//    pix_points_to_empty, src/boxtree/node.rs:311-333): the DDA through a brick issues no voxel loads, the voxel
//    value is loaded once, on the hit;
//  * the 4-entry NodeStack ring (cpu.rs:18-76) lives in four scalar registers, selected without dynamic indexing.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/vhx.h"

namespace vhx {

#define VHX_MAX_ITERS (1u << 22)  // same bound as the oracle (iteration bound)

// VHX_PROF (diagnostic builds only, scripts/probes/probe_blocks.py): per pass and per block of the traversal, the number
// of wave executions and the lanes active in them (wave ballot), accumulated in g_prof and read by
// vhx_profile_counters. The pass is told apart by its budget (pass_of_budget); 16 blocks per pass.
#ifndef VHX_PROF
#define VHX_PROF 0
#endif
#if VHX_PROF
__device__ unsigned long long g_prof[5 * 16 * 2];
#define VHX_PROF_BLOCK(pass, id)                                                                                  \
    do {                                                                                                          \
        const uint64_t m_ = __ballot(1);                                                                          \
        if ((threadIdx.x & 63u) == (uint32_t)__builtin_ctzll(m_)) {                                               \
            atomicAdd(&vhx::g_prof[((pass) * 16u + (id)) * 2u], 1ull);                                            \
            atomicAdd(&vhx::g_prof[((pass) * 16u + (id)) * 2u + 1u], (unsigned long long)__popcll(m_));           \
        }                                                                                                         \
    } while (0)
#else
#define VHX_PROF_BLOCK(pass, id) \
    do {                         \
    } while (0)
#endif
// pass slots of the profile counters: {24, 72, 216, 648} uses slots 0-3, the default {32, 128, 768} slots 0, 2, 3
__device__ __forceinline__ uint32_t pass_of_budget(uint32_t b) {
    return b >= VHX_MAX_ITERS ? 4u : (b <= 32u ? 0u : (b <= 96u ? 1u : (b <= 256u ? 2u : 3u)));
}

struct DevTree {
    const uint4 *hdr;          // {occ_lo, occ_hi, type, 0} per node
    const uint32_t *children;  // 64 per node
    const uint32_t *voxels;    // raw PaletteIndexValues, bd^3 per brick
    const uint64_t *brick_occ; // occ_words per brick; bit = flat cell index
    // brick_dim <= 4 (one occupancy word per brick): per child entry {children[i] (a UniformLeaf's brick in all 64
    // entries), occupancy word of that brick (lo, hi; 0 unless a Parted brick of a leaf), 0}, so a node iteration
    // gets the push target, the brick descriptor and the brick's occupancy with one load
    const uint4 *child_rec;
    const uint32_t *solid;
    const uint32_t *color;
    // node_mips (vhx_set_node_mips): per node its MIP brick descriptor; nullptr = MIPs off (the reference path)
    const uint32_t *mips;
    uint32_t color_count;
    uint32_t node_count;
    uint32_t size;
    uint32_t bd;
    uint32_t occ_words;  // max(1, bd^3/64)
};

// VHX_CHAIN (diagnostic builds only, libvhx_chain.so, scripts/chain_profile.py): the dependent chain of one ray traced
// alone in its wave, broken down per node iteration by s_memtime stamps (MI355X_MICROARCH.md: tick = shader cycle) --
// the wait for the iteration's node loads (header + child record, issued together), the leaf probe (brick walk), the
// POP / PUSH bookkeeping, the ADVANCE walk (or POP's step), and the loop overhead between iterations -- with a
// histogram of the node-load waits in 64-cycle buckets (the cache level that served them). vhx_chain_profile.
#ifndef VHX_CHAIN
#define VHX_CHAIN 0
#endif
#define VHX_CHAIN_HIST 48u
struct ChainAcc {
    unsigned long long load, probe, move, adv, other, last;
    uint32_t nload, nprobe, nadv, npad;
    uint32_t hist[VHX_CHAIN_HIST];
};
#if VHX_CHAIN
// one stamp, the wait for its own result inside the statement (the guide's recipe); the scheduling barriers keep the
// traversal's instructions on their side of it
__device__ __forceinline__ unsigned long long chain_stamp() {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#endif

struct HitOut {
    uint32_t value, cell, vx, vy, vz, bytes;
    uint32_t iters;  // loop steps of the whole traversal at its end (0 for a ray that misses the root cube)
    float ix, iy, iz, nx, ny, nz;
    bool hit;
#if VHX_CHAIN
    ChainAcc chain;
#endif
};

struct F3d {
    float x, y, z;
};
// (x, y) pairs for the walk loops: arithmetic on this type issues v_pk_add_f32 / v_pk_mul_f32 (two IEEE f32 ops per
// lane per instruction, each rounded exactly like the scalar op), z stays scalar
typedef float F2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ F2 mk2(float x, float y) { return F2{x, y}; }

__device__ __forceinline__ F3d mk(float x, float y, float z) { return F3d{x, y, z}; }
__device__ __forceinline__ F3d vadd(F3d a, F3d b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ F3d vsub(F3d a, F3d b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ F3d vmul(F3d a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ F3d vdiv(F3d a, float s) { return mk(a.x / s, a.y / s, a.z / s); }
__device__ __forceinline__ float vlen(F3d a) { return __builtin_sqrtf((a.x * a.x + a.y * a.y) + a.z * a.z); }
__device__ __forceinline__ F3d vnorm(F3d a) { return vdiv(a, vlen(a)); }

__device__ __forceinline__ float rsignum(float a) { return __builtin_isnan(a) ? a : __builtin_copysignf(1.0f, a); }
// Rust `as` casts (saturating, NaN -> 0). CDNA's v_cvt_i32_f32 / v_cvt_u32_f32 implement exactly this (out-of-range
// inputs incl. infinities saturate, NaN converts to 0), so each cast is one instruction; written as inline asm because
// the C++ conversion is undefined out of range and the compiler would otherwise guard it with branches.
__device__ __forceinline__ int32_t ras_i32(float f) {
    int32_t r;
    asm("v_cvt_i32_f32 %0, %1" : "=v"(r) : "v"(f));
    return r;
}
__device__ __forceinline__ uint32_t ras_u32(float f) {
    uint32_t r;
    asm("v_cvt_u32_f32 %0, %1" : "=v"(r) : "v"(f));
    return r;
}
__device__ __forceinline__ uint32_t ras_u8(float f) {
    const uint32_t r = ras_u32(f);
    return r < 255u ? r : 255u;
}

// x - fmod(x, s) for s a power of two: fmod(x, s) = x - q*s with q = trunc(x/s) exact, so the difference is q*s
// exactly, except that x - x is +0 where q*s may be -0; adding +0.0 maps -0 to +0 and leaves every other value alone
__device__ __forceinline__ float floor_to_pow2(float x, float s);

// exact 1/s for s a normal power of two: exponent e -> -e
__device__ __forceinline__ float rcp_pow2(float s) { return __uint_as_float(0x7F000000u - __float_as_uint(s)); }
// fmodf(x, s) for s a power of two (exact: x*(1/s) and trunc(.)*s are exact scalings, the difference is exact by
// Sterbenz); the sign of a zero result follows x like C fmod
__device__ __forceinline__ float fmod_pow2(float x, float s) {
    const float q = __builtin_truncf(x * rcp_pow2(s));
    const float r = x - q * s;
    return r == 0.0f ? __builtin_copysignf(0.0f, x) : r;
}

__device__ __forceinline__ float floor_to_pow2(float x, float s) {
    return __builtin_truncf(x * rcp_pow2(s)) * s + 0.0f;
}

// RAY_TO_NODE_OCCUPANCY_BITMASK_LUT[s][o] (src/spatial/lut.rs:96-161): sectants t with t_k on the ray's side of
// s_k on every axis; o = (dx>=0) + 2(dz>=0) + 4(dy>=0).
__host__ __device__ constexpr uint64_t occ_lut(uint32_t s, uint32_t o) {
    const uint32_t sx = s & 3u, sy = (s >> 2) & 3u, sz = s >> 4;
    const uint32_t mx = (o & 1u) ? (0xFu << sx) & 0xFu : (0xFu >> (3u - sx));
    const uint32_t my = (o & 4u) ? (0xFu << sy) & 0xFu : (0xFu >> (3u - sy));
    const uint32_t mz = (o & 2u) ? (0xFu << sz) & 0xFu : (0xFu >> (3u - sz));
    uint32_t row16 = 0;
#pragma unroll
    for (uint32_t y = 0; y < 4; ++y) row16 |= ((my >> y) & 1u) ? (mx << (4u * y)) : 0u;
    uint64_t m = 0;
#pragma unroll
    for (uint32_t z = 0; z < 4; ++z) m |= ((mz >> z) & 1u) ? ((uint64_t)row16 << (16u * z)) : 0ull;
    return m;
}

// step_sectant (src/spatial/mod.rs:23-26) for s < 64 and integer steps dk in {-1,0,1}: move each coordinate;
// if any leaves [0,3] the result is 64 + the wrapped sectant (sectant_step_result_lut.rs:48-93)
__device__ __forceinline__ uint32_t step_sectant_i(uint32_t s, int32_t dx, int32_t dy, int32_t dz) {
    const int32_t x = (int32_t)(s & 3u) + dx, y = (int32_t)((s >> 2) & 3u) + dy, z = (int32_t)(s >> 4) + dz;
    const uint32_t out = ((uint32_t)x > 3u) | ((uint32_t)y > 3u) | ((uint32_t)z > 3u);
    return ((uint32_t)x & 3u) | (((uint32_t)y & 3u) << 2) | (((uint32_t)z & 3u) << 4) | (out << 6);
}

// offset_sectant, src/spatial/math/mod.rs:27-44 ((off * 4) / size with size a power of two)
// (off * 4) / size: two scalings by powers of two, one multiply by 4/size gives the same value (at most one rounding,
// on underflow, in either order)
__device__ __forceinline__ uint32_t offset_sectant(F3d off, float size) {
    const float rs4 = 4.0f * rcp_pow2(size);
    F3d idx = mk(off.x * rs4, off.y * rs4, off.z * rs4);
    idx = mk(__builtin_floorf(idx.x), __builtin_floorf(idx.y), __builtin_floorf(idx.z));
    idx = mk(__builtin_fminf(idx.x, 3.0f), __builtin_fminf(idx.y, 3.0f), __builtin_fminf(idx.z, 3.0f));
    return ras_u8(idx.x + (idx.y * 4.0f) + (idx.z * 16.0f));
}

struct CubeD {
    F3d min;
    float size;
};
// Cube::child_bounds_for, src/spatial/mod.rs:72-77; SECTANT_OFFSET_LUT[s] = (s&3, (s>>2)&3, s>>4) / 4
// min + (k * 0.25) * size with k in 0..3: every term is an exact multiple of size / 4 (cube coordinates are such
// multiples below 2^24 * size / 4), so one fma per axis gives the reference's value bit for bit.
__device__ __forceinline__ CubeD child_bounds(CubeD c, uint32_t s) {
    CubeD r;
    r.size = c.size * 0.25f;
    r.min = mk(__builtin_fmaf((float)(s & 3u), r.size, c.min.x), __builtin_fmaf((float)((s >> 2) & 3u), r.size, c.min.y),
               __builtin_fmaf((float)(s >> 4), r.size, c.min.z));
    return r;
}
// cube_impact_normal, src/spatial/raytracing/mod.rs:97-125
__device__ __forceinline__ F3d impact_normal(CubeD c, F3d p) {
    const float h = c.size * 0.5f;
    F3d m = vsub(vadd(c.min, mk(h, h, h)), p);
    const float mc = __builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(m.x), __builtin_fabsf(m.y)), __builtin_fabsf(m.z));
    F3d n = mk(__builtin_fabsf(m.x) == mc ? -m.x : 0.0f, __builtin_fabsf(m.y) == mc ? -m.y : 0.0f,
               __builtin_fabsf(m.z) == mc ? -m.z : 0.0f);
    return vnorm(n);
}

// The signs of a ray's direction live in sg only (signum(d): +-1, NaN for a NaN component); the reference's
// max(sg, 0) and `sg as i32` are formed where used (three registers fewer than carrying them: pass 0 fits 64 VGPRs)
// d and sf are kept as an (x, y) pair plus z: the walk loops' packed f32 instructions read them in place, where
// separate x / y registers had to be copied into aligned pairs that stayed live beside the originals
struct RayD {
    F3d o, sg;
    F2 dxy, sfxy;
    float dz, sfz;
};
__device__ __forceinline__ F3d dvec(const RayD &r) { return mk(r.dxy.x, r.dxy.y, r.dz); }
// sg_k > 0 <=> (sg_k as i32) > 0 (NaN: false both ways); max(sg_k, 0) is 1 exactly then, else 0
__device__ __forceinline__ bool spos(float s) { return s > 0.0f; }

__device__ __forceinline__ void ray_setup(RayD &r, F3d o, F3d d) {
    r.o = o;
    r.dxy = mk2(d.x, d.y);
    r.dz = d.z;
    r.sg = mk(rsignum(d.x), rsignum(d.y), rsignum(d.z));
}
// get_dda_scale_factors, cpu.rs:79-92 (only needed once the ray enters the root cube)
__device__ __forceinline__ void ray_scale_factors(RayD &r) {
    const F3d d = dvec(r);
    const float zx = d.z / d.x, yx = d.y / d.x, xy = d.x / d.y, zy = d.z / d.y, xz = d.x / d.z, yz = d.y / d.z;
    r.sfxy = mk2(__builtin_sqrtf((1.0f + zx * zx) + yx * yx), __builtin_sqrtf((xy * xy + 1.0f) + zy * zy));
    r.sfz = __builtin_sqrtf((xz * xz + 1.0f) + yz * yz);
}

// dda_step_to_next_sibling, src/raytracing/cpu.rs:104-132. Returns the axis mask of the step (bit k set where
// min_step == d_k); the float step of the reference is sg_k on those axes and 0.0 elsewhere.
__device__ __forceinline__ uint32_t dda_step(const RayD &r, F3d &p, CubeD b) {
    const F3d diff = vsub(p, b.min);
    const F3d st = mk(b.size * __builtin_fmaxf(r.sg.x, 0.0f) - r.sg.x * diff.x,
                      b.size * __builtin_fmaxf(r.sg.y, 0.0f) - r.sg.y * diff.y,
                      b.size * __builtin_fmaxf(r.sg.z, 0.0f) - r.sg.z * diff.z);
    const float dx = __builtin_fabsf(st.x * r.sfxy.x), dy = __builtin_fabsf(st.y * r.sfxy.y),
                dz = __builtin_fabsf(st.z * r.sfz);
    const float m = __builtin_fminf(__builtin_fminf(dx, dy), dz);
    p = vadd(p, vmul(dvec(r), m));
    return (m == dx ? 1u : 0u) | (m == dy ? 2u : 0u) | (m == dz ? 4u : 0u);
}
__device__ __forceinline__ F3d step_vec(const RayD &r, uint32_t sel) {
    return mk((sel & 1u) ? r.sg.x : 0.0f, (sel & 2u) ? r.sg.y : 0.0f, (sel & 4u) ? r.sg.z : 0.0f);
}
__device__ __forceinline__ uint32_t step_sectant(const RayD &r, uint32_t s, uint32_t sel) {
    return step_sectant_i(s, (sel & 1u) ? ras_i32(r.sg.x) : 0, (sel & 2u) ? ras_i32(r.sg.y) : 0,
                          (sel & 4u) ? ras_i32(r.sg.z) : 0);
}

// brick geometry helpers
template <int BD>
struct Brick {
    static constexpr int N3 = BD * BD * BD;
    static constexpr uint32_t WORDS = N3 >= 64 ? (uint32_t)(N3 / 64) : 1u;
    static constexpr float INV = 1.0f / (float)BD;  // exact: BD is a power of two
};

template <bool COUNT>
__device__ __forceinline__ uint32_t pal_bytes(uint32_t v) {
    return COUNT ? ((v & 0xFFFFu) != 0xFFFFu ? 4u : 0u) + ((v >> 16) != 0xFFFFu ? 4u : 0u) : 0u;
}

__device__ __forceinline__ void fill_hit(HitOut &h, uint32_t v, uint32_t cell, F3d p, CubeD hb) {
    h.value = v;
    h.cell = cell;
    h.ix = p.x;
    h.iy = p.y;
    h.iz = p.z;
    const F3d n = impact_normal(hb, p);
    h.nx = n.x;
    h.ny = n.y;
    h.nz = n.z;
    h.vx = ras_u32(hb.min.x);
    h.vy = ras_u32(hb.min.y);
    h.vz = ras_u32(hb.min.z);
}

// probe_brick (cpu.rs:236-292) incl. traverse_brick (cpu.rs:136-232).
// The entry cell is tested before the loop; the loop steps from an empty cell and tests the next one, so every
// iteration commits its step unconditionally and the loop has a single exit (left the brick, or hit). A brick walk
// is at most 3*BD cells, so the step budget of a pass is checked by the caller once per node iteration; inside the
// walk only the VHX_MAX_ITERS bound is checked (the DDA arithmetic is described at the loop). Returns true on a hit,
// with the hit cell's flat index in `hflat` (-1 for a Solid brick); the hit record itself is filled after the
// traversal loop (finish_hit), so the loop carries two registers for it instead of a dozen.
template <bool COUNT, int BD>
__device__ __forceinline__ bool probe_brick(const DevTree &t, const RayD &r, F3d &p, uint32_t desc, uint64_t cocc,
                                            CubeD bb, HitOut &h, uint32_t &iters, int32_t &hflat, uint32_t pp = 0) {
    // one branch (a Parted brick's walk); Empty and Solid (cpu.rs:249-260) resolve by selects. VHX_EMPTY has the
    // Solid bit set, so "Parted" is simply the bit clear.
    const bool solid = (desc & VHX_SOLID_BIT) != 0u && desc != VHX_EMPTY;
    if (COUNT && solid) h.bytes += 4;
    bool hit = solid;
    int32_t flat = -1;  // hflat of a Solid brick
    if ((desc & VHX_SOLID_BIT) == 0u) {
        VHX_PROF_BLOCK(pp, 8);
        using B = Brick<BD>;
        // (p - min) * dim / size: both scalings are by powers of two, so one multiply by dim/size is the same value
        const F3d pib = vmul(vsub(p, bb.min), (float)BD * rcp_pow2(bb.size));
        int32_t ix = ras_i32(pib.x), iy = ras_i32(pib.y), iz = ras_i32(pib.z);
        ix = ix < 0 ? 0 : (ix > BD - 1 ? BD - 1 : ix);
        iy = iy < 0 ? 0 : (iy > BD - 1 ? BD - 1 : iy);
        iz = iz < 0 ? 0 : (iz > BD - 1 ? BD - 1 : iz);
        const float unit = bb.size * B::INV;
        const uint64_t *occw = t.brick_occ + (uint64_t)desc * B::WORDS;
        const uint32_t *vox = t.voxels + (uint64_t)desc * (uint64_t)B::N3;
        flat = ix + iy * BD + iz * (BD * BD);
        int32_t word_idx = flat >> 6;
        uint64_t word = B::WORDS == 1 ? cocc : occw[word_idx];  // cocc: the child record's copy of occw[0]
        hit = ((word >> (flat & 63)) & 1ull) != 0ull;
        if (COUNT) h.bytes += 4 + pal_bytes<COUNT>(vox[flat]);  // the reference reads the palettes of every cell
        if (!hit) {
            VHX_PROF_BLOCK(pp, 9);
            // Cell walk in exit-plane form. The reference's st_k = unit * max(sg_k, 0) - sg_k * (p_k - cmin_k): the
            // difference p_k - cmin_k is exact (cmin_k is a multiple of unit and p_k lies within a unit of it, so
            // Sterbenz applies, or cmin_k = 0), hence for sg_k = +1 st_k = unit - (p_k - cmin_k) and
            // (cmin_k + unit) - p_k are the same real number rounded once, and for sg_k = -1 st_k = p_k - cmin_k
            // exactly. With the exit plane e_k = cmin_k + unit * max(sg_k, 0) (exact), |st_k * sf_k| =
            // |(e_k - p_k) * sf_k| bit for bit.
            // Cell indices are carried direction-normalised (j_k = i_k, or BD-1-i_k for a negative direction), so a
            // step adds 1 and the flat index is j-flat ^ F.
            // e_k = min_k + (i_k + max(sg_k, 0)) * unit: every term is an exact multiple of unit below 2^24 * unit,
            // so the fused form is the value of the reference-order sum (min + i*unit) + unit*max(sg, 0) exactly
            F2 exy = mk2(__builtin_fmaf((float)(ix + (int32_t)spos(r.sg.x)), unit, bb.min.x),
                         __builtin_fmaf((float)(iy + (int32_t)spos(r.sg.y)), unit, bb.min.y));
            float ez = __builtin_fmaf((float)(iz + (int32_t)spos(r.sg.z)), unit, bb.min.z);
            const F2 sguxy = mk2(r.sg.x * unit, r.sg.y * unit);
            const float sguz = r.sg.z * unit;
            const F2 sfxy = r.sfxy, dxy = r.dxy;
            F2 pxy = mk2(p.x, p.y);
            float pz = p.z;
            const uint32_t fx = spos(r.sg.x) ? 0u : BD - 1u, fy = spos(r.sg.y) ? 0u : BD - 1u,
                           fz = spos(r.sg.z) ? 0u : BD - 1u;
            const uint32_t F = fx + fy * BD + fz * (BD * BD);
            uint32_t jx = (uint32_t)ix ^ fx, jy = (uint32_t)iy ^ fy, jz = (uint32_t)iz ^ fz;
            for (;;) {
                VHX_PROF_BLOCK(pp, 2);
                ++iters;
                // dda_step_to_next_sibling (cpu.rs:104-132) on the cell {cmin, unit}
                const F2 sxy = (exy - pxy) * sfxy;
                const float dx = __builtin_fabsf(sxy.x), dy = __builtin_fabsf(sxy.y),
                            dz = __builtin_fabsf((ez - pz) * r.sfz);
                const float m = __builtin_fminf(__builtin_fminf(dx, dy), dz);
                pxy = pxy + dxy * m;
                pz = pz + r.dz * m;
                const bool mx = m == dx, my = m == dy, mz = m == dz;
                const F2 en = exy + sguxy;
                exy = mk2(mx ? en.x : exy.x, my ? en.y : exy.y);
                ez = mz ? ez + sguz : ez;
                jx += (uint32_t)mx;
                jy += (uint32_t)my;
                jz += (uint32_t)mz;
                // the exit test is one integer word (left the brick | occupied cell | iteration bound), so the loop's
                // control costs one compare instead of a chain of mask operations
                const uint32_t oob = (jx | jy | jz) & ~(uint32_t)(BD - 1);  // non-zero iff the walk left the brick
                const uint32_t uflat = (jx + jy * BD + jz * (BD * BD)) ^ F;
                if (B::WORDS > 1) {
                    const int32_t wi = (int32_t)(uflat >> 6);
                    if (oob == 0u && wi != word_idx) {
                        word_idx = wi;
                        word = occw[wi];
                    }
                }
                const uint32_t bit = (uint32_t)(word >> (uflat & 63u)) & 1u;  // meaningless once oob (exit anyway)
                if (COUNT && oob == 0u) h.bytes += 4 + pal_bytes<COUNT>(vox[uflat]);
                // the bound only ends a ray whose steps make no progress (a zero or NaN direction); at the bound the
                // oracle tests the cell it stepped into and stops before the next step, like this exit
                static_assert(VHX_MAX_ITERS == (1u << 22), "bound test below");
                if ((oob | bit | (iters >> 22)) != 0u) break;
            }
            // hit = the exit test, recomputed once from the final cell instead of carrying the loop's booleans out of
            // it (opaque copies keep the compiler from reusing the in-loop values, which costs mask bookkeeping per
            // cell)
            p = mk(pxy.x, pxy.y, pz);
            asm volatile("" : "+v"(jx), "+v"(jy), "+v"(jz));
            flat = (int32_t)((jx + jy * BD + jz * (BD * BD)) ^ F);
            hit = (jx | jy | jz) < (uint32_t)BD && ((word >> (flat & 63)) & 1ull) != 0ull;
        }
    }
    hflat = flat;
    return hit;
}

// The hit record of probe_brick (cpu.rs:249-260 for a Solid brick, cpu.rs:268-289 for a cell of a Parted brick):
// the voxel value, the cell bounds and the impact normal, computed once after the traversal loop.
template <int BD>
__device__ __forceinline__ void finish_hit(const DevTree &t, HitOut &h, uint32_t desc, int32_t hflat, F3d p, CubeD bb) {
    using B = Brick<BD>;
    if (hflat < 0) {
        fill_hit(h, t.solid[desc & 0x7FFFFFFFu], VHX_EMPTY, p, bb);
        return;
    }
    const uint32_t ix = (uint32_t)hflat % BD, iy = ((uint32_t)hflat / BD) % BD, iz = (uint32_t)hflat / (BD * BD);
    const uint32_t v = t.voxels[(uint64_t)desc * (uint64_t)B::N3 + (uint32_t)hflat];
    CubeD hb;
    hb.size = bb.size * B::INV;
    hb.min = vadd(bb.min, vmul(vmul(mk((float)ix, (float)iy, (float)iz), bb.size), B::INV));
    fill_hit(h, v, (uint32_t)hflat, p, hb);
}

// RAY_TO_NODE_OCCUPANCY_BITMASK_LUT, tabulated at compile time (occ_tab[s * 8 + o] = occ_lut(s, o), 4 KB in constant
// memory) and copied into LDS by every block before tracing (a copy instead of 512 evaluations per block).
struct OccTab {
    uint64_t v[512];
};
constexpr OccTab make_occ_tab() {
    OccTab t{};
    for (uint32_t i = 0; i < 512u; ++i) t.v[i] = occ_lut(i >> 3, i & 7u);
    return t;
}
__constant__ OccTab g_occ_tab = make_occ_tab();
#define OCC_TAB_WORDS 512u
__device__ __forceinline__ void fill_occ_tab(uint64_t *occ_tab) {
    for (uint32_t i = threadIdx.x; i < 512u; i += blockDim.x) occ_tab[i] = g_occ_tab.v[i];
}

// Saved traversal state of a ray abandoned at a pass budget (multi-pass scheduling): everything the loop below
// carries from one node iteration to the next, 64 bytes. Cube sizes are powers of two (zero mantissa), so the
// current cube's size word also holds the target sectant (7 bits) and the stack depth (3 bits).
struct St4 {
    uint4 a, b, c, e;
};
__device__ __forceinline__ St4 pack_state(F3d p, uint32_t iters, CubeD cur, CubeD tb, uint32_t target, uint32_t count,
                                          uint32_t node, uint32_t s1, uint32_t s2, uint32_t s3) {
    St4 s;
    s.a = make_uint4(__float_as_uint(p.x), __float_as_uint(p.y), __float_as_uint(p.z), iters);
    s.b = make_uint4(__float_as_uint(cur.min.x), __float_as_uint(cur.min.y), __float_as_uint(cur.min.z),
                     __float_as_uint(cur.size) | target | (count << 8));
    s.c = make_uint4(__float_as_uint(tb.min.x), __float_as_uint(tb.min.y), __float_as_uint(tb.min.z),
                     __float_as_uint(tb.size));
    s.e = make_uint4(node, s1, s2, s3);
    return s;
}
__device__ __forceinline__ void save_state(uint4 *st, F3d p, uint32_t iters, CubeD cur, CubeD tb, uint32_t target,
                                           uint32_t count, uint32_t node, uint32_t s1, uint32_t s2, uint32_t s3) {
    const St4 s = pack_state(p, iters, cur, tb, target, count, node, s1, s2, s3);
    st[0] = s.a;
    st[1] = s.b;
    st[2] = s.c;
    st[3] = s.e;
}

// BoxTree::get_by_ray, src/raytracing/cpu.rs:296-458, as a traversal state with three steps: begin (ray setup and the
// root intersection, or a resumed state), step (one iteration of the node loop) and end (save an abandoned ray's
// state, or fill the hit record). get_by_ray runs them back to back; a caller may also interleave rays per lane.
// `budget` bounds the loop iterations (node, advance and brick steps, counted from the ray's start; checked at the end
// of each node iteration, so a pass may overrun it by one brick walk and one advance). With budget == VHX_MAX_ITERS
// this is the full traversal (a ray exceeding the bound is a miss, as in the oracle) and end() always returns true.
// A smaller budget makes a pass of the multi-pass scheduler: false = the ray was abandoned after `budget` steps; with
// `sbase` given, its state is saved at sbase[4 * sidx] and a later pass continues it (`resume`) exactly where it
// stopped, otherwise the later pass traces it again from scratch. Either way the result is bit-identical to one
// uninterrupted traversal (the state is saved whole; the traversal is deterministic). h.bytes is the caller's running
// byte count (COUNT builds): 0 for a fresh ray, the count at the abandon for a resumed one.
//
// Control flow: the reference's two nested loops (restart from the root / walk the NodeStack) are one loop here, and
// every way out of it sets the exit code `ex` and leaves through a single exit at the bottom of the iteration. The
// NodeStack<u32, 4> ring (cpu.rs:18-76) is a shift register: `node` is its top, s1..s3 the entries below; a push onto
// a full stack drops the oldest entry, a pop that empties it ends the walk and restarts from the root.
template <bool COUNT, int BD, bool MIP = false>
struct Trav {
    RayD r;
    uint32_t dir_idx;
    float tsize;
    CubeD cur;
    F3d p;
    uint32_t target;
    CubeD tb;
    uint32_t node, s1, s2, s3, count, iters;
    // how the loop ended, one integer instead of several booleans (kept in a VGPR; boolean flags set in divergent
    // branches become 64-bit lane masks merged by scalar instructions at every join): 0 = still running, 1 = hit,
    // 2 = miss (left the tree, invalid key, or the iteration bound), 3 = abandoned at the pass budget, 4 = hit in a
    // node's MIP brick (MIPs on, vhx_set_node_mips)
    uint32_t ex;
    // tbok: target_bounds equals child_bounds(current, target) (kept by PUSH, POP and ADVANCE; not after a restart,
    // which leaves it stale, cpu.rs:317-320), so a leaf probe takes its brick cube from tb instead of recomputing it.
    // A resumed ray starts with 0 (recompute), which is always correct.
    uint32_t tbok;
    uint32_t hdesc;
    int32_t hflat;

    // false: the ray misses the root cube (a miss, nothing more to do)
    // START (the opt-in depth-prepass mode, not the reference path): the ray enters the tree no earlier than `start`
    // along its direction (the prepass's min-of-4 distance, viewport_render.wgsl:714-726); the exact path is START =
    // false and compiles to the same code as before.
    template <bool START = false>
    __device__ __forceinline__ bool begin(const DevTree &t, F3d o, F3d d, HitOut &h, const uint4 *sbase, uint32_t sidx,
                                          bool resume, float start = 0.0f) {
        // sbase + 4 * sidx: the resumed ray's saved state (by output index, or by queue position in the queue-state
        // mode, where the compaction moved every abandoned ray's state into the next pass's queue order)
        h.hit = false;
        ray_setup(r, o, d);
        {
            const F3d od = vadd(mk(1.0f, 1.0f, 1.0f), d);
            dir_idx = (uint32_t)(od.x >= 1.0f) + (uint32_t)(od.z >= 1.0f) * 2u + (uint32_t)(od.y >= 1.0f) * 4u;
        }
        tsize = (float)t.size;
        ex = 0;
        hdesc = 0;
        hflat = 0;
        if (resume) {
            const uint4 *st = sbase + 4ull * sidx;
            const uint4 a = st[0], b = st[1], c = st[2], e = st[3];
            p = mk(__uint_as_float(a.x), __uint_as_float(a.y), __uint_as_float(a.z));
            iters = a.w;
            cur.min = mk(__uint_as_float(b.x), __uint_as_float(b.y), __uint_as_float(b.z));
            cur.size = __uint_as_float(b.w & 0xFF800000u);
            target = b.w & 0x7Fu;
            count = (b.w >> 8) & 7u;
            tb.min = mk(__uint_as_float(c.x), __uint_as_float(c.y), __uint_as_float(c.z));
            tb.size = __uint_as_float(c.w);
            node = e.x;
            s1 = e.y;
            s2 = e.z;
            s3 = e.w;
        } else {
            cur.min = mk(0.0f, 0.0f, 0.0f);
            cur.size = tsize;
            // Cube::intersect_ray, src/spatial/raytracing/mod.rs:33-62 (root: min 0, max = 0 + size = size)
            const float t1 = (0.0f - o.x) / d.x, t2 = (tsize - o.x) / d.x;
            const float t3 = (0.0f - o.y) / d.y, t4 = (tsize - o.y) / d.y;
            const float t5 = (0.0f - o.z) / d.z, t6 = (tsize - o.z) / d.z;
            const float tmin = __builtin_fmaxf(__builtin_fmaxf(__builtin_fminf(t1, t2), __builtin_fminf(t3, t4)),
                                               __builtin_fminf(t5, t6));
            const float tmax = __builtin_fminf(__builtin_fminf(__builtin_fmaxf(t1, t2), __builtin_fmaxf(t3, t4)),
                                               __builtin_fmaxf(t5, t6));
            if (tmax < 0.0f || tmin > tmax) {  // the outer loop never runs: a miss
                ex = 2u;
                return false;
            }
            float t0 = tmin < 0.0f ? 0.0f : tmin;
            if (START) {
                if (!(start <= tmax)) {  // the neighbourhood's prepass rays left the tree (or start is +inf): a miss
                    ex = 2u;
                    return false;
                }
                t0 = __builtin_fmaxf(t0, start);
            }
            p = vadd(o, vmul(d, t0));
            target = offset_sectant(p, cur.size);
            tb = child_bounds(cur, target);
            node = 0, s1 = 0, s2 = 0, s3 = 0, count = 1;  // push(ROOT)
            iters = 1;  // the first node iteration
        }
        ray_scale_factors(r);
        tbok = resume ? 0u : 1u;
        return true;
    }

    __device__ __forceinline__ void step(const DevTree &t, const uint64_t *occ_tab, HitOut &h, uint32_t budget) {
        // the child slot is read by both the leaf probe and the push: issue it with the header load so the
        // iteration waits for one memory latency instead of two (with brick_dim <= 4 the child record also carries
        // the brick's occupancy word, so a probe waits for no further load)
        uint4 lh;
        uint32_t slot;
        uint64_t cocc = 0;
#if VHX_CHAIN
        const unsigned long long tA = chain_stamp();
        if (h.chain.last) h.chain.other += tA - h.chain.last;
#endif
        if (Brick<BD>::WORDS == 1) {
            lh = t.hdr[node];
            const uint4 cr = t.child_rec[(uint64_t)node * 64u + (target & 63u)];
            slot = cr.x;
            cocc = ((uint64_t)cr.z << 32) | (uint64_t)cr.y;
        } else {
            lh = t.hdr[node];
            slot = t.children[(uint64_t)node * 64u + (target & 63u)];
        }
        // the pop test's LUT word, read from LDS while the node loads are in flight (the empty asm keeps the read
        // here instead of next to its use after the probe, where its latency was exposed)
        uint64_t omask = occ_tab[(target & 63u) * 8u + dir_idx];
        asm volatile("" : "+v"(omask));
#if VHX_CHAIN
        asm volatile("" ::"v"(lh.x), "v"(lh.y), "v"(lh.z), "v"(slot), "v"((uint32_t)cocc));  // the loads have landed
        const unsigned long long tB = chain_stamp();
        h.chain.load += tB - tA;
        h.chain.nload += 1;
        h.chain.hist[min((uint32_t)((tB - tA) >> 6), VHX_CHAIN_HIST - 1u)] += 1;
#endif
        const uint64_t occ = ((uint64_t)lh.y << 32) | (uint64_t)lh.x;
        const uint32_t ntype = lh.z;
        if (COUNT) h.bytes += 12;
        const bool uniform = ntype == VHX_NODE_UNIFORM_LEAF;
        const uint32_t pp = VHX_PROF ? pass_of_budget(budget) : 0u;
        // the hit descriptor and cell are defined afresh in every iteration (they are read only after the iteration
        // that sets ex to 1 or 4): not loop-carried, two registers fewer across the loop
        hdesc = slot;
        hflat = -1;
        if (target < 64u && (uniform || ntype == VHX_NODE_LEAF)) {
            VHX_PROF_BLOCK(pp, 1);
            if (COUNT) h.bytes += 4;
            hdesc = Brick<BD>::WORDS == 1 || !uniform ? slot : t.children[(uint64_t)node * 64u];
            CubeD bb = uniform ? cur : tb;
            if (!uniform && tbok == 0u) bb = child_bounds(cur, target);
            ex = probe_brick<COUNT, BD>(t, r, p, hdesc, cocc, bb, h, iters, hflat, pp) ? 1u : 0u;
#if VHX_CHAIN
            h.chain.nprobe += 1;
#endif
        }
#if VHX_CHAIN
        const unsigned long long tP = chain_stamp();
        h.chain.probe += tP - tB;
        unsigned long long tQ = tP;
#endif
        // MIP stand-in (viewport_render.wgsl:438-454, probe_MIP 328-364): the target sectant is occupied but its child
        // entry is absent (a view that does not hold it). The node's MIP brick is traced over the node's cube from a
        // copy of the ray point; a hit ends the ray, a miss ADVANCEs past the sectant instead of pushing into the
        // missing child. Compiled only into the MIP kernels (their own instantiations), so the reference path's code
        // and register allocation are untouched.
        bool mip_adv = false;
        if (MIP) {
            if (target < 64u && slot == VHX_EMPTY && ((occ >> target) & 1ull) != 0ull &&
                (ntype == VHX_NODE_INTERNAL || ntype == VHX_NODE_LEAF)) {
                mip_adv = true;
                const uint32_t mdesc = t.mips[node];
                if (COUNT) h.bytes += 4;
                if (mdesc != VHX_EMPTY) {
                    const uint64_t mocc =
                        Brick<BD>::WORDS == 1 && (mdesc & VHX_SOLID_BIT) == 0u ? t.brick_occ[mdesc] : 0ull;
                    F3d pm = p;
                    int32_t mflat;
                    if (probe_brick<COUNT, BD>(t, r, pm, mdesc, mocc, cur, h, iters, mflat)) {
                        p = pm;
                        hdesc = mdesc;
                        hflat = mflat;
                        ex = 4u;
                    }
                }
            }
        }
        if (ex == 0u) {
            // the three moves are sequential ifs over precomputed conditions rather than an if / else-if chain: each
            // updates the loop state in place, where the chain's join made the compiler copy every unchanged state
            // register twice per iteration
            const bool pop = uniform || target >= 64u || occ == 0 || (occ & omask) == 0;
            const bool push = !pop && !mip_adv && ntype == VHX_NODE_INTERNAL && ((occ >> target) & 1ull) != 0;
            if (pop) {
                VHX_PROF_BLOCK(pp, 3);
                // POP (cpu.rs:368-393). Its step to the next sibling (dda_step_to_next_sibling on the popped cube,
                // step_sectant, target_bounds += step * size) is one trip of the walk below, which the lanes that
                // advance run anyway: one copy of the DDA code per iteration instead of two.
                count -= 1;
                node = s1;
                s1 = s2;
                s2 = s3;
                tb = cur;
                cur.size *= 4.0f;
                cur.min = mk(floor_to_pow2(cur.min.x, cur.size), floor_to_pow2(cur.min.y, cur.size),
                             floor_to_pow2(cur.min.z, cur.size));  // min -= min % size
                // offset_sectant(tb.center - cur.min, cur.size) is the popped cube's sectant k in its parent: tb.min =
                // cur.min + k * tb.size (node cubes are aligned to their size, the parent is the aligned 4x cube), so
                // center - cur.min = (k + 1/2) * tb.size exactly and floor((k + 1/2) * 4 / cur.size) = k; k is formed
                // directly from the exact difference tb.min - cur.min
                {
                    const float rs = rcp_pow2(tb.size);
                    const uint32_t kx = (uint32_t)((tb.min.x - cur.min.x) * rs),
                                   ky = (uint32_t)((tb.min.y - cur.min.y) * rs),
                                   kz = (uint32_t)((tb.min.z - cur.min.z) * rs);
                    target = kx + ky * 4u + kz * 16u;
                }
            }
            if (push) {
                VHX_PROF_BLOCK(pp, 4);
                // PUSH (cpu.rs:401-411)
                if (COUNT) h.bytes += 4;
                s3 = s2;
                s2 = s1;
                s1 = node;
                node = slot;
                count = count + 1 < 4 ? count + 1 : 4;
                cur = tb;
                target = offset_sectant(vsub(p, tb.min), tb.size);
                tb = child_bounds(cur, target);
                tbok = 1u;
                ex = slot >= t.node_count ? 2u : 0u;  // the reference would panic on an invalid key: a miss here
            }
#if VHX_CHAIN
            tQ = chain_stamp();
            h.chain.move += tQ - tP;
#endif
            if (!push) {
                VHX_PROF_BLOCK(pp, 5);
#if VHX_CHAIN
                h.chain.nadv += 1;
#endif
                // ADVANCE (cpu.rs:416-437), or POP's single step: at most 9 steps across the node, the pass budget
                // is checked after it. Same form as the brick walk (exit planes, direction-normalised sectant
                // coordinates); the exit-plane difference equals the reference's dda_step_to_next_sibling for a point
                // on or inside the stepped cube (§4), which the popped cube is. Every step is committed: tb.min after
                // a step out of the node is dead (the next iteration pops and overwrites it). The reference's target
                // (step_sectant) is formed once at the end (>= 64: the walk left the node; POP's step_sectant gives
                // 64 + the wrapped sectant there, which the next iteration's POP never reads).
                // A POP lane walks with every sectant occupied: it stops after its one step.
                const uint64_t wocc = pop ? ~0ull : occ;
                // tb.size * max(sg, 0): tb.size or 0 (the reference's product, exactly)
                const F3d usg = mk(spos(r.sg.x) ? tb.size : 0.0f, spos(r.sg.y) ? tb.size : 0.0f,
                                   spos(r.sg.z) ? tb.size : 0.0f);
                const F3d sgs = mk(r.sg.x * tb.size, r.sg.y * tb.size, r.sg.z * tb.size);
                const uint32_t fx = spos(r.sg.x) ? 0u : 3u, fy = spos(r.sg.y) ? 0u : 3u, fz = spos(r.sg.z) ? 0u : 3u;
                const uint32_t F = fx + fy * 4u + fz * 16u;
                uint32_t jx = (target & 3u) ^ fx, jy = ((target >> 2) & 3u) ^ fy, jz = (target >> 4) ^ fz;
                F2 exy = mk2(tb.min.x + usg.x, tb.min.y + usg.y);
                float ez = tb.min.z + usg.z;
                const F2 sgsxy = mk2(sgs.x, sgs.y), sfxy = r.sfxy, dxy = r.dxy;
                F2 pxy = mk2(p.x, p.y);
                float pz = p.z;
                for (;;) {
                    VHX_PROF_BLOCK(pp, 6);
                    ++iters;
                    const F2 sxy = (exy - pxy) * sfxy;
                    const float dx = __builtin_fabsf(sxy.x), dy = __builtin_fabsf(sxy.y),
                                dz = __builtin_fabsf((ez - pz) * r.sfz);
                    const float m = __builtin_fminf(__builtin_fminf(dx, dy), dz);
                    pxy = pxy + dxy * m;
                    pz = pz + r.dz * m;
                    const bool mx = m == dx, my = m == dy, mz = m == dz;
                    const F2 en = exy + sgsxy;
                    exy = mk2(mx ? en.x : exy.x, my ? en.y : exy.y);
                    ez = mz ? ez + sgs.z : ez;
                    jx += (uint32_t)mx;
                    jy += (uint32_t)my;
                    jz += (uint32_t)mz;
                    const uint32_t oob = (jx | jy | jz) & ~3u;  // non-zero iff the walk left the node
                    const uint32_t tg = (jx + jy * 4u + jz * 16u) ^ F;
                    const uint32_t bit = (uint32_t)(wocc >> (tg & 63u)) & 1u;
                    if ((oob | bit | ((iters - 1u) >> 22)) != 0u) break;  // left | occupied | iters > 2^22
                }
                p = mk(pxy.x, pxy.y, pz);
                asm volatile("" : "+v"(jx), "+v"(jy), "+v"(jz));
                target = (jx | jy | jz) < 4u ? (jx + jy * 4u + jz * 16u) ^ F : 64u;
                tb.min = mk(exy.x - usg.x, exy.y - usg.y, ez - usg.z);  // exact: undoes the exact e = tb.min + usg
                if (pop) {
                    iters -= 1u;  // POP's step is not one of the walk's steps
                    tbok = 1u;
                    if (count == 0) {
                        VHX_PROF_BLOCK(pp, 7);
                        // the stack ran empty: restart from the root (cpu.rs:441-455); target_bounds stays stale
                        p = vadd(p, vmul(dvec(r), 0.1f));
                        if (p.x < tsize && p.y < tsize && p.z < tsize && p.x > 0.0f && p.y > 0.0f && p.z > 0.0f) {
                            target = offset_sectant(p, tsize);
                            tbok = 0u;  // target_bounds stays stale
                            node = 0;
                            count = 1;
                            cur.min = mk(0.0f, 0.0f, 0.0f);
                            cur.size = tsize;
                        } else {
                            ex = 2u;  // left the tree: a miss
                        }
                    }
                }
            }
            // the next node iteration; past the iteration bound the ray ends as a miss in every pass (the reference
            // stops at the top of that iteration): a ray whose walks ran past the bound inside a budgeted pass must
            // not be resumed for one more iteration (its probe could hit; tests/test_gpu_parity.py, degenerate rays)
            if (ex == 0u && ++iters > budget) ex = budget >= VHX_MAX_ITERS || iters > VHX_MAX_ITERS ? 2u : 3u;
        }
#if VHX_CHAIN
        const unsigned long long tR = chain_stamp();
        h.chain.adv += tR - tQ;
        h.chain.last = tR;
#endif
    }

    __device__ __forceinline__ bool end(const DevTree &t, HitOut &h, uint4 *sbase, uint32_t sidx, bool slots = false) {
        h.iters = iters;
        // slots (queue-state mode): sidx is the first slot of this wave's chunk list, and the wave's abandoned rays take
        // consecutive slots in lane order -- the positions its chunk list gives them (wave_append, the queue pass's
        // chunk append), so the compaction can move the states along with the list
        if (slots) {
            const uint64_t m = __ballot(ex == 3u);
            sidx += (uint32_t)__popcll(m & ((1ull << (threadIdx.x & 63u)) - 1ull));
        }
        // an abandoned ray's state is the loop state at its exit (saved here, outside the hot loop)
        if (ex == 3u && sbase) save_state(sbase + 4ull * sidx, p, iters, cur, tb, target, count, node, s1, s2, s3);
        if (ex == 1u) {  // the loop left on the hit: node, cur, target and p are those of the probe
            h.hit = true;
            const bool huni = t.hdr[node].z == VHX_NODE_UNIFORM_LEAF;
            finish_hit<BD>(t, h, hdesc, hflat, p, huni ? cur : child_bounds(cur, target));
        } else if (ex == 4u) {  // a MIP hit: the MIP brick spans the node's cube
            h.hit = true;
            finish_hit<BD>(t, h, hdesc, hflat, p, cur);
        }
        return ex != 3u;
    }
};

// sparse (a budgeted pass with saved state): once fewer than `sparse` lanes of the wave still trace, they are abandoned
// like rays over the budget (their state saved, the next pass resumes them packed into full waves) instead of keeping
// the wave's issue slots for a few lanes. 0 = off. The result is the same either way (the traversal is deterministic).
// rbase (queue-state mode): a resumed ray's state is read at rbase + 4 * ridx and an abandoned ray's is saved at
// sbase + 4 * (sidx + its rank among the wave's abandoned rays) (Trav::end); without it both use sbase + 4 * sidx.
template <bool COUNT, int BD, bool START = false, bool MIP = false>
__device__ __forceinline__ bool get_by_ray(const DevTree &t, const uint64_t *occ_tab, F3d o, F3d d, HitOut &h,
                                           uint32_t budget, uint4 *sbase = nullptr, uint32_t sidx = 0,
                                           bool resume = false, float start = 0.0f, uint32_t sparse = 0,
                                           const uint4 *rbase = nullptr, uint32_t ridx = 0, bool slots = false) {
    Trav<COUNT, BD, MIP> tr;
    VHX_PROF_BLOCK(pass_of_budget(budget), 10);
    h.iters = 0;
    if (!tr.template begin<START>(t, o, d, h, rbase ? rbase : sbase, rbase ? ridx : sidx, resume, start)) return true;
    VHX_PROF_BLOCK(pass_of_budget(budget), 11);
    for (;;) {
        VHX_PROF_BLOCK(pass_of_budget(budget), 0);
        tr.step(t, occ_tab, h, budget);
        if (tr.ex != 0u) break;
        if (sparse && (uint32_t)__popcll(__ballot(1)) < sparse) {
            tr.ex = 3u;
            break;
        }
    }
    VHX_PROF_BLOCK(pass_of_budget(budget), 12);
    return tr.end(t, h, sbase, sidx, slots);
}

}  // namespace vhx
