// Persistent, wavefront-refilled primary-ray kernel for gfx950.
//
// Per-ray work of the reference traversal (get_by_ray, src/raytracing/cpu.rs:296-458) is heavily skewed: on the
// 1024^3 scene S frame a ray takes ~14 node/advance/brick steps on average and up to ~2000. With one ray per lane for
// the lane's lifetime every wave is as slow as its slowest lane. Here each wave owns a task of rays and every lane
// runs the traversal as an explicit state machine, one step per loop trip; lanes that finish are counted by a
// wave-wide ballot and take the next rays of the task (rank by popcount of the lower lanes), so the wave stays full
// until its task drains. Balance across waves is left to the hardware dispatcher (many more tasks than wave slots).
//
// ls_step performs exactly the operations of get_by_ray<COUNT> in trace.hpp, in the same order, so results and the
// instrumented byte counts are bit-identical; only the interleaving across lanes changes.
//   S_NODE     top of the inner loop (cpu.rs:321-411): stack check / restart (441-455), node record, probe,
//              then POP (368-393) / PUSH (401-411) / switch to ADVANCE
//   S_BRICK    one cell of traverse_brick (cpu.rs:172-231)
//   S_ADVANCE  one DDA step of the advance loop (cpu.rs:416-437)
#pragma once

namespace vhx {

enum : uint32_t { S_NODE = 0, S_BRICK = 1, S_ADVANCE = 2 };

struct LaneState {
    RayD r;
    F3d p;
    CubeD cur, tb;
    uint32_t target, node, dir_idx, iters;
    uint32_t s0, s1, s2, s3, head, count;
    uint64_t occ;
    uint32_t ntype;
    // traverse_brick state
    int32_t ix, iy, iz, flat, word_idx;
    uint32_t desc;
    uint64_t word;
    CubeD bcur, bb;
    uint32_t sel;  // axis mask of the last brick DDA step
    uint32_t state;
    uint32_t bytes;
};

__device__ __forceinline__ uint32_t ls_top(const LaneState &s) {
    return s.head == 0 ? s.s0 : (s.head == 1 ? s.s1 : (s.head == 2 ? s.s2 : s.s3));
}
__device__ __forceinline__ void ls_push(LaneState &s, uint32_t v) {
    s.head = (s.head + 1) & 3u;
    s.count = s.count + 1 < 4 ? s.count + 1 : 4;
    s.s0 = s.head == 0 ? v : s.s0;
    s.s1 = s.head == 1 ? v : s.s1;
    s.s2 = s.head == 2 ? v : s.s2;
    s.s3 = s.head == 3 ? v : s.s3;
}

// ray setup of get_by_ray (cpu.rs:298-314) + the first OUTER iteration; false = the ray misses the root cube
__device__ __forceinline__ bool ls_begin(const DevTree &t, LaneState &s, F3d o, F3d d) {
    ray_setup(s.r, o, d);
    {
        const F3d od = vadd(mk(1.0f, 1.0f, 1.0f), d);
        s.dir_idx = (uint32_t)(od.x >= 1.0f) + (uint32_t)(od.z >= 1.0f) * 2u + (uint32_t)(od.y >= 1.0f) * 4u;
    }
    const float tsize = (float)t.size;
    s.cur.min = mk(0.0f, 0.0f, 0.0f);
    s.cur.size = tsize;
    // Cube::intersect_ray (src/spatial/raytracing/mod.rs:33-62) on the root; max corner = min + size = size
    const float t1 = (0.0f - o.x) / d.x, t2 = (tsize - o.x) / d.x;
    const float t3 = (0.0f - o.y) / d.y, t4 = (tsize - o.y) / d.y;
    const float t5 = (0.0f - o.z) / d.z, t6 = (tsize - o.z) / d.z;
    const float tmin = __builtin_fmaxf(__builtin_fmaxf(__builtin_fminf(t1, t2), __builtin_fminf(t3, t4)),
                                       __builtin_fminf(t5, t6));
    const float tmax = __builtin_fminf(__builtin_fminf(__builtin_fmaxf(t1, t2), __builtin_fmaxf(t3, t4)),
                                       __builtin_fmaxf(t5, t6));
    s.s0 = s.s1 = s.s2 = s.s3 = 0;
    s.head = 0;
    s.count = 0;
    s.iters = 0;
    s.bytes = 0;
    if (tmax < 0.0f || tmin > tmax) return false;
    ray_scale_factors(s.r);
    s.p = vadd(o, vmul(d, tmin < 0.0f ? 0.0f : tmin));
    s.target = offset_sectant(s.p, tsize);
    s.tb = child_bounds(s.cur, s.target);
    s.node = 0;
    ls_push(s, 0u);
    s.state = S_NODE;
    return true;
}

__device__ __forceinline__ void ls_hit_solid(const DevTree &t, const LaneState &s, HitOut &h) {
    fill_hit(h, t.solid[s.desc & 0x7FFFFFFFu], VHX_EMPTY, s.p, s.bb);
    h.hit = true;
}

// After a probe missed (or no probe): POP / PUSH / ADVANCE (cpu.rs:361-438). Returns true if the ray ended.
template <bool COUNT>
__device__ __forceinline__ bool ls_after_probe(const DevTree &t, LaneState &s, bool backtrack) {
    if (backtrack || s.target >= 64 || s.occ == 0 || (s.occ & occ_lut(s.target, s.dir_idx)) == 0) {
        if (s.count != 0) {
            s.count -= 1;
            s.head = (s.head - 1) & 3u;
        }
        s.tb = s.cur;
        s.cur.size *= 4.0f;
        s.cur.min = vsub(s.cur.min, mk(fmod_pow2(s.cur.min.x, s.cur.size), fmod_pow2(s.cur.min.y, s.cur.size),
                                       fmod_pow2(s.cur.min.z, s.cur.size)));
        const float hs = s.tb.size * 0.5f;
        s.target = offset_sectant(vsub(vadd(s.tb.min, mk(hs, hs, hs)), s.cur.min), s.cur.size);
        const uint32_t sel = dda_step(s.r, s.p, s.tb);
        s.target = step_sectant(s.r, s.target, sel);
        s.tb.min = vadd(s.tb.min, vmul(step_vec(s.r, sel), s.tb.size));
        if (s.count != 0) s.node = ls_top(s);
        s.state = S_NODE;
        return false;
    }
    if (s.ntype == VHX_NODE_INTERNAL && ((s.occ >> s.target) & 1ull) != 0) {
        if (COUNT) s.bytes += 4;
        const uint32_t child = t.children[(uint64_t)s.node * 64u + s.target];
        if (child >= t.node_count) return true;  // the reference would panic on an invalid key
        s.node = child;
        s.cur = s.tb;
        s.target = offset_sectant(vsub(s.p, s.tb.min), s.tb.size);
        s.tb = child_bounds(s.cur, s.target);
        ls_push(s, child);
        s.state = S_NODE;
        return false;
    }
    s.state = S_ADVANCE;
    return false;
}

// One traversal step. Returns true when the ray is finished (h holds the result, h.hit = false for a miss).
template <bool COUNT, int BD>
__device__ __forceinline__ bool ls_step(const DevTree &t, LaneState &s, HitOut &h) {
    using B = Brick<BD>;
    h.hit = false;
    if (s.state == S_BRICK) {
        if ((uint32_t)s.ix >= (uint32_t)BD || (uint32_t)s.iy >= (uint32_t)BD || (uint32_t)s.iz >= (uint32_t)BD)
            return ls_after_probe<COUNT>(t, s, s.ntype == VHX_NODE_UNIFORM_LEAF);  // brick missed
        const uint32_t sel = s.sel;
        s.flat += ((sel & 1u) ? s.r.isx : 0) + ((sel & 2u) ? s.r.isy * BD : 0) + ((sel & 4u) ? s.r.isz * (BD * BD) : 0);
        if (B::WORDS > 1) {
            const int32_t wi = s.flat >> 6;
            if (wi != s.word_idx) {
                s.word_idx = wi;
                s.word = t.brick_occ[(uint64_t)s.desc * B::WORDS + (uint32_t)wi];
            }
        }
        if (COUNT) s.bytes += 4;
        const uint64_t vbase = (uint64_t)s.desc * (uint64_t)B::N3;
        if ((s.word >> (s.flat & 63)) & 1ull) {
            const uint32_t v = t.voxels[vbase + (uint32_t)s.flat];
            if (COUNT) s.bytes += pal_bytes<COUNT>(v);
            CubeD hb;
            hb.size = s.bb.size * B::INV;
            hb.min = vadd(s.bb.min, vmul(vmul(mk((float)s.ix, (float)s.iy, (float)s.iz), s.bb.size), B::INV));
            fill_hit(h, v, (uint32_t)s.flat, s.p, hb);
            h.hit = true;
            return true;
        }
        if (COUNT) s.bytes += pal_bytes<COUNT>(t.voxels[vbase + (uint32_t)s.flat]);
        if (++s.iters > VHX_MAX_ITERS) return true;
        const uint32_t nsel = dda_step(s.r, s.p, s.bcur);
        s.sel = nsel;
        s.bcur.min = vadd(s.bcur.min, vmul(step_vec(s.r, nsel), s.bcur.size));
        s.ix += (nsel & 1u) ? s.r.isx : 0;
        s.iy += (nsel & 2u) ? s.r.isy : 0;
        s.iz += (nsel & 4u) ? s.r.isz : 0;
        return false;
    }
    if (s.state == S_ADVANCE) {
        if (++s.iters > VHX_MAX_ITERS) return true;
        const uint32_t sel = dda_step(s.r, s.p, s.tb);
        s.target = step_sectant(s.r, s.target, sel);
        if (s.target < 64) s.tb.min = vadd(s.tb.min, vmul(step_vec(s.r, sel), s.tb.size));
        if (s.target >= 64 || ((s.occ >> s.target) & 1ull) != 0) s.state = S_NODE;
        return false;
    }
    // S_NODE
    if (s.count == 0) {
        // inner loop exhausted: restart from the root (cpu.rs:441-455, then 317-320)
        const float tsize = (float)t.size;
        s.p = vadd(s.p, vmul(s.r.d, 0.1f));
        if (!(s.p.x < tsize && s.p.y < tsize && s.p.z < tsize && s.p.x > 0.0f && s.p.y > 0.0f && s.p.z > 0.0f))
            return true;
        s.target = offset_sectant(s.p, tsize);
        s.node = 0;
        s.cur.min = mk(0.0f, 0.0f, 0.0f);
        s.cur.size = tsize;
        ls_push(s, 0u);
    }
    if (++s.iters > VHX_MAX_ITERS) return true;
    const uint32_t last = ls_top(s);
    const uint4 lh = t.hdr[last];
    s.occ = ((uint64_t)lh.y << 32) | (uint64_t)lh.x;
    s.ntype = last == s.node ? lh.z : t.hdr[s.node].z;
    if (COUNT) s.bytes += 12;
    const bool uniform = s.ntype == VHX_NODE_UNIFORM_LEAF;
    if (s.target < 64 && (uniform || s.ntype == VHX_NODE_LEAF)) {
        if (COUNT) s.bytes += 4;
        s.desc = t.children[(uint64_t)s.node * 64u + (uniform ? 0u : s.target)];
        s.bb = uniform ? s.cur : child_bounds(s.cur, s.target);
        if (s.desc != VHX_EMPTY) {
            if (s.desc & VHX_SOLID_BIT) {
                if (COUNT) s.bytes += 4;
                ls_hit_solid(t, s, h);
                return true;
            }
            // Parted: traverse_brick setup (cpu.rs:146-168)
            const float rs = rcp_pow2(s.bb.size);
            const F3d pib = vmul(vmul(vsub(s.p, s.bb.min), (float)BD), rs);
            int32_t ix = ras_i32(pib.x), iy = ras_i32(pib.y), iz = ras_i32(pib.z);
            s.ix = ix < 0 ? 0 : (ix > BD - 1 ? BD - 1 : ix);
            s.iy = iy < 0 ? 0 : (iy > BD - 1 ? BD - 1 : iy);
            s.iz = iz < 0 ? 0 : (iz > BD - 1 ? BD - 1 : iz);
            s.flat = s.ix + s.iy * BD + s.iz * BD * BD;
            const float unit = s.bb.size * B::INV;
            s.bcur.min = vadd(s.bb.min, vmul(mk((float)s.ix, (float)s.iy, (float)s.iz), unit));
            s.bcur.size = unit;
            s.word_idx = s.flat >> 6;
            s.word = t.brick_occ[(uint64_t)s.desc * B::WORDS + (uint32_t)s.word_idx];
            s.sel = 0;
            s.state = S_BRICK;
            return false;
        }
    }
    return ls_after_probe<COUNT>(t, s, uniform);
}

}  // namespace vhx
