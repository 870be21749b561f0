/*
 * vhx_oracle.c — CPU restatement of VoxelHex's reference raytracer. TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library, and only as the
 * checker / reported CPU baseline. The product path (libvhx.so, voxelhex_amd) never links or calls it.
 *
 * What it restates (paths relative to the VoxelHex repository, commit mounted at /root/reference):
 *   get_by_ray              src/raytracing/cpu.rs:296-458
 *   NodeStack<u32,4>        src/raytracing/cpu.rs:18-76   (ring buffer: push overwrites the oldest entry)
 *   get_dda_scale_factors   src/raytracing/cpu.rs:79-92
 *   dda_step_to_next_sibling src/raytracing/cpu.rs:104-132
 *   traverse_brick          src/raytracing/cpu.rs:136-232
 *   probe_brick             src/raytracing/cpu.rs:236-292
 *   Cube::intersect_ray     src/spatial/raytracing/mod.rs:33-62
 *   cube_impact_normal      src/spatial/raytracing/mod.rs:97-125
 *   Cube::child_bounds_for  src/spatial/mod.rs:72-77,   step_sectant src/spatial/mod.rs:23-26
 *   offset_sectant          src/spatial/math/mod.rs:27-44, hash_direction src/spatial/math/mod.rs:48-52
 *   V3c arithmetic          src/spatial/math/vector.rs (length 71-73, normalized 75-77, modulo 62-67,
 *                           From<V3c<f32>> for V3c<i32> = round, 373-383)
 *   pix_points_to_empty     src/boxtree/node.rs:311-333
 *   LUTs                    src/spatial/lut.rs:4-161, regenerated with the logic of
 *                           src/bin/sectant_region_offset_lut.rs:12-26 and src/bin/sectant_step_result_lut.rs:48-114;
 *                           RAY_TO_NODE_OCCUPANCY_BITMASK_LUT (lut.rs:96-161, no generator in the reference) is
 *                           regenerated from its observable rule and pinned against the table in tests/golden/.
 *   primary rays            benches/performance.rs:32-61 (glass), examples/gpu_render.rs:203-224 (inverse VP)
 *   shading                 examples/gpu_render.rs:199, 236-251
 *
 * Float semantics follow Rust: IEEE f32 ops in source order, no FMA contraction (build with -ffp-contract=off),
 * f32::min/max ignore NaN (fminf/fmaxf), signum(+-0) = +-1, `as` casts saturate (NaN -> 0), % on f32 is fmodf,
 * powf(x, 2.) is x*x (LLVM folds it so), V3c<f32> -> V3c<i32> rounds half away from zero.
 *
 * MIP stand-ins (vhx_oracle_set_node_mips; not the reference CPU path, which never reads MIPs): with node MIPs set,
 * a node iteration whose target sectant is occupied but whose child entry is absent traces the node's MIP brick over
 * the node's cube first -- the WGSL path's probe_MIP (src/raytracing/bevy/viewport_render.wgsl:328-364, 438-454) --
 * and ADVANCEs past the sectant on a miss instead of pushing into the missing child (docs/DESIGN_LOG.md §10b).
 *
 * Deviation (documented in DESIGN.md): the reference loops have no iteration bound; this restatement stops a ray
 * after VHX_ORACLE_MAX_ITERS inner iterations and reports a miss (the GPU kernel uses the same bound).
 */
#include "../include/vhx.h"

#include <math.h>
#include <stdint.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define VHX_ORACLE_MAX_ITERS (1u << 22)
static _Thread_local uint32_t g_brick_steps; /* per-thread scratch for the work statistics */
/* optional per-ray event trace (diagnostics: wave-divergence simulation in scripts/sim_divergence.py):
 * N node iteration, P brick probe, B brick cell step, O pop, U push, A advance step, R restart */
static _Thread_local uint8_t *g_ev;
static _Thread_local uint32_t g_ev_n, g_ev_cap;
#define EV(ch)                                                     \
    do {                                                           \
        if (g_ev && g_ev_n < g_ev_cap) g_ev[g_ev_n++] = (uint8_t)(ch); \
    } while (0)
/* optional: the node key of every N event (the node the iteration visits), for the queue-order simulations */
static _Thread_local uint32_t *g_evn;
static _Thread_local uint32_t g_evn_n, g_evn_cap;
#define EVN(key)                                                       \
    do {                                                               \
        if (g_evn && g_evn_n < g_evn_cap) g_evn[g_evn_n++] = (uint32_t)(key); \
    } while (0)

typedef struct { float x, y, z; } v3;
typedef struct { v3 min; float size; } cube;

/* ---------------------------------------------------------------- Rust scalar semantics --------------------- */
static inline float r_min(float a, float b) { return fminf(a, b); }
static inline float r_max(float a, float b) { return fmaxf(a, b); }
static inline float r_signum(float a) { return isnan(a) ? a : copysignf(1.0f, a); }
static inline int32_t r_as_i32(float f) {
    if (isnan(f)) return 0;
    if (f >= 2147483648.0f) return INT32_MAX;
    if (f <= -2147483648.0f) return INT32_MIN;
    return (int32_t)f;
}
static inline uint32_t r_as_u32(float f) {
    if (isnan(f) || f <= 0.0f) return 0;
    if (f >= 4294967296.0f) return UINT32_MAX;
    return (uint32_t)f;
}
static inline uint8_t r_as_u8(float f) {
    if (isnan(f) || f <= 0.0f) return 0;
    if (f >= 255.0f) return 255;
    return (uint8_t)f;
}

/* ---------------------------------------------------------------- V3c<f32> ---------------------------------- */
static inline v3 V(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v3 v_add(v3 a, v3 b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 v_sub(v3 a, v3 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 v_mul(v3 a, float s) { return V(a.x * s, a.y * s, a.z * s); }
static inline v3 v_div(v3 a, float s) { return V(a.x / s, a.y / s, a.z / s); }
static inline float v_length(v3 a) { return sqrtf((a.x * a.x + a.y * a.y) + a.z * a.z); }
static inline v3 v_normalized(v3 a) { return v_div(a, v_length(a)); }
static inline float v_dot(v3 a, v3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }

/* ---------------------------------------------------------------- LUTs -------------------------------------- */
static float SECTANT_OFFSET[64][3];
static uint8_t STEP_LUT[64][3][3][3];
static uint64_t OCC_LUT[64][8];
static int luts_ready = 0;

/* sectant_region_offset_lut.rs:12-26: offset of sectant flat(x,y,z) = (x/4, y/4, z/4) */
static void gen_offset_lut(void) {
    for (int x = 0; x < 4; ++x)
        for (int y = 0; y < 4; ++y)
            for (int z = 0; z < 4; ++z) {
                int s = x + y * 4 + z * 16;
                SECTANT_OFFSET[s][0] = (float)x / 4.0f;
                SECTANT_OFFSET[s][1] = (float)y / 4.0f;
                SECTANT_OFFSET[s][2] = (float)z / 4.0f;
            }
}

/* sectant_step_result_lut.rs: hash_region 10-23, sectant_after_step 48-93 */
static uint8_t hash_region_unit(v3 o) {
    int ix = (int)floorf(o.x * 4.0f / 1.0f), iy = (int)floorf(o.y * 4.0f / 1.0f), iz = (int)floorf(o.z * 4.0f / 1.0f);
    return (uint8_t)(ix + iy * 4 + iz * 16);
}
static uint8_t sectant_after_step(int sx, int sy, int sz, int sectant) {
    v3 sg = V((float)((sx > 0) - (sx < 0)), (float)((sy > 0) - (sy < 0)), (float)((sz > 0) - (sz < 0)));
    v3 off = V(SECTANT_OFFSET[sectant][0], SECTANT_OFFSET[sectant][1], SECTANT_OFFSET[sectant][2]);
    float ssize = 1.0f / 4.0f;
    v3 center = v_add(off, V(ssize / 2.0f, ssize / 2.0f, ssize / 2.0f));
    v3 after = v_add(center, V(ssize * sg.x, ssize * sg.y, ssize * sg.z));
    if (after.x < 0.f || after.x > 1.f || after.y < 0.f || after.y > 1.f || after.z < 0.f || after.z > 1.f) {
        v3 w = V(fmodf(after.x, 1.f), fmodf(after.y, 1.f), fmodf(after.z, 1.f));
        if (w.x < 0.f) w.x += 1.f;
        if (w.y < 0.f) w.y += 1.f;
        if (w.z < 0.f) w.z += 1.f;
        return (uint8_t)(64 + hash_region_unit(w));
    }
    return hash_region_unit(after);
}
static void gen_step_lut(void) {
    for (int s = 0; s < 64; ++s)
        for (int z = -1; z <= 1; ++z)
            for (int y = -1; y <= 1; ++y)
                for (int x = -1; x <= 1; ++x) STEP_LUT[s][x + 1][y + 1][z + 1] = sectant_after_step(x, y, z, s);
}
/* RAY_TO_NODE_OCCUPANCY_BITMASK_LUT[s][o]: sectants reachable from s moving monotonically in octant o, where
 * o = (dx>=0) + 2*(dz>=0) + 4*(dy>=0) (hash_direction, math/mod.rs:48-52). Pinned by tests against lut.rs. */
static void gen_occ_lut(void) {
    for (int s = 0; s < 64; ++s) {
        int sx = s % 4, sy = (s / 4) % 4, sz = s / 16;
        for (int o = 0; o < 8; ++o) {
            int px = o & 1, pz = (o >> 1) & 1, py = (o >> 2) & 1;
            uint64_t m = 0;
            for (int t = 0; t < 64; ++t) {
                int tx = t % 4, ty = (t / 4) % 4, tz = t / 16;
                int okx = px ? (tx >= sx) : (tx <= sx);
                int oky = py ? (ty >= sy) : (ty <= sy);
                int okz = pz ? (tz >= sz) : (tz <= sz);
                if (okx && oky && okz) m |= (uint64_t)1 << t;
            }
            OCC_LUT[s][o] = m;
        }
    }
}
static void ensure_luts(void) {
    if (luts_ready) return;
    gen_offset_lut();
    gen_step_lut();
    gen_occ_lut();
    luts_ready = 1;
}

/* ---------------------------------------------------------------- spatial ----------------------------------- */
/* step_sectant, spatial/mod.rs:23-26 */
static inline uint8_t step_sectant(uint8_t s, v3 step) {
    int ix = r_as_i32(step.x), iy = r_as_i32(step.y), iz = r_as_i32(step.z);
    return STEP_LUT[s][((ix > 0) - (ix < 0)) + 1][((iy > 0) - (iy < 0)) + 1][((iz > 0) - (iz < 0)) + 1];
}
/* Cube::child_bounds_for, spatial/mod.rs:72-77 */
static inline cube child_bounds_for(cube c, uint8_t s) {
    cube r;
    r.min = v_add(c.min, v_mul(V(SECTANT_OFFSET[s][0], SECTANT_OFFSET[s][1], SECTANT_OFFSET[s][2]), c.size));
    r.size = c.size / 4.0f;
    return r;
}
/* offset_sectant, math/mod.rs:27-44 */
static inline uint8_t offset_sectant(v3 off, float size) {
    v3 idx = v_div(v_mul(off, 4.0f), size);
    idx = V(floorf(idx.x), floorf(idx.y), floorf(idx.z));
    idx = V(r_min(idx.x, 3.0f), r_min(idx.y, 3.0f), r_min(idx.z, 3.0f));
    return r_as_u8(idx.x + (idx.y * 4.0f) + (idx.z * 16.0f));
}
/* hash_direction, math/mod.rs:48-52 */
static inline unsigned hash_direction(v3 d) {
    v3 o = v_add(V(1.f, 1.f, 1.f), d);
    return (unsigned)(o.x >= 1.f) + (unsigned)(o.z >= 1.f) * 2u + (unsigned)(o.y >= 1.f) * 4u;
}
/* Cube::intersect_ray, spatial/raytracing/mod.rs:33-62. returns 0 = None, 1 = Some(None), 2 = Some(Some(t)) */
static int intersect_ray(cube c, v3 o, v3 d, float *t) {
    v3 mx = v_add(c.min, V(c.size, c.size, c.size));
    float t1 = (c.min.x - o.x) / d.x, t2 = (mx.x - o.x) / d.x;
    float t3 = (c.min.y - o.y) / d.y, t4 = (mx.y - o.y) / d.y;
    float t5 = (c.min.z - o.z) / d.z, t6 = (mx.z - o.z) / d.z;
    float tmin = r_max(r_max(r_min(t1, t2), r_min(t3, t4)), r_min(t5, t6));
    float tmax = r_min(r_min(r_max(t1, t2), r_max(t3, t4)), r_max(t5, t6));
    if (tmax < 0.f || tmin > tmax) return 0;
    if (tmin < 0.0f) return 1;
    *t = tmin;
    return 2;
}
/* cube_impact_normal, spatial/raytracing/mod.rs:97-125 */
static v3 cube_impact_normal(cube c, v3 p) {
    v3 m = v_sub(v_add(c.min, V(c.size / 2.f, c.size / 2.f, c.size / 2.f)), p);
    float mc = r_max(r_max(fabsf(m.x), fabsf(m.y)), fabsf(m.z));
    v3 n = V(fabsf(m.x) == mc ? -m.x : 0.f, fabsf(m.y) == mc ? -m.y : 0.f, fabsf(m.z) == mc ? -m.z : 0.f);
    return v_normalized(n);
}

/* ---------------------------------------------------------------- raytracer --------------------------------- */
typedef struct {
    v3 o, d, sf;
} ray_t;

typedef struct {
    uint32_t value, cell, voxel[3], bytes, hit;
    v3 impact, normal;
    uint32_t n_node, n_advance, n_brick, n_pop, n_push, n_restart, n_probe; /* work statistics */
} hit_t;

/* get_dda_scale_factors, cpu.rs:79-92 */
static v3 dda_scale_factors(v3 d) {
    float zx = d.z / d.x, yx = d.y / d.x, xy = d.x / d.y, zy = d.z / d.y, xz = d.x / d.z, yz = d.y / d.z;
    return V(sqrtf((1.f + zx * zx) + yx * yx), sqrtf((xy * xy + 1.f) + zy * zy), sqrtf((xz * xz + 1.f) + yz * yz));
}
/* dda_step_to_next_sibling, cpu.rs:104-132 */
static v3 dda_step(const ray_t *r, v3 *p, cube b) {
    v3 sg = V(r_signum(r->d.x), r_signum(r->d.y), r_signum(r->d.z));
    v3 diff = v_sub(*p, b.min);
    v3 st = V(b.size * r_max(sg.x, 0.f) - sg.x * diff.x, b.size * r_max(sg.y, 0.f) - sg.y * diff.y,
              b.size * r_max(sg.z, 0.f) - sg.z * diff.z);
    float dx = fabsf(st.x * r->sf.x), dy = fabsf(st.y * r->sf.y), dz = fabsf(st.z * r->sf.z);
    float m = r_min(r_min(dx, dy), dz);
    *p = v_add(*p, v_mul(r->d, m));
    return V(m == dx ? sg.x : 0.f, m == dy ? sg.y : 0.f, m == dz ? sg.z : 0.f);
}
/* NodeContent::pix_points_to_empty, node.rs:311-333 (palette index beyond the palette = that half is none) */
static int points_to_empty(const vhx_tree_desc *t, uint32_t v, uint32_t *bytes) {
    uint32_t ci = v & 0xFFFFu, di = v >> 16;
    int color_empty = 1, data_empty = 1;
    if (ci != 0xFFFFu) {
        *bytes += 4;
        if (ci < t->color_count) color_empty = ((t->color_palette[ci] >> 24) & 0xFFu) == 0;
    }
    if (di != 0xFFFFu) {
        *bytes += 4;
        if (di < t->data_count) data_empty = t->data_palette[di] == 0;
    }
    return color_empty && data_empty;
}
/* traverse_brick, cpu.rs:136-232 */
static int traverse_brick(const vhx_tree_desc *t, const ray_t *r, v3 *p, const uint32_t *brick, cube bb, int bd,
                          int32_t idx_out[3], int32_t *flat_out, uint32_t *bytes, uint32_t *iters) {
    v3 pib = v_div(v_mul(v_sub(*p, bb.min), (float)bd), bb.size);
    int32_t ix = r_as_i32(pib.x), iy = r_as_i32(pib.y), iz = r_as_i32(pib.z);
    ix = ix < 0 ? 0 : (ix > bd - 1 ? bd - 1 : ix);
    iy = iy < 0 ? 0 : (iy > bd - 1 ? bd - 1 : iy);
    iz = iz < 0 ? 0 : (iz > bd - 1 ? bd - 1 : iz);
    int32_t fdx = 1, fdy = bd, fdz = bd * bd;
    int32_t flat = ix + iy * bd + iz * bd * bd;
    float unit = bb.size / (float)bd;
    cube cur;
    cur.min = v_add(bb.min, v_mul(V((float)ix, (float)iy, (float)iz), unit));
    cur.size = unit;
    v3 step = V(0.f, 0.f, 0.f);
    for (;;) {
        if (ix < 0 || ix >= bd || iy < 0 || iy >= bd || iz < 0 || iz >= bd) return 0;
        flat += r_as_i32(step.x) * fdx + r_as_i32(step.y) * fdy + r_as_i32(step.z) * fdz;
        *bytes += 4;
        if (!points_to_empty(t, brick[flat], bytes)) {
            idx_out[0] = ix;
            idx_out[1] = iy;
            idx_out[2] = iz;
            *flat_out = flat;
            return 1;
        }
        if (++*iters > VHX_ORACLE_MAX_ITERS) return 0;
        (*bytes) += 0; /* keep byte model unchanged */
        g_brick_steps += 1;
        EV('B');
        step = dda_step(r, p, cur);
        cur.min = v_add(cur.min, v_mul(step, unit));
        ix += r_as_i32(roundf(step.x));
        iy += r_as_i32(roundf(step.y));
        iz += r_as_i32(roundf(step.z));
    }
}
/* probe_brick, cpu.rs:236-292 */
static int probe_brick(const vhx_tree_desc *t, const ray_t *r, v3 *p, uint32_t desc, cube bb, hit_t *h,
                       uint32_t *iters) {
    if (desc == VHX_EMPTY) return 0;
    if (desc & VHX_SOLID_BIT) {
        h->bytes += 4;
        h->value = t->solid_values[desc & 0x7FFFFFFFu];
        h->cell = VHX_EMPTY;
        h->impact = *p;
        h->normal = cube_impact_normal(bb, *p);
        h->voxel[0] = r_as_u32(bb.min.x);
        h->voxel[1] = r_as_u32(bb.min.y);
        h->voxel[2] = r_as_u32(bb.min.z);
        return 1;
    }
    int bd = (int)t->brick_dim;
    const uint32_t *brick = t->voxels + (uint64_t)desc * (uint64_t)bd * (uint64_t)bd * (uint64_t)bd;
    int32_t idx[3], flat;
    if (!traverse_brick(t, r, p, brick, bb, bd, idx, &flat, &h->bytes, iters)) return 0;
    cube hb;
    hb.size = bb.size / (float)bd;
    hb.min = v_add(bb.min, v_div(v_mul(V((float)idx[0], (float)idx[1], (float)idx[2]), bb.size), (float)bd));
    h->value = brick[flat];
    h->cell = (uint32_t)flat;
    h->impact = *p;
    h->normal = cube_impact_normal(hb, *p);
    h->voxel[0] = r_as_u32(hb.min.x);
    h->voxel[1] = r_as_u32(hb.min.y);
    h->voxel[2] = r_as_u32(hb.min.z);
    return 1;
}

/* NodeStack<u32, SIZE>, cpu.rs:18-76 */
typedef struct { uint32_t data[4]; uint32_t head, count; } node_stack;
static inline void ns_push(node_stack *s, uint32_t v) {
    s->head = (s->head + 1) % 4;
    s->count = s->count + 1 < 4 ? s->count + 1 : 4;
    s->data[s->head] = v;
}
static inline void ns_pop(node_stack *s) {
    if (s->count == 0) return;
    s->count -= 1;
    s->head = s->head == 0 ? 3 : s->head - 1;
}

/* node MIP descriptors (vhx_oracle_set_node_mips), NULL = the reference path */
static const uint32_t *g_node_mips;
static uint32_t g_node_mips_count;

/* BoxTree::get_by_ray, cpu.rs:296-458 */
static void get_by_ray(const vhx_tree_desc *t, v3 o, v3 d, hit_t *h) {
    memset(h, 0, sizeof(*h));
    h->value = VHX_EMPTY;
    h->cell = VHX_EMPTY;
    h->voxel[0] = h->voxel[1] = h->voxel[2] = VHX_EMPTY;
    ray_t r;
    r.o = o;
    r.d = d;
    r.sf = dda_scale_factors(d);
    unsigned dir_idx = hash_direction(d);
    float tsize = (float)t->boxtree_size;
    node_stack stack;
    memset(&stack, 0, sizeof(stack));
    cube cur = {V(0.f, 0.f, 0.f), tsize};
    v3 p;
    uint8_t target;
    cube tb;
    float tt = 0.f;
    int isect = intersect_ray(cur, o, d, &tt);
    if (isect) {
        p = v_add(o, v_mul(d, isect == 2 ? tt : 0.f));
        target = offset_sectant(p, cur.size);
        tb = child_bounds_for(cur, target);
    } else {
        p = o;
        target = 64;
        tb = cur;
    }
    uint32_t node = 0;
    uint32_t iters = 0;
    while (target < 64) {
        node = 0;
        cur.min = V(0.f, 0.f, 0.f);
        cur.size = tsize;
        ns_push(&stack, 0);
        while (stack.count != 0) {
            if (++iters > VHX_ORACLE_MAX_ITERS) return;
            h->n_node++;
            EV('N');
            EVN(node);
            uint64_t occ = t->node_ocbits[stack.data[stack.head]];
            uint32_t ntype = t->node_type[node];
            h->bytes += 12;
            int backtrack = ntype == VHX_NODE_UNIFORM_LEAF;
            if (target < 64) {
                if (ntype == VHX_NODE_UNIFORM_LEAF) {
                    h->bytes += 4;
                    h->n_probe++;
                    EV('P');
                    if (probe_brick(t, &r, &p, t->node_children[(uint64_t)node * 64], cur, h, &iters)) {
                        h->hit = 1;
                        return;
                    }
                    backtrack = 1;
                } else if (ntype == VHX_NODE_LEAF) {
                    h->bytes += 4;
                    h->n_probe++;
                    EV('P');
                    if (probe_brick(t, &r, &p, t->node_children[(uint64_t)node * 64 + target],
                                    child_bounds_for(cur, target), h, &iters)) {
                        h->hit = 1;
                        return;
                    }
                }
            }
            int mip_adv = 0; /* MIP stand-in for an occupied but absent child (see the header) */
            if (g_node_mips && target < 64 && (ntype == VHX_NODE_INTERNAL || ntype == VHX_NODE_LEAF) &&
                t->node_children[(uint64_t)node * 64 + target] == VHX_EMPTY && (occ & ((uint64_t)1 << target)) != 0) {
                mip_adv = 1;
                h->bytes += 4;
                const uint32_t mdesc = node < g_node_mips_count ? g_node_mips[node] : VHX_EMPTY;
                v3 pm = p;
                if (probe_brick(t, &r, &pm, mdesc, cur, h, &iters)) {
                    h->hit = 1;
                    return;
                }
            }
            if (backtrack || target >= 64 || occ == 0 || (occ & OCC_LUT[target][dir_idx]) == 0) {
                /* POP */
                h->n_pop++;
                EV('O');
                ns_pop(&stack);
                tb = cur;
                cur.size *= 4.0f;
                cur.min = v_sub(cur.min, V(fmodf(cur.min.x, cur.size), fmodf(cur.min.y, cur.size),
                                           fmodf(cur.min.z, cur.size)));
                target = offset_sectant(v_sub(v_add(tb.min, V(tb.size / 2.f, tb.size / 2.f, tb.size / 2.f)), cur.min),
                                        cur.size);
                v3 sv = dda_step(&r, &p, tb);
                target = step_sectant(target, sv);
                tb.min = v_add(tb.min, v_mul(sv, tb.size));
                if (stack.count != 0) node = stack.data[stack.head];
                continue;
            }
            if (ntype == VHX_NODE_INTERNAL && (occ & ((uint64_t)1 << target)) != 0 && !mip_adv) {
                /* PUSH */
                h->n_push++;
                EV('U');
                h->bytes += 4;
                uint32_t child = t->node_children[(uint64_t)node * 64 + target];
                if (child >= t->node_count) return; /* reference would panic on the invalid key */
                node = child;
                cur = tb;
                target = offset_sectant(v_sub(p, tb.min), tb.size);
                tb = child_bounds_for(cur, target);
                ns_push(&stack, child);
            } else {
                /* ADVANCE */
                for (;;) {
                    if (++iters > VHX_ORACLE_MAX_ITERS) return;
                    h->n_advance++;
                    EV('A');
                    v3 sv = dda_step(&r, &p, tb);
                    target = step_sectant(target, sv);
                    if (target < 64) tb.min = v_add(tb.min, v_mul(sv, tb.size));
                    if (target >= 64 || (occ & ((uint64_t)1 << target)) != 0) break;
                }
            }
        }
        h->n_restart++;
        EV('R');
        p = v_add(p, v_mul(d, 0.1f));
        if (p.x < tsize && p.y < tsize && p.z < tsize && p.x > 0.f && p.y > 0.f && p.z > 0.f)
            target = offset_sectant(p, tsize);
        else
            target = 64;
    }
}

/* examples/gpu_render.rs:199, 236-251 */
static uint32_t shade(const vhx_tree_desc *t, const hit_t *h) {
    if (!h->hit) return 128u | (128u << 8) | (128u << 16) | (255u << 24);
    uint32_t ci = h->value & 0xFFFFu;
    if (ci == 0xFFFFu || ci >= t->color_count) return 255u << 24;
    uint32_t c = t->color_palette[ci];
    v3 L = v_normalized(V(0.f, -1.f, 1.f));
    float s = 1.f - (v_dot(h->normal, L) / 2.f + 0.5f);
    uint32_t rr = r_as_u8((float)(c & 0xFFu) * s), gg = r_as_u8((float)((c >> 8) & 0xFFu) * s),
             bb = r_as_u8((float)((c >> 16) & 0xFFu) * s);
    return rr | (gg << 8) | (bb << 16) | (255u << 24);
}

static void store_hit(const vhx_tree_desc *t, const vhx_hits *out, uint64_t i, v3 o, const hit_t *h) {
    if (out->value) out->value[i] = h->hit ? h->value : VHX_EMPTY;
    if (out->cell) out->cell[i] = h->hit ? h->cell : VHX_EMPTY;
    if (out->voxel) {
        for (int k = 0; k < 3; ++k) out->voxel[3 * i + k] = h->hit ? h->voxel[k] : VHX_EMPTY;
    }
    if (out->impact) {
        out->impact[3 * i] = h->hit ? h->impact.x : 0.f;
        out->impact[3 * i + 1] = h->hit ? h->impact.y : 0.f;
        out->impact[3 * i + 2] = h->hit ? h->impact.z : 0.f;
    }
    if (out->normal) {
        out->normal[3 * i] = h->hit ? h->normal.x : 0.f;
        out->normal[3 * i + 1] = h->hit ? h->normal.y : 0.f;
        out->normal[3 * i + 2] = h->hit ? h->normal.z : 0.f;
    }
    if (out->depth) out->depth[i] = h->hit ? v_length(v_sub(h->impact, o)) : INFINITY;
    if (out->rgba) out->rgba[i] = shade(t, h);
    if (out->bytes) out->bytes[i] = h->bytes;
}

/* benches/performance.rs:54-61 and examples/gpu_render.rs:203-224 (glam Mat4*Vec4, Vec3::normalize) */
static void primary_ray(const vhx_camera *c, uint32_t px, uint32_t py, v3 *o, v3 *d) {
    uint32_t x = px, y = c->height - 1u - py; /* image rows are flipped: gpu_render.rs:198 */
    *o = V(c->origin[0], c->origin[1], c->origin[2]);
    if (c->ray_model == VHX_RAY_GLASS) {
        v3 bl = V(c->glass_bottom_left[0], c->glass_bottom_left[1], c->glass_bottom_left[2]);
        v3 rt = V(c->glass_right[0], c->glass_right[1], c->glass_right[2]);
        v3 up = V(c->glass_up[0], c->glass_up[1], c->glass_up[2]);
        v3 gp = v_add(v_add(bl, v_mul(v_mul(rt, (float)x), c->pixel_width)), v_mul(v_mul(up, (float)y), c->pixel_height));
        *d = v_normalized(v_sub(gp, *o));
    } else {
        const float *m = c->inv_view_proj;
        float nx = ((float)x + 0.5f) / (float)c->width * 2.0f - 1.0f;
        float ny = ((float)y + 0.5f) / (float)c->height * 2.0f - 1.0f;
        float nr[4], fr[4];
        for (int k = 0; k < 4; ++k) {
            nr[k] = ((m[k] * nx + m[4 + k] * ny) + m[8 + k] * -1.0f) + m[12 + k] * 1.0f;
            fr[k] = ((m[k] * nx + m[4 + k] * ny) + m[8 + k] * 1.0f) + m[12 + k] * 1.0f;
        }
        v3 np = V(nr[0] / nr[3], nr[1] / nr[3], nr[2] / nr[3]);
        v3 fp = V(fr[0] / fr[3], fr[1] / fr[3], fr[2] / fr[3]);
        v3 dd = v_sub(fp, np);
        float rcp = 1.0f / sqrtf((dd.x * dd.x + dd.y * dd.y) + dd.z * dd.z);
        *d = v_mul(dd, rcp);
    }
}

/* ---------------------------------------------------------------- exported API ------------------------------ */
/* Sets (or with NULL clears) the node MIP descriptors every following trace uses (process-wide). */
void vhx_oracle_set_node_mips(const uint32_t *node_mips, uint32_t count) {
    g_node_mips = node_mips;
    g_node_mips_count = node_mips ? count : 0;
}

int vhx_oracle_trace_rays(const vhx_tree_desc *t, const float *rays, uint64_t n, const vhx_hits *out, int threads) {
    if (!t || !rays || !out) return VHX_E_INVALID_ARG;
    ensure_luts();
#ifdef _OPENMP
    if (threads <= 0) threads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 64) num_threads(threads)
#endif
    for (int64_t i = 0; i < (int64_t)n; ++i) {
        hit_t h;
        v3 o = V(rays[6 * i], rays[6 * i + 1], rays[6 * i + 2]);
        v3 d = V(rays[6 * i + 3], rays[6 * i + 4], rays[6 * i + 5]);
        get_by_ray(t, o, d, &h);
        store_hit(t, out, (uint64_t)i, o, &h);
    }
    (void)threads;
    return VHX_OK;
}

/* Traces the pixel rectangle [x0,x0+w) x [y0,y0+h) of the frame; output row-major inside the rectangle. */
int vhx_oracle_trace_primary(const vhx_tree_desc *t, const vhx_camera *cam, uint32_t x0, uint32_t y0, uint32_t w,
                             uint32_t h, const vhx_hits *out, int threads) {
    if (!t || !cam || !out) return VHX_E_INVALID_ARG;
    ensure_luts();
#ifdef _OPENMP
    if (threads <= 0) threads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 64) num_threads(threads)
#endif
    for (int64_t i = 0; i < (int64_t)w * (int64_t)h; ++i) {
        uint32_t col = (uint32_t)(i % w), row = (uint32_t)(i / w);
        uint32_t px = x0 + col, py = y0 + row;
        hit_t hh;
        v3 o, d;
        primary_ray(cam, px, py, &o, &d);
        get_by_ray(t, o, d, &hh);
        store_hit(t, out, (uint64_t)i, o, &hh);
    }
    (void)threads;
    return VHX_OK;
}

/* Hard shadows (BASELINE config 5; no reference counterpart — docs/DESIGN_LOG.md §9 defines them): for every hit record i
 * (value[i] != 0xFFFFFFFF) one shadow ray from impact + normal * 1e-3 (multiply, then add) toward `light`, direction
 * normalised like V3c::normalized; shadowed[i] = hit ? 1 : 0; rgba (optional) gets rgb >> 1 where shadowed; bytes
 * (optional) the shadow ray's algorithmic bytes. */
int vhx_oracle_trace_shadows(const vhx_tree_desc *t, const float light[3], uint64_t n, const uint32_t *value,
                             const float *impact, const float *normal, uint32_t *shadowed, uint32_t *rgba,
                             uint32_t *bytes, int threads) {
    if (!t || !light || (n && (!value || !impact || !normal || !shadowed))) return VHX_E_INVALID_ARG;
    ensure_luts();
#ifdef _OPENMP
    if (threads <= 0) threads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 64) num_threads(threads)
#endif
    for (int64_t i = 0; i < (int64_t)n; ++i) {
        shadowed[i] = 0;
        if (bytes) bytes[i] = 0;
        if (value[i] == VHX_EMPTY) continue;
        const float *ip = impact + 3 * i, *np = normal + 3 * i;
        v3 o = V(ip[0] + np[0] * 1e-3f, ip[1] + np[1] * 1e-3f, ip[2] + np[2] * 1e-3f);
        v3 d = v_normalized(V(light[0] - o.x, light[1] - o.y, light[2] - o.z));
        hit_t h;
        get_by_ray(t, o, d, &h);
        shadowed[i] = h.hit ? 1u : 0u;
        if (rgba && h.hit) rgba[i] = ((rgba[i] >> 1) & 0x007F7F7Fu) | (rgba[i] & 0xFF000000u);
        if (bytes) bytes[i] = h.bytes;
    }
    (void)threads;
    return VHX_OK;
}

/* Generates the three lookup tables (for pinning against the reference tables in tests/golden). */
void vhx_oracle_luts(float offset[64 * 3], uint8_t step[64 * 27], uint64_t occ[64 * 8]) {
    ensure_luts();
    memcpy(offset, SECTANT_OFFSET, sizeof(SECTANT_OFFSET));
    memcpy(step, STEP_LUT, sizeof(STEP_LUT));
    memcpy(occ, OCC_LUT, sizeof(OCC_LUT));
}

/* Primitive entry points, for the spatial known-answer tests of src/spatial/{tests.rs,raytracing/tests.rs,
 * math/tests.rs}. */
uint32_t vhx_oracle_offset_sectant(const float off[3], float size) {
    ensure_luts();
    return offset_sectant(V(off[0], off[1], off[2]), size);
}
uint32_t vhx_oracle_step_sectant(uint32_t s, const float step[3]) {
    ensure_luts();
    return step_sectant((uint8_t)s, V(step[0], step[1], step[2]));
}
uint32_t vhx_oracle_hash_direction(const float d[3]) { return hash_direction(V(d[0], d[1], d[2])); }
/* returns 0 None, 1 Some(impact_distance None), 2 Some(Some(t)) */
int vhx_oracle_intersect_ray(const float cmin[3], float csize, const float ray[6], float *t) {
    cube c = {V(cmin[0], cmin[1], cmin[2]), csize};
    return intersect_ray(c, V(ray[0], ray[1], ray[2]), V(ray[3], ray[4], ray[5]), t);
}
void vhx_oracle_cube_impact_normal(const float cmin[3], float csize, const float p[3], float n[3]) {
    cube c = {V(cmin[0], cmin[1], cmin[2]), csize};
    v3 r = cube_impact_normal(c, V(p[0], p[1], p[2]));
    n[0] = r.x;
    n[1] = r.y;
    n[2] = r.z;
}
/* Ring-buffer NodeStack<i32, size> (cpu.rs:18-76) for the node_stack_tests (cpu.rs tests 812-902).
 * ops: value >= 0 = push(value), -1 = pop, -2 = last; results: popped/last value or INT32_MIN for None. */
int vhx_oracle_nodestack_run(int size, const int32_t *ops, int n, int32_t *results) {
    if (size <= 0 || size > 64) return VHX_E_INVALID_ARG;
    int32_t data[64] = {0};
    int head = 0, count = 0;
    for (int i = 0; i < n; ++i) {
        results[i] = INT32_MIN;
        if (ops[i] >= 0) {
            head = (head + 1) % size;
            count = count + 1 < size ? count + 1 : size;
            data[head] = ops[i];
        } else if (ops[i] == -1) {
            if (count != 0) {
                count -= 1;
                results[i] = data[head];
                head = head == 0 ? size - 1 : head - 1;
            }
        } else if (count != 0) {
            results[i] = data[head];
        }
    }
    return VHX_OK;
}

/* Work statistics over a pixel rectangle (instrumentation for DESIGN.md): sums of per-ray counters
 * [rays, hits, node iterations, advance steps, brick steps, pops, pushes, restarts, probes, bytes] and the max of
 * node+advance+brick steps over rays in stats[10]. */
int vhx_oracle_work_stats(const vhx_tree_desc *t, const vhx_camera *cam, uint32_t x0, uint32_t y0, uint32_t w,
                          uint32_t h, double stats[11]) {
    ensure_luts();
    for (int k = 0; k < 11; ++k) stats[k] = 0;
    for (uint32_t row = 0; row < h; ++row)
        for (uint32_t col = 0; col < w; ++col) {
            hit_t hh;
            v3 o, d;
            primary_ray(cam, x0 + col, y0 + row, &o, &d);
            g_brick_steps = 0;
            get_by_ray(t, o, d, &hh);
            stats[0] += 1;
            stats[1] += hh.hit;
            stats[2] += hh.n_node;
            stats[3] += hh.n_advance;
            stats[4] += g_brick_steps;
            stats[5] += hh.n_pop;
            stats[6] += hh.n_push;
            stats[7] += hh.n_restart;
            stats[8] += hh.n_probe;
            stats[9] += hh.bytes;
            double tot = (double)hh.n_node + hh.n_advance + g_brick_steps;
            if (tot > stats[10]) stats[10] = tot;
        }
    return VHX_OK;
}

/* Per-ray total steps (node iterations + advance steps + brick steps) over a pixel rectangle, row-major. */
int vhx_oracle_ray_steps(const vhx_tree_desc *t, const vhx_camera *cam, uint32_t x0, uint32_t y0, uint32_t w,
                         uint32_t h, uint32_t *steps, int threads) {
    ensure_luts();
#ifdef _OPENMP
    if (threads <= 0) threads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 64) num_threads(threads)
#endif
    for (int64_t i = 0; i < (int64_t)w * (int64_t)h; ++i) {
        hit_t hh;
        v3 o, d;
        primary_ray(cam, x0 + (uint32_t)(i % w), y0 + (uint32_t)(i / w), &o, &d);
        g_brick_steps = 0;
        get_by_ray(t, o, d, &hh);
        steps[i] = hh.n_node + hh.n_advance + g_brick_steps;
    }
    (void)threads;
    return VHX_OK;
}

/* Per-ray event sequences (see EV above) for the primary rays of the given pixels: events of ray i are
 * buf[off[i] .. off[i+1]); returns the total length, or -1 if cap was too small. Diagnostics only. */
int64_t vhx_oracle_ray_events(const vhx_tree_desc *t, const vhx_camera *cam, const uint32_t *px, const uint32_t *py,
                              uint64_t n, uint8_t *buf, uint64_t cap, uint64_t *off) {
    ensure_luts();
    uint64_t used = 0;
    for (uint64_t i = 0; i < n; ++i) {
        hit_t hh;
        v3 o, d;
        primary_ray(cam, px[i], py[i], &o, &d);
        g_ev = buf + used;
        g_ev_n = 0;
        g_ev_cap = (uint32_t)(cap - used > 0xFFFFFFFFull ? 0xFFFFFFFFull : cap - used);
        get_by_ray(t, o, d, &hh);
        off[i] = used;
        if (g_ev_n >= g_ev_cap) {
            g_ev = 0;
            return -1;
        }
        used += g_ev_n;
    }
    off[n] = used;
    g_ev = 0;
    return (int64_t)used;
}

/* vhx_oracle_ray_events plus the node key of every N event: nodes[noff[i] .. noff[i+1]) for ray i (as many as its N
 * events); -1 if either capacity was too small. Diagnostics only. */
int64_t vhx_oracle_ray_events_nodes(const vhx_tree_desc *t, const vhx_camera *cam, const uint32_t *px,
                                    const uint32_t *py, uint64_t n, uint8_t *buf, uint64_t cap, uint64_t *off,
                                    uint32_t *nodes, uint64_t ncap, uint64_t *noff) {
    uint64_t nused = 0;
    ensure_luts();
    uint64_t used = 0;
    for (uint64_t i = 0; i < n; ++i) {
        hit_t hh;
        v3 o, d;
        primary_ray(cam, px[i], py[i], &o, &d);
        g_ev = buf + used;
        g_ev_n = 0;
        g_ev_cap = (uint32_t)(cap - used > 0xFFFFFFFFull ? 0xFFFFFFFFull : cap - used);
        g_evn = nodes + nused;
        g_evn_n = 0;
        g_evn_cap = (uint32_t)(ncap - nused > 0xFFFFFFFFull ? 0xFFFFFFFFull : ncap - nused);
        get_by_ray(t, o, d, &hh);
        off[i] = used;
        noff[i] = nused;
        if (g_ev_n >= g_ev_cap || g_evn_n >= g_evn_cap) {
            g_ev = 0;
            g_evn = 0;
            return -1;
        }
        used += g_ev_n;
        nused += g_evn_n;
    }
    off[n] = used;
    noff[n] = nused;
    g_ev = 0;
    g_evn = 0;
    return (int64_t)used;
}
