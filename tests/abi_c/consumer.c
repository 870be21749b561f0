/* A compiled C consumer of libvhx's C ABI (include/vhx.h), built with `gcc -std=c99` and linked against libvhx.so by
 * tests/test_abi_c.py. It makes the calls the reference's Rust renderer would make through the `extern "C"` block of
 * INTEGRATION.md, in the same order: create the context (BoxTreeGPUHost::new, src/raytracing/bevy/mod.rs:164-180),
 * upload the flattened tree (prepare_bind_groups, pipeline/mod.rs:242-402), dispatch a frame (VhxRenderNode::run,
 * pipeline/mod.rs:96-155), a second context for a frame in flight, a ranged write (write_range_to_buffer,
 * streaming/mod.rs:344-370) and a retrace, refused calls with vhx_last_error, and the one-rank multi-GPU split.
 *
 * usage: consumer TREE_FILE OUT_DIR
 *   TREE_FILE: "VHXT", u32 version 1, u32 sizeof(vhx_camera), the 8 u32 counts of vhx_tree_desc, the vhx_camera bytes,
 *              then the 7 arrays in VHX_BUF_* order (sizes from the counts)
 *   OUT_DIR:   frame0.bin  value|cell|voxel|impact|normal|depth|rgba of the uploaded tree
 *              batch.bin   value|depth|rgba of the 5 frames of two back-to-back vhx_trace_primary_batch calls, then
 *                          the shadowed flags of the 2 frames of one vhx_trace_shadows_batch (light (S, S, S))
 *              frame1.bin  value|depth|rgba after clearing the first `clear` voxels (the count is printed)
 *              mgpu.bin    rgba|depth of the one-rank vhx_mgpu render of the uploaded tree
 * exit 0 = every call behaved as expected; 3 = no HIP device (vhx_create returned VHX_E_NO_DEVICE); 1 = failure. */
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "vhx.h"

#define CHECK(call)                                                                                               \
    do {                                                                                                          \
        int rc_ = (call);                                                                                         \
        if (rc_ != VHX_OK) {                                                                                      \
            fprintf(stderr, "%s:%d %s = %d (%s)\n", __FILE__, __LINE__, #call, rc_, vhx_last_error(ctx));        \
            return 1;                                                                                             \
        }                                                                                                         \
    } while (0)

static void *read_exact(FILE *f, size_t bytes) {
    void *p = malloc(bytes ? bytes : 1);
    if (p && bytes && fread(p, 1, bytes, f) != bytes) {
        free(p);
        return NULL;
    }
    return p;
}

static int write_parts(const char *dir, const char *name, const void *const *parts, const size_t *bytes, int n) {
    char path[4096];
    snprintf(path, sizeof(path), "%s/%s", dir, name);
    FILE *f = fopen(path, "wb");
    if (!f) return 1;
    for (int i = 0; i < n; ++i)
        if (fwrite(parts[i], 1, bytes[i], f) != bytes[i]) {
            fclose(f);
            return 1;
        }
    return fclose(f) != 0;
}

int main(int argc, char **argv) {
    vhx_ctx *ctx = NULL;
    if (argc != 3) {
        fprintf(stderr, "usage: consumer TREE_FILE OUT_DIR\n");
        return 1;
    }
    if (vhx_abi_version() != VHX_ABI_VERSION) {
        fprintf(stderr, "ABI version %u, header %u\n", vhx_abi_version(), VHX_ABI_VERSION);
        return 1;
    }
    /* ---- the tree and the camera, as the host side would hand them over ---- */
    FILE *f = fopen(argv[1], "rb");
    if (!f) return 1;
    char magic[4];
    uint32_t head[2], counts[8];
    if (fread(magic, 1, 4, f) != 4 || memcmp(magic, "VHXT", 4) != 0 || fread(head, 4, 2, f) != 2 || head[0] != 1 ||
        head[1] != sizeof(vhx_camera) || fread(counts, 4, 8, f) != 8) {
        fprintf(stderr, "bad tree file\n");
        return 1;
    }
    vhx_camera cam;
    if (fread(&cam, sizeof(cam), 1, f) != 1) return 1;
    vhx_tree_desc t;
    memset(&t, 0, sizeof(t));
    t.boxtree_size = counts[0];
    t.brick_dim = counts[1];
    t.node_count = counts[2];
    t.brick_count = counts[3];
    t.solid_count = counts[4];
    t.color_count = counts[5];
    t.data_count = counts[6];
    const uint64_t n3 = (uint64_t)t.brick_dim * t.brick_dim * t.brick_dim;
    const size_t sizes[7] = {4ull * t.node_count,   8ull * t.node_count, 256ull * t.node_count, 4ull * n3 * t.brick_count,
                             4ull * t.solid_count, 4ull * t.color_count, 4ull * t.data_count};
    void *arrays[7];
    for (int i = 0; i < 7; ++i)
        if (!(arrays[i] = read_exact(f, sizes[i]))) {
            fprintf(stderr, "short tree file\n");
            return 1;
        }
    fclose(f);
    t.node_type = (const uint32_t *)arrays[0];
    t.node_ocbits = (const uint64_t *)arrays[1];
    t.node_children = (const uint32_t *)arrays[2];
    t.voxels = (const uint32_t *)arrays[3];
    t.solid_values = (const uint32_t *)arrays[4];
    t.color_palette = (const uint32_t *)arrays[5];
    t.data_palette = (const uint32_t *)arrays[6];

    /* ---- context and upload ---- */
    int ndev = 0;
    if (vhx_device_count(&ndev) != VHX_OK) return 1;
    int rc = vhx_create(0, &ctx);
    if (rc == VHX_E_NO_DEVICE) {
        printf("no_device 1 devices %d\n", ndev);
        return 3;
    }
    if (rc != VHX_OK) return 1;
    CHECK(vhx_upload_tree(ctx, &t));

    /* ---- frame 0: every field, host outputs ---- */
    const uint64_t n = (uint64_t)cam.width * cam.height;
    uint32_t *value = malloc(4 * n), *cell = malloc(4 * n), *voxel = malloc(12 * n), *rgba = malloc(4 * n);
    float *impact = malloc(12 * n), *normal = malloc(12 * n), *depth = malloc(4 * n);
    if (!value || !cell || !voxel || !rgba || !impact || !normal || !depth) return 1;
    vhx_hits h = {value, cell, voxel, impact, normal, depth, rgba, NULL, NULL};
    CHECK(vhx_trace_primary(ctx, &cam, 0, 0, 1, VHX_LAYOUT_FRAMEBUFFER, &h, 0));
    float ms = 0.0f;
    CHECK(vhx_sync(ctx, &ms));
    {
        const void *parts[7] = {value, cell, voxel, impact, normal, depth, rgba};
        const size_t bytes[7] = {4 * n, 4 * n, 12 * n, 12 * n, 12 * n, 4 * n, 4 * n};
        if (write_parts(argv[2], "frame0.bin", parts, bytes, 7)) return 1;
    }
    uint64_t hits = 0;
    for (uint64_t i = 0; i < n; ++i) hits += value[i] != VHX_EMPTY;
    printf("frame0 %ux%u hits %llu trace_ms %.3f\n", cam.width, cam.height, (unsigned long long)hits, ms);

    /* ---- batches (vhx_trace_primary_batch), device outputs: two batches back to back on ONE context (3 + 2 frames
     * of the same camera; with the staging ring on, "stage_slots=4", the second call queues behind the first without a
     * host wait), an
     * aliasing batch that must be refused, then the hard shadows of two frames as one vhx_trace_shadows_batch ---- */
    {
        enum { NB = 5 };
        void *dv[NB], *dd[NB], *dr[NB], *di[2], *dn[2], *ds[2];
        for (int k = 0; k < NB; ++k)
            if (hipMalloc(&dv[k], 4 * n) != hipSuccess || hipMalloc(&dd[k], 4 * n) != hipSuccess ||
                hipMalloc(&dr[k], 4 * n) != hipSuccess)
                return 1;
        for (int k = 0; k < 2; ++k)
            if (hipMalloc(&di[k], 12 * n) != hipSuccess || hipMalloc(&dn[k], 12 * n) != hipSuccess ||
                hipMalloc(&ds[k], 4 * n) != hipSuccess)
                return 1;
        vhx_camera bc[NB];
        vhx_hits bh[NB];
        for (int k = 0; k < NB; ++k) {
            bc[k] = cam;
            vhx_hits z = {(uint32_t *)dv[k], NULL, NULL, k < 2 ? (float *)di[k] : NULL, k < 2 ? (float *)dn[k] : NULL,
                          (float *)dd[k], (uint32_t *)dr[k], NULL, NULL};
            bh[k] = z;
        }
        CHECK(vhx_set_tuning(ctx, "stage_slots=4"));
        CHECK(vhx_trace_primary_batch(ctx, bc, 3, bh));
        CHECK(vhx_trace_primary_batch(ctx, bc + 3, 2, bh + 3));
        vhx_hits alias[2] = {bh[0], bh[0]};
        alias[1].value = (uint32_t *)dv[1];
        alias[1].depth = (float *)dd[1];
        rc = vhx_trace_primary_batch(ctx, bc, 2, alias); /* both frames would write one rgba array */
        printf("batch_overlap %d \"%s\"\n", rc, vhx_last_error(ctx));
        if (rc != VHX_E_INVALID_ARG) return 1;
        const float light[3] = {(float)t.boxtree_size, (float)t.boxtree_size, (float)t.boxtree_size};
        vhx_shadow_frame sf[2];
        for (int k = 0; k < 2; ++k) {
            vhx_shadow_frame z = {(const uint32_t *)dv[k], (const float *)di[k], (const float *)dn[k], (uint32_t *)ds[k],
                                  NULL};
            sf[k] = z;
        }
        CHECK(vhx_trace_shadows_batch(ctx, light, 2, n, sf));
        CHECK(vhx_sync(ctx, &ms));
        uint32_t *host = malloc(4 * n * (3 * NB + 2));
        if (!host) return 1;
        for (int k = 0; k < NB; ++k)
            if (hipMemcpy(host + (3 * k) * n, dv[k], 4 * n, hipMemcpyDeviceToHost) != hipSuccess ||
                hipMemcpy(host + (3 * k + 1) * n, dd[k], 4 * n, hipMemcpyDeviceToHost) != hipSuccess ||
                hipMemcpy(host + (3 * k + 2) * n, dr[k], 4 * n, hipMemcpyDeviceToHost) != hipSuccess)
                return 1;
        for (int k = 0; k < 2; ++k)
            if (hipMemcpy(host + (3 * NB + k) * n, ds[k], 4 * n, hipMemcpyDeviceToHost) != hipSuccess) return 1;
        const void *parts[1] = {host};
        const size_t bytes[1] = {4 * n * (3 * NB + 2)};
        if (write_parts(argv[2], "batch.bin", parts, bytes, 1)) return 1;
        printf("batch frames %d shadow_frames 2\n", NB);
        free(host);
        for (int k = 0; k < NB; ++k) (void)hipFree(dv[k]), (void)hipFree(dd[k]), (void)hipFree(dr[k]);
        for (int k = 0; k < 2; ++k) (void)hipFree(di[k]), (void)hipFree(dn[k]), (void)hipFree(ds[k]);
    }

    /* ---- a second context on the same tree (a frame in flight) traces the same frame ---- */
    vhx_ctx *sh = NULL;
    CHECK(vhx_create_shared(ctx, &sh));
    uint32_t *value2 = malloc(4 * n), *rgba2 = malloc(4 * n);
    float *depth2 = malloc(4 * n);
    if (!value2 || !rgba2 || !depth2) return 1;
    vhx_hits h2 = {value2, NULL, NULL, NULL, NULL, depth2, rgba2, NULL, NULL};
    CHECK(vhx_trace_primary(sh, &cam, 0, 0, 1, VHX_LAYOUT_FRAMEBUFFER, &h2, 0));
    const int shared_equal = !memcmp(value, value2, 4 * n) && !memcmp(rgba, rgba2, 4 * n) && !memcmp(depth, depth2, 4 * n);
    printf("shared_equal %d\n", shared_equal);

    /* ---- a ranged write through the owner, then the shared context retraces (ordered by libvhx) ---- */
    const uint64_t clear = (t.brick_count / 3) * n3;
    uint32_t *empty = malloc(4 * (clear ? clear : 1));
    if (!empty) return 1;
    for (uint64_t i = 0; i < clear; ++i) empty[i] = VHX_EMPTY;
    CHECK(vhx_update_range(ctx, VHX_BUF_VOXELS, 0, clear, empty));
    memset(empty, 0, 4 * (clear ? clear : 1)); /* the source may be reused as soon as the call returns */
    CHECK(vhx_trace_primary(sh, &cam, 0, 0, 1, VHX_LAYOUT_FRAMEBUFFER, &h2, 0));
    {
        const void *parts[3] = {value2, depth2, rgba2};
        const size_t bytes[3] = {4 * n, 4 * n, 4 * n};
        if (write_parts(argv[2], "frame1.bin", parts, bytes, 3)) return 1;
    }
    printf("frame1 cleared_voxels %llu\n", (unsigned long long)clear);

    /* ---- refused calls and their messages ---- */
    uint32_t small[8] = {0};
    const uint64_t nvox = n3 * t.brick_count;
    rc = vhx_update_range(ctx, VHX_BUF_VOXELS, nvox - 4, 8, small);
    printf("past_end %d \"%s\"\n", rc, vhx_last_error(ctx));
    if (rc != VHX_E_CAPACITY) return 1;
    rc = vhx_update_range(sh, VHX_BUF_VOXELS, 0, 4, small);
    printf("through_shared %d \"%s\"\n", rc, vhx_last_error(sh));
    if (rc != VHX_E_STATE) return 1;
    vhx_camera bad = cam;
    bad.width = 0;
    rc = vhx_trace_primary(ctx, &bad, 0, 0, 1, VHX_LAYOUT_FRAMEBUFFER, &h, 0);
    printf("empty_frame %d \"%s\"\n", rc, vhx_last_error(ctx));
    if (rc != VHX_E_INVALID_ARG) return 1;

    /* ---- the multi-GPU split on a one-rank communicator: broadcast (re-upload) and render ---- */
    uint8_t id[VHX_MGPU_ID_BYTES];
    rc = vhx_mgpu_unique_id(id);
    if (rc == VHX_E_RCCL) {
        printf("mgpu skipped (RCCL not loadable)\n");
    } else {
        CHECK(rc);
        vhx_mgpu *m = NULL;
        CHECK(vhx_mgpu_create(ctx, id, 1, 0, 64, &m));
        CHECK(vhx_mgpu_broadcast_tree(m, &t)); /* rank 0 uploads the original tree again */
        vhx_tile_plan plan;
        CHECK(vhx_mgpu_tile_plan(1, 1, 64, cam.width, cam.height, 0, &plan));
        void *fb = NULL, *fbd = NULL;
        if (hipMalloc(&fb, 4 * n) != hipSuccess || hipMalloc(&fbd, 4 * n) != hipSuccess) return 1;
        CHECK(vhx_mgpu_render(m, &cam, (uint32_t *)fb, (float *)fbd));
        CHECK(vhx_mgpu_sync(m, &ms));
        if (hipMemcpy(rgba2, fb, 4 * n, hipMemcpyDeviceToHost) != hipSuccess ||
            hipMemcpy(depth2, fbd, 4 * n, hipMemcpyDeviceToHost) != hipSuccess)
            return 1;
        const void *parts[2] = {rgba2, depth2};
        const size_t bytes[2] = {4 * n, 4 * n};
        if (write_parts(argv[2], "mgpu.bin", parts, bytes, 2)) return 1;
        printf("mgpu tiles %u slots %u trace_ms %.3f\n", plan.tiles, plan.slots, ms);
        vhx_mgpu_destroy(m);
        (void)hipFree(fb);
        (void)hipFree(fbd);
    }
    vhx_destroy(sh);
    vhx_destroy(ctx);
    for (int i = 0; i < 7; ++i) free(arrays[i]);
    free(value), free(cell), free(voxel), free(rgba), free(impact), free(normal), free(depth);
    free(value2), free(rgba2), free(depth2), free(empty);
    printf("ok\n");
    return 0;
}
