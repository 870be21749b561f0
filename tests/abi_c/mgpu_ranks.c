/* Multi-rank driver of the vhx_mgpu ABI (include/vhx.h), C99 + pthreads, one thread per rank, every rank with its own
 * vhx_ctx on HIP device 0. Run by tests/test_gpu_mgpu_ranks.py with VHX_RCCL_LIB pointing at the loopback communicator
 * (tests/loopback/loopback_rccl.cpp), so that the N > 1 code of vhx_mgpu -- the tree broadcast's receive side, the
 * tile deal over R + N - 1 slots, the point-to-point group into rank 0's slot-major buffer, the untile, frames in
 * flight and vhx_mgpu_balance with peers -- runs on one GPU. Each rank makes the calls a rank process of the reference
 * renderer would make (multi-GPU).
 *
 * usage: mgpu_ranks TREE_FILE CAMB_FILE OUT_FILE NRANKS ROOT_SLOTS FRAMES_IN_FLIGHT OVERLAP FRAMES MODE
 *   TREE_FILE  the consumer.c tree file (tree + camera A);  CAMB_FILE  raw vhx_camera bytes of camera B
 *   ROOT_SLOTS R (MODE "balance": chosen by vhx_mgpu_balance instead)
 *   FRAMES     frames rendered, alternating camera A and B (A first), every one submitted without waiting
 *   MODE       "plain" | "balance" | "rgba" (plain with one plane: vhx_mgpu_set_planes(m, 1) on every rank, rank 0
 *              passes fb_depth = NULL, so its depth framebuffers keep their 0xAB fill; first a set_planes call with
 *              different counts on rank 0 and the others, which every rank must refuse) | "batch" / "batchrgba" (plain /
 *              rgba with the frames submitted as vhx_mgpu_render_batch calls of 3 frames)
 *   OUT_FILE   rank 0's framebuffers after the last frame of each camera: rgbaA | depthA | rgbaB | depthB
 * prints one line per rank (rays, measured trace / transfer ms, bytes into rank 0 per frame) and "root_slots R", then
 * "ok"; exit 1 on failure. */
#define _POSIX_C_SOURCE 200809L
#include <hip/hip_runtime_api.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "vhx.h"

#define MAX_RANKS 8

static vhx_tree_desc g_tree;
static vhx_camera g_cam[2];
static uint8_t g_id[VHX_MGPU_ID_BYTES];
static int g_n, g_R, g_F, g_overlap, g_frames, g_balance, g_rgba, g_batch;
static const char *g_out;

typedef struct {
    int rank;
    int rc;
    char err[512];
    uint64_t rays;
    float trace_ms, xfer_ms;
    uint32_t R;
    uint64_t root_bytes;
} rank_state;

#define RCHECK(call)                                                                                              \
    do {                                                                                                          \
        int rc_ = (call);                                                                                         \
        if (rc_ != VHX_OK) {                                                                                      \
            snprintf(s->err, sizeof(s->err), "%s = %d (%s)", #call, rc_, ctx ? vhx_last_error(ctx) : "");        \
            s->rc = rc_ ? rc_ : -1;                                                                               \
            goto done;                                                                                            \
        }                                                                                                         \
    } while (0)

static void *rank_main(void *arg) {
    rank_state *s = (rank_state *)arg;
    vhx_ctx *ctx = NULL;
    vhx_mgpu *m = NULL;
    void *fb[2] = {NULL, NULL}, *fbd[2] = {NULL, NULL};
    uint32_t *host = NULL;
    const uint64_t n = (uint64_t)g_cam[0].width * g_cam[0].height;
    RCHECK(vhx_create(0, &ctx));
    RCHECK(vhx_mgpu_create(ctx, g_id, g_n, s->rank, 64, &m));
    RCHECK(vhx_mgpu_set_frames_in_flight(m, (uint32_t)g_F));
    RCHECK(vhx_mgpu_set_overlap(m, g_overlap));
    RCHECK(vhx_mgpu_broadcast_tree(m, s->rank == 0 ? &g_tree : NULL));
    if (g_rgba) {
        /* a disagreement first (rank 0 asks for one plane, the others for two): every rank is refused alike */
        const int drc = vhx_mgpu_set_planes(m, s->rank == 0 ? 1u : 2u);
        if (drc != VHX_E_INVALID_ARG) {
            snprintf(s->err, sizeof(s->err), "set_planes with different counts returned %d", drc);
            s->rc = -1;
            goto done;
        }
        RCHECK(vhx_mgpu_set_planes(m, 1));
    }
    if (g_balance) {
        RCHECK(vhx_mgpu_balance(m, &g_cam[0], 3, &s->R, NULL, NULL));
    } else {
        RCHECK(vhx_mgpu_set_root_slots(m, (uint32_t)g_R));
        s->R = (uint32_t)g_R;
    }
    if (s->rank == 0)
        for (int c = 0; c < 2; ++c)
            if (hipMalloc(&fb[c], 4 * n) != hipSuccess || hipMalloc(&fbd[c], 4 * n) != hipSuccess ||
                hipMemset(fb[c], 0xAB, 4 * n) != hipSuccess || hipMemset(fbd[c], 0xAB, 4 * n) != hipSuccess) {
                snprintf(s->err, sizeof(s->err), "hipMalloc");
                s->rc = -1;
                goto done;
            }
    /* every frame submitted back to back: frames in flight on F contexts, gathers overlapping the next traces */
    if (g_batch) {
        /* batches of g_batch frames (the last one shorter); frame k still alternates the cameras and framebuffers */
        for (int k0 = 0; k0 < g_frames; k0 += g_batch) {
            vhx_camera bc[8];
            uint32_t *bf[8];
            float *bd[8];
            const int nb = g_frames - k0 < g_batch ? g_frames - k0 : g_batch;
            for (int j = 0; j < nb; ++j) {
                bc[j] = g_cam[(k0 + j) & 1];
                bf[j] = (uint32_t *)fb[(k0 + j) & 1];
                bd[j] = (float *)fbd[(k0 + j) & 1];
            }
            RCHECK(vhx_mgpu_render_batch(m, bc, (uint32_t)nb, s->rank == 0 ? bf : NULL,
                                         s->rank == 0 && !g_rgba ? bd : NULL));
        }
    } else {
        for (int k = 0; k < g_frames; ++k)
            RCHECK(vhx_mgpu_render(m, &g_cam[k & 1], (uint32_t *)fb[k & 1], g_rgba ? NULL : (float *)fbd[k & 1]));
    }
    RCHECK(vhx_mgpu_sync(m, NULL));
    RCHECK(vhx_mgpu_info(m, g_cam[0].width, g_cam[0].height, NULL, NULL, &s->rays));
    RCHECK(vhx_mgpu_frame_bytes(m, g_cam[0].width, g_cam[0].height, &s->root_bytes));
    RCHECK(vhx_mgpu_measure(m, &g_cam[0], 2, &s->trace_ms, &s->xfer_ms));
    if (s->rank == 0) {
        host = (uint32_t *)malloc(16 * n);
        if (!host) {
            s->rc = -1;
            goto done;
        }
        for (int c = 0; c < 2; ++c)
            if (hipMemcpy(host + (2 * c) * n, fb[c], 4 * n, hipMemcpyDeviceToHost) != hipSuccess ||
                hipMemcpy(host + (2 * c + 1) * n, fbd[c], 4 * n, hipMemcpyDeviceToHost) != hipSuccess) {
                s->rc = -1;
                goto done;
            }
        FILE *f = fopen(g_out, "wb");
        if (!f || fwrite(host, 4, 4 * n, f) != 4 * n || fclose(f) != 0) {
            snprintf(s->err, sizeof(s->err), "writing %s", g_out);
            s->rc = -1;
        }
    }
done:
    if (m) vhx_mgpu_destroy(m);
    for (int c = 0; c < 2; ++c) {
        if (fb[c]) (void)hipFree(fb[c]);
        if (fbd[c]) (void)hipFree(fbd[c]);
    }
    free(host);
    if (ctx) vhx_destroy(ctx);
    return NULL;
}

static void *read_exact(FILE *f, size_t bytes) {
    void *p = malloc(bytes ? bytes : 1);
    if (p && bytes && fread(p, 1, bytes, f) != bytes) {
        free(p);
        return NULL;
    }
    return p;
}

int main(int argc, char **argv) {
    if (argc != 10) {
        fprintf(stderr, "usage: mgpu_ranks TREE_FILE CAMB_FILE OUT_FILE NRANKS ROOT_SLOTS FRAMES_IN_FLIGHT OVERLAP "
                        "FRAMES MODE\n");
        return 1;
    }
    g_out = argv[3];
    g_n = atoi(argv[4]);
    g_R = atoi(argv[5]);
    g_F = atoi(argv[6]);
    g_overlap = atoi(argv[7]);
    g_frames = atoi(argv[8]);
    g_balance = strcmp(argv[9], "balance") == 0;
    g_rgba = strcmp(argv[9], "rgba") == 0 || strcmp(argv[9], "batchrgba") == 0;
    g_batch = strncmp(argv[9], "batch", 5) == 0 ? 3 : 0;
    if (g_n < 1 || g_n > MAX_RANKS || g_frames < 2) return 1;
    FILE *f = fopen(argv[1], "rb");
    char magic[4];
    uint32_t head[2], counts[8];
    if (!f || fread(magic, 1, 4, f) != 4 || memcmp(magic, "VHXT", 4) != 0 || fread(head, 4, 2, f) != 2 ||
        head[0] != 1 || head[1] != sizeof(vhx_camera) || fread(counts, 4, 8, f) != 8 ||
        fread(&g_cam[0], sizeof(vhx_camera), 1, f) != 1) {
        fprintf(stderr, "bad tree file\n");
        return 1;
    }
    vhx_tree_desc *t = &g_tree;
    t->boxtree_size = counts[0];
    t->brick_dim = counts[1];
    t->node_count = counts[2];
    t->brick_count = counts[3];
    t->solid_count = counts[4];
    t->color_count = counts[5];
    t->data_count = counts[6];
    const uint64_t n3 = (uint64_t)t->brick_dim * t->brick_dim * t->brick_dim;
    const size_t sizes[7] = {4ull * t->node_count,   8ull * t->node_count, 256ull * t->node_count,
                             4ull * n3 * t->brick_count, 4ull * t->solid_count, 4ull * t->color_count,
                             4ull * t->data_count};
    void *arrays[7];
    for (int i = 0; i < 7; ++i)
        if (!(arrays[i] = read_exact(f, sizes[i]))) {
            fprintf(stderr, "short tree file\n");
            return 1;
        }
    fclose(f);
    t->node_type = (const uint32_t *)arrays[0];
    t->node_ocbits = (const uint64_t *)arrays[1];
    t->node_children = (const uint32_t *)arrays[2];
    t->voxels = (const uint32_t *)arrays[3];
    t->solid_values = (const uint32_t *)arrays[4];
    t->color_palette = (const uint32_t *)arrays[5];
    t->data_palette = (const uint32_t *)arrays[6];
    f = fopen(argv[2], "rb");
    if (!f || fread(&g_cam[1], sizeof(vhx_camera), 1, f) != 1 || g_cam[1].width != g_cam[0].width ||
        g_cam[1].height != g_cam[0].height) {
        fprintf(stderr, "bad camera file\n");
        return 1;
    }
    fclose(f);
    if (vhx_mgpu_unique_id(g_id) != VHX_OK) {
        fprintf(stderr, "vhx_mgpu_unique_id failed (VHX_RCCL_LIB?)\n");
        return 1;
    }
    rank_state st[MAX_RANKS];
    pthread_t th[MAX_RANKS];
    memset(st, 0, sizeof(st));
    for (int r = 0; r < g_n; ++r) {
        st[r].rank = r;
        if (pthread_create(&th[r], NULL, rank_main, &st[r]) != 0) return 1;
    }
    int bad = 0;
    uint64_t rays = 0;
    for (int r = 0; r < g_n; ++r) {
        pthread_join(th[r], NULL);
        printf("rank %d rc %d rays %llu trace_ms %.4f transfer_ms %.4f R %u root_bytes %llu %s\n", r, st[r].rc,
               (unsigned long long)st[r].rays, st[r].trace_ms, st[r].xfer_ms, st[r].R,
               (unsigned long long)st[r].root_bytes, st[r].err);
        bad |= st[r].rc != 0 || st[r].R != st[0].R;
        rays += st[r].rays;
    }
    printf("root_slots %u rays %llu\n", st[0].R, (unsigned long long)rays);
    for (int i = 0; i < 7; ++i) free(arrays[i]);
    if (bad) return 1;
    printf("ok\n");
    return 0;
}
