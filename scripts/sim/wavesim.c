/* Wave-level simulation of the traversal kernels' SIMT schedule (diagnostics for DESIGN.md §3 / §12; not product code).
 *
 * Per-ray event sequences come from the oracle (vhx_oracle_ray_events: N node iteration, P probe, B brick cell step,
 * O pop, U push, A advance step, R restart) and are cut into node iterations. The simulator replays the multi-pass
 * schedule of libvhx (pass 0 over 8x8-pixel waves with a step budget and sparse-wave abandonment, queue passes over
 * 64 consecutive rays in frame order, budgets counted like Trav: node iterations + brick steps + advance steps) and,
 * per wave iteration, counts the wave executions and active lanes of every block of Trav::step, the block structure of
 * the kernel. `design` selects alternative loop structures:
 *   0  current: per iteration top, probe, brick walk loop (max brick steps), pop / push / walk setup, advance loop
 *   1  capped brick walks: at most `cap` brick trips per iteration; a lane whose walk is unfinished carries it into
 *      the next iteration (it skips the node blocks there)
 *   5  merged walk: pop / push / walk setup first, then one loop over brick and node steps (block 15: switch)
 * Output: per pass and block, waves and lanes (same blocks as the VHX_PROF kernel build), so that design 0 can be
 * checked against the GPU counts of scripts/probes/probe_blocks.py.
 *
 * Build: gcc -O2 -fopenmp -shared -fPIC scripts/sim/wavesim.c -o scripts/sim/_build/libwavesim.so
 * Driver: scripts/sim/wavesim.py */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/vhx.h"

int64_t vhx_oracle_ray_events_nodes(const vhx_tree_desc *t, const vhx_camera *cam, const uint32_t *px,
                                    const uint32_t *py, uint64_t n, uint8_t *buf, uint64_t cap, uint64_t *off,
                                    uint32_t *nodes, uint64_t ncap, uint64_t *noff);

#define VHX_MAX_ITERS_SIM (1u << 22)

typedef struct {
    uint8_t probe, nb, pop, push, na, restart;
    uint32_t node;  /* the node the iteration visits */
} it_t;

static it_t *g_its;
static uint64_t *g_off; /* per pixel: first iteration; g_off[n] = total */
static uint32_t g_W, g_H;

/* events of every pixel, cut into iterations (rows in parallel) */
int64_t wavesim_build(const vhx_tree_desc *t, const vhx_camera *cam, uint32_t W, uint32_t H) {
    const uint64_t n = (uint64_t)W * H;
    free(g_its);
    free(g_off);
    g_W = W;
    g_H = H;
    g_off = (uint64_t *)calloc(n + 1, sizeof(uint64_t));
    it_t **rows = (it_t **)calloc(H, sizeof(it_t *));
    uint64_t *row_n = (uint64_t *)calloc(H, sizeof(uint64_t));
    int bad = 0;
#pragma omp parallel for schedule(dynamic, 4)
    for (uint32_t y = 0; y < H; ++y) {
        uint32_t *px = (uint32_t *)malloc(W * 4), *py = (uint32_t *)malloc(W * 4);
        for (uint32_t x = 0; x < W; ++x) px[x] = x, py[x] = y;
        uint64_t cap = (uint64_t)W * 64;
        uint8_t *buf = NULL;
        uint32_t *nodes = NULL;
        uint64_t *off = (uint64_t *)malloc((W + 1) * 8), *noff = (uint64_t *)malloc((W + 1) * 8);
        int64_t used;
        for (;;) {
            buf = (uint8_t *)realloc(buf, cap);
            nodes = (uint32_t *)realloc(nodes, cap * 4);
            used = vhx_oracle_ray_events_nodes(t, cam, px, py, W, buf, cap, off, nodes, cap, noff);
            if (used >= 0) break;
            cap *= 4;
        }
        /* count iterations */
        uint64_t nit = 0;
        for (int64_t i = 0; i < used; ++i) nit += buf[i] == 'N';
        it_t *its = (it_t *)calloc(nit ? nit : 1, sizeof(it_t));
        uint64_t k = 0;
        for (uint32_t x = 0; x < W; ++x) {
            uint64_t cnt = 0;
            it_t *cur = NULL;
            for (uint64_t i = off[x]; i < off[x + 1]; ++i) {
                const uint8_t ch = buf[i];
                if (ch == 'N') {
                    cur = &its[k];
                    cur->node = nodes[noff[x] + cnt];
                    ++k;
                    ++cnt;
                } else if (cur) {
                    switch (ch) {
                        case 'P': cur->probe = 1; break;
                        case 'B': cur->nb = (uint8_t)(cur->nb < 255 ? cur->nb + 1 : 255); break;
                        case 'O': cur->pop = 1; break;
                        case 'U': cur->push = 1; break;
                        case 'A': cur->na = (uint8_t)(cur->na < 255 ? cur->na + 1 : 255); break;
                        case 'R': cur->restart = 1; break;
                    }
                }
            }
            g_off[(uint64_t)y * W + x] = cnt;  /* count for now */
        }
        if (k != nit) bad = 1;
        rows[y] = its;
        row_n[y] = nit;
        free(px), free(py), free(buf), free(off), free(nodes), free(noff);
    }
    if (bad) return -1;
    uint64_t total = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t c = g_off[i];
        g_off[i] = total;
        total += c;
    }
    g_off[n] = total;
    g_its = (it_t *)malloc(total * sizeof(it_t) + 1);
    uint64_t at = 0;
    for (uint32_t y = 0; y < H; ++y) {
        memcpy(g_its + at, rows[y], row_n[y] * sizeof(it_t));
        at += row_n[y];
        free(rows[y]);
    }
    free(rows), free(row_n);
    return (int64_t)total;
}

/* blocks (as the VHX_PROF build): 0 iteration, 1 leaf target (probe), 2 brick trip, 3 pop, 4 push, 5 walk setup,
 * 6 advance trip, 7 restart, 13 iteration-end bookkeeping, 14 carried walk (design 1), 16 regroup exchange (6, 7) */
#define NB 17
#define NP 8 /* passes */
typedef struct {
    uint64_t waves[NP][NB], lanes[NP][NB];
    uint64_t rays_in[NP], waves_pass[NP];
    double max_wave[NP]; /* the costliest wave of each pass (cost units: the instructions of cfg.cost per block) */
} stats_t;

typedef struct {
    uint32_t budgets[NP]; /* budget of pass p (p < npass - 1); the last pass is unbounded */
    uint32_t npass;
    uint32_t sparse0;    /* pass-0 sparse-wave threshold */
    uint32_t design, cap;
    uint32_t rpw[NP];    /* rays per wave of queue pass p (0 = 64) */
    uint32_t cost[NB];   /* instructions per wave execution of each block */
    uint32_t order;      /* queue order of the queue passes: 0 frame rows, 1 64x64 tiles Morton inside ("64z"), 2 bucketed
                            by the ray's total steps (perfect prediction, sqrt(2) buckets, longest first), 64z inside */
    uint32_t nwaves;     /* design 3 / 4: persistent waves of a refill pass */
    uint32_t seg;        /* order 5: the 64z queue sorted by (node, position) inside segments of `seg` entries */
} cfg_t;

typedef struct {
    uint32_t ray;  /* pixel index */
    uint32_t cur;  /* next iteration index */
    uint32_t iters;
    uint32_t carry; /* design 1: brick steps still to walk of the current iteration */
} lane_t;

static const cfg_t *g_cfg;
static double g_wave_cost; /* cost of the wave being simulated */
static void add(stats_t *s, int p, int b, uint32_t lanes) {
    s->waves[p][b] += 1;
    s->lanes[p][b] += lanes;
    g_wave_cost += g_cfg->cost[b];
}

/* one wave of a pass; abandoned rays are appended to `out` (in lane order) */
static void sim_wave(const cfg_t *c, int p, lane_t *L, int n, uint32_t budget, uint32_t sparse, stats_t *s,
                     lane_t *out, uint64_t *nout) {
    int done[64] = {0};
    for (;;) {
        int act[64], na = 0;
        for (int i = 0; i < n; ++i)
            if (!done[i]) act[na++] = i;
        if (!na) break;
        add(s, p, 13, na);  /* a trip of the wave's loop */
        /* this iteration's records */
        const it_t *r[64];
        uint32_t mb = 0, ma = 0, npr = 0, npop = 0, npush = 0, nws = 0, nres = 0, nb_now[64];
        int fresh[64];
        for (int a = 0; a < na; ++a) {
            lane_t *l = &L[act[a]];
            r[a] = &g_its[g_off[l->ray] + l->cur];
            fresh[a] = l->carry == 0;
            uint32_t nbw = fresh[a] ? r[a]->nb : l->carry;
            if (c->design == 1 && nbw > c->cap) nbw = c->cap;
            nb_now[a] = nbw;
            if (nbw > mb) mb = nbw;
        }
        /* node iteration top (loads, decode): fresh lanes; probe block: fresh lanes with a probe */
        uint32_t nfresh = 0;
        for (int a = 0; a < na; ++a) nfresh += fresh[a];
        if (nfresh) add(s, p, 0, nfresh);
        for (int a = 0; a < na; ++a) npr += fresh[a] && r[a]->probe;
        if (npr) add(s, p, 1, npr);
        if (c->design == 5) {
            /* merged walk: pop / push / walk setup before one walk loop in which a lane walks its brick and then (a
               miss) its node-level walk: trips = max over lanes of brick steps + node steps, plus a transition block
               (block 15) in every trip where some lane switches from its brick to its node walk */
            uint32_t npop5 = 0, npush5 = 0, nws5 = 0, nres5 = 0, mt = 0, tr[64], tot[64];
            for (int a = 0; a < na; ++a) {
                npop5 += r[a]->pop;
                npush5 += r[a]->push;
                if (r[a]->pop || r[a]->na) ++nws5;
                nres5 += r[a]->restart;
                const uint32_t w = r[a]->pop ? 1u : r[a]->na;
                tr[a] = w ? r[a]->nb : 0xFFFFFFFFu;  /* the trip at which the lane switches (none: no node walk) */
                tot[a] = r[a]->nb + w;
                if (tot[a] > mt) mt = tot[a];
            }
            if (npop5) add(s, p, 3, npop5);
            if (npush5) add(s, p, 4, npush5);
            if (nws5) add(s, p, 5, nws5);
            for (uint32_t t = 0; t < mt; ++t) {
                uint32_t k = 0, sw = 0;
                for (int a = 0; a < na; ++a) {
                    k += tot[a] > t;
                    sw += tr[a] == t;
                }
                if (sw) add(s, p, 15, sw);
                add(s, p, 2, k);
            }
            if (nres5) add(s, p, 7, nres5);
            uint32_t still5 = 0;
            for (int a = 0; a < na; ++a) {
                lane_t *l = &L[act[a]];
                l->iters += r[a]->nb + r[a]->na;
                l->cur += 1;
                const uint32_t nit = (uint32_t)(g_off[l->ray + 1] - g_off[l->ray]);
                if (l->cur >= nit) {
                    done[act[a]] = 1;
                    continue;
                }
                l->iters += 1;
                if (l->iters > budget) {
                    done[act[a]] = 1;
                    out[(*nout)++] = *l;
                    continue;
                }
                ++still5;
            }
            if (sparse && still5 && still5 < sparse) {
                for (int i = 0; i < n; ++i)
                    if (!done[i]) {
                        done[i] = 1;
                        out[(*nout)++] = L[i];
                    }
            }
            continue;
        }
        for (uint32_t t = 0; t < mb; ++t) {
            uint32_t k = 0;
            for (int a = 0; a < na; ++a) k += nb_now[a] > t;
            add(s, p, 2, k);
        }
        /* lanes that finish their brick walk this iteration go on with the rest of the iteration */
        int cont[64];
        for (int a = 0; a < na; ++a) {
            lane_t *l = &L[act[a]];
            const uint32_t left = (fresh[a] ? r[a]->nb : l->carry) - nb_now[a];
            cont[a] = left == 0;
            l->carry = left;
        }
        for (int a = 0; a < na; ++a) {
            if (!cont[a]) continue;
            npop += r[a]->pop;
            npush += r[a]->push;
            const uint32_t w = r[a]->pop ? 1u : r[a]->na;
            if (r[a]->pop || r[a]->na) ++nws;
            if (w > ma) ma = w;
            nres += r[a]->restart;
        }
        if (npop) add(s, p, 3, npop);
        if (npush) add(s, p, 4, npush);
        if (nws) add(s, p, 5, nws);
        for (uint32_t t = 0; t < ma; ++t) {
            uint32_t k = 0;
            for (int a = 0; a < na; ++a) k += cont[a] && (r[a]->pop ? 1u : r[a]->na) > t;
            add(s, p, 6, k);
        }
        if (nres) add(s, p, 7, nres);
        /* end of iteration: finished, abandoned at the budget, or on */
        uint32_t still = 0;
        for (int a = 0; a < na; ++a) {
            lane_t *l = &L[act[a]];
            if (!cont[a]) {  /* carried walk: the budget is checked when the iteration completes */
                l->iters += nb_now[a];
                ++still;
                continue;
            }
            l->iters += nb_now[a] + r[a]->na;
            l->cur += 1;
            const uint32_t nit = (uint32_t)(g_off[l->ray + 1] - g_off[l->ray]);
            if (l->cur >= nit) {
                done[act[a]] = 1;
                continue;
            }
            l->iters += 1;  /* the next node iteration */
            if (l->iters > budget) {
                done[act[a]] = 1;
                out[(*nout)++] = *l;
                continue;
            }
            ++still;
        }
        if (sparse && still && still < sparse) {
            for (int i = 0; i < n; ++i)
                if (!done[i]) {
                    done[i] = 1;
                    out[(*nout)++] = L[i];
                }
        }
    }
}

/* designs 6 / 7 (workgroup regroup): the 4 waves of a workgroup (pass 0: the 4 waves of a 16x16
 * block; queue passes: 4 consecutive chunks) run each node iteration in lockstep (a barrier per iteration). The node
 * blocks run per wave as in design 0; the brick walks (design 6), or the brick and the ADVANCE walks (design 7), of
 * every lane of the 4 waves that needs one are compacted through LDS into ceil(k / 64) full waves (in wave-major lane
 * order, as a prefix-sum compaction gives them), walked there, and the results handed back: block 16 is that exchange,
 * charged once per source wave with a walker and once per packed wave (write + read of the walk state and result). */
static void walk_blocks(const cfg_t *c, int p, int blk, const uint32_t *len, int nk, int packed, stats_t *s) {
    (void)c;
    for (int i = 0; i < nk; i += 64) {
        const int e = nk - i < 64 ? nk - i : 64;
        uint32_t mx = 0;
        for (int j = i; j < i + e; ++j)
            if (len[j] > mx) mx = len[j];
        for (uint32_t t = 0; t < mx; ++t) {
            uint32_t k = 0;
            for (int j = i; j < i + e; ++j) k += len[j] > t;
            add(s, p, blk, k);
        }
        if (packed) add(s, p, 16, (uint32_t)e);
    }
}
static void sim_group(const cfg_t *c, int p, lane_t *const *Lw, const int *nw, int G, uint32_t budget, uint32_t sparse,
                      stats_t *s, lane_t *out, uint64_t *nout) {
    int done[4][64];
    memset(done, 0, sizeof(done));
    for (;;) {
        int any = 0;
        uint32_t blen[256], alen[256];
        int nbk = 0, nak = 0;
        const it_t *rr[4][64];
        int actv[4][64], nav[4];
        for (int w = 0; w < G; ++w) {
            nav[w] = 0;
            for (int i = 0; i < nw[w]; ++i)
                if (!done[w][i]) actv[w][nav[w]++] = i;
            if (!nav[w]) continue;
            any = 1;
            const int na = nav[w];
            add(s, p, 13, na);
            add(s, p, 0, na);
            uint32_t npr = 0, wb = 0;
            for (int a = 0; a < na; ++a) {
                const lane_t *l = &Lw[w][actv[w][a]];
                rr[w][a] = &g_its[g_off[l->ray] + l->cur];
                npr += rr[w][a]->probe;
                if (rr[w][a]->nb) {
                    blen[nbk++] = rr[w][a]->nb;
                    ++wb;
                }
            }
            if (npr) add(s, p, 1, npr);
            if (wb && c->design >= 6) add(s, p, 16, wb);  /* the source wave's exchange */
            if (c->design < 6) walk_blocks(c, p, 2, blen + nbk - wb, (int)wb, 0, s);
        }
        if (!any) break;
        if (c->design >= 6) walk_blocks(c, p, 2, blen, nbk, 1, s);
        for (int w = 0; w < G; ++w) {
            const int na = nav[w];
            if (!na) continue;
            uint32_t npop = 0, npush = 0, nws = 0, nres = 0, wa = 0;
            for (int a = 0; a < na; ++a) {
                const it_t *r = rr[w][a];
                npop += r->pop, npush += r->push, nres += r->restart;
                const uint32_t k = r->pop ? 1u : r->na;
                if (r->pop || r->na) ++nws;
                if (k) {
                    alen[nak++] = k;
                    ++wa;
                }
            }
            if (npop) add(s, p, 3, npop);
            if (npush) add(s, p, 4, npush);
            if (nws) add(s, p, 5, nws);
            if (wa && c->design >= 7) add(s, p, 16, wa);
            if (c->design < 7) walk_blocks(c, p, 6, alen + nak - wa, (int)wa, 0, s);
            if (nres) add(s, p, 7, nres);
        }
        if (c->design >= 7) walk_blocks(c, p, 6, alen, nak, 1, s);
        for (int w = 0; w < G; ++w) {
            uint32_t still = 0;
            for (int a = 0; a < nav[w]; ++a) {
                const int i = actv[w][a];
                lane_t *l = &Lw[w][i];
                const it_t *r = rr[w][a];
                l->iters += r->nb + r->na;
                l->cur += 1;
                const uint32_t nit = (uint32_t)(g_off[l->ray + 1] - g_off[l->ray]);
                if (l->cur >= nit) { done[w][i] = 1; continue; }
                l->iters += 1;
                if (l->iters > budget) { done[w][i] = 1; out[(*nout)++] = *l; continue; }
                ++still;
            }
            if (sparse && still && still < sparse)
                for (int i = 0; i < nw[w]; ++i)
                    if (!done[w][i]) { done[w][i] = 1; out[(*nout)++] = Lw[w][i]; }
        }
    }
}

/* design 2 (vote-aligned phases): a lane is at PRE (next: top + probe setup of iteration cur), WALK (brick steps
 * pending) or POST (the rest of iteration cur: pop / push / walk setup / advance / end). A wave trip runs an N-phase
 * (POST lanes do their post and go on with the next iteration's pre; PRE lanes do their pre) and/or a W-phase (WALK
 * lanes walk to the end of their bricks), each only when enough lanes need it (kn, kw) or nothing else is pending. */
enum { ST_PRE = 0, ST_WALK = 1, ST_POST = 2 };
static void sim_wave2(const cfg_t *c, int p, lane_t *L, int n, uint32_t budget, uint32_t sparse, stats_t *s,
                      lane_t *out, uint64_t *nout) {
    int done[64] = {0}, st[64];
    for (int i = 0; i < n; ++i) st[i] = ST_PRE;
    const uint32_t kn = c->cap & 0xFF, kw = c->cap >> 8;
    for (;;) {
        uint32_t nN = 0, nW = 0, nact = 0;
        for (int i = 0; i < n; ++i)
            if (!done[i]) {
                ++nact;
                if (st[i] == ST_WALK) ++nW; else ++nN;
            }
        if (!nact) break;
        add(s, p, 13, nact);
        int doN = nN && (nN >= kn || nW == 0), doW = nW && (nW >= kw || nN == 0);
        if (!doN && !doW) doN = doW = 1;
        if (doN) {
            /* post stage */
            uint32_t npost = 0, npop = 0, npush = 0, nws = 0, nres = 0, ma = 0;
            for (int i = 0; i < n; ++i) {
                if (done[i] || st[i] != ST_POST) continue;
                const it_t *r = &g_its[g_off[L[i].ray] + L[i].cur];
                ++npost;
                npop += r->pop, npush += r->push, nres += r->restart;
                const uint32_t w = r->pop ? 1u : r->na;
                if (r->pop || r->na) ++nws;
                if (w > ma) ma = w;
            }
            if (npost) add(s, p, 8, npost);
            if (npop) add(s, p, 3, npop);
            if (npush) add(s, p, 4, npush);
            if (nws) add(s, p, 5, nws);
            for (uint32_t t = 0; t < ma; ++t) {
                uint32_t k = 0;
                for (int i = 0; i < n; ++i) {
                    if (done[i] || st[i] != ST_POST) continue;
                    const it_t *r = &g_its[g_off[L[i].ray] + L[i].cur];
                    k += (r->pop ? 1u : r->na) > t;
                }
                add(s, p, 6, k);
            }
            if (nres) add(s, p, 7, nres);
            /* end of iteration for the POST lanes: done, abandoned, or on to the next iteration's pre */
            uint32_t still = 0;
            for (int i = 0; i < n; ++i) {
                if (done[i] || st[i] != ST_POST) continue;
                const it_t *r = &g_its[g_off[L[i].ray] + L[i].cur];
                L[i].iters += r->nb + r->na;
                L[i].cur += 1;
                const uint32_t nit = (uint32_t)(g_off[L[i].ray + 1] - g_off[L[i].ray]);
                if (L[i].cur >= nit) { done[i] = 1; continue; }
                L[i].iters += 1;
                if (L[i].iters > budget) { done[i] = 1; out[(*nout)++] = L[i]; continue; }
                st[i] = ST_PRE;
                ++still;
            }
            (void)still;
            /* pre stage */
            uint32_t npre = 0, npr = 0;
            for (int i = 0; i < n; ++i) {
                if (done[i] || st[i] != ST_PRE) continue;
                const it_t *r = &g_its[g_off[L[i].ray] + L[i].cur];
                ++npre;
                npr += r->probe;
                if (r->nb) { st[i] = ST_WALK; L[i].carry = r->nb; }
                else if (r->probe && (uint32_t)(g_off[L[i].ray + 1] - g_off[L[i].ray]) == L[i].cur + 1 && !r->pop &&
                         !r->na && !r->push) { done[i] = 1; }  /* hit at the entry cell: the ray ends */
                else st[i] = ST_POST;
            }
            if (npre) add(s, p, 0, npre);
            if (npr) add(s, p, 1, npr);
        }
        if (doW) {
            uint32_t mb = 0;
            for (int i = 0; i < n; ++i)
                if (!done[i] && st[i] == ST_WALK && L[i].carry > mb) mb = L[i].carry;
            for (uint32_t t = 0; t < mb; ++t) {
                uint32_t k = 0;
                for (int i = 0; i < n; ++i) k += !done[i] && st[i] == ST_WALK && L[i].carry > t;
                add(s, p, 2, k);
            }
            for (int i = 0; i < n; ++i) {
                if (done[i] || st[i] != ST_WALK) continue;
                L[i].carry = 0;
                const it_t *r = &g_its[g_off[L[i].ray] + L[i].cur];
                const uint32_t nit = (uint32_t)(g_off[L[i].ray + 1] - g_off[L[i].ray]);
                /* a walk that ends the ray (hit) with nothing after it in the iteration */
                if (L[i].cur + 1 == nit && !r->pop && !r->na && !r->push && !r->restart) { done[i] = 1; continue; }
                st[i] = ST_POST;
            }
        }
        if (sparse) {
            uint32_t left = 0;
            for (int i = 0; i < n; ++i) left += !done[i];
            if (left && left < sparse)
                for (int i = 0; i < n; ++i)
                    if (!done[i]) { done[i] = 1; out[(*nout)++] = L[i]; }
        }
    }
}

/* design 3 (lane refill, persistent waves): a queue pass runs `nw` waves round-robin, one node iteration per turn;
 * a wave whose empty lanes number at least `refill` (or that holds no ray) takes that many rays from the shared
 * queue (block 9, one execution per refill, its lanes the rays taken) and goes on; a ray over the pass budget is
 * abandoned to the next pass, a finished ray frees its lane. Block 14: the per-iteration refill check. */
static uint64_t g_qpos;
static void sim_refill_pass(const cfg_t *c, int p, lane_t *q, uint64_t nq, uint32_t budget, uint32_t nw,
                            uint32_t refill, stats_t *s, lane_t *out, uint64_t *nout) {
    lane_t *L = (lane_t *)malloc((size_t)nw * 64 * sizeof(lane_t));
    uint8_t *has = (uint8_t *)calloc((size_t)nw * 64, 1);
    double *cost = (double *)calloc(nw, sizeof(double));
    uint32_t *busy = (uint32_t *)calloc(nw, sizeof(uint32_t));
    g_qpos = 0;
    uint32_t live = nw;
    uint8_t *gone = (uint8_t *)calloc(nw, 1);
    while (live) {
        for (uint32_t w = 0; w < nw; ++w) {
            if (gone[w]) continue;
            lane_t *W = L + (size_t)w * 64;
            uint8_t *H = has + (size_t)w * 64;
            const uint32_t empty = 64 - busy[w];
            if (g_qpos < nq && (empty >= refill || busy[w] == 0)) {
                uint32_t k = 0;
                for (int i = 0; i < 64 && g_qpos < nq; ++i)
                    if (!H[i]) {
                        W[i] = q[g_qpos++];
                        W[i].carry = 0;
                        H[i] = 1;
                        ++k;
                    }
                busy[w] += k;
                s->rays_in[p] += k;
                s->waves[p][9] += 1;
                s->lanes[p][9] += k;
                cost[w] += c->cost[9];
            }
            if (busy[w] == 0) {
                gone[w] = 1;
                --live;
                continue;
            }
            /* one node iteration of the wave's rays (design 0 blocks) */
            g_wave_cost = 0;
            s->waves[p][14] += 1;
            s->lanes[p][14] += busy[w];
            g_wave_cost += c->cost[14];
            int act[64], na = 0;
            for (int i = 0; i < 64; ++i)
                if (H[i]) act[na++] = i;
            add(s, p, 13, na);
            const it_t *r[64];
            uint32_t mb = 0, ma = 0, npr = 0, npop = 0, npush = 0, nws = 0, nres = 0;
            for (int a = 0; a < na; ++a) {
                r[a] = &g_its[g_off[W[act[a]].ray] + W[act[a]].cur];
                if (r[a]->nb > mb) mb = r[a]->nb;
                npr += r[a]->probe;
                npop += r[a]->pop;
                npush += r[a]->push;
                const uint32_t wk = r[a]->pop ? 1u : r[a]->na;
                if (r[a]->pop || r[a]->na) ++nws;
                if (wk > ma) ma = wk;
                nres += r[a]->restart;
            }
            add(s, p, 0, na);
            if (npr) add(s, p, 1, npr);
            for (uint32_t t = 0; t < mb; ++t) {
                uint32_t k = 0;
                for (int a = 0; a < na; ++a) k += r[a]->nb > t;
                add(s, p, 2, k);
            }
            if (npop) add(s, p, 3, npop);
            if (npush) add(s, p, 4, npush);
            if (nws) add(s, p, 5, nws);
            for (uint32_t t = 0; t < ma; ++t) {
                uint32_t k = 0;
                for (int a = 0; a < na; ++a) k += (r[a]->pop ? 1u : r[a]->na) > t;
                add(s, p, 6, k);
            }
            if (nres) add(s, p, 7, nres);
            for (int a = 0; a < na; ++a) {
                lane_t *l = &W[act[a]];
                l->iters += r[a]->nb + r[a]->na;
                l->cur += 1;
                const uint32_t nit = (uint32_t)(g_off[l->ray + 1] - g_off[l->ray]);
                if (l->cur >= nit) {
                    H[act[a]] = 0;
                    --busy[w];
                    continue;
                }
                l->iters += 1;
                if (l->iters > budget) {
                    H[act[a]] = 0;
                    --busy[w];
                    out[(*nout)++] = *l;
                }
            }
            cost[w] += g_wave_cost;
        }
    }
    double mx = 0;
    for (uint32_t w = 0; w < nw; ++w)
        if (cost[w] > mx) mx = cost[w];
    if (mx > s->max_wave[p]) s->max_wave[p] = mx;
    s->waves_pass[p] += nw;
    free(L), free(has), free(cost), free(busy), free(gone);
}

static uint32_t g_order;
static uint32_t spread_bits(uint32_t v) {
    v &= 0xFFFF;
    v = (v | (v << 8)) & 0x00FF00FF;
    v = (v | (v << 4)) & 0x0F0F0F0F;
    v = (v | (v << 2)) & 0x33333333;
    return (v | (v << 1)) & 0x55555555;
}
static uint64_t steps_of(uint32_t ray) {
    uint64_t st = 0;
    for (uint64_t i = g_off[ray]; i < g_off[ray + 1]; ++i) st += 1u + g_its[i].nb + g_its[i].na;
    return st;
}
static uint64_t order_key(uint32_t ray) {
    if (g_order == 0) return ray;
    const uint32_t x = ray % g_W, y = ray / g_W, tx = (g_W + 63) / 64;
    const uint64_t tile = (uint64_t)(y / 64) * tx + x / 64;
    const uint64_t pos = (tile << 12) | (spread_bits(x & 63) | (spread_bits(y & 63) << 1));
    if (g_order == 1) return pos;
    const uint64_t st = steps_of(ray);
    uint32_t b = 0;  /* sqrt(2) buckets: b = floor(2 log2(steps)) */
    while (b < 63 && (1ull << ((b + 1) / 2)) * ((b + 1) % 2 ? 181ull : 128ull) / 128ull <= st) ++b;
    return ((uint64_t)(63 - b) << 40) | pos;
}
static uint32_t g_mode;
static int cmp_ray(const void *a, const void *b) {
    const lane_t *la = (const lane_t *)a, *lb = (const lane_t *)b;
    uint64_t x, y;
    if (g_mode == 3 || g_mode == 4 || g_mode == 5) {
        g_order = 1;
        const uint64_t pa = order_key(la->ray), pb = order_key(lb->ray);
        g_order = g_mode;
        const uint64_t na = g_its[g_off[la->ray] + la->cur].node, nb = g_its[g_off[lb->ray] + lb->cur].node;
        if (g_mode == 3 || g_mode == 5) {
            x = (na << 40) | pa;
            y = (nb << 40) | pb;
        } else {  /* tile (pos >> 12), node, Morton inside */
            x = ((pa >> 12) << 44) | (na << 12) | (pa & 4095);
            y = ((pb >> 12) << 44) | (nb << 12) | (pb & 4095);
        }
    } else {
        x = order_key(la->ray);
        y = order_key(lb->ray);
    }
    return x < y ? -1 : x > y;
}

int wavesim_run(const cfg_t *c, stats_t *s) {
    memset(s, 0, sizeof(*s));
    g_cfg = c;
    g_order = c->order;
    g_mode = c->order;
    const uint32_t W = g_W, H = g_H;
    const uint64_t n = (uint64_t)W * H;
    lane_t *q = (lane_t *)malloc(n * sizeof(lane_t)), *q2 = (lane_t *)malloc(n * sizeof(lane_t));
    uint64_t nq = 0;
    /* pass 0: 8x8-pixel waves (four per 16x16 workgroup, blocks in raster order) */
    const uint32_t bx = (W + 15) / 16, by = (H + 15) / 16;
    const uint32_t b0 = c->npass > 1 ? c->budgets[0] : VHX_MAX_ITERS_SIM;
    if (c->design == 4) { /* pass 0 as a refill pass over the pixels in wave-tile order */
        uint64_t np = 0;
        for (uint32_t b = 0; b < bx * by; ++b)
            for (uint32_t w = 0; w < 4; ++w)
                for (uint32_t k = 0; k < 64; ++k) {
                    const uint32_t x = (b % bx) * 16 + (w & 1) * 8 + (k & 7), y = (b / bx) * 16 + (w >> 1) * 8 + (k >> 3);
                    if (x >= W || y >= H) continue;
                    const uint32_t ray = y * W + x;
                    if (g_off[ray + 1] == g_off[ray]) continue;
                    q2[np].ray = ray, q2[np].cur = 0, q2[np].iters = 1, q2[np].carry = 0;
                    ++np;
                }
        sim_refill_pass(c, 0, q2, np, b0, c->nwaves, c->cap, s, q, &nq);
    } else if (c->design >= 6) {
        for (uint32_t b = 0; b < bx * by; ++b) {
            lane_t L4[4][64];
            lane_t *Lw[4] = {L4[0], L4[1], L4[2], L4[3]};
            int nw[4] = {0, 0, 0, 0};
            for (uint32_t w = 0; w < 4; ++w) {
                for (uint32_t k = 0; k < 64; ++k) {
                    const uint32_t x = (b % bx) * 16 + (w & 1) * 8 + (k & 7), y = (b / bx) * 16 + (w >> 1) * 8 + (k >> 3);
                    if (x >= W || y >= H) continue;
                    const uint32_t ray = y * W + x;
                    s->rays_in[0] += 1;
                    if (g_off[ray + 1] == g_off[ray]) continue;
                    lane_t *l = &L4[w][nw[w]++];
                    l->ray = ray, l->cur = 0, l->iters = 1, l->carry = 0;
                }
                s->waves_pass[0] += 1;
            }
            sim_group(c, 0, Lw, nw, 4, b0, c->npass > 1 ? c->sparse0 : 0, s, q, &nq);
        }
    } else
    for (uint32_t b = 0; b < bx * by; ++b)
        for (uint32_t w = 0; w < 4; ++w) {
            lane_t L[64];
            int nl = 0;
            for (uint32_t k = 0; k < 64; ++k) {
                const uint32_t x = (b % bx) * 16 + (w & 1) * 8 + (k & 7), y = (b / bx) * 16 + (w >> 1) * 8 + (k >> 3);
                if (x >= W || y >= H) continue;
                const uint32_t ray = y * W + x;
                s->rays_in[0] += 1;
                if (g_off[ray + 1] == g_off[ray]) continue; /* misses the root: no iteration */
                L[nl].ray = ray, L[nl].cur = 0, L[nl].iters = 1, L[nl].carry = 0;
                ++nl;
            }
            s->waves_pass[0] += 1;
            g_wave_cost = 0;
            if (nl) (c->design == 2 ? sim_wave2 : sim_wave)(c, 0, L, nl, b0, c->npass > 1 ? c->sparse0 : 0, s, q, &nq);
            if (g_wave_cost > s->max_wave[0]) s->max_wave[0] = g_wave_cost;
        }
    for (uint32_t p = 1; p < c->npass; ++p) {
        if (c->order == 5) { /* 64z order, then each segment of c->seg entries by (node, position) */
            g_mode = 1;
            g_order = 1;
            qsort(q, nq, sizeof(lane_t), cmp_ray);
            g_mode = 5;
            for (uint64_t i = 0; i < nq; i += c->seg)
                qsort(q + i, nq - i < c->seg ? nq - i : c->seg, sizeof(lane_t), cmp_ray);
        } else
        qsort(q, nq, sizeof(lane_t), cmp_ray); /* frame order (pass 1: flag compaction; later: chunk order) */
        const int last = p + 1 >= c->npass;
        const uint32_t budget = last ? VHX_MAX_ITERS_SIM : c->budgets[p];
        const int slot = (int)p;
        const uint32_t rpw = c->rpw[p] ? c->rpw[p] : 64u;
        uint64_t nq2 = 0;
        if (c->design >= 3 && c->design < 6) {
            sim_refill_pass(c, slot, q, nq, budget, c->nwaves, c->cap, s, q2, &nq2);
            lane_t *t = q;
            q = q2;
            q2 = t;
            nq = nq2;
            continue;
        }
        s->rays_in[slot] += nq;
        if (c->design >= 6) {
            for (uint64_t i = 0; i < nq; i += 4 * (uint64_t)rpw) {
                lane_t *Lw[4];
                int nw[4] = {0, 0, 0, 0}, G = 0;
                for (int w = 0; w < 4 && i + (uint64_t)w * rpw < nq; ++w) {
                    const uint64_t o = i + (uint64_t)w * rpw;
                    Lw[w] = q + o;
                    nw[w] = (int)(nq - o < rpw ? nq - o : rpw);
                    s->waves_pass[slot] += 1;
                    G = w + 1;
                }
                sim_group(c, slot, Lw, nw, G, budget, 0, s, q2, &nq2);
            }
            lane_t *t = q;
            q = q2;
            q2 = t;
            nq = nq2;
            continue;
        }
        for (uint64_t i = 0; i < nq; i += rpw) {
            const int nl = (int)(nq - i < rpw ? nq - i : rpw);
            s->waves_pass[slot] += 1;
            g_wave_cost = 0;
            (c->design == 2 ? sim_wave2 : sim_wave)(c, slot, q + i, nl, budget, 0, s, q2, &nq2);
            if (g_wave_cost > s->max_wave[slot]) s->max_wave[slot] = g_wave_cost;
        }
        lane_t *t = q;
        q = q2;
        q2 = t;
        nq = nq2;
    }
    free(q), free(q2);
    return 0;
}
