"""Issue-cost simulation of pass 0 with lane refill (diagnostic for DESIGN.md §12): per-ray event sequences from the
oracle, truncated at the pass-0 budget; "cur" = one wave per 8x8 tile (today's k_trace_primary), (T, G) = persistent
waves over G rays in tile order that hand new rays to their idle lanes once T lanes are idle (cost CINIT per refill).
Costs per node iteration follow sim_divergence.py. usage: sim_refill.py [CINIT]"""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "scripts"))
import voxelhex_amd as vhx
from voxelhex_amd import _native as N
from sim_divergence import events, iterations, C
W, H = 3840, 2160
flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 1024, 4)
cam = vhx.glass_camera(1024, W, H, target=(512.0, 512.0, 512.0))
BUD = 64
CINIT = int(sys.argv[1]) if len(sys.argv) > 1 else 300
def trunc(its):
    out = []; it = 0
    for a in its:
        out.append(a); it += 1 + a['B'] + a['A']
        if it > BUD: break
    return out
def it_cost(act):
    c = C['N']
    if any(a['P'] for a in act): c += C['P']
    c += C['B'] * max(a['B'] + a['P'] for a in act) + C['A'] * max(a['A'] for a in act)
    if any(a['O'] for a in act): c += C['O']
    if any(a['R'] for a in act): c += C['R']
    if any(a['U'] for a in act): c += C['U']
    return c
res = {}
for y0 in (1000, 600, 1400):
    rows = range(y0, y0 + 32)
    # 8x8 wave tiles over 32 rows
    waves = []
    for ty in range(y0, y0 + 32, 8):
        for tx in range(0, W, 8):
            waves.append([(ty + j) * W + tx + i for j in range(8) for i in range(8)])
    pix = np.array([p for w in waves for p in w])
    ev = events(flat, cam, pix, W, H)
    its = [trunc(iterations(s)) for s in ev]
    # current: one wave per tile
    cur = 0
    for w in range(len(waves)):
        L = its[w * 64:(w + 1) * 64]
        cur += CINIT
        K = max(len(l) for l in L)
        for k in range(K):
            act = [l[k] for l in L if k < len(l)]
            if act: cur += it_cost(act)
    # refill: persistent waves each taking the pixel stream in tile order; G rays per persistent wave
    for T in (8, 16, 32, 48):
        for G in (64 * 8, 64 * 32):
            ref = 0
            for w0 in range(0, len(its), G):
                queue = list(range(w0, min(w0 + G, len(its))))
                lanes = [None] * 64; pos = [0] * 64
                qi = 0
                # initial fill
                for l in range(64):
                    if qi < len(queue): lanes[l] = queue[qi]; qi += 1
                ref += CINIT
                while any(x is not None for x in lanes):
                    act = []
                    for l in range(64):
                        r = lanes[l]
                        if r is None: continue
                        if pos[l] < len(its[r]): act.append(its[r][pos[l]])
                    if act: ref += it_cost(act)
                    for l in range(64):
                        r = lanes[l]
                        if r is None: continue
                        pos[l] += 1
                        if pos[l] >= len(its[r]): lanes[l] = None
                    free = sum(x is None for x in lanes)
                    if qi < len(queue) and (free >= T or free == 64):
                        for l in range(64):
                            if lanes[l] is None and qi < len(queue):
                                lanes[l] = queue[qi]; pos[l] = 0; qi += 1
                        ref += CINIT + 8  # init cost + ballot/atomic
                    ref += 4  # per-iteration refill test
            res.setdefault((T, G), []).append(ref)
    res.setdefault("cur", []).append(cur)
    print(y0, "cur", cur, {k: v[-1] for k, v in res.items() if k != "cur"}, flush=True)
c = sum(res["cur"])
for k, v in res.items():
    if k != "cur": print(k, f"{sum(v)/c:.3f}")
