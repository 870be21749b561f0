"""Wave-divergence simulation of traversal loop structures (diagnostics for DESIGN.md §3).

Per-ray event sequences come from the oracle (vhx_oracle_ray_events: N node iteration, P probe, B brick cell step,
O pop, U push, A advance step, R restart). Rays of a wave run in lockstep over node iterations; a loop inside an
iteration costs (max over lanes of its trip count) x (body instructions). Body costs are instruction counts of the
current gfx950 ISA (approximate).

usage: sim_divergence.py PIXELS.npz [key]   (key = array of pixel indices, default t64)
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

C = dict(N=60, P=60, B=55, O=90, U=45, A=58, R=40, BA=66, T=25)


def events(flat, cam, pix, W, H):
    from tests._oracle import ORACLE_LIB
    lib = ctypes.CDLL(ORACLE_LIB)
    f = lib.vhx_oracle_ray_events
    f.restype = ctypes.c_int64
    px = (pix % W).astype(np.uint32)
    py = (pix // W).astype(np.uint32)
    cap = int(len(pix) * 3000)
    buf = np.zeros(cap, np.uint8)
    off = np.zeros(len(pix) + 1, np.uint64)
    u32p = ctypes.POINTER(ctypes.c_uint32)
    n = f(ctypes.byref(flat.desc), ctypes.byref(cam), px.ctypes.data_as(u32p), py.ctypes.data_as(u32p),
          ctypes.c_uint64(len(pix)), buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_uint64(cap),
          off.ctypes.data_as(ctypes.c_void_p))
    assert n >= 0
    return [bytes(buf[off[i]:off[i + 1]]).decode() for i in range(len(pix))]


def iterations(seq):
    """Split a ray's events into node iterations: list of dicts with counts per event kind."""
    its = []
    cur = None
    for ch in seq:
        if ch == 'N':
            cur = dict(P=0, B=0, O=0, U=0, A=0, R=0)
            its.append(cur)
        elif cur is not None:
            cur[ch] += 1
    return its


def wave_cost(lanes, model):
    its = [iterations(s) for s in lanes]
    K = max(len(i) for i in its)
    total = 0
    for k in range(K):
        act = [i[k] for i in its if k < len(i)]
        if not act:
            continue
        c = C['N']
        if any(a['P'] for a in act):
            c += C['P']
        if model == "current":
            c += C['B'] * max(a['B'] + a['P'] for a in act)  # brick trips ~ steps (+ the tested cell)
            c += C['A'] * max(a['A'] for a in act)
        elif model == "merged":
            walk = max(a['B'] + a['P'] + a['A'] for a in act)
            c += C['BA'] * walk + (C['T'] if any(a['A'] and a['P'] for a in act) else 0)
        if any(a['O'] for a in act):
            c += C['O']
        if any(a['R'] for a in act):
            c += C['R']
        if any(a['U'] for a in act):
            c += C['U']
        total += c
    return total


def main():
    import voxelhex_amd as vhx
    from voxelhex_amd import _native as N
    z = np.load(sys.argv[1])
    key = sys.argv[2] if len(sys.argv) > 2 else "t64"
    W, H = 3840, 2160
    flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 1024, 4)
    cam = vhx.glass_camera(1024, W, H, target=(512.0, 512.0, 512.0))
    pix = z[key]
    seqs = events(flat, cam, pix, W, H)
    top = events(flat, cam, z["top64"], W, H)
    for model in ("current", "merged"):
        single = wave_cost(top[:1], model)
        tw = wave_cost(top, model)
        waves = [wave_cost(seqs[i:i + 64], model) for i in range(0, len(seqs), 64)]
        print(f"{model:8s} single {single:8d}  top64-wave {tw:8d} ({tw / single:.2f}x)  "
              f"{key}: max wave {max(waves):8d} ({max(waves) / single:.2f}x), sum {sum(waves) / 1e6:.1f}M")


if __name__ == "__main__":
    main()


def breakdown(lanes):
    """Per-component cost of the current structure for one wave."""
    its = [iterations(s) for s in lanes]
    K = max(len(i) for i in its)
    comp = dict(N=0, P=0, B=0, A=0, O=0, U=0, R=0)
    for k in range(K):
        act = [i[k] for i in its if k < len(i)]
        if not act:
            continue
        comp['N'] += C['N']
        if any(a['P'] for a in act):
            comp['P'] += C['P']
        comp['B'] += C['B'] * max(a['B'] + a['P'] for a in act)
        comp['A'] += C['A'] * max(a['A'] for a in act)
        for kk in "OUR":
            if any(a[kk] for a in act):
                comp[kk] += C[kk]
    return comp, K


def tokens(seq):
    """Per-trip tokens of a one-step-per-trip machine: N+outcome (O/U/R folded into the node trip), P, B, A."""
    out = []
    for ch in seq:
        if ch == 'N':
            out.append(['N'])
        elif ch in "OUR":
            if out and out[-1][0] == 'N':
                out[-1].append(ch)
            else:
                out.append(['N', ch])
        else:
            out.append([ch])
    return out


def ifif_cost(lanes, merge_ba=False):
    toks = [tokens(s) for s in lanes]
    T = max(len(t) for t in toks)
    total = 0
    for k in range(T):
        act = [t[k] for t in toks if k < len(t)]
        kinds = set(a[0] for a in act)
        c = 0
        if 'N' in kinds:
            c += C['N'] + sum(C[x] for x in "OUR" if any(x in a for a in act))
        if 'P' in kinds:
            c += C['P']
        if merge_ba and ('B' in kinds or 'A' in kinds):
            c += C['BA']
        else:
            c += (C['B'] if 'B' in kinds else 0) + (C['A'] if 'A' in kinds else 0)
        total += c
    return total
