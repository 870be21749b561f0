"""Driver of the wave-level SIMT simulator (scripts/sim/wavesim.c; diagnostics, not product code).

Builds the bench frame's per-ray iteration records from the oracle's event traces and replays the multi-pass schedule
with a loop-structure design, printing per pass and block the wave executions and mean active lanes (the blocks of the
VHX_PROF kernel build, so that design 0 can be compared with scripts/probes/probe_blocks.py on the GPU) and a VALU
estimate from per-block instruction costs (COSTS, read off the gfx950 ISA of k_trace_queue<false, 4>).
    python scripts/sim/wavesim.py [--size 1024] [--designs 0,1:4,1:2] [--budgets 24,96,768]
"""
import argparse
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
LIB = os.path.join(ROOT, "scripts", "sim", "_build", "libwavesim.so")
BLOCKS = {13: "loop trip", 0: "iteration top", 1: "probe", 2: "brick trip", 8: "post", 3: "pop", 4: "push",
          5: "walk setup", 6: "advance trip", 7: "restart", 9: "refill", 14: "refill check", 15: "walk switch",
          16: "regroup exchange"}
# VALU instructions per wave execution of each block (ISA of the bd-4 queue kernel, round 3)
COSTS = {13: 15, 0: 25, 1: 55, 2: 28, 8: 15, 3: 30, 4: 40, 5: 20, 6: 28, 7: 55, 9: 300, 14: 4, 15: 12,
         16: int(os.environ.get("REGROUP_COST", "30"))}  # 16: LDS write + read of a walk's state and result, per wave
RAY_SETUP = 250  # ray generation + begin (divisions, square roots) per pass-0 wave


NP = 8
NB = 17  # blocks (wavesim.c)


class Stats(ctypes.Structure):
    _fields_ = [("waves", (ctypes.c_uint64 * NB) * NP), ("lanes", (ctypes.c_uint64 * NB) * NP),
                ("rays_in", ctypes.c_uint64 * NP), ("waves_pass", ctypes.c_uint64 * NP),
                ("max_wave", ctypes.c_double * NP)]


class Cfg(ctypes.Structure):
    _fields_ = [("budgets", ctypes.c_uint32 * NP), ("npass", ctypes.c_uint32), ("sparse0", ctypes.c_uint32),
                ("design", ctypes.c_uint32), ("cap", ctypes.c_uint32), ("rpw", ctypes.c_uint32 * NP),
                ("cost", ctypes.c_uint32 * NB), ("order", ctypes.c_uint32), ("nwaves", ctypes.c_uint32), ("seg", ctypes.c_uint32)]


def build():
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    subprocess.run(["gcc", "-O2", "-fopenmp", "-shared", "-fPIC", "-Wall", os.path.join(ROOT, "scripts/sim/wavesim.c"),
                    "-o", LIB, "-L", os.path.join(ROOT, "oracle/_build"), "-loracle",
                    "-Wl,-rpath," + os.path.join(ROOT, "oracle/_build")], check=True)
    return ctypes.CDLL(LIB)


def run(lib, budgets, design, cap, sparse0=12, rpw=(), order=0, nwaves=768, seg=1024):
    c = Cfg()
    c.seg = seg
    c.order = order
    c.nwaves = nwaves
    for i, b in enumerate(budgets):
        c.budgets[i] = b
    for i, r in enumerate(rpw):
        c.rpw[i] = r
    for b, v in COSTS.items():
        c.cost[b] = v
    c.npass = len(budgets) + 1
    c.sparse0, c.design, c.cap = sparse0, design, cap
    s = Stats()
    assert lib.wavesim_run(ctypes.byref(c), ctypes.byref(s)) == 0
    return s


def report(s, label):
    tot = 0.0
    print(f"== {label}")
    for p in range(NP):
        if not s.waves_pass[p]:
            continue
        refill = s.waves[p][9] > 0  # a refill pass charges its ray setup per refill (block 9)
        valu = 0 if refill else (RAY_SETUP * s.waves_pass[p] if p == 0 or s.rays_in[p] else 0)
        line = []
        for b, name in BLOCKS.items():
            w, l = s.waves[p][b], s.lanes[p][b]
            if w:
                valu += w * COSTS[b]
                line.append(f"{name} {w} ({l / w:.1f})")
        tot += valu
        print(f"  pass {p}: rays {s.rays_in[p]} waves {s.waves_pass[p]} VALU~{valu / 1e6:.1f}M max-wave {s.max_wave[p] / 1e3:.0f}k"
              f" | " + "; ".join(line))
    print(f"  total VALU~{tot / 1e6:.1f}M")
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--bd", type=int, default=4)
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--budgets", default="24,96,768")
    ap.add_argument("--designs", default="0")
    ap.add_argument("--seg", type=int, default=1024, help="order 5: segment length of the node sort")
    ap.add_argument("--nwaves", type=int, default=768, help="persistent waves of a refill pass (designs 3, 4)")
    ap.add_argument("--orders", default="0", help="queue orders to compare: 0 frame rows, 1 64z tiles, 2 step buckets")
    a = ap.parse_args()
    import time
    import voxelhex_amd as vhx
    lib = build()
    lib.wavesim_build.restype = ctypes.c_int64
    flat = vhx.FlatTree.build_scene(1, a.size, a.bd, threads=8)
    cam = vhx.glass_camera(a.size, a.width, a.height, target=(a.size / 2,) * 3)
    t0 = time.time()
    n = lib.wavesim_build(ctypes.byref(flat.desc), ctypes.byref(cam), a.width, a.height)
    print(f"iteration records: {n} ({time.time() - t0:.1f} s)")
    budgets = tuple(int(b) for b in a.budgets.split(",") if b)
    for d in a.designs.split(","):
        design, _, cap = d.partition(":")
        for o in a.orders.split(","):
            s = run(lib, budgets, int(design), int(cap or 0), order=int(o), nwaves=a.nwaves, seg=a.seg)
            report(s, f"design {d} budgets {budgets} order {o}")


if __name__ == "__main__":
    main()
