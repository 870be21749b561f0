"""Block profile of the traversal (diagnostics): with a VHX_PROF build of libvhx (VHX_LIB=voxelhex_amd/_lib/prof/
libvhx.so), traces the bench frame (scene S 1024^3 bd 4, 3840x2160, glass camera) once per schedule and prints, per
pass and block, the wave executions and the mean active lanes (wave ballot).
    VHX_LIB=voxelhex_amd/_lib/prof/libvhx.so python scripts/probes/probe_blocks.py [--size 1024] [--budgets 24,96,768]
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

BLOCKS = {0: "iteration", 1: "leaf target", 2: "brick walk trip", 3: "pop", 4: "push", 5: "walk setup (!push)",
          6: "advance walk trip", 7: "restart", 8: "parted probe", 9: "cell walk entered", 10: "ray start",
          11: "ray in tree", 12: "ray end"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--bd", type=int, default=4)
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--budgets", default="24,96,768")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    import voxelhex_amd as vhx
    from voxelhex_amd import _native as N
    flat = vhx.FlatTree.build_scene(1, a.size, a.bd, threads=16)
    rt = vhx.Raytracer(0)
    rt.upload(flat)
    rt.set_pass_budgets(tuple(int(b) for b in a.budgets.split(",") if b))
    cam = vhx.glass_camera(a.size, a.width, a.height, target=(a.size / 2,) * 3)
    buf = (ctypes.c_uint64 * 160)()
    rt.trace_primary(cam, fields=("rgba",))  # warm-up
    N.check(N.lib().vhx_profile_counters(rt._h, buf, 160, 1), rt._h)
    rt.trace_primary(cam, fields=("rgba",))
    N.check(N.lib().vhx_profile_counters(rt._h, buf, 160, 1), rt._h)
    out = {}
    for p in range(5):  # pass slots (vhx.h, vhx_profile_counters)
        for b, name in BLOCKS.items():
            n, lanes = buf[2 * (p * 16 + b)], buf[2 * (p * 16 + b) + 1]
            if n:
                out[f"p{p}.{b}"] = {"block": name, "waves": int(n), "lanes": int(lanes), "mean_lanes": round(lanes / n, 2)}
                print(f"pass {p} {b:2d} {name:20s} waves {n:12d} lanes {lanes:14d} mean {lanes / n:6.2f}")
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)
    rt.close()


if __name__ == "__main__":
    main()
