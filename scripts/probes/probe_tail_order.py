"""Diagnostic: does ordering the tail rays by a predicted length shorten the tail pass?

The bench frame's rays that exceed the pass-0 budget (steps > 64, from PIXELS.npz) are traced as an explicit ray batch
(pass 0 + one unbounded queue pass, as in the frame) in several orders: frame order (today's queue), bucketed by a
geometric predictor (the ray's path length inside the root cube, 8 linear buckets, longest first, frame order inside
a bucket), and sorted by the true step count (an upper bound). Prints the launch time of each (median of 5).
usage: probe_tail_order.py PIXELS.npz"""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import voxelhex_amd as vhx
from voxelhex_amd import _native as N

W, H, S = 3840, 2160, 1024.0
z = np.load(sys.argv[1])
steps = z["steps"].astype(np.int64)
t = np.nonzero(steps > 64)[0]
flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 1024, 4, threads=16)
rt = vhx.Raytracer(0)
rt.upload(flat)
cam = vhx.glass_camera(1024, W, H, target=(512.0, 512.0, 512.0))
f = np.float32
o = np.array(cam.origin, f)
bl, r, u = (np.array(v, f) for v in (cam.glass_bottom_left, cam.glass_right, cam.glass_up))
px = (t % W).astype(f)
py = (H - 1 - t // W).astype(f)
gp = (bl[None] + (r[None] * px[:, None]) * f(cam.pixel_width)) + (u[None] * py[:, None]) * f(cam.pixel_height)
d = gp - o[None]
d = (d / np.sqrt((d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2])[:, None]).astype(f)
orig = np.repeat(o[None], len(t), 0)
with np.errstate(divide="ignore", invalid="ignore"):
    t1 = (0 - o[None].astype(np.float64)) / d
    t2 = (S - o[None].astype(np.float64)) / d
L = np.min(np.maximum(t1, t2), 1) - np.maximum(np.max(np.minimum(t1, t2), 1), 0)
b = np.minimum(7, (L / S * 8 / 1.74).astype(np.int64))
orders = {"frame": np.arange(len(t)), "bucket8": np.lexsort((np.arange(len(t)), -b)),
          "sorted(oracle)": np.argsort(-steps[t], kind="stable")}
rt.set_pass_budgets((64,))
for name, ordr in orders.items():
    ts = []
    for _ in range(6):
        rt.trace_rays(orig[ordr], d[ordr], fields=("value",))
        ts.append(rt.sync())
    print(f"{name:16s} {len(t)} rays: {np.median(ts[1:]):.3f} ms", flush=True)
