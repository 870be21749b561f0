"""Diagnostic (PMC runs): one configuration of probe_spread.py -- k copies of the bench frame's longest ray (or the k
longest distinct rays), one real ray every `gap` lanes, single-pass launches, 3 repetitions.
usage: probe_cfg.py PIXELS.npz GAP K [dup|distinct]"""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import voxelhex_amd as vhx
from voxelhex_amd import _native as N

z = np.load(sys.argv[1])
gap, k = int(sys.argv[2]), int(sys.argv[3])
mode = sys.argv[4] if len(sys.argv) > 4 else "dup"
W, H = 3840, 2160
flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 1024, 4)
rt = vhx.Raytracer(0)
rt.upload(flat)
cam = vhx.glass_camera(1024, W, H, target=(512.0, 512.0, 512.0))
o = np.array(cam.origin, np.float32)
bl, r, u = (np.array(v, np.float32) for v in (cam.glass_bottom_left, cam.glass_right, cam.glass_up))
steps = z["steps"].astype(np.int64)
order = np.argsort(-steps, kind="stable")[:4096]
px = (order % W).astype(np.float32); py = (H - 1 - order // W).astype(np.float32)
gp = bl[None] + (r[None] * px[:, None]) * np.float32(cam.pixel_width) + (u[None] * py[:, None]) * np.float32(cam.pixel_height)
d = gp - o[None]
d = (d / np.sqrt((d * d).sum(1, keepdims=True))).astype(np.float32)
rt.set_pass_budgets(())
n = k * gap
dd = np.repeat(-d[:1], n, 0)
dd[::gap] = d[:k] if mode == "distinct" else np.repeat(d[:1], k, 0)
ts = []
for _ in range(3):
    rt.trace_rays(np.repeat(o[None], n, 0), dd, fields=("value",))
    ts.append(rt.sync())
print(f"gap={gap} k={k} mode={mode} ms={min(ts[1:]):.3f}", flush=True)
