"""Diagnostic: device time of the k longest rays (by step count) as k grows, one ray per wave (VHX_RPW=1,
budgets (1,)) and 64 per wave (single pass). Shows whether concurrent single-ray waves slow each other down."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import voxelhex_amd as vhx
from voxelhex_amd import _native as N

z = np.load(sys.argv[1])
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
dup = os.environ.get("DUP") == "1"
if dup:
    d = np.repeat(d[:1], len(d), 0)
for sched in ((1,), ()):
    rt.set_pass_budgets(sched)
    for k in (1, 2, 4, 8, 16, 32, 64, 128, 256, 1024, 4096):
        ts = []
        for _ in range(3):
            rt.trace_rays(np.repeat(o[None], k, 0), d[:k], fields=("value",))
            ts.append(rt.sync())
        print(f"rpw={os.environ.get('VHX_RPW')} dup={dup} sched={sched} k={k:5d} ms={min(ts[1:]):.3f}", flush=True)
