"""Diagnostic: k copies of the bench frame's longest ray in one single-pass launch, one real ray every `gap` lanes
(the other lanes hold rays that miss the tree at once). gap 64 = one ray per wave (4 per workgroup), gap 256 = one
per workgroup, gap 1024 = one per 4 workgroups. Separates wave-placement effects from divergence."""
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
rt.set_pass_budgets(())
mode = os.environ.get("MODE", "dup")
for gap in (1, 64, 256, 1024):
    for k in (1, 16, 64, 256, 1024, 4096):
        n = k * gap
        oo = np.repeat(o[None], n, 0)
        dd = np.repeat(-d[:1], n, 0)  # points away from the tree: a miss at the root test
        sel = d[:k] if mode == "distinct" else np.repeat(d[:1], k, 0)
        dd[::gap] = sel
        ts = []
        for _ in range(3):
            rt.trace_rays(oo, dd, fields=("value",))
            ts.append(rt.sync())
        print(f"mode={mode} gap={gap:5d} k={k:5d} ms={min(ts[1:]):.3f}", flush=True)
