"""Diagnostic: device time of the bench frame's rays > 64 steps traced in different orders (single pass)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
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
rt.set_pass_budgets(())
for name in z.files:
    pix = z[name]
    px = (pix % W).astype(np.float32); py = (H - 1 - pix // W).astype(np.float32)
    gp = bl[None] + (r[None] * px[:, None]) * np.float32(cam.pixel_width) + (u[None] * py[:, None]) * np.float32(cam.pixel_height)
    d = gp - o[None]
    d = (d / np.sqrt((d * d).sum(1, keepdims=True))).astype(np.float32)
    oo = np.repeat(o[None], len(pix), 0)
    ts = []
    for _ in range(4):
        rt.trace_rays(oo, d, fields=("value",))
        ts.append(rt.sync())
    print(f"{name:22s} n={len(pix)} ms={min(ts[1:]):.3f}", flush=True)
