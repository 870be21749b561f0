"""Diagnostic: device time of each of the bench frame's longest rays traced alone (one ray, one wave).
Pixel lists: scratch/tail_pixels.npz (scripts/make_tail_pixels.py). Prints the slowest rays with their step counts."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import voxelhex_amd as vhx
from voxelhex_amd import _native as N

z = np.load(sys.argv[1])
n = int(sys.argv[2]) if len(sys.argv) > 2 else 256
W, H = 3840, 2160
flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 1024, 4)
rt = vhx.Raytracer(0)
rt.upload(flat)
cam = vhx.glass_camera(1024, W, H, target=(512.0, 512.0, 512.0))
o = np.array(cam.origin, np.float32)
bl, r, u = (np.array(v, np.float32) for v in (cam.glass_bottom_left, cam.glass_right, cam.glass_up))
steps = z["steps"].astype(np.int64)
order = np.argsort(-steps, kind="stable")[:n]
px = (order % W).astype(np.float32); py = (H - 1 - order // W).astype(np.float32)
gp = bl[None] + (r[None] * px[:, None]) * np.float32(cam.pixel_width) + (u[None] * py[:, None]) * np.float32(cam.pixel_height)
d = gp - o[None]
d = (d / np.sqrt((d * d).sum(1, keepdims=True))).astype(np.float32)
rt.set_pass_budgets(())
res = []
for i in range(n):
    ts = []
    for _ in range(3):
        rt.trace_rays(o[None], d[i:i + 1], fields=("value",))
        ts.append(rt.sync())
    res.append(min(ts[1:]))
res = np.array(res)
top = np.argsort(-res)[:24]
for k in top:
    print(f"pix={order[k]} steps={steps[order[k]]} ms={res[k]:.3f}")
np.savez("gpurun_out/single_times.npz", pix=order, ms=res)
