"""Diagnostic: trace only the bench frame's longest ray (one wave, single pass) a few times, for PMC counters."""
import sys
import numpy as np
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
import voxelhex_amd as vhx
from voxelhex_amd import _native as N

z = np.load(sys.argv[1])
which = sys.argv[2] if len(sys.argv) > 2 else "longest"
W, H = 3840, 2160
flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 1024, 4)
rt = vhx.Raytracer(0)
rt.upload(flat)
cam = vhx.glass_camera(1024, W, H, target=(512.0, 512.0, 512.0))
o = np.array(cam.origin, np.float32)
bl, r, u = (np.array(v, np.float32) for v in (cam.glass_bottom_left, cam.glass_right, cam.glass_up))
pix = z["top64"][:1] if which == "longest" else z["top64"]
px = (pix % W).astype(np.float32); py = (H - 1 - pix // W).astype(np.float32)
gp = bl[None] + (r[None] * px[:, None]) * np.float32(cam.pixel_width) + (u[None] * py[:, None]) * np.float32(cam.pixel_height)
d = gp - o[None]
d = (d / np.sqrt((d * d).sum(1, keepdims=True))).astype(np.float32)
rt.set_pass_budgets(())
for _ in range(3):
    rt.trace_rays(np.repeat(o[None], len(pix), 0), d, fields=("value",))
    print(which, rt.sync(), flush=True)
