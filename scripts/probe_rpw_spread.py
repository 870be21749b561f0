"""Diagnostic: divergence factor vs rays per wave. The R longest rays of the bench frame (by step count) are packed k
per wave, one real wave per 256-thread workgroup (the other lanes hold rays that miss at the root test), so waves do
not share a CU. Single-pass launches."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import voxelhex_amd as vhx
from voxelhex_amd import _native as N

z = np.load(sys.argv[1])
R = int(sys.argv[2]) if len(sys.argv) > 2 else 256
off = int(sys.argv[3]) if len(sys.argv) > 3 else 0
W, H = 3840, 2160
flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 1024, 4)
rt = vhx.Raytracer(0)
rt.upload(flat)
cam = vhx.glass_camera(1024, W, H, target=(512.0, 512.0, 512.0))
o = np.array(cam.origin, np.float32)
bl, r, u = (np.array(v, np.float32) for v in (cam.glass_bottom_left, cam.glass_right, cam.glass_up))
steps = z["steps"].astype(np.int64)
order = np.sort(np.argsort(-steps, kind="stable")[off:off + R])  # frame order within the selection
px = (order % W).astype(np.float32); py = (H - 1 - order // W).astype(np.float32)
gp = bl[None] + (r[None] * px[:, None]) * np.float32(cam.pixel_width) + (u[None] * py[:, None]) * np.float32(cam.pixel_height)
d = gp - o[None]
d = (d / np.sqrt((d * d).sum(1, keepdims=True))).astype(np.float32)
rt.set_pass_budgets(())
print(f"rays {off}..{off + R} by step count: steps {steps[order].min()}..{steps[order].max()}")
for k in (1, 2, 4, 8, 16, 32, 64):
    nw = (R + k - 1) // k
    n = nw * 256
    dd = np.repeat(-d[:1], n, 0)
    for w in range(nw):
        sel = d[w * k:(w + 1) * k]
        dd[w * 256:w * 256 + len(sel)] = sel
    ts = []
    for _ in range(3):
        rt.trace_rays(np.repeat(o[None], n, 0), dd, fields=("value",))
        ts.append(rt.sync())
    print(f"rays/wave={k:3d} waves={nw:4d} ms={min(ts[1:]):.3f}", flush=True)
