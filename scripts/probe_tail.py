"""Diagnostic: device time of the longest rays of the bench frame (traced through vhx_trace_rays, single pass).
Pixel lists come from the oracle's per-ray step counts (vhx_oracle_ray_steps), computed off-box."""
import sys, time
import numpy as np
import torch
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
import voxelhex_amd as vhx
from voxelhex_amd import _native as N

def main():
    z = np.load(sys.argv[1])
    W, H = 3840, 2160
    flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 1024, 4)
    rt = vhx.Raytracer(0)
    rt.upload(flat)
    cam = vhx.glass_camera(1024, W, H, target=(512.0, 512.0, 512.0))
    o = np.array(cam.origin, np.float32)
    bl, r, u = (np.array(v, np.float32) for v in (cam.glass_bottom_left, cam.glass_right, cam.glass_up))
    def rays(pix):
        px = (pix % W).astype(np.float32); py = (H - 1 - pix // W).astype(np.float32)
        gp = bl[None] + (r[None] * px[:, None]) * np.float32(cam.pixel_width) + (u[None] * py[:, None]) * np.float32(cam.pixel_height)
        d = gp - o[None]
        d = d / np.sqrt((d * d).sum(1, keepdims=True))
        return np.repeat(o[None], len(pix), 0), d.astype(np.float32)
    for sched in ((), (32, 256)):
        rt.set_pass_budgets(sched)
        for name, pix in (("longest", z["top64"][:1]), ("top64", z["top64"]), ("top64x16", np.tile(z["top64"], 16)),
                          ("tail>256", z["tail"]), ("tail>1024", z["tail"][z["steps"][z["tail"]] > 1024]),
                          ("tail>256 shuffled", z["tail_shuf"]), ("tail>64", z["t64"]), ("tail>64 shuffled", z["t64_shuf"])):
            oo, dd = rays(pix)
            ts = []
            for _ in range(4):
                rt.trace_rays(oo, dd, fields=("value",))
                ts.append(rt.sync())
            print(f"sched={sched} {name:18s} n={len(pix):7d} ms={min(ts[1:]):.3f}", flush=True)

main()
