"""Diagnostic: does overlapping one band's tail pass with the next band's pass 0 shorten the frame?

The bench frame is cut into K horizontal bands (band cameras: the glass origin shifted by whole pixel rows -- the
same rays up to rounding of the bottom-left corner, timing only). Bands are traced on C contexts (each its own tree
copy and HIP stream), band b on context b % C, so band b's tail can run while band b+1's pass 0 does.
usage: probe_bands.py K C [frames]"""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import voxelhex_amd as vhx
from voxelhex_amd import _native as N

K, C = int(sys.argv[1]), int(sys.argv[2])
frames = int(sys.argv[3]) if len(sys.argv) > 3 else 10
W, H = 3840, 2160
flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 1024, 4, threads=16)
dev = torch.device("cuda", 0)
full = vhx.glass_camera(1024, W, H, target=(512.0, 512.0, 512.0))
Hb = H // K
cams = []
for b in range(K):
    cam = vhx.glass_camera(1024, W, Hb, target=(512.0, 512.0, 512.0))
    cam.pixel_height, cam.glass_up[:] = full.pixel_height, full.glass_up[:]
    shift = np.float32(full.pixel_height) * np.float32((K - 1 - b) * Hb)
    cam.glass_bottom_left[:] = [float(np.float32(v) + np.float32(u) * shift)
                                for v, u in zip(full.glass_bottom_left, full.glass_up)]
    cams.append(cam)
rts, streams = [], []
for c in range(C):
    rt = vhx.Raytracer(0)
    s = torch.cuda.Stream(dev)
    rt.set_stream(s.cuda_stream)
    rt.upload(flat)
    rts.append(rt)
    streams.append(s)
outs = [{"rgba": torch.zeros(W * Hb, dtype=torch.int32, device=dev),
         "depth": torch.zeros(W * Hb, dtype=torch.float32, device=dev)} for _ in range(K)]


def frame():
    for b in range(K):
        rts[b % C].trace_primary(cams[b], out=outs[b])


for _ in range(3):
    frame()
torch.cuda.synchronize()
ts = []
for _ in range(frames):
    t0 = time.perf_counter()
    frame()
    torch.cuda.synchronize()
    ts.append((time.perf_counter() - t0) * 1e3)
print(f"K={K} C={C} ms/frame median={np.median(ts):.3f} min={min(ts):.3f}", flush=True)
