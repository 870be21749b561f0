"""Diagnostic: the bench frame with the outputs handed over in host memory (vhx_trace_primary with on_device = 0: the
C ABI copies the results back over PCIe before returning), against device-resident outputs. Wall time per frame,
median of 10 after 2 warm-up frames.  usage: probe_host_outputs.py"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
import voxelhex_amd as vhx
from voxelhex_amd import _native as N

W, H = 3840, 2160
flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 1024, 4, threads=16)
rt = vhx.Raytracer(0)
rt.upload(flat)
cam = vhx.glass_camera(1024, W, H, target=(512.0, 512.0, 512.0))
dev = {"rgba": torch.zeros(W * H, dtype=torch.int32, device="cuda"),
       "depth": torch.zeros(W * H, dtype=torch.float32, device="cuda")}


def run(f):
    for _ in range(2):
        f()
    ts = []
    for _ in range(10):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        f()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    return float(np.median(ts))


reuse = {"rgba": np.zeros(W * H, np.uint32), "depth": np.zeros(W * H, np.float32)}
pinned = {"rgba": torch.zeros(W * H, dtype=torch.int32).pin_memory(),
          "depth": torch.zeros(W * H, dtype=torch.float32).pin_memory()}


cases = {"device outputs (rgba + depth)": lambda: rt.trace_primary(cam, out=dev),
         "host rgba + depth, reused arrays": lambda: rt.trace_primary(cam, out=reuse),
         "host rgba + depth, pinned arrays": lambda: rt.trace_primary(cam, out=pinned),
         "host rgba + depth, fresh arrays": lambda: rt.trace_primary(cam, fields=("rgba", "depth")),
         "host rgba, fresh arrays": lambda: rt.trace_primary(cam, fields=("rgba",))}
for name, f in cases.items():
    ms = run(f)
    print(f"{name:36s} {ms:7.3f} ms/frame  {W * H / ms / 1e3:8.0f} Mrays/s", flush=True)
