"""A short frames-in-flight run (F from argv, default 3) for rocprofv3 --kernel-trace: the timeline of overlapping
frames. Usage: probe_inflight_trace.py [F] [frames]"""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import voxelhex_amd as vhx
from voxelhex_amd import _native as N

F = int(sys.argv[1]) if len(sys.argv) > 1 else 3
K = int(sys.argv[2]) if len(sys.argv) > 2 else 12
flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 1024, 4, threads=16)
W, H = 3840, 2160
cam = vhx.glass_camera(1024, W, H, target=(512.0,) * 3)
owner = vhx.Raytracer(0); owner.upload(flat)
ctxs = [owner] + [owner.shared() for _ in range(F - 1)]
streams = [torch.cuda.Stream() for _ in ctxs]
for r, s in zip(ctxs, streams):
    r.set_stream(s.cuda_stream)
outs = [{"rgba": torch.zeros(W * H, dtype=torch.int32, device="cuda"),
         "depth": torch.zeros(W * H, dtype=torch.float32, device="cuda")} for _ in ctxs]
for i in range(K):
    ctxs[i % F].trace_primary(cam, out=outs[i % F])
torch.cuda.synchronize()
print("done", flush=True)
