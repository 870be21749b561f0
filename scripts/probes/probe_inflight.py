"""Frames in flight: F contexts (each with its own copy of the tree), each on its own stream, frames dealt round-robin.
Steady-state wall time per frame vs F (does frame k's latency-bound tail overlap frame k+1's pass 0?)."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np, torch
import voxelhex_amd as vhx
from voxelhex_amd import _native as N

flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 1024, 4, threads=16)
W, H = 3840, 2160
cam = vhx.glass_camera(1024, W, H, target=(512.0,) * 3)
ctxs, streams, outs = [], [], []
for f in range(4):
    rt = vhx.Raytracer(0); rt.upload(flat)
    s = torch.cuda.Stream(); rt.set_stream(s.cuda_stream)
    ctxs.append(rt); streams.append(s)
    outs.append({"rgba": torch.zeros(W * H, dtype=torch.int32, device="cuda"),
                 "depth": torch.zeros(W * H, dtype=torch.float32, device="cuda")})
prio = [torch.cuda.Stream(priority=-1) for _ in range(4)]
for F in (1, 2, 3, 4):
    for mode in ("plain",):
        K = 40
        for i in range(6):
            ctxs[i % F].trace_primary(cam, out=outs[i % F])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(K):
            ctxs[i % F].trace_primary(cam, out=outs[i % F])
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / K
        ok = all(torch.equal(outs[0]["rgba"], outs[f]["rgba"]) for f in range(F))
        print(f"F={F} {mode}: {dt*1e3:.4f} ms/frame  {W*H/dt/1e6:.0f} Mrays/s  frames equal {ok}", flush=True)
