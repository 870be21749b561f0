"""Host submission time per frame against the frame period (is a small frame launch-bound?).
Usage: probe_launch_rate.py SIZE BD W H  (eight frames in flight, own streams)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ["GPU_MAX_HW_QUEUES"] = "12"  # one hardware queue per frame in flight (the box exports 4)
import torch  # noqa: E402

import voxelhex_amd as vhx  # noqa: E402
from voxelhex_amd import _native as N  # noqa: E402

size, bd, W, H = (int(x) for x in sys.argv[1:5])
flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, size, bd, threads=16)
cam = vhx.glass_camera(size, W, H, target=(size / 2,) * 3)
F = 8
owner = vhx.Raytracer(0)
owner.upload(flat)
ctxs = [owner] + [owner.shared() for _ in range(F - 1)]
outs = [{"rgba": torch.zeros(W * H, dtype=torch.int32, device="cuda"),
         "depth": torch.zeros(W * H, dtype=torch.float32, device="cuda")} for _ in ctxs]
for i in range(16):
    ctxs[i % F].trace_primary(cam, out=outs[i % F])
torch.cuda.synchronize()
for K in (50, 200):
    t0 = time.perf_counter()
    for i in range(K):
        ctxs[i % F].trace_primary(cam, out=outs[i % F])
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"{W}x{H} {size}^3 bd{bd} K={K}: submit {(t1 - t0) / K * 1e3:.4f} ms/frame, period {(t2 - t0) / K * 1e3:.4f} "
          f"ms/frame", flush=True)
