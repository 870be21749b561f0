"""The lone frame (one vhx_trace_primary at a time, the reference's call shape) of the headline workload under tuning
specs, alternated: median device time of the frames after the first two (the early tail's list is recorded by the
first). usage: probe_lone.py [frames] [spec|spec|...]   ("-" = defaults)"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import voxelhex_amd as vhx  # noqa: E402
from voxelhex_amd import _native as N  # noqa: E402

F = int(sys.argv[1]) if len(sys.argv) > 1 else 12
SPECS = (sys.argv[2] if len(sys.argv) > 2 else "-|tail=0").split("|")
S, W, H = 1024, 3840, 2160
flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, S, 4, threads=16)
cam = vhx.glass_camera(S, W, H, target=(S / 2.0,) * 3)
out = {"rgba": torch.zeros(W * H, dtype=torch.int32, device="cuda"),
       "depth": torch.zeros(W * H, dtype=torch.float32, device="cuda")}
rts = {}
for spec in SPECS:
    rt = vhx.Raytracer(0, tune=None if spec == "-" else spec)
    rt.upload(flat)
    rts[spec] = rt
torch.cuda.synchronize()
res = {s: ([], []) for s in SPECS}
for rep in range(2):
    for spec in SPECS:
        rt = rts[spec]
        for k in range(F):
            t0 = time.perf_counter()
            rt.trace_primary(cam, out=out)
            ms = rt.sync()
            if k >= 2:
                res[spec][0].append(ms)
                res[spec][1].append((time.perf_counter() - t0) * 1e3)
        print(f"{spec:40s} rep {rep}: median {np.median(res[spec][0][-(F - 2):]):.4f} ms device, "
              f"{np.median(res[spec][1][-(F - 2):]):.4f} ms wall, tail list {rt.tail_info()[0]}, "
              f"schedule {rt.pass_budgets()}", flush=True)
