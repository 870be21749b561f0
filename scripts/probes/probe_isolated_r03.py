"""Isolated-frame latency (one frame at a time, synchronised; libvhx's own events, like bench.py's kernel_ms_isolated)
of the bench frame for each pass schedule given on the command line ("" = one pass); env knobs such as VHX_QWAVES
apply.   usage: probe_isolated_r03.py "64" "24,72,216,648" adaptive ..."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import voxelhex_amd as vhx  # noqa: E402
from voxelhex_amd import _native as N  # noqa: E402

flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 1024, 4, threads=16)
W, H = 3840, 2160
cam = vhx.glass_camera(1024, W, H, target=(512.0,) * 3)
rt = vhx.Raytracer(0)
rt.upload(flat)
out = {"rgba": torch.zeros(W * H, dtype=torch.int32, device="cuda"),
       "depth": torch.zeros(W * H, dtype=torch.float32, device="cuda")}
torch.cuda.synchronize()
ref = None
env = " ".join(f"{k}={v}" for k, v in sorted(os.environ.items()) if k.startswith("VHX_"))
for spec in sys.argv[1:]:
    if spec != "adaptive":  # "adaptive": the library's own choice (the lone-frame schedule here)
        rt.set_pass_budgets(tuple(int(x) for x in spec.split(",") if x))
    ms = []
    for i in range(23):
        rt.trace_primary(cam, out=out)
        t = rt.sync()
        if i >= 3:
            ms.append(t)
    if ref is None:
        ref = out["rgba"].clone()
    handed, err = rt.split_stats()
    print(f"{env:30s} budgets={spec or '()':>22}: isolated {np.median(ms):.4f} ms (min {min(ms):.4f})  "
          f"equal {torch.equal(ref, out['rgba'])}  split handed {handed} err {err}", flush=True)
rt.close()
