"""Lone-frame latency (one frame at a time, synchronised; libvhx's events, like bench.py's `lone`) of the bench frame
for each vhx_set_tuning spec on the command line (docs/DESIGN_LOG.md §15), interleaved over REPS rounds so that box drift hits
every spec alike; also a lone orbiting frame (every frame a different view).
usage: probe_lone.py "" "budgets=64,1024" ..."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import voxelhex_amd as vhx  # noqa: E402
from voxelhex_amd import _native as N  # noqa: E402

REPS = int(os.environ.get("REPS", "2"))
flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 1024, 4, threads=16)
W, H = 3840, 2160
cam = vhx.glass_camera(1024, W, H, target=(512.0,) * 3)
orbit = [vhx.glass_camera(1024, W, H, angle=40.0 + 0.01 * k, target=(512.0,) * 3) for k in range(40)]
rts = {}
for spec in sys.argv[1:]:
    rt = vhx.Raytracer(0, tune=spec)
    rt.upload(flat)
    rts[spec] = rt
out = {"rgba": torch.zeros(W * H, dtype=torch.int32, device="cuda"),
       "depth": torch.zeros(W * H, dtype=torch.float32, device="cuda")}
torch.cuda.synchronize()
ref = None
res = {s: {"static": [], "orbit": []} for s in rts}
for rep in range(REPS):
    for spec, rt in rts.items():
        for i in range(13):
            rt.trace_primary(cam, out=out)
            t = rt.sync()
            if i >= 3:
                res[spec]["static"].append(t)
        if ref is None:
            ref = out["rgba"].clone()
        assert torch.equal(ref, out["rgba"]), spec
        for k, c in enumerate(orbit[:20]):
            rt.trace_primary(c, out=out)
            t = rt.sync()
            if k >= 3:
                res[spec]["orbit"].append(t)
for spec, r in res.items():
    print(f"{spec:40s} lone static {np.median(r['static']):.4f} ms (min {min(r['static']):.4f})   "
          f"lone orbit {np.median(r['orbit']):.4f} ms (min {min(r['orbit']):.4f})", flush=True)
