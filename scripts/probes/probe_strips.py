"""A lone frame traced as S interleaved tile sets on S contexts of one tree at once (tile_start = k, tile_stride = S,
framebuffer layout: every context writes its own pixels of the same framebuffer), each on its own stream: the sets'
tails overlap the other sets' first passes, as frames in flight do. Timed from the first submission to the last
completion (host clock around synchronisations), median of REPS, against the one-context lone frame; the frame is
compared bit for bit with it. usage: probe_strips.py SPEC...  with SPEC = S[:tune][:hi]  (tune = a vhx_set_tuning
spec for every context, "-" for none; hi = the first context's stream at high priority)"""
import os
import sys

os.environ["GPU_MAX_HW_QUEUES"] = "24"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import time  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402

import voxelhex_amd as vhx  # noqa: E402
from voxelhex_amd import _native as N  # noqa: E402

REPS = int(os.environ.get("REPS", "10"))
W, H, T = 3840, 2160, 64
dev = torch.device("cuda", 0)
lo, hi = torch.cuda.Stream.priority_range()
flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 1024, 4, threads=16)
cam = vhx.glass_camera(1024, W, H, target=(512.0,) * 3)
owner = vhx.Raytracer(0)
owner.upload(flat)
ref = {"rgba": torch.zeros(W * H, dtype=torch.int32, device=dev), "depth": torch.zeros(W * H, dtype=torch.float32, device=dev)}
owner.trace_primary(cam, out=ref)
owner.sync()
lone = []
for _ in range(REPS + 2):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    owner.trace_primary(cam, out=ref)
    owner.sync()
    lone.append((time.perf_counter() - t0) * 1e3)
print(f"{'lone (one context)':40s} {np.median(lone[2:]):.4f} ms (min {min(lone[2:]):.4f})", flush=True)
for spec in sys.argv[1:]:
    parts = spec.split(":")
    S = int(parts[0])
    tune = parts[1] if len(parts) > 1 and parts[1] != "-" else None
    high = len(parts) > 2 and parts[2] == "hi"
    streams = [torch.cuda.Stream(device=dev, priority=hi if (high and k == 0) else lo) for k in range(S)]
    rts = [owner.shared() for _ in range(S)]
    for r, s in zip(rts, streams):
        r.set_stream(s.cuda_stream)
        if tune:
            r.set_tuning(tune)
    out = {"rgba": torch.zeros(W * H, dtype=torch.int32, device=dev),
           "depth": torch.zeros(W * H, dtype=torch.float32, device=dev)}
    torch.cuda.synchronize()
    ts = []
    for rep in range(REPS + 2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k, r in enumerate(rts):
            r.trace_primary(cam, tile_size=T, tile_start=k, tile_stride=S, out=out)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    ok = torch.equal(out["rgba"], ref["rgba"]) and torch.equal(out["depth"], ref["depth"])
    print(f"{spec:40s} {np.median(ts[2:]):.4f} ms (min {min(ts[2:]):.4f}) equal {ok}", flush=True)
    for r in rts:
        r.close()
