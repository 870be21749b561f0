"""The driver's timed window (20 frames, F = 20 in flight, one frame per context) against a 100-frame window, with the
contexts on their own streams (as bench.py) or on torch streams of two priorities handed over with vhx_set_stream
before anything runs (the first H contexts high, the rest low), to see how much of the 20-step figure is pipeline fill
and drain and whether stream priorities shorten it. One configuration per process (each stream its own hardware
queue); bench frame, default schedules; the frames compared bit for bit with the first context's.
usage: probe_batch.py own|low|hiH   (REPS rounds, default 5)"""
import os
import sys

F = 20
os.environ["GPU_MAX_HW_QUEUES"] = str(F + 4)  # as bench.py: a queue per stream (the box presets 4)
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import time  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402

import voxelhex_amd as vhx  # noqa: E402
from voxelhex_amd import _native as N  # noqa: E402

mode = sys.argv[1]
REPS = int(os.environ.get("REPS", "5"))
W, H = 3840, 2160
dev = torch.device("cuda", 0)
lo, hi = torch.cuda.Stream.priority_range()
streams = None
if mode != "own":  # the streams first, so that each takes a hardware queue of its own
    nhi = 0 if mode == "low" else int(mode[2:])
    streams = [torch.cuda.Stream(device=dev, priority=hi if k < nhi else lo) for k in range(F)]
owner = vhx.Raytracer(0)
if streams:
    owner.set_stream(streams[0].cuda_stream)
owner.upload(vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 1024, 4, threads=16))
rts = [owner] + [owner.shared() for _ in range(F - 1)]
if streams:
    for r, s in zip(rts[1:], streams[1:]):
        r.set_stream(s.cuda_stream)
cam = vhx.glass_camera(1024, W, H, target=(512.0,) * 3)
outs = [{"rgba": torch.zeros(W * H, dtype=torch.int32, device=dev),
         "depth": torch.zeros(W * H, dtype=torch.float32, device=dev)} for _ in rts]
torch.cuda.synchronize()


def batch(n):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(n):
        rts[k % F].trace_primary(cam, out=outs[k % F])
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / n


for r in rts:  # setup frame per context
    r.trace_primary(cam, out=outs[0])
res = {20: [], 100: []}
for rep in range(REPS):
    batch(5)
    res[20].append(batch(20))
    res[100].append(batch(100))
for k in range(1, F):
    assert torch.equal(outs[0]["rgba"], outs[k]["rgba"]), k
print(f"{mode:6s} 20 frames {np.median(res[20]):.4f} ms/frame (min {min(res[20]):.4f})   "
      f"100 frames {np.median(res[100]):.4f} (min {min(res[100]):.4f})", flush=True)
