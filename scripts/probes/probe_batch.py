"""The driver's timed window (20 frames, F = 20 in flight, one frame per context) against longer windows, and the same
20-frame batch with stream priorities (torch streams handed to the contexts with vhx_set_stream), to see how much of
the 20-step figure is pipeline fill and drain. Bench frame, default schedules; frames compared bit for bit.
usage: probe_batch.py   (REPS rounds, default 5)"""
import os
import sys

F = 20
os.environ.setdefault("GPU_MAX_HW_QUEUES", str(F + 4))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import time  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402

import voxelhex_amd as vhx  # noqa: E402
from voxelhex_amd import _native as N  # noqa: E402

REPS = int(os.environ.get("REPS", "5"))
W, H = 3840, 2160
dev = torch.device("cuda", 0)
flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 1024, 4, threads=16)
cam = vhx.glass_camera(1024, W, H, target=(512.0,) * 3)
print("stream priority range (low, high):", torch.cuda.Stream.priority_range(), flush=True)


def contexts(prios):
    """F contexts of one tree; prios None: their own streams, else torch streams of these priorities (created back to
    back, one hardware queue each)."""
    owner = vhx.Raytracer(0)
    owner.upload(flat)
    rts = [owner] + [owner.shared() for _ in range(F - 1)]
    keep = []
    if prios is None:
        streams = [torch.cuda.ExternalStream(r.stream(), device=dev) for r in rts]
    else:
        streams = [torch.cuda.Stream(device=dev, priority=p) for p in prios]
        for r, s in zip(rts, streams):
            r.set_stream(s.cuda_stream)
        keep = streams
    outs = [{"rgba": torch.zeros(W * H, dtype=torch.int32, device=dev),
             "depth": torch.zeros(W * H, dtype=torch.float32, device=dev)} for _ in rts]
    torch.cuda.synchronize()
    return rts, streams, outs, keep


def batch(rts, outs, n):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(n):
        rts[k % F].trace_primary(cam, out=outs[k % F])
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / n


lo, hi = torch.cuda.Stream.priority_range()
configs = {
    "own streams": None,
    "torch streams, all low": [lo] * F,
    "torch streams, first 10 high": [hi] * 10 + [lo] * 10,
    "torch streams, first 5 high": [hi] * 5 + [lo] * 15,
    "torch streams, first 15 high": [hi] * 15 + [lo] * 5,
}
built = {name: contexts(p) for name, p in configs.items()}
ref = None
res = {name: {20: [], 100: []} for name in configs}
for rep in range(REPS):
    for name, (rts, streams, outs, keep) in built.items():
        batch(rts, outs, 5)  # warm-up
        res[name][20].append(batch(rts, outs, 20))
        if name in ("own streams", "torch streams, first 10 high"):
            res[name][100].append(batch(rts, outs, 100))
        got = outs[7]["rgba"].clone()
        if ref is None:
            ref = got
        assert torch.equal(ref, got), name
for name, r in res.items():
    s = f"{name:32s} 20 frames {np.median(r[20]):.4f} ms/frame (min {min(r[20]):.4f})"
    if r[100]:
        s += f"   100 frames {np.median(r[100]):.4f} (min {min(r[100]):.4f})"
    print(s, flush=True)
