"""Streaming-frame timing: a device view of the 256^3 scene-S tree (brick_dim 4) around a viewport that
moves every frame, at the reference's default rates (node_uploads_per_frame 25, brick_uploads_per_frame 50,
view.rs:109-111). Per frame: the producer's host time (vhx_stream_upload: decisions + packing + one staged copy), the
device time of the frame's ranged writes (HIP events around the upload on the context's stream) and the trace of a
1920x1080 frame of the view. usage: bench_streaming.py [frames]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import voxelhex_amd as vhx
from voxelhex_amd import _native as N

frames = int(sys.argv[1]) if len(sys.argv) > 1 else 200
t = vhx.BoxTree(256, 4)
t.insert_scene(N.VHX_SCENE_LATTICE_CUBE)
rt = vhx.Raytracer(0)
stream = torch.cuda.ExternalStream(rt.stream())
torch.cuda.set_stream(stream)
S = 256.0
s = vhx.StreamingView(t, rt, (S / 2, S / 2, S / 2), 64.0)
s.set_rates(25, 50, 10)
out = {"rgba": torch.zeros(1920 * 1080, dtype=torch.int32, device="cuda"),
       "depth": torch.zeros(1920 * 1080, dtype=torch.float32, device="cuda")}
host, dev, trace, written, resizes = [], [], [], [], 0
for k in range(frames):
    a = 2.0 * np.pi * k / frames
    c = (S / 2 + 60.0 * np.cos(a), S / 2, S / 2 + 60.0 * np.sin(a))
    s.set_viewport(c, 64.0)
    e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    e0.record(stream)
    t0 = time.perf_counter()
    st, grow = s.upload()
    host.append((time.perf_counter() - t0) * 1e3)
    if grow:
        s.resize()
        resizes += 1
    e1.record(stream)
    cam = vhx.glass_camera(256, 1920, 1080, angle=40.0 + a, target=c)
    rt.trace_primary(cam, out=out)
    e2.record(stream)
    written.append(st["bytes_written"])
    torch.cuda.synchronize()
    dev.append(e0.elapsed_time(e1))
    trace.append(e1.elapsed_time(e2))
q = lambda v: f"median {np.median(v):.3f} p90 {np.percentile(v, 90):.3f} max {np.max(v):.3f}"
print(f"{frames} frames, {resizes} resizes, bytes written per frame median {int(np.median(written))} max {max(written)}")
print(f"producer host ms (vhx_stream_upload): {q(host)}")
print(f"ranged writes device ms (update batch on the stream): {q(dev)}")
print(f"trace 1920x1080 of the view ms: {q(trace)}")
s.close()
rt.close()
