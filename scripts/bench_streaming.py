"""Streaming-frame timing (docs/DESIGN_LOG.md §9c, §14.2): a device view of the 256^3 scene-S tree (brick_dim 4) around a viewport
that moves every frame, at the reference's default rates (node_uploads_per_frame 25, brick_uploads_per_frame 50,
view.rs:109-111), each frame a 1920x1080 trace of the view -- the reference's render loop (upload::<T> then dispatch,
streaming/mod.rs:420-635, pipeline/mod.rs:96-155).

--inflight 1 (default): one frame at a time; per frame the producer's host time (vhx_stream_upload: decisions +
packing + one staged copy), the device time of the frame's ranged writes (HIP events around the upload on the context's
stream) and the trace.
--inflight F > 1: F contexts share the device view (vhx_create_shared), frame k is traced by context k % F into its own
outputs, the uploads go through the owner, and nothing is synchronised between frames (libvhx orders every write after
the frames submitted before it and every frame after the writes submitted before it); the figure is the frame period
(wall time / frames) next to the same loop at F = 1 without per-frame synchronisation.
--batches K1,K2,... (with --inflight F): the uploads of K frames written once every K frames
(vhx_stream_upload_frames), so that K frames in flight share one tree version; each K runs the same frames of the orbit,
rounds interleaved (docs/DESIGN_LOG.md §15.4).
--size / --width / --height: the tree (scene S, brick_dim 4; 1024 builds the host tree from the bulk image,
BoxTree.from_scene) and the frame.
usage: bench_streaming.py [frames] [--inflight F] [--batches 1,4,8] [--size 1024 --width 3840 --height 2160]"""
import argparse
import os
import sys
import time

ap = argparse.ArgumentParser()
ap.add_argument("frames", nargs="?", type=int, default=200)
ap.add_argument("--inflight", type=int, default=1)
ap.add_argument("--batches", default=None)
ap.add_argument("--size", type=int, default=256)
ap.add_argument("--width", type=int, default=1920)
ap.add_argument("--height", type=int, default=1080)
ap.add_argument("--rounds", type=int, default=2)
args = ap.parse_args()
if args.inflight > 1 and int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < args.inflight + 4:
    os.environ["GPU_MAX_HW_QUEUES"] = str(min(32, args.inflight + 4))  # before HIP starts (bench.py's hw_queues)

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import voxelhex_amd as vhx  # noqa: E402
from voxelhex_amd import _native as N  # noqa: E402

frames = args.frames
SZ, WD, HT = args.size, args.width, args.height
if SZ >= 512:
    t = vhx.BoxTree.from_scene(N.VHX_SCENE_LATTICE_CUBE, SZ, 4, threads=16)
else:
    t = vhx.BoxTree(SZ, 4)
    t.insert_scene(N.VHX_SCENE_LATTICE_CUBE)
rt = vhx.Raytracer(0)
stream = torch.cuda.ExternalStream(rt.stream())
torch.cuda.set_stream(stream)
S = float(SZ)
VD = S / 4  # view distance (64 at 256^3)
s = vhx.StreamingView(t, rt, (S / 2, S / 2, S / 2), VD)
s.set_rates(25, 50, 10)


def view(k):
    a = 2.0 * np.pi * k / frames
    c = (S / 2 + 0.234 * S * np.cos(a), S / 2, S / 2 + 0.234 * S * np.sin(a))
    return a, c


def outputs():
    return {"rgba": torch.zeros(WD * HT, dtype=torch.int32, device="cuda"),
            "depth": torch.zeros(WD * HT, dtype=torch.float32, device="cuda")}


q = lambda v: f"median {np.median(v):.3f} p90 {np.percentile(v, 90):.3f} max {np.max(v):.3f}"  # noqa: E731

if args.inflight <= 1:
    out = outputs()
    host, dev, trace, written, resizes = [], [], [], [], 0
    for k in range(frames):
        a, c = view(k)
        s.set_viewport(c, VD)
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        e0.record(stream)
        t0 = time.perf_counter()
        st, grow = s.upload()
        host.append((time.perf_counter() - t0) * 1e3)
        if grow:
            s.resize()
            resizes += 1
        e1.record(stream)
        cam = vhx.glass_camera(SZ, WD, HT, angle=40.0 + a, target=c)
        rt.trace_primary(cam, out=out)
        e2.record(stream)
        written.append(st["bytes_written"])
        torch.cuda.synchronize()
        dev.append(e0.elapsed_time(e1))
        trace.append(e1.elapsed_time(e2))
    print(f"{frames} frames, {resizes} resizes, bytes written per frame median {int(np.median(written))} max {max(written)}")
    print(f"producer host ms (vhx_stream_upload): {q(host)}")
    print(f"ranged writes device ms (update batch on the stream): {q(dev)}")
    print(f"trace {WD}x{HT} of the view ms: {q(trace)}")
else:
    F = args.inflight
    ctxs = [rt] + [rt.shared() for _ in range(F - 1)]
    for r in ctxs:
        r.stream()  # each context's own stream, created back to back (one hardware queue each)
    outs = [outputs() for _ in range(F)]
    torch.cuda.synchronize()

    def loop(nctx, k0):
        host, resizes = [], 0
        t0 = time.perf_counter()
        for k in range(k0, k0 + frames):
            a, c = view(k)
            s.set_viewport(c, VD)
            h0 = time.perf_counter()
            _, grow = s.upload()  # through the owner, no host wait
            host.append((time.perf_counter() - h0) * 1e3)
            if grow:
                s.resize()
                resizes += 1
            cam = vhx.glass_camera(SZ, WD, HT, angle=40.0 + a, target=c)
            ctxs[k % nctx].trace_primary(cam, out=outs[k % nctx])
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3 / frames, host, resizes

    loop(F, 0)  # warm-up: every context allocates its queues, the view reaches its size
    if args.batches:
        def batched(K, k0):
            t0 = time.perf_counter()
            resizes = 0
            for k in range(k0, k0 + frames):
                a, c = view(k)
                s.set_viewport(c, VD)
                if (k - k0) % K == 0:
                    _, grow = s.upload(frames=K)  # K frames' uploads, one tree version for the next K frames
                    if grow:
                        s.resize()
                        resizes += 1
                cam = vhx.glass_camera(SZ, WD, HT, angle=40.0 + a, target=c)
                ctxs[k % F].trace_primary(cam, out=outs[k % F])
            torch.cuda.synchronize()
            return (time.perf_counter() - t0) * 1e3 / frames, resizes
        Ks = [int(x) for x in args.batches.split(",")]
        res = {K: [] for K in Ks}
        for rnd in range(args.rounds):
            for K in Ks:
                period, resizes = batched(K, frames)  # the same frames of the orbit for every K
                res[K].append(period)
                print(f"round {rnd} batch K={K}: {frames} frames on {F} contexts, period {period:.4f} ms per frame "
                      f"(upload + {WD}x{HT} trace), {resizes} resizes", flush=True)
        base = min(res[Ks[0]])
        for K in Ks:
            print(f"batch K={K}: best period {min(res[K]):.4f} ms per frame = {min(res[K]) / base:.3f} x K={Ks[0]}")
    for nctx in (1, F):
        period, host, resizes = loop(nctx, frames)
        print(f"frames in flight {nctx}: {frames} frames, period {period:.4f} ms per frame (upload + {WD}x{HT} trace), "
              f"producer host ms {q(host)}, {resizes} resizes")
    for r in ctxs[1:]:
        r.close()
s.close()
rt.close()
