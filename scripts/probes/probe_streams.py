"""Stream layout vs frames in flight (hardware-queue sharing): ms per frame of the bench frame at F = 3, 4 for
layouts: own = each context's own stream (lazy); dummyK = K unused streams first, then own; torch = torch pool
streams; eager = 4 unused streams then torch pool streams (the layout before lazy context streams).
Usage: probe_streams.py LAYOUT"""
import ctypes, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import voxelhex_amd as vhx
from voxelhex_amd import _native as N

lay = sys.argv[1]
hip = ctypes.CDLL("libamdhip64.so")
dummies = []
def dummy(k):
    for _ in range(k):
        s = ctypes.c_void_p()
        assert hip.hipStreamCreateWithFlags(ctypes.byref(s), 1) == 0
        dummies.append(s)
flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 1024, 4, threads=16)
W, H = 3840, 2160
cam = vhx.glass_camera(1024, W, H, target=(512.0,) * 3)
torch.zeros(1, device="cuda")
if lay.startswith("dummy"):
    dummy(int(lay[5:]))
owner = vhx.Raytracer(0)
owner.upload(flat)  # creates the owner's own stream
ctxs = [owner] + [owner.shared() for _ in range(3)]
if lay == "eager":
    dummy(4)
if lay in ("torch", "eager"):
    streams = [torch.cuda.Stream() for _ in ctxs]
    for r, s in zip(ctxs, streams):
        r.set_stream(s.cuda_stream)
else:
    streams = [torch.cuda.ExternalStream(r.stream()) for r in ctxs]
outs = [{"rgba": torch.zeros(W * H, dtype=torch.int32, device="cuda"),
         "depth": torch.zeros(W * H, dtype=torch.float32, device="cuda")} for _ in ctxs]
for F in (3, 4):
    K = 40
    for i in range(8):
        ctxs[i % F].trace_primary(cam, out=outs[i % F])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(K):
        ctxs[i % F].trace_primary(cam, out=outs[i % F])
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / K
    print(f"layout {lay:8s} F={F}: {dt * 1e3:.4f} ms/frame", flush=True)
