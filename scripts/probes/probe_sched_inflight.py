"""Pass-budget schedules under frames in flight: ms per frame (3840x2160 bench frame) for each schedule at F = 1 and 3.
Usage: probe_sched_inflight.py "64" "32,256" ...  (env knobs such as VHX_QWAVES apply to every context)."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import voxelhex_amd as vhx
from voxelhex_amd import _native as N

flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 1024, 4, threads=16)
W, H = 3840, 2160
cam = vhx.glass_camera(1024, W, H, target=(512.0,) * 3)
owner = vhx.Raytracer(0); owner.upload(flat)
FS = [int(x) for x in os.environ.get("VHX_PROBE_F", "1,3").split(",")]
ctxs = [owner] + [owner.shared() for _ in range(max(FS) - 1)]
# each context on its own stream (created back to back: one hardware queue each)
streams = [torch.cuda.ExternalStream(r.stream()) for r in ctxs]
outs = [{"rgba": torch.zeros(W * H, dtype=torch.int32, device="cuda"),
         "depth": torch.zeros(W * H, dtype=torch.float32, device="cuda")} for _ in ctxs]
ref = None
for spec in sys.argv[1:] or ["64"]:
    b = tuple(int(x) for x in spec.split(",") if x)
    for r in ctxs:
        r.set_pass_budgets(b)
    for F in FS:
        K = int(os.environ.get("VHX_PROBE_K", "40"))
        for i in range(6):
            ctxs[i % F].trace_primary(cam, out=outs[i % F])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(K):
            ctxs[i % F].trace_primary(cam, out=outs[i % F])
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / K
        if ref is None:
            ref = outs[0]["rgba"].clone()
        ok = all(torch.equal(ref, outs[f]["rgba"]) for f in range(F))
        print(f"budgets={spec:>12} F={F}: {dt*1e3:.4f} ms/frame  {W*H/dt/1e6:.0f} Mrays/s  equal {ok}", flush=True)
