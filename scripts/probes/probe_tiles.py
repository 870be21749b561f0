"""Config 4 (7680x4320, scene S 1024^3 bd 4) on one GPU, frames in flight, by output layout: whole
framebuffer frames, the same frame as one tile set (VHX_LAYOUT_TILES, 64x64 tiles, every tile), one rank's tile set of
an N-rank split (tiles r, r+N, ...), and the vhx_mgpu one-rank path (tile set + untile), so that the cost of the tile
layout and of the multi-GPU plumbing are told apart. usage: probe_tiles.py [F] [N] [tune spec]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
F = int(sys.argv[1]) if len(sys.argv) > 1 else 16
NR = int(sys.argv[2]) if len(sys.argv) > 2 else 8
TUNE = sys.argv[3] if len(sys.argv) > 3 else None
os.environ.setdefault("GPU_MAX_HW_QUEUES", str(min(32, F + 4)))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import voxelhex_amd as vhx  # noqa: E402
from voxelhex_amd import _native as N  # noqa: E402
from voxelhex_amd import multigpu as M  # noqa: E402

W, H, T, S = 7680, 4320, 64, 1024
flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, S, 4, threads=16)
cam = vhx.glass_camera(S, W, H, target=(S / 2.0,) * 3)
rt = vhx.Raytracer(0, tune=TUNE)
rt.upload(flat)
rts = [rt] + [rt.shared() for _ in range(F - 1)]
if TUNE:
    for r in rts[1:]:
        r.set_tuning(TUNE)
dev = torch.device("cuda", 0)


def outs(n):
    return [{"rgba": torch.zeros(n, dtype=torch.int32, device=dev), "depth": torch.zeros(n, dtype=torch.float32,
                                                                                           device=dev)} for _ in rts]


def run(label, n_out, kw, frames=40, warm=F + 5):
    o = outs(n_out)
    torch.cuda.synchronize()
    for k in range(warm):
        rts[k % F].trace_primary(cam, out=o[k % F], **kw)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(frames):
        rts[k % F].trace_primary(cam, out=o[k % F], **kw)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / frames
    print(f"{label:52s} {ms:.4f} ms per frame  {n_out / ms / 1e3:9.0f} Mentries/s  schedule {rts[-1].pass_budgets()}",
          flush=True)
    return o


fb = run("framebuffer 7680x4320", W * H, {})
ntile = M.tiles_per_rank(W, H, T, 1) * T * T
tl = run("tile set, every 64x64 tile", ntile, dict(tile_size=T, tile_start=0, tile_stride=1,
                                                 layout=N.VHX_LAYOUT_TILES))
fbs = fb[-1]["rgba"].cpu().numpy()
un = M.untile_numpy(tl[-1]["rgba"].cpu().numpy(), 1, M.tiles_per_rank(W, H, T, 1), T, W, H)
print("tile set untiled == framebuffer:", bool(np.array_equal(un, fbs)))
nr = M.tiles_per_rank(W, H, T, NR) * T * T
run(f"tile set of rank 0 of {NR} (tiles 0, {NR}, ...)", nr, dict(tile_size=T, tile_start=0, tile_stride=NR,
                                                                  layout=N.VHX_LAYOUT_TILES))
run(f"tile set of rank 1 of {NR}", nr, dict(tile_size=T, tile_start=1, tile_stride=NR, layout=N.VHX_LAYOUT_TILES))
mg = M.MgpuRenderer(rt, M.mgpu_unique_id(), 1, 0, tile_size=T, overlap=True)
mg.set_frames_in_flight(min(F, N.VHX_MGPU_MAX_INFLIGHT))
mg.set_planes(1)
fbr = torch.zeros(W * H, dtype=torch.int32, device=dev)
for k in range(F + 5):
    mg.render(cam, fbr)
mg.sync()
t0 = time.perf_counter()
for k in range(40):
    mg.render(cam, fbr)
mg.sync()
torch.cuda.synchronize()
ms = (time.perf_counter() - t0) * 1e3 / 40
print(f"{'vhx_mgpu one rank, RGBA plane, untile':52s} {ms:.4f} ms per frame  equal {bool(np.array_equal(fbr.cpu().numpy(), fbs))}",
      flush=True)
mg.close()


def run_batches(label, n_out, T_, start, stride, K, C, frames=42):
    """batches of K tile sets (vhx_trace_tiles_batch) on C contexts round-robin"""
    o = [outs(n_out) for _ in range(K)]  # K output sets per context slot (reused round-robin)
    ctxs = rts[:C]
    torch.cuda.synchronize()

    def go(nb):
        for b in range(nb):
            r = ctxs[b % C]
            oo = [o[j][b % C] for j in range(K)]
            r.trace_tiles_batch([cam] * K, T_, [start] * K, stride, oo)

    go(2 * C)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    nb = frames // K
    go(nb)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / (nb * K)
    print(f"{label:52s} {ms:.4f} ms per frame  batches of {K} on {C} contexts", flush=True)


if len(rts) >= 3:
    for K, C in ((7, 3), (4, 2), (14, 2)):
        run_batches(f"batched tile set, every tile", ntile, T, 0, 1, K, C)
        run_batches(f"batched tile set of rank 0 of {NR}", nr, T, 0, NR, K, C)
