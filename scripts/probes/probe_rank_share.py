"""Diagnostic: one rank's share of the weak-scaling bench frame (bench.py --gpus N), traced alone on one GPU.

Rank r of N traces the 64x64 tiles r, r+N, ... of the frame_size(3840, 2160, N) frame in the tile layout, exactly
as in bench.py; this times that launch for each rank of N = 1, 2, 4, 8 (N = 1: the framebuffer launch), so the
per-rank time behind the multi-GPU bench line can be seen on a single GPU.
usage: probe_rank_share.py [frames]"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
import voxelhex_amd as vhx
from voxelhex_amd import _native as N
from voxelhex_amd import multigpu as M
from bench import frame_size

frames = int(sys.argv[1]) if len(sys.argv) > 1 else 10
flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 1024, 4, threads=16)
rt = vhx.Raytracer(0)
s = torch.cuda.Stream()
torch.cuda.set_stream(s)
rt.set_stream(s.cuda_stream)
rt.upload(flat)
T = 64
for world in (1, 2, 4, 8):
    W, H = frame_size(3840, 2160, world)
    cam = vhx.glass_camera(1024, W, H, target=(512.0, 512.0, 512.0))
    for rank in range(world):
        if world == 1:
            n, kw = W * H, dict(tile_size=0, tile_start=0, tile_stride=1, layout=N.VHX_LAYOUT_FRAMEBUFFER)
        else:
            n = M.tiles_per_rank(W, H, T, world) * T * T
            kw = dict(tile_size=T, tile_start=rank, tile_stride=world, layout=N.VHX_LAYOUT_TILES)
        out = {"rgba": torch.zeros(n, dtype=torch.int32, device="cuda"),
               "depth": torch.zeros(n, dtype=torch.float32, device="cuda")}
        for _ in range(2):
            rt.trace_primary(cam, out=out, **kw)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(frames):
            rt.trace_primary(cam, out=out, **kw)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / frames
        rays = M.rank_rays(W, H, T, rank, world) if world > 1 else W * H
        print(f"N={world} {W}x{H} rank {rank}: {rays} rays, {ms:.3f} ms, {rays / ms / 1e3:.0f} Mrays/s", flush=True)
