"""World-size-2 gloo run of the screen-tile split + gather + untile path (CPU; the oracle traces each rank's tiles).

Checks that the tile plan covers the frame exactly once, that per-rank tile-major buffers gathered to rank 0 and
scattered with untile_numpy reproduce the single-rank frame, and the per-rank ray counts bench.py reports.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from voxelhex_amd import multigpu as M

W, H, T = 200, 136, 64


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import voxelhex_amd as vhx
    from tests._oracle import Oracle
    flat = vhx.FlatTree.build_scene(vhx.native.VHX_SCENE_LATTICE_CUBE, 64, 4)
    cam = vhx.glass_camera(64, W, H, target=(32.0, 32.0, 32.0))
    orc = Oracle()
    per = M.tiles_per_rank(W, H, T, world)
    local = np.zeros(per * T * T, np.uint32)
    for j, tile in enumerate(M.rank_tiles(W, H, T, rank, world)):
        x0, y0, w, h = M.tile_rect(tile, W, H, T)
        rgba = orc.trace_primary(flat, cam, x0, y0, w, h, threads=1, fields=("rgba",))["rgba"].reshape(h, w)
        local[j * T * T:(j + 1) * T * T].reshape(T, T)[:h, :w] = rgba
    g = M.gather_to_root(torch.from_numpy(local.view(np.int32)), world, rank, dist)
    if rank == 0:
        fb = M.untile_numpy(g.numpy().view(np.uint32), world, per, T, W, H)
        full = orc.trace_primary(flat, cam, 0, 0, W, H, threads=1, fields=("rgba",))["rgba"]
        np.save(out_path, np.stack([fb, full]))
    dist.destroy_process_group()


def test_tile_plan_covers_frame_once():
    for world in (1, 2, 3, 8):
        seen = np.zeros((H, W), np.int32)
        for r in range(world):
            for t in M.rank_tiles(W, H, T, r, world):
                x0, y0, w, h = M.tile_rect(t, W, H, T)
                seen[y0:y0 + h, x0:x0 + w] += 1
        assert (seen == 1).all()
        assert sum(M.rank_rays(W, H, T, r, world) for r in range(world)) == W * H


def test_two_rank_gloo_gather_matches_single_frame(tmp_path):
    out = str(tmp_path / "frames.npy")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    fb, full = np.load(out)
    assert np.array_equal(fb, full)
    assert (full != 0).all()


def _pipeline_worker(rank, world, port, out_path, overlap):
    """Frames with step-dependent content through GatherPipeline (gloo, CPU tensors); rank 0 records every untiled
    frame, so a buffer mix-up between in-flight frames shows as a wrong frame."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    per = M.tiles_per_rank(W, H, T, world)
    n_out = per * T * T
    seen = []

    def untile(gathered, slot):
        seen.append(M.untile_numpy(gathered.numpy().view(np.uint32), world, per, T, W, H))

    pipe = M.GatherPipeline(n_out, world, rank, dist, "cpu", untile, overlap=overlap)
    frames = 5
    for k in range(frames):
        buf = pipe.out_buffer().numpy().view(np.uint32)
        for j, tile in enumerate(M.rank_tiles(W, H, T, rank, world)):
            x0, y0, w, h = M.tile_rect(tile, W, H, T)
            ys, xs = np.mgrid[y0:y0 + h, x0:x0 + w]
            buf[j * T * T:(j + 1) * T * T].reshape(T, T)[:h, :w] = (ys * W + xs) * 16 + k
        pipe.submit()
    pipe.drain()
    if rank == 0:
        np.save(out_path, np.stack(seen))
    dist.destroy_process_group()


@pytest.mark.parametrize("overlap", [True, False])
def test_gather_pipeline_keeps_frames_apart(tmp_path, overlap):
    out = str(tmp_path / "seen.npy")
    mp.spawn(_pipeline_worker, args=(2, _free_port(), out, overlap), nprocs=2, join=True)
    seen = np.load(out)
    ys, xs = np.mgrid[0:H, 0:W]
    assert seen.shape[0] == 5
    for k in range(5):
        assert np.array_equal(seen[k], ((ys * W + xs) * 16 + k).ravel().astype(np.uint32)), k


def _planes_worker(rank, world, port, out_path):
    """The vhx_mgpu data path restated on the CPU: the RCCL id made by libvhx on rank 0 reaches every rank through
    the gloo group (as bench.py sends it), each rank's [RGBA | depth] tile planes are gathered rank-major and
    untile_planes_numpy (k_untile_planes) rebuilds both framebuffers."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import voxelhex_amd as vhx
    from tests._oracle import Oracle
    obj = [M.mgpu_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    ids = [None] * world
    dist.all_gather_object(ids, obj[0])
    flat = vhx.FlatTree.build_scene(vhx.native.VHX_SCENE_LATTICE_CUBE, 64, 4)
    cam = vhx.glass_camera(64, W, H, target=(32.0, 32.0, 32.0))
    orc = Oracle()
    per = M.tiles_per_rank(W, H, T, world)
    n = per * T * T
    local = np.zeros(2 * n, np.uint32)
    for j, tile in enumerate(M.rank_tiles(W, H, T, rank, world)):
        x0, y0, w, h = M.tile_rect(tile, W, H, T)
        r = orc.trace_primary(flat, cam, x0, y0, w, h, threads=1, fields=("rgba", "depth"))
        local[j * T * T:(j + 1) * T * T].reshape(T, T)[:h, :w] = r["rgba"].reshape(h, w)
        local[n + j * T * T:n + (j + 1) * T * T].reshape(T, T)[:h, :w] = r["depth"].view(np.uint32).reshape(h, w)
    g = M.gather_to_root(torch.from_numpy(local.view(np.int32)), world, rank, dist)
    if rank == 0:
        rgba, depth = M.untile_planes_numpy(g.numpy().view(np.uint32), 2, world, per, T, W, H)
        full = orc.trace_primary(flat, cam, 0, 0, W, H, threads=1, fields=("rgba", "depth"))
        same_id = all(i == ids[0] for i in ids) and len(ids[0]) == 128
        np.save(out_path, np.stack([rgba, full["rgba"], depth, full["depth"].view(np.uint32),
                                    np.full(W * H, int(same_id), np.uint32)]))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_rank_planes_gather_and_rccl_id_exchange(tmp_path, world):
    out = str(tmp_path / "planes.npy")
    mp.spawn(_planes_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    rgba, full_rgba, depth, full_depth, same_id = np.load(out)
    assert same_id.all(), "ranks received different RCCL ids"
    assert np.array_equal(rgba, full_rgba)
    assert np.array_equal(depth, full_depth)
