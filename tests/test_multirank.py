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


# ---- the C tile plan of vhx_mgpu (vhx_mgpu_tile_plan) with rank 0 holding R slots ----------------------------------
def test_c_tile_plan_deals_every_tile_once():
    """vhx_mgpu_tile_plan for N in {1, 2, 3, 8} and R in {1..4}, incl. frames with fewer tiles than slots: the slots of
    all ranks partition 0..V-1, slot s traces tiles s, s + V, ... (at most tiles_per_slot of them), and every tile of
    the frame is traced exactly once."""
    for (w, h) in ((W, H), (3840, 2160), (64, 64), (130, 70)):
        for n in (1, 2, 3, 8):
            for r_slots in (1, 2, 3, 4):
                plans = [M.tile_plan(n, r_slots, T, w, h, q) for q in range(n)]
                V = r_slots + n - 1
                assert all(p["slots"] == V for p in plans)
                owned = sorted(s for p in plans for s in range(p["first_slot"], p["first_slot"] + p["slot_count"]))
                assert owned == list(range(V))
                assert plans[0]["slot_count"] == r_slots and all(p["slot_count"] == 1 for p in plans[1:])
                tiles = plans[0]["tiles"]
                assert tiles == ((w + T - 1) // T) * ((h + T - 1) // T)
                seen = np.zeros(tiles, np.int32)
                for s_ in range(V):
                    mine = list(range(s_, tiles, V))
                    assert len(mine) <= plans[0]["tiles_per_slot"]
                    seen[mine] += 1
                assert (seen == 1).all()
    with pytest.raises(ValueError):
        M.tile_plan(2, 0, T, W, H, 0)  # R >= 1
    with pytest.raises(ValueError):
        M.tile_plan(2, 1, T, W, H, 2)  # rank < N


def _slots_worker(rank, world, port, out_path, r_slots, w, h):
    """vhx_mgpu_render's data path restated on the CPU with the C plan: each rank traces its slots (oracle) into
    [RGBA | depth] parts of tiles_per_slot tiles, ranks >= 1 send their part to rank 0 point to point (gloo send/recv,
    as the RCCL group does), rank 0 places each at its slot's offset and untiles the slot-major buffer."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import voxelhex_amd as vhx
    from tests._oracle import Oracle
    flat = vhx.FlatTree.build_scene(vhx.native.VHX_SCENE_LATTICE_CUBE, 64, 4)
    cam = vhx.glass_camera(64, w, h, target=(32.0, 32.0, 32.0))
    orc = Oracle()
    plan = M.tile_plan(world, r_slots, T, w, h, rank)
    V, per, n = plan["slots"], plan["tiles_per_slot"], plan["tiles_per_slot"] * T * T
    parts = np.zeros(plan["slot_count"] * 2 * n, np.uint32)
    for k in range(plan["slot_count"]):
        s_ = plan["first_slot"] + k
        for j, tile in enumerate(range(s_, plan["tiles"], V)):
            x0, y0, tw, th = M.tile_rect(tile, w, h, T)
            r = orc.trace_primary(flat, cam, x0, y0, tw, th, threads=1, fields=("rgba", "depth"))
            base = k * 2 * n
            parts[base + j * T * T:base + (j + 1) * T * T].reshape(T, T)[:th, :tw] = r["rgba"].reshape(th, tw)
            parts[base + n + j * T * T:base + n + (j + 1) * T * T].reshape(T, T)[:th, :tw] = \
                r["depth"].view(np.uint32).reshape(th, tw)
    if rank == 0:
        gathered = np.zeros(V * 2 * n, np.uint32)
        gathered[:parts.size] = parts
        for q in range(1, world):
            qp = M.tile_plan(world, r_slots, T, w, h, q)
            buf = torch.zeros(2 * n, dtype=torch.int32)
            dist.recv(buf, src=q)
            gathered[qp["first_slot"] * 2 * n:(qp["first_slot"] + 1) * 2 * n] = buf.numpy().view(np.uint32)
        rgba, depth = M.untile_planes_numpy(gathered, 2, V, per, T, w, h)
        full = orc.trace_primary(flat, cam, 0, 0, w, h, threads=1, fields=("rgba", "depth"))
        np.save(out_path, np.stack([rgba, full["rgba"], depth, full["depth"].view(np.uint32)]))
    else:
        dist.send(torch.from_numpy(parts.view(np.int32)), dst=0)
    dist.destroy_process_group()


@pytest.mark.parametrize("world,r_slots,w,h", [(2, 1, W, H), (2, 3, W, H), (3, 2, W, H), (3, 3, 130, 70)])
def test_root_slots_split_reassembles_the_frame(tmp_path, world, r_slots, w, h):
    """R > 1 and a frame with fewer tiles than slots ((3, 3, 130x70): 6 tiles, 5 slots, rank 2's slot holds one)."""
    out = str(tmp_path / "slots.npy")
    mp.spawn(_slots_worker, args=(world, _free_port(), out, r_slots, w, h), nprocs=world, join=True)
    rgba, full_rgba, depth, full_depth = np.load(out)
    assert np.array_equal(rgba, full_rgba)
    assert np.array_equal(depth, full_depth)
