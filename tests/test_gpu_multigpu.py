"""BASELINE config 4 (8 x MI355X screen-tile split + gather, 7680x4320, 1024^3) on one GPU, and the multi-GPU C ABI.

* The 7680x4320 frame of the bench tree is traced as the 8 rank tile sets of config 4 (64x64 tiles dealt round-robin,
  VHX_LAYOUT_TILES), concatenated rank-major as the gather delivers them ([RGBA plane | depth plane] per rank),
  scattered with vhx_untile_frame and compared with the oracle's whole 7680x4320 frame (RGBA and depth bit-exact).
  With rank 0 holding R = 2 slots (a weighted split) the 8 ranks deal over 9 slots; the same check covers that layout.
* vhx_mgpu_* (RCCL behind the C ABI) with a one-rank communicator: the tree broadcast, the per-frame transfers and
  the untile on rank 0 reproduce the same frame, with and without overlapped frames, with rank 0 tracing 1-3 slots,
  and after vhx_mgpu_balance. (RCCL refuses two ranks on one GPU, so N > 1 runs first on the driver's 8-GPU node; the
  code path is the same apart from the point-to-point sends to rank 0 and RCCL's own transport.)
"""
import numpy as np
import pytest

import voxelhex_amd as vhx
from voxelhex_amd import _native as N
from voxelhex_amd import multigpu as M

pytestmark = pytest.mark.gpu

W4, H4, T4, R4 = 7680, 4320, 64, 8


@pytest.fixture(scope="module")
def config4(oracle):
    flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 1024, 4)
    cam = vhx.glass_camera(1024, W4, H4, target=(512.0, 512.0, 512.0))
    ref = oracle.trace_primary(flat, cam, 0, 0, W4, H4, fields=("rgba", "depth"))
    return flat, cam, ref


def _check_frame(rgba, depth, ref, what):
    got_rgba = rgba.cpu().numpy().view(np.uint32)
    got_depth = depth.cpu().numpy().view(np.uint32)
    bad = np.count_nonzero(got_rgba != ref["rgba"])
    assert bad == 0, f"{what}: rgba differs at {bad} pixels"
    bad = np.count_nonzero(got_depth != ref["depth"].view(np.uint32))
    assert bad == 0, f"{what}: depth differs at {bad} pixels"


@pytest.mark.parametrize("root_slots", [1, 2])
def test_config4_eight_rank_tile_sets_vs_oracle(gpu, config4, root_slots):
    import torch
    flat, cam, ref = config4
    gpu.upload(flat)
    V = R4 + root_slots - 1  # slots: rank 0 owns 0..root_slots-1, rank r >= 1 slot root_slots + r - 1
    per = M.tiles_per_rank(W4, H4, T4, V)
    n_out = per * T4 * T4
    gathered = torch.zeros(V * 2 * n_out, dtype=torch.int32, device="cuda")
    for r in range(V):
        part = gathered[r * 2 * n_out:(r + 1) * 2 * n_out]
        gpu.trace_primary(cam, tile_size=T4, tile_start=r, tile_stride=V, layout=N.VHX_LAYOUT_TILES,
                          out={"rgba": part[:n_out], "depth": part[n_out:].view(torch.float32)})
    rgba = torch.zeros(W4 * H4, dtype=torch.int32, device="cuda")
    depth = torch.zeros(W4 * H4, dtype=torch.float32, device="cuda")
    gpu.untile_frame(gathered.data_ptr(), 2, V, per, T4, W4, H4, rgba.data_ptr(), depth.data_ptr())
    gpu.sync()
    _check_frame(rgba, depth, ref, f"config 4, 8 rank tile sets over {V} slots")
    assert (ref["rgba"] != 0xFF808080).mean() > 0.1  # a frame with geometry, not the background


@pytest.mark.parametrize("overlap,inflight,root_slots", [(True, 1, 1), (False, 1, 1), (True, 3, 1), (True, 3, 3),
                                                         (False, 2, 2)])
def test_mgpu_one_rank_rccl_frame_vs_oracle(config4, overlap, inflight, root_slots):
    """root_slots > 1: rank 0 traces several tile slots (tiles s, s + V, ... for s < R) straight into its slot-major
    buffer and untiles V = R slots -- the rank-0 side of a weighted split, with no peer at N = 1."""
    import torch
    flat, cam, ref = config4
    rt = vhx.Raytracer(0)
    try:
        m = M.MgpuRenderer(rt, M.mgpu_unique_id(), 1, 0, tile_size=T4, overlap=overlap)
        m.set_frames_in_flight(inflight)
        m.broadcast_tree(flat)
        m.set_root_slots(root_slots)
        assert m.rays(W4, H4) == W4 * H4
        fbs = [(torch.zeros(W4 * H4, dtype=torch.int32, device="cuda"),
                torch.zeros(W4 * H4, dtype=torch.float32, device="cuda")) for _ in range(4)]
        for rgba, depth in fbs:  # frames in flight through the alternating tile buffers (and contexts)
            m.render(cam, rgba, depth)
        m.sync()
        for k, (rgba, depth) in enumerate(fbs):
            _check_frame(rgba, depth, ref, f"vhx_mgpu frame {k} (overlap={overlap})")
        m.close()
    finally:
        rt.close()


@pytest.mark.parametrize("batch,inflight,root_slots,planes", [(3, 1, 1, 2), (4, 2, 1, 1), (2, 2, 3, 2), (5, 3, 2, 1)])
def test_mgpu_render_batch_one_rank_vs_oracle(config4, batch, inflight, root_slots, planes):
    """vhx_mgpu_render_batch: K frames' tile slots traced as one vhx_trace_tiles_batch, transferred as one RCCL group
    and untiled per frame; every frame of two back-to-back batches (successive contexts) equals the oracle's frame."""
    import torch
    flat, cam, ref = config4
    rt = vhx.Raytracer(0)
    try:
        m = M.MgpuRenderer(rt, M.mgpu_unique_id(), 1, 0, tile_size=T4)
        m.set_frames_in_flight(inflight)
        m.broadcast_tree(flat)
        m.set_root_slots(root_slots)
        m.set_planes(planes)
        fr = [torch.zeros(W4 * H4, dtype=torch.int32, device="cuda") for _ in range(2 * batch)]
        fd = [torch.zeros(W4 * H4, dtype=torch.float32, device="cuda") for _ in range(2 * batch)] if planes == 2 else None
        for b in range(2):
            m.render_batch([cam] * batch, fr[b * batch:(b + 1) * batch],
                           None if fd is None else fd[b * batch:(b + 1) * batch])
        m.sync()
        for k in range(2 * batch):
            got = fr[k].cpu().numpy().view(np.uint32)
            assert np.array_equal(got, ref["rgba"]), f"batch frame {k}: rgba"
            if fd is not None:
                assert np.array_equal(fd[k].cpu().numpy().view(np.uint32), ref["depth"].view(np.uint32)), k
        m.close()
    finally:
        rt.close()


def test_mgpu_balance_one_rank(config4):
    """vhx_mgpu_balance at N = 1: there is no transfer, every share models the same period, so R stays 1; the frames
    rendered after it match the oracle."""
    import torch
    flat, cam, ref = config4
    rt = vhx.Raytracer(0)
    try:
        m = M.MgpuRenderer(rt, M.mgpu_unique_id(), 1, 0, tile_size=T4)
        m.broadcast_tree(flat)
        m.set_root_slots(2)
        R, trace_ms, transfer_ms = m.balance(cam, frames=2)
        assert R == 1 and trace_ms > 0.0 and transfer_ms >= 0.0
        rgba = torch.zeros(W4 * H4, dtype=torch.int32, device="cuda")
        depth = torch.zeros(W4 * H4, dtype=torch.float32, device="cuda")
        m.render(cam, rgba, depth)
        m.sync()
        _check_frame(rgba, depth, ref, "after vhx_mgpu_balance")
        with pytest.raises(N.VhxError):
            m.set_root_slots(N.VHX_MGPU_MAX_ROOT_SLOTS + 1)
        m.close()
    finally:
        rt.close()


def test_mgpu_planes_and_frame_bytes_through_python(config4):
    """MgpuRenderer.set_planes / frame_bytes (the calls bench.py makes on every rank of the vhx_mgpu path) through the
    Python wrapper: RGBA-only frames (fb_depth None) equal the oracle, rank 0 receives no bytes at N = 1, and a plane
    count other than 1 or 2 is refused."""
    import torch
    flat, cam, ref = config4
    rt = vhx.Raytracer(0)
    try:
        m = M.MgpuRenderer(rt, M.mgpu_unique_id(), 1, 0, tile_size=T4)
        m.broadcast_tree(flat)
        m.set_planes(1)
        assert m.frame_bytes(W4, H4) == 0  # one rank: nothing crosses a link
        rgba = torch.zeros(W4 * H4, dtype=torch.int32, device="cuda")
        m.render(cam, rgba, None)
        m.sync()
        assert np.array_equal(rgba.cpu().numpy().view(np.uint32), ref["rgba"])
        m.set_planes(2)
        assert m.frame_bytes(W4, H4) == 0
        with pytest.raises(N.VhxError):
            m.set_planes(3)
        m.close()
    finally:
        rt.close()


def test_bench_mgpu_path_one_rank():
    """bench.py's vhx_mgpu path end to end (VHX_BENCH_MGPU1=1: gloo setup, RCCL id exchange, renderer, set_planes,
    balance, tree broadcast, timed frames, frame_bytes, the untimed multi-GPU check) on a small workload; the line
    reports the gathered frame equal to a lone trace in both plane counts."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, VHX_BENCH_MGPU1="1", MASTER_ADDR="127.0.0.1", MASTER_PORT="29541")
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--size", "64", "--width", "512", "--height", "256",
           "--steps", "3", "--warmup", "1", "--inflight", "2", "--no-cpu-baseline", "--no-pmc", "--no-extra"]
    p = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-4000:]
    line = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
    assert line["multi_gpu_check"]["frame_equal"] and line["multi_gpu_check"]["two_plane_frame_equal"]
    assert line["mgpu_split"]["bytes_into_rank0_per_frame"] == 0 and "mgpu_fallback" not in line


def test_mgpu_argument_errors(gpu):
    import ctypes
    flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 64, 4)
    uid = M.mgpu_unique_id()
    rt = vhx.Raytracer(0)
    try:
        idbuf = (ctypes.c_uint8 * 128).from_buffer_copy(uid)
        h = ctypes.c_void_p()
        assert N.lib().vhx_mgpu_create(rt._h, idbuf, 1, 1, 64, ctypes.byref(h)) == N.VHX_E_INVALID_ARG  # rank >= N
        assert N.lib().vhx_mgpu_create(rt._h, idbuf, 1, 0, 0, ctypes.byref(h)) == N.VHX_E_INVALID_ARG  # tile 0
        m = M.MgpuRenderer(rt, uid, 1, 0, tile_size=32)
        with pytest.raises(N.VhxError):
            m.broadcast_tree(None)  # rank 0 must pass the tree
        with pytest.raises(N.VhxError):
            m.render(vhx.glass_camera(64, 64, 64))  # rank 0 without a framebuffer (and no tree yet)
        m.broadcast_tree(flat)
        m.close()
    finally:
        rt.close()


def test_shared_contexts_frames_in_flight(oracle):
    """vhx_create_shared: contexts tracing one uploaded tree on their own streams, frames in flight, each frame equal to
    the oracle's; uploads and updates through a shared context are refused; the tree outlives its owner."""
    import torch
    flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 256, 4)
    W, H = 320, 200
    cams = [vhx.glass_camera(256, W, H, angle=40.0 + 0.05 * k, target=(128.0, 128.0, 128.0)) for k in range(6)]
    refs = [oracle.trace_primary(flat, c, 0, 0, W, H, fields=("rgba", "depth", "value")) for c in cams]
    owner = vhx.Raytracer(0)
    owner.upload(flat)
    ctxs = [owner] + [owner.shared() for _ in range(2)]
    streams = [torch.cuda.Stream() for _ in ctxs]
    for r, s in zip(ctxs, streams):
        r.set_stream(s.cuda_stream)
    outs = [{"rgba": torch.zeros(W * H, dtype=torch.int32, device="cuda"),
             "depth": torch.zeros(W * H, dtype=torch.float32, device="cuda"),
             "value": torch.zeros(W * H, dtype=torch.int32, device="cuda")} for _ in cams]
    for k, (c, o) in enumerate(zip(cams, outs)):  # six frames, three in flight
        ctxs[k % 3].trace_primary(c, out=o)
    torch.cuda.synchronize()
    for k, (o, ref) in enumerate(zip(outs, refs)):
        for f in ("rgba", "depth", "value"):
            assert np.array_equal(o[f].cpu().numpy().view(np.uint32), ref[f].view(np.uint32)), (k, f)
    with pytest.raises(N.VhxError):
        ctxs[1].update_range(N.VHX_BUF_VOXELS, 0, flat.voxels[:4])
    with pytest.raises(N.VhxError):
        N.check(N.lib().vhx_upload_tree(ctxs[2]._h, __import__("ctypes").byref(flat.desc)), ctxs[2]._h)
    owner.close()  # the shared contexts keep the tree alive
    got = ctxs[2].trace_primary(cams[0], fields=("rgba",))
    assert np.array_equal(got["rgba"], refs[0]["rgba"])
    for r in ctxs[1:]:
        r.close()
