"""The one-launch frame (k_trace_frame): a framebuffer frame's whole pass ladder in one persistent
launch, rays handed from pass to pass inside it (XCD-local queues). Only the schedule changes: every frame equals the
oracle / the golden digests for every ladder (down to a one-step first pass, every ray handed over many times), every
brick_dim, repeated frames on one context (slot tags by frame epoch), a frame size that grows the slots, and frames
interleaved with the per-pass launches."""
import json
import os

import numpy as np
import pytest

import voxelhex_amd as vhx
from tests.golden.make_frame_fixture import FIELDS, digest
from tests.test_gpu_parity import assert_same
from voxelhex_amd import _native as N

pytestmark = pytest.mark.gpu

META = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "frames.json")))


@pytest.mark.parametrize("budgets", [None, (24, 72, 216, 648), (3, 20), (1,), (1, 2, 3, 4, 5, 6)])
def test_frame1_vs_oracle(oracle, budgets):
    size, W, H = 256, 320, 200
    flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, size, 4)
    cams = [vhx.glass_camera(size, W, H, angle=40.0 + 0.3 * k, target=(size / 2,) * 3) for k in range(3)]
    refs = [oracle.trace_primary(flat, c, 0, 0, W, H) for c in cams]
    rt = vhx.Raytracer(0, tune="one=1")
    try:
        rt.upload(flat)
        if budgets is not None:
            rt.set_pass_budgets(budgets)
        for rep in range(2):  # the same slots again under the next frames' epochs
            for k, c in enumerate(cams):
                assert_same(rt.trace_primary(c), refs[k], f"{budgets} view {k} #{rep}")
        # byte counting keeps the per-pass launches; the next one-launch frame still matches
        assert_same(rt.trace_primary(cams[0], count_bytes=True), refs[0], f"{budgets} byte counting")
        assert_same(rt.trace_primary(cams[1]), refs[1], f"{budgets} after a per-pass frame")
    finally:
        rt.close()


@pytest.mark.parametrize("bd,size", [(1, 64), (2, 128), (8, 128), (16, 256), (32, 128)])
def test_frame1_brick_dims(oracle, bd, size):
    W, H = 200, 136
    flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, size, bd)
    cam = vhx.glass_camera(size, W, H, target=(size / 2,) * 3)
    ref = oracle.trace_primary(flat, cam, 0, 0, W, H)
    rt = vhx.Raytracer(0, tune="one=1")
    try:
        rt.upload(flat)
        for budgets in (None, (2, 9, 30)):
            if budgets is not None:
                rt.set_pass_budgets(budgets)
            assert_same(rt.trace_primary(cam), ref, f"bd {bd} {budgets}")
        small = vhx.glass_camera(size, 96, 64, target=(size / 2,) * 3)  # a smaller frame in the same slots
        assert_same(rt.trace_primary(small), oracle.trace_primary(flat, small, 0, 0, 96, 64), f"bd {bd} small")
    finally:
        rt.close()


def test_frame1_bench_frame_matches_golden():
    """The lone bench frame (3840x2160, scene S 1024^3 bd 4) in one launch, under the lone-frame ladder and the
    frames-in-flight ladder, three times each: every field equals the golden digests."""
    name = "c3_1024_bd4_3840x2160"
    rt = vhx.Raytracer(0, tune="one=1")
    try:
        rt.upload(vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 1024, 4))
        cam = vhx.glass_camera(1024, 3840, 2160, target=(512.0,) * 3)
        for budgets in (None, (24, 72, 216, 648)):
            if budgets is not None:
                rt.set_pass_budgets(budgets)
            for rep in range(3):
                f = rt.trace_primary(cam, fields=FIELDS)
                bad = [k for k in FIELDS if digest(f[k]) != META[name]["sha256"][k]]
                assert not bad, f"{budgets} frame {rep}: fields {bad} differ from the golden frame"
    finally:
        rt.close()


def test_frame1_frames_in_flight(oracle):
    """One-launch frames on several contexts of one tree at once (each its own slots and counters)."""
    size, W, H = 256, 256, 160
    flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, size, 4)
    cams = [vhx.glass_camera(size, W, H, angle=40.0 + 0.2 * k, target=(size / 2,) * 3) for k in range(6)]
    refs = [oracle.trace_primary(flat, c, 0, 0, W, H, fields=("rgba", "depth")) for c in cams]
    import torch
    owner = vhx.Raytracer(0, tune="one=1")
    try:
        owner.upload(flat)
        ctxs = [owner] + [owner.shared() for _ in range(2)]
        for r in ctxs[1:]:
            r.set_tuning("one=1")
        outs = [{"rgba": torch.zeros(W * H, dtype=torch.int32, device="cuda"),
                 "depth": torch.zeros(W * H, dtype=torch.float32, device="cuda")} for _ in cams]
        torch.cuda.synchronize()
        for k, c in enumerate(cams):
            ctxs[k % 3].trace_primary(c, out=outs[k])
        for r in ctxs:
            r.sync()
        for k in range(len(cams)):
            got = {"rgba": outs[k]["rgba"].cpu().numpy().view(np.uint32), "depth": outs[k]["depth"].cpu().numpy()}
            assert_same(got, {n: refs[k][n] for n in ("rgba", "depth")}, f"frame {k}")
        for r in ctxs[1:]:
            r.close()
    finally:
        owner.close()
