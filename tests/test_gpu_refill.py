"""Lane refill of the unbounded last pass (k_trace_refill): persistent waves resume a new queued ray in
a lane as soon as enough lanes are idle. Only which lane traces a ray changes, so rays, frames and shadow rays equal
the oracle at every refill threshold (1: a take per idle lane; 64: only fully idle waves take) and pass ladder, and the
lone bench frame equals the golden digests of every field."""
import json
import os

import numpy as np
import pytest

import voxelhex_amd as vhx
from tests.golden.make_frame_fixture import FIELDS, digest
from tests.test_gpu_parity import _device_hits, assert_same, rand_rays
from voxelhex_amd import _native as N

pytestmark = pytest.mark.gpu

META = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "frames.json")))


@pytest.mark.parametrize("tune", ["refill=1", "refill=8", "refill=32", "refill=64", "refill=32;qsort=0",
                                  "refill=16;qwaves=64"])
def test_refill_vs_oracle(oracle, tune):
    rt = vhx.Raytracer(0, tune=tune)
    try:
        flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 256, 4)
        rt.upload(flat)
        rng = np.random.default_rng(5)
        o, d = rand_rays(rng, 256, 8000)
        cam = vhx.glass_camera(256, 200, 120, target=(128.0, 128.0, 128.0))
        ref_rays = oracle.trace_rays(flat, o, d)
        ref_frame = oracle.trace_primary(flat, cam, 0, 0, 200, 120)
        for budgets in (None, (64,), (1,), (2, 9, 30), (16,)):
            if budgets is not None:
                rt.set_pass_budgets(budgets)
            assert_same(rt.trace_rays(o, d), ref_rays, f"rays {tune} {budgets}")
            for rep in range(2):  # the pass counter and the queue are reused by the next frame
                assert_same(rt.trace_primary(cam), ref_frame, f"frame {tune} {budgets} #{rep}")
    finally:
        rt.close()


@pytest.mark.parametrize("bd,size", [(1, 64), (2, 128), (8, 128), (16, 256), (32, 128)])
def test_refill_brick_dims(oracle, bd, size):
    rt = vhx.Raytracer(0, tune="refill=24")
    try:
        flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, size, bd)
        rt.upload(flat)
        cam = vhx.glass_camera(size, 160, 104, target=(size / 2,) * 3)
        ref = oracle.trace_primary(flat, cam, 0, 0, 160, 104)
        for budgets in ((3,), (2, 9, 30)):
            rt.set_pass_budgets(budgets)
            assert_same(rt.trace_primary(cam), ref, f"bd {bd} {budgets}")
    finally:
        rt.close()


def test_refill_shadow_rays(oracle):
    """Shadow rays (config 5) go through the same unbounded pass: flags and darkened rgba equal the oracle's."""
    rt = vhx.Raytracer(0, tune="refill=32")
    try:
        size, W, H = 256, 192, 112
        flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, size, 4)
        rt.upload(flat)
        cam = vhx.glass_camera(size, W, H, target=(size / 2,) * 3)
        light = (float(size),) * 3
        ref_primary = oracle.trace_primary(flat, cam, 0, 0, W, H, fields=("value", "impact", "normal", "rgba"))
        ref = oracle.trace_shadows(flat, light, ref_primary)
        for budgets in ((64,), (2, 9, 30)):
            rt.set_pass_budgets(budgets)
            hits = rt.trace_primary(cam, out=_device_hits(W * H))
            res = rt.trace_shadows(light, hits)
            rt.sync()
            sh = res["shadowed"].cpu().numpy().view(np.uint32)
            assert np.array_equal(sh, ref["shadowed"]), f"{budgets}: shadow flags differ at {np.count_nonzero(sh != ref['shadowed'])}"
            assert np.array_equal(hits["rgba"].cpu().numpy().view(np.uint32), ref["rgba"]), f"{budgets}: rgba"
    finally:
        rt.close()


def test_refill_bench_frame_matches_golden():
    """The lone bench frame (3840x2160, scene S 1024^3 bd 4) with refill in its unbounded pass: every field equals the
    golden digests, three frames in a row."""
    name = "c3_1024_bd4_3840x2160"
    rt = vhx.Raytracer(0, tune="refill=32")
    try:
        rt.upload(vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 1024, 4))
        cam = vhx.glass_camera(1024, 3840, 2160, target=(512.0,) * 3)
        for rep in range(3):
            f = rt.trace_primary(cam, fields=FIELDS)
            bad = [k for k in FIELDS if digest(f[k]) != META[name]["sha256"][k]]
            assert not bad, f"frame {rep}: fields {bad} differ from the golden frame"
    finally:
        rt.close()
