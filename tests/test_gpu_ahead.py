"""The ahead stream of a lone frame: the rays that were long in the previous frame on the context are
traced on a second stream from the start of the frame while pass 0 skips them. Only the schedule changes: every frame is
bit-identical to the oracle / the golden digests, whatever the prediction (the same view, a different view, a different
frame size, thresholds and caps that make every abandoned ray or none an ahead ray, one ray per wave)."""
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


@pytest.mark.parametrize("tune", ["ahead=1", "ahead=1;ahead_min=1", "ahead=1;ahead_min=65;ahead_rpw=1",
                                  "ahead=1;ahead_min=1;ahead_cap=7", "ahead=1;ahead_min=4000000", "ahead=0"])
def test_ahead_frames_vs_oracle(oracle, tune):
    size, W, H = 256, 320, 200
    flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, size, 4)
    cams = [vhx.glass_camera(size, W, H, angle=40.0 + 0.3 * k, target=(size / 2,) * 3) for k in range(3)]
    small = vhx.glass_camera(size, 200, 136, target=(size / 2,) * 3)
    refs = [oracle.trace_primary(flat, c, 0, 0, W, H) for c in cams]
    ref_small = oracle.trace_primary(flat, small, 0, 0, 200, 136)
    rt = vhx.Raytracer(0, tune=tune)
    try:
        rt.upload(flat)
        # the lone-frame schedule (one context, nothing else in flight): the ahead stream from the second frame on
        for rep in range(2):
            for k, c in enumerate(cams):
                assert rt.pass_budgets()[1] in ("idle", "fixed")
                assert_same(rt.trace_primary(c), refs[k], f"{tune} view {k} #{rep}")
            assert_same(rt.trace_primary(small), ref_small, f"{tune} other frame size")
            assert_same(rt.trace_primary(cams[0], count_bytes=True), refs[0], f"{tune} byte counting")
        rt.set_pass_budgets((3, 20))  # a fixed multi-pass schedule with the ahead stream forced on
        for k, c in enumerate(cams):
            assert_same(rt.trace_primary(c), refs[k], f"{tune} fixed budgets view {k}")
    finally:
        rt.close()


def test_ahead_bench_frame_matches_golden():  # (ahead forced on below)
    """The lone bench frame (3840x2160, scene S 1024^3 bd 4) three times on one context (the ahead stream is on in the
    lone-frame schedule): the first frame records the prediction, the next two trace their long rays ahead; every field
    equals the golden digests."""
    name = "c3_1024_bd4_3840x2160"
    rt = vhx.Raytracer(0, tune="ahead=1")
    try:
        rt.upload(vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 1024, 4))
        cam = vhx.glass_camera(1024, 3840, 2160, target=(512.0,) * 3)
        for rep in range(3):
            f = rt.trace_primary(cam, fields=FIELDS)
            assert rt.pass_budgets() == ((64,), "idle")
            bad = [k for k in FIELDS if digest(f[k]) != META[name]["sha256"][k]]
            assert not bad, f"frame {rep}: fields {bad} differ from the golden frame"
    finally:
        rt.close()
