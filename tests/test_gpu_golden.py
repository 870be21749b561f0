"""GPU frames against the committed golden frames (tests/golden/frames.json: SHA-256 of every field of the oracle's
BASELINE config 1-3 frames, pinned by tests/test_golden_frames.py): bit-exact without running the oracle, for the
default four-pass schedule and one unbounded pass."""
import json
import os

import pytest

import voxelhex_amd as vhx
from tests.golden.make_frame_fixture import CASES, FIELDS, MIP_CASES, digest, mip_view
from tests.test_gpu_parity import DEFAULT_BUDGETS

pytestmark = pytest.mark.gpu

META = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "frames.json")))


@pytest.mark.parametrize("name", sorted(CASES))
def test_gpu_frame_matches_golden(gpu, name):
    scene, size, bd, W, H = CASES[name]
    flat = vhx.FlatTree.build_scene(scene, size, bd)
    gpu.upload(flat)
    cam = vhx.glass_camera(size, W, H, target=(size / 2,) * 3)
    try:
        for budgets in (DEFAULT_BUDGETS, ()):
            gpu.set_pass_budgets(budgets)
            f = gpu.trace_primary(cam, fields=FIELDS)
            got = {k: digest(f[k]) for k in FIELDS}
            bad = [k for k in FIELDS if got[k] != META[name]["sha256"][k]]
            assert not bad, f"{name} budgets {budgets}: fields {bad} differ from the golden frame"
    finally:
        gpu.set_pass_budgets(DEFAULT_BUDGETS)


@pytest.mark.parametrize("name", sorted(MIP_CASES))
def test_gpu_mip_view_matches_golden(name):
    scene, size, bd, W, H, depth = MIP_CASES[name]
    flat = mip_view(scene, size, bd, depth)
    rt = vhx.Raytracer(0)
    try:
        rt.upload(flat)
        rt.set_node_mips(flat.node_mips)
        cam = vhx.glass_camera(size, W, H, target=(size / 2,) * 3)
        f = rt.trace_primary(cam, fields=FIELDS)
        bad = [k for k in FIELDS if digest(f[k]) != META[name]["sha256"][k]]
        assert not bad, f"{name}: fields {bad} differ from the golden MIP view"
    finally:
        rt.close()
