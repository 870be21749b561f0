"""The oracle reproduces the committed golden frames (tests/golden/frames.json, made by
tests/golden/make_frame_fixture.py): SHA-256 of every field of the BASELINE config 1-3 frames and their 64x64 crops.
Guards the checker itself against drift; the GPU side is tests/test_gpu_golden.py."""
import json
import os

import numpy as np
import pytest

from tests.golden.make_frame_fixture import CASES, FIELDS, MIP_CASES, crop, digest, frame, mip_frame

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
META = json.load(open(os.path.join(HERE, "frames.json")))
CROPS = np.load(os.path.join(HERE, "frame_crops.npz"))


@pytest.mark.parametrize("name", sorted(CASES))
def test_oracle_matches_golden_frame(oracle, name):
    m = META[name]
    scene, size, bd, W, H = CASES[name]
    assert (m["scene"], m["size"], m["brick_dim"], m["width"], m["height"]) == (scene, size, bd, W, H)
    _, _, f = frame(oracle, scene, size, bd, W, H)
    assert {k: digest(f[k]) for k in FIELDS} == m["sha256"]
    for k in ("value", "depth", "rgba"):
        assert np.array_equal(crop(f[k], W, H).view(np.uint32), CROPS[f"{name}__{k}"].view(np.uint32)), k


@pytest.mark.parametrize("name", sorted(MIP_CASES))
def test_oracle_matches_golden_mip_view(oracle, name):
    m = META[name]
    scene, size, bd, W, H, depth = MIP_CASES[name]
    assert m["mip_lod_depth"] == depth
    _, _, f = mip_frame(oracle, scene, size, bd, W, H, depth)
    assert {k: digest(f[k]) for k in FIELDS} == m["sha256"]
    for k in ("value", "depth", "rgba"):
        assert np.array_equal(crop(f[k], W, H).view(np.uint32), CROPS[f"{name}__{k}"].view(np.uint32)), k
