"""Pass 0's per-wave lists in the queue order (docs/DESIGN_LOG.md §16.6): a single frame on the frames-in-flight schedule
(adaptive=0: the busy ladder, qorder 38, so pass 0 lists its abandoned rays itself) equals the same frame on the lone
schedule (output order, per-pixel flags) and the oracle, at frame sizes that leave partial 64x64 tiles, partial 16x16
blocks and partial 8x8 waves; and the flag path (p0lists=0) equals both."""
import numpy as np
import pytest

import voxelhex_amd as vhx
from voxelhex_amd import _native as N

FIELDS = ("value", "cell", "voxel", "impact", "normal", "depth", "rgba")


@pytest.mark.gpu
@pytest.mark.parametrize("W,H", [(1, 1), (97, 33), (17, 250), (320, 180), (641, 65), (1920, 1080)])
def test_listed_pass0_equals_flags_and_lone(W, H):
    flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 256, 4)
    cam = vhx.glass_camera(256, W, H, target=(128.0,) * 3)
    outs = {}
    for tag, tune in (("lone", None), ("lists", "adaptive=0"), ("flags", "adaptive=0;p0lists=0")):
        rt = vhx.Raytracer(0, tune=tune)
        try:
            rt.upload(flat)
            outs[tag] = rt.trace_primary(cam, fields=FIELDS)
        finally:
            rt.close()
    for tag in ("lists", "flags"):
        for f in FIELDS:
            a, b = outs[tag][f].view(np.uint32), outs["lone"][f].view(np.uint32)
            assert np.array_equal(a, b), f"{tag} {W}x{H}: {f} differs at {int((a != b).sum())} entries"


@pytest.mark.gpu
def test_listed_pass0_vs_oracle(oracle):
    flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 64, 4)
    cam = vhx.glass_camera(64, 211, 97, angle=40.3, target=(32.0,) * 3)
    rt = vhx.Raytracer(0, tune="adaptive=0")
    try:
        rt.upload(flat)
        got = rt.trace_primary(cam, fields=FIELDS)
    finally:
        rt.close()
    ref = oracle.trace_primary(flat, cam, 0, 0, cam.width, cam.height, fields=FIELDS)
    for f in FIELDS:
        assert np.array_equal(got[f].view(np.uint32), ref[f].view(np.uint32)), f
    assert (got["value"] != N.VHX_EMPTY).sum() > 1000
