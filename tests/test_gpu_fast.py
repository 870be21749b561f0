"""Depth-prepass fast mode (vhx_set_depth_prepass; SURVEY.md 8f #4, the WGSL path's prepass,
src/raytracing/bevy/viewport_render.wgsl:702-726): opt-in and outside the parity bar. These tests check that it never
touches the exact path and measure how far it strays from it (the pixels whose hit differs; docs/DESIGN_LOG.md §10)."""
import numpy as np
import pytest

import voxelhex_amd as vhx
from voxelhex_amd import _native as N
from tests.test_gpu_parity import assert_same

pytestmark = pytest.mark.gpu


def _differing(a, b):
    return float(np.mean(a["value"] != b["value"]))


@pytest.mark.parametrize("size,bd,W,H,margin,bound", [(256, 4, 1920, 1080, 0.0, 0.05), (256, 4, 1920, 1080, 2.0, 0.05),
                                                     (1024, 4, 3840, 2160, 0.0, 0.05)])
def test_depth_prepass_mode(oracle, size, bd, W, H, margin, bound):
    flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, size, bd)
    cam = vhx.glass_camera(size, W, H, target=(size / 2,) * 3)
    rt = vhx.Raytracer(0)
    try:
        rt.upload(flat)
        fields = ("value", "depth", "rgba")
        exact = rt.trace_primary(cam, fields=fields)
        rt.set_depth_prepass(True, margin)
        fast = rt.trace_primary(cam, fields=fields)
        frac = _differing(fast, exact)
        print(f"depth prepass {size}^3 bd{bd} {W}x{H} margin {margin}: {100 * frac:.3f} % of pixels hit differently")
        assert frac < bound
        # where both hit the same voxel value the fast ray can only have started later, never earlier
        same = (fast["value"] == exact["value"]) & (exact["value"] != N.VHX_EMPTY)
        assert same.mean() > 0.05
        # the exact path is untouched by the mode: byte counting, tiles and ray batches stay exact
        counted = rt.trace_primary(cam, fields=("value",), count_bytes=True)
        ref = oracle.trace_primary(flat, cam, 0, 0, W, H, fields=("value",), count_bytes=True)
        assert_same(counted, ref, "byte counting with the mode on")
        part = rt.trace_primary(cam, tile_size=64, tile_start=1, tile_stride=3, layout=N.VHX_LAYOUT_TILES,
                                fields=("value",))
        rt.set_depth_prepass(False)
        part_exact = rt.trace_primary(cam, tile_size=64, tile_start=1, tile_stride=3, layout=N.VHX_LAYOUT_TILES,
                                      fields=("value",))
        assert np.array_equal(part["value"], part_exact["value"])
        assert_same(rt.trace_primary(cam, fields=fields), exact, "mode off again")
        assert_same({k: exact[k] for k in ("value", "depth")},
                    oracle.trace_primary(flat, cam, 0, 0, W, H, fields=("value", "depth")), "exact = oracle")
    finally:
        rt.close()


def test_depth_prepass_frames_in_flight_and_validation():
    flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 256, 4)
    cam = vhx.glass_camera(256, 640, 360, target=(128.0,) * 3)
    rt = vhx.Raytracer(0)
    try:
        rt.upload(flat)
        with pytest.raises(N.VhxError):
            rt.set_depth_prepass(True, -1.0)
        rt.set_depth_prepass(True, 0.0)
        a = rt.trace_primary(cam, fields=("value",))
        sh = rt.shared()  # a shared context inherits the mode
        b = sh.trace_primary(cam, fields=("value",))
        assert np.array_equal(a["value"], b["value"])
        sh.close()
    finally:
        rt.close()
