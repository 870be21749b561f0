"""Streaming on the device with the tree edited mid-stream (handle_tree_updates, src/raytracing/bevy/streaming/mod.rs:
35-286, restated in voxelhex_amd/csrc/stream.cpp): every frame's ranged writes go to HBM as one vhx_update_ranges
call; after each round of edits the GPU traces the device view exactly like the oracle traces the host mirror and like
the edited tree, inside the streamed region."""
import numpy as np
import pytest

import voxelhex_amd as vhx
from voxelhex_amd import _native as N
from tests.test_gpu_parity import assert_same
from tests.test_streaming import FIELDS, _edit, _rays_in_box, _tree

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("size,bd", [(64, 4), (128, 8)])
def test_tree_edits_mid_stream_on_device(oracle, size, bd):
    t = _tree(size, bd)
    rt = vhx.Raytracer(0)
    try:
        S = float(size)
        s = vhx.StreamingView(t, rt, (S / 2, S / 2, S / 2), S)
        s.set_rates(8, 32, 10)
        for _ in range(3):  # a few frames into the stream, then the first edits
            s.upload()
        rng = np.random.default_rng(bd)
        lo, hi = np.full(3, 1.0), np.full(3, S - 1)
        for rnd in range(3):
            _edit(t, rng, size)
            stats, frames, _ = s.upload_all()
            assert stats["pending"] == 0
            o, d = _rays_in_box(rng, lo, hi, 12000)
            got = rt.trace_rays(o, d, fields=FIELDS, count_bytes=True)
            assert_same(got, oracle.trace_rays(s.view(), o, d, fields=FIELDS, count_bytes=True),
                        f"device view vs host mirror, round {rnd}")
            full = oracle.trace_rays(t.flatten(), o, d, fields=FIELDS)
            assert_same({k: got[k] for k in FIELDS}, full, f"device view vs edited tree, round {rnd}")
            assert (full["value"] != N.VHX_EMPTY).sum() > 500
        s.close()
    finally:
        rt.close()


def test_streamed_mips_on_device_match_the_mirror(oracle):
    """A MIP-enabled stream on a device context: the device view (ranged writes + vhx_set_node_mips from the stream)
    traces exactly like the oracle on the host mirror with the mirror's node MIPs, before and after a viewport move."""
    from tests.test_streaming import FIELDS, _mip_stream, _rays_in_box
    rt = vhx.Raytracer(0)
    try:
        t, s = _mip_stream(rt)
        rng = np.random.default_rng(9)
        for step in range(2):
            o, d = _rays_in_box(rng, np.array([0.0, 0.0, 0.0]), np.array([256.0, 256.0, 256.0]), 20000)
            got = rt.trace_rays(o, d, fields=FIELDS)
            with oracle.node_mips(s.node_mips()):
                ref = oracle.trace_rays(s.view(), o, d, fields=FIELDS)
            assert_same(got, ref, f"streamed MIP view, step {step}")
            assert (ref["value"] != N.VHX_EMPTY).mean() > 0.2
            s.set_viewport((180.0, 170.0, 160.0), 40.0)
            s.upload_all()
        s.close()
    finally:
        rt.close()
