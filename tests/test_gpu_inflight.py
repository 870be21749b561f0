"""The headline configuration checked as it is timed: F contexts sharing the 1024^3 bd-4 tree
(vhx_create_shared), each on its own stream with a hardware queue of its own (tests/conftest.py raises
GPU_MAX_HW_QUEUES before HIP starts), frames in flight on every stream at once, 3840x2160; F = 16 is the bench's
default, F = 8 the round-2/3 setting.

Every in-flight frame of the golden camera must equal tests/golden/frames.json `c3_1024_bd4_3840x2160` (the oracle's
frame, SHA-256 per field); frames of a second camera interleaved with them on the same contexts must equal the owner
context tracing that camera alone. A cross-stream race (shared queues, counters or state of one context read by
another) shows up as a digest mismatch.
"""
import json
import os

import numpy as np
import pytest

import voxelhex_amd as vhx
from tests.golden.make_frame_fixture import digest
from voxelhex_amd import _native as N

pytestmark = pytest.mark.gpu

META = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "frames.json")))
CASE = "c3_1024_bd4_3840x2160"


def _outs(n, dev):
    import torch
    return {"value": torch.zeros(n, dtype=torch.int32, device=dev),
            "cell": torch.zeros(n, dtype=torch.int32, device=dev),
            "voxel": torch.zeros((n, 3), dtype=torch.int32, device=dev),
            "impact": torch.zeros((n, 3), dtype=torch.float32, device=dev),
            "normal": torch.zeros((n, 3), dtype=torch.float32, device=dev),
            "depth": torch.zeros(n, dtype=torch.float32, device=dev),
            "rgba": torch.zeros(n, dtype=torch.int32, device=dev)}


@pytest.mark.parametrize("F", [8, 16])
def test_frames_in_flight_match_golden(F):
    import torch
    m = META[CASE]
    size, W, H = m["size"], m["width"], m["height"]
    assert int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) >= F + 1, "conftest.py sets GPU_MAX_HW_QUEUES"
    flat = vhx.FlatTree.build_scene(m["scene"], size, m["brick_dim"], threads=min(16, os.cpu_count() or 1))
    cam_a = vhx.glass_camera(size, W, H, target=(size / 2,) * 3)  # the golden camera
    cam_b = vhx.glass_camera(size, W, H, angle=40.5, target=(size / 2,) * 3)
    owner = vhx.Raytracer(0)
    ctxs = [owner]
    try:
        owner.upload(flat)
        ctxs += [owner.shared() for _ in range(F - 1)]
        dev = torch.device("cuda", 0)
        streams = [torch.cuda.ExternalStream(r.stream(), device=dev) for r in ctxs]  # each context's own stream
        outs = [_outs(W * H, dev) for _ in ctxs]
        torch.cuda.synchronize()  # the zero fills (torch's stream) complete before the context streams write
        ref_b = owner.trace_primary(cam_b, fields=("rgba", "depth", "value"))  # one frame alone
        for rnd in range(2):
            # round 0: even contexts trace the golden camera, odd ones camera B; round 1 swaps them. Every context's
            # frame is launched before any is waited for: eight frames in flight on eight streams
            cams = [(cam_a if (f + rnd) % 2 == 0 else cam_b) for f in range(F)]
            for r, c, o in zip(ctxs, cams, outs):
                r.trace_primary(c, out=o)
            # the adaptive schedule (vhx.h, vhx_get_pass_budgets): the first frame of a round is submitted with nothing
            # in flight (the lone-frame schedule), every later one while the first is still running (a 3840x2160
            # frame takes > 1 ms; the frames-in-flight schedule) -- and the frames are the same either way
            sched = [r.pass_budgets() for r in ctxs]
            assert sched[0] == ((64,), "idle"), sched[0]
            assert all(sc == ((32, 128, 768), "busy") for sc in sched[1:]), sched
            for s in streams:
                s.synchronize()
            for f, (c, o) in enumerate(zip(cams, outs)):
                if c is cam_a:
                    got = {k: digest(o[k].cpu().numpy().view(np.uint32)) for k in m["sha256"]}
                    bad = [k for k in m["sha256"] if got[k] != m["sha256"][k]]
                    assert not bad, f"round {rnd} context {f}: fields {bad} differ from the golden frame"
                else:
                    for k in ("rgba", "depth", "value"):
                        a = o[k].cpu().numpy().view(np.uint32)
                        assert np.array_equal(a, ref_b[k].view(np.uint32)), \
                            f"round {rnd} context {f}: {k} differs from the lone frame at {(a != ref_b[k].view(np.uint32)).sum()}"
    finally:
        for r in ctxs[1:]:
            r.close()
        owner.close()
