"""Early tail of lone frames (vhx_ctx::tail_*, vhx_tail_info; VERDICT r05 next 5, the reference's call shape
VhxRenderNode::run, src/raytracing/bevy/pipeline/mod.rs:96-155): a lone frame records the pixels of its longest rays
and the context's next lone frame of the same size traces them from its start on a second stream while pass 0 skips
them. Scheduling only -- every frame must stay bit-identical to the oracle / the golden digests whatever the list
holds: the same camera again (the list exact), another camera (the list stale), a list cut at its cap, every
rays-per-wave setting, a frame size change, frames in flight in between, and tree updates between lone frames."""
import json
import os

import numpy as np
import pytest

import voxelhex_amd as vhx
from tests.golden.make_frame_fixture import CASES, FIELDS, digest
from voxelhex_amd import _native as N

pytestmark = pytest.mark.gpu

META = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "frames.json")))


def _u32(f):
    return {k: np.ascontiguousarray(v).view(np.uint32) for k, v in f.items()}


def _same(a, b, what):
    for k in b:
        x, y = a[k].reshape(-1), b[k].reshape(-1)
        bad = int(np.count_nonzero(x != y))
        assert bad == 0, f"{what}: field {k} differs at {bad} entries"


@pytest.mark.parametrize("tune", ["tail=1", "tail=1;tail_min=65", "tail=1;tail_min=65;tail_cap=100",
                                  "tail=1;tail_min=100;tail_rpw=1", "tail=1;tail_min=100;tail_rpw=64;tail_prio=3",
                                  "tail=1;tail_min=1;tail_cap=1000000", "tail=0"])
def test_tail_frames_vs_oracle(oracle, tune):
    size, W, H = 256, 320, 240
    flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, size, 4)
    cams = [vhx.glass_camera(size, W, H, angle=40.0 + 0.3 * k, target=(size / 2,) * 3) for k in range(2)]
    refs = [_u32(oracle.trace_primary(flat, c, 0, 0, W, H, fields=FIELDS)) for c in cams]
    rt = vhx.Raytracer(0, tune=tune)
    try:
        rt.upload(flat)
        for k, ci in enumerate((0, 0, 1, 0, 0)):  # the list exact, stale (another camera), then exact again
            got = _u32(rt.trace_primary(cams[ci], fields=FIELDS))
            assert rt.pass_budgets()[1] == "idle"
            _same(got, refs[ci], f"tune {tune} frame {k}")
        n, wh = rt.tail_info()
        if tune == "tail=0":
            assert n == 0
        elif tune and "tail_min=" in tune:
            assert wh == (W, H) and n > 0, (n, wh)
            if tune.endswith("tail_cap=100"):
                assert n <= 100
    finally:
        rt.close()


def test_tail_frame_size_change_and_frames_in_flight(oracle):
    """A list of another frame size is not used; busy frames (another context in flight) neither record nor use it;
    a tree update between lone frames leaves the list a mere (stale) prediction."""
    import torch
    size = 256
    flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, size, 4)
    big = vhx.glass_camera(size, 400, 300, target=(size / 2,) * 3)
    small = vhx.glass_camera(size, 320, 240, target=(size / 2,) * 3)
    ref_big = _u32(oracle.trace_primary(flat, big, 0, 0, 400, 300, fields=FIELDS))
    ref_small = _u32(oracle.trace_primary(flat, small, 0, 0, 320, 240, fields=FIELDS))
    rt = vhx.Raytracer(0, tune="tail=1;tail_min=65")
    try:
        rt.upload(flat)
        _same(_u32(rt.trace_primary(big, fields=FIELDS)), ref_big, "big 1")
        assert rt.tail_info()[1] == (400, 300)
        _same(_u32(rt.trace_primary(small, fields=FIELDS)), ref_small, "small after big (list of another size)")
        _same(_u32(rt.trace_primary(small, fields=FIELDS)), ref_small, "small with its list")
        n_small = rt.tail_info()[0]
        assert n_small > 0
        # frames in flight on a shared context: the busy schedule, no recording
        other = rt.shared()
        outs = [{"rgba": torch.zeros(320 * 240, dtype=torch.int32, device="cuda"),
                 "depth": torch.zeros(320 * 240, dtype=torch.float32, device="cuda")} for _ in range(4)]
        torch.cuda.synchronize()
        for k in range(4):
            (rt if k % 2 == 0 else other).trace_primary(small, out=outs[k])
        rt.sync()
        other.sync()
        for o in outs:
            assert np.array_equal(o["rgba"].cpu().numpy().view(np.uint32), ref_small["rgba"])
            assert np.array_equal(o["depth"].cpu().numpy().view(np.uint32), ref_small["depth"])
        other.close()
        # a tree update (a brick's voxels rewritten): the recorded list is now a stale prediction; the frame must equal
        # the same context's frame with the early tail off
        rt.update_range(N.VHX_BUF_VOXELS, 0, np.full(4 * 64, 0xFFFFFFFF, np.uint32))
        got = _u32(rt.trace_primary(small, fields=FIELDS))
        rt.set_tuning("tail=0")
        _same(got, _u32(rt.trace_primary(small, fields=FIELDS)), "after the update")
        rt.set_tuning("tail=1")
        rt.update_range(N.VHX_BUF_VOXELS, 0, np.ascontiguousarray(flat.voxels[:4 * 64]))
        _same(_u32(rt.trace_primary(small, fields=FIELDS)), ref_small, "restored tree")
    finally:
        rt.close()


def test_tail_headline_lone_frames_match_golden():
    """Three lone frames of the headline workload on one context (the second and third trace the recorded tail
    early): every field equals the committed golden digests, and the tail list is not empty."""
    name = "c3_1024_bd4_3840x2160"
    scene, size, bd, W, H = CASES[name]
    flat = vhx.FlatTree.build_scene(scene, size, bd, threads=min(16, os.cpu_count() or 1))
    cam = vhx.glass_camera(size, W, H, target=(size / 2,) * 3)
    rt = vhx.Raytracer(0, tune="tail=1;tail_min=1024;tail_cap=100000;tail_prio=3")
    try:
        rt.upload(flat)
        for k in range(3):
            f = rt.trace_primary(cam, fields=FIELDS)
            bad = [x for x in FIELDS if digest(f[x]) != META[name]["sha256"][x]]
            assert not bad, f"lone frame {k}: fields {bad} differ from the golden frame"
            n, wh = rt.tail_info()
            assert wh == (W, H) and n > 0, (k, n, wh)
    finally:
        rt.close()
