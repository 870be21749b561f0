"""Tail split of the lone-frame schedule's unbounded last pass (k_trace_queue_split): rays handed
from one wave to another in the middle of their traversal -- loop state packed into overflow slots, taken by waves
that ran out of work -- must give the oracle's results bit for bit (the reference's get_by_ray, cpu.rs:296-458), and
the hand-offs must actually happen (vhx_get_split_stats). The split pass is the non-counting kernel, so these traces
request no byte counts; the counting path keeps k_trace_queue."""
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

# split=1 puts the split on every fixed schedule; more queue waves or one-wave workgroups change how many waves
# wait and how often tracing waves split; few adaptive rays per wave make the main queue itself thin
SPLIT_TUNES = ["split=1", "split=1;qwaves=8192", "split=1;qblock=64;qxcd=0", "split=1;rpw=0,0,0,0;tw=7"]


@pytest.mark.parametrize("tune", SPLIT_TUNES)
def test_split_pass_vs_oracle(oracle, tune):
    rt = vhx.Raytracer(0, tune=tune)
    try:
        flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 256, 4)
        rt.upload(flat)
        rng = np.random.default_rng(23)
        o, d = rand_rays(rng, 256, 20000)
        W, H = 320, 200
        cam = vhx.glass_camera(256, W, H, target=(128.0, 128.0, 128.0))
        ref_rays = oracle.trace_rays(flat, o, d)
        ref_frame = oracle.trace_primary(flat, cam, 0, 0, W, H)
        handed = 0
        for budgets in ((64,), (2, 9, 30), (4, 40), (1,)):
            rt.set_pass_budgets(budgets)
            assert_same(rt.trace_rays(o, d), ref_rays, f"rays {tune} {budgets}")
            h, err = rt.split_stats()
            assert err == 0, f"{err} hand-offs never completed ({tune} {budgets})"
            handed += h
            for rep in range(2):  # the second frame reuses the slots under the next epoch
                assert_same(rt.trace_primary(cam), ref_frame, f"frame {tune} {budgets} #{rep}")
                h, err = rt.split_stats()
                assert err == 0
                handed += h
        assert handed > 0, "no ray was handed over: the split path did not run"
    finally:
        rt.close()


def test_split_shadow_rays_vs_oracle(oracle):
    """Shadow rays (config 5) resume through the same split pass."""
    rt = vhx.Raytracer(0, tune="split=1")
    try:
        size, w, h = 256, 256, 192
        flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, size, 4)
        rt.upload(flat)
        cam = vhx.glass_camera(size, w, h, target=(size / 2,) * 3)
        light = (float(size),) * 3
        ref_primary = oracle.trace_primary(flat, cam, 0, 0, w, h, fields=("value", "impact", "normal", "rgba"))
        ref = oracle.trace_shadows(flat, light, ref_primary)
        for budgets in ((1,), (4, 40)):
            rt.set_pass_budgets(budgets)
            hits = rt.trace_primary(cam, out=_device_hits(w * h))
            res = rt.trace_shadows(light, hits)
            rt.sync()
            _, err = rt.split_stats()
            assert err == 0
            sh = res["shadowed"].cpu().numpy().view(np.uint32)
            assert np.array_equal(sh, ref["shadowed"]), f"{budgets}: flags differ at {np.count_nonzero(sh != ref['shadowed'])}"
            assert np.array_equal(hits["rgba"].cpu().numpy().view(np.uint32), ref["rgba"])
    finally:
        rt.close()


def test_lone_bench_frame_splits_and_matches_golden():
    """The adaptive lone frame at the headline size -- 3840x2160 on scene S 1024^3 bd 4, the bench's isolated frame --
    with the split on runs it and equals the golden digests of every field; so does a second frame (next epoch)."""
    name = "c3_1024_bd4_3840x2160"
    rt = vhx.Raytracer(0, tune="split=1")
    try:
        flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 1024, 4)
        rt.upload(flat)
        cam = vhx.glass_camera(1024, 3840, 2160, target=(512.0,) * 3)
        for rep in range(2):
            f = rt.trace_primary(cam, fields=FIELDS)
            handed, err = rt.split_stats()
            budgets, sched = rt.pass_budgets()
            assert sched == "idle" and budgets == (64,)
            assert err == 0 and handed > 0, (handed, err)
            bad = [k for k in FIELDS if digest(f[k]) != META[name]["sha256"][k]]
            assert not bad, f"frame {rep}: fields {bad} differ from the golden frame"
    finally:
        rt.close()
