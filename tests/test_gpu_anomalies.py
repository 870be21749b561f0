"""Regression tests for the two GPU anomalies of round 1 (docs/DESIGN_LOG.md §13).

1. Stale staging data: vhx_trace_rays once staged host rays in a stream-ordered hipMallocAsync buffer, and the kernel
   intermittently read data of an earlier call. scripts/anomalies/mallocasync_stale.hip reproduces it on the ROCm 7.2
   runtime without libvhx (profiles/r02/anomalies/). libvhx stages through a context-owned hipMalloc buffer; the test
   below drives that path the way the repro fails most often: host ray batches of changing size and content, each
   call on the other of two streams.
2. The shadow-pass hang of a 1-step first budget, seen while the order-preserving compaction was written: the
   script that debugged it (64^3 scene, 64x48 frame, budgets (), (1,), (4, 40)) runs here on a fresh context.
"""
import numpy as np
import pytest

import voxelhex_amd as vhx
from voxelhex_amd import _native as N
from tests.test_gpu_parity import assert_same, rand_rays

pytestmark = pytest.mark.gpu


def test_host_ray_staging_is_fresh_every_call(gpu, oracle):
    import torch
    flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 64, 4)
    gpu.upload(flat)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    rng = np.random.default_rng(5)
    try:
        for k in range(48):
            n = 1 + (k * 7919) % 5000
            o, d = rand_rays(rng, 64, n)
            gpu.set_stream(streams[k & 1].cuda_stream)
            got = gpu.trace_rays(o, d, fields=("value", "impact", "depth"))
            ref = oracle.trace_rays(flat, o, d)
            assert_same(got, {f: ref[f] for f in ("value", "impact", "depth")}, f"call {k} ({n} rays)")
    finally:
        gpu.set_stream(None)


def test_shadow_one_step_budget_fresh_context(oracle):
    import torch
    flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 64, 4)
    cam = vhx.glass_camera(64, 64, 48, target=(32.0, 32.0, 32.0))
    light = (64.0, 64.0, 64.0)
    ref = oracle.trace_primary(flat, cam, 0, 0, 64, 48, fields=("value", "impact", "normal", "rgba"))
    ref_sh = oracle.trace_shadows(flat, light, ref)
    rt = vhx.Raytracer(0)
    try:
        rt.upload(flat)
        for budgets in ((), (1,), (4, 40), (1, 2, 3, 4)):
            rt.set_pass_budgets(budgets)
            hits = {"value": torch.empty(64 * 48, dtype=torch.int32, device="cuda"),
                    "impact": torch.empty((64 * 48, 3), dtype=torch.float32, device="cuda"),
                    "normal": torch.empty((64 * 48, 3), dtype=torch.float32, device="cuda"),
                    "rgba": torch.empty(64 * 48, dtype=torch.int32, device="cuda")}
            rt.trace_primary(cam, out=hits)
            res = rt.trace_shadows(light, hits)
            rt.sync()
            assert np.array_equal(res["shadowed"].cpu().numpy().view(np.uint32), ref_sh["shadowed"]), budgets
            assert np.array_equal(hits["rgba"].cpu().numpy().view(np.uint32), ref_sh["rgba"]), budgets
    finally:
        rt.close()
