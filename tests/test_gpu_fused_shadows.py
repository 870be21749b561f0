"""Fused hard shadows (vhx_set_shadow_light; BASELINE config 5): with a light set, a lane that
finishes a primary ray with a hit goes on with the hit's shadow ray in the same pass, and leftover shadow rays travel
the queue passes tagged. The frame must equal vhx_trace_primary followed by vhx_trace_shadows bit for bit -- value,
depth, RGBA (darkened where shadowed) and the shadowed flags -- under the frames-in-flight schedule (fused), the lone
frame's schedule (the shadows traced after the primary rays), batches of frames and tile sets, every brick_dim, and
schedules that abandon rays at every step; the separate path is itself pinned by the oracle
(tests/test_gpu_parity.py::test_shadow_rays_vs_oracle, the full-size config-5 frame)."""
import numpy as np
import pytest

import voxelhex_amd as vhx
from voxelhex_amd import _native as N

pytestmark = pytest.mark.gpu

FIELDS = ("value", "depth", "rgba", "shadowed")


def _outs(n):
    import torch
    d = "cuda"
    return {"value": torch.full((n,), -1, dtype=torch.int32, device=d),
            "impact": torch.zeros((n, 3), dtype=torch.float32, device=d),
            "normal": torch.zeros((n, 3), dtype=torch.float32, device=d),
            "depth": torch.zeros(n, dtype=torch.float32, device=d),
            "rgba": torch.zeros(n, dtype=torch.int32, device=d),
            "shadowed": torch.full((n,), 7, dtype=torch.int32, device=d)}


def _host(o):
    return {k: o[k].cpu().numpy().view(np.uint32).reshape(-1) for k in FIELDS}


def _separate(rt, cam, light, **kw):
    import torch
    n = cam.width * cam.height if not kw else None
    if kw:
        T = kw["tile_size"]
        nt = ((cam.width + T - 1) // T) * ((cam.height + T - 1) // T)
        n = max(0, (nt - kw["tile_start"] + kw["tile_stride"] - 1) // kw["tile_stride"]) * T * T
    o = _outs(n)
    torch.cuda.synchronize()
    rt.trace_primary(cam, out=o, **kw)
    rt.trace_shadows(light, o, shadowed=o["shadowed"])
    rt.sync()
    return _host(o)


def _assert_same(a, b, what):
    for f in FIELDS:
        bad = int(np.count_nonzero(a[f] != b[f]))
        assert bad == 0, f"{what}: field {f} differs at {bad} entries"


@pytest.mark.parametrize("size,bd", [(64, 4), (256, 4), (128, 8), (32, 2), (16, 1)])
@pytest.mark.parametrize("tune", ["adaptive=0", "adaptive=0;budgets=1,3,7,15", "adaptive=0;sparse=60,60,60",
                                  "adaptive=0;sbudget=40", "adaptive=0;sbudget=1", None])
def test_fused_frame_equals_primary_then_shadows(size, bd, tune):
    """adaptive=0 keeps the frames-in-flight schedule for a lone frame, so pass 0 lists its rays and the shadows fuse;
    tune None is the lone frame's schedule, where they are traced after the primary rays."""
    import torch
    flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, size, bd)
    light = (float(size),) * 3
    cams = [vhx.glass_camera(size, 200, 136, angle=40.0 + 0.4 * k, target=(size / 2,) * 3) for k in range(2)]
    sep = vhx.Raytracer(0, tune=tune)
    fus = vhx.Raytracer(0, tune=tune)
    try:
        sep.upload(flat)
        fus.upload(flat)
        fus.set_shadow_light(light)
        for k, cam in enumerate(cams):
            ref = _separate(sep, cam, light)
            o = _outs(cam.width * cam.height)
            torch.cuda.synchronize()
            fus.trace_primary(cam, out=o)
            fus.sync()
            got = _host(o)
            _assert_same(got, ref, f"{size}^3 bd {bd} tune {tune} camera {k}")
            assert (ref["shadowed"] == 1).sum() > 0 and (ref["value"] != N.VHX_EMPTY).sum() > 100
    finally:
        sep.close()
        fus.close()


def test_fused_batches_and_tile_sets():
    """vhx_trace_primary_batch and vhx_trace_tiles_batch with a light (always the batch schedule: fused) against the
    separate traces of each frame; tile padding entries stay untouched in both."""
    import torch
    size, W, H, T = 256, 200, 136, 64
    flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, size, 4)
    light = (float(size),) * 3
    cams = [vhx.glass_camera(size, W, H, angle=40.0 + 0.3 * k, target=(size / 2,) * 3) for k in range(3)]
    sep = vhx.Raytracer(0)
    fus = vhx.Raytracer(0)
    try:
        sep.upload(flat)
        fus.upload(flat)
        fus.set_shadow_light(light)
        outs = [_outs(W * H) for _ in cams]
        torch.cuda.synchronize()
        fus.trace_primary_batch(cams, outs)
        fus.sync()
        for k, cam in enumerate(cams):
            _assert_same(_host(outs[k]), _separate(sep, cam, light), f"batch frame {k}")
        starts, stride = (0, 1, 2), 3
        nt = ((W + T - 1) // T) * ((H + T - 1) // T)
        sizes = [max(0, (nt - s + stride - 1) // stride) * T * T for s in starts]
        touts = [_outs(n) for n in sizes]
        torch.cuda.synchronize()
        fus.trace_tiles_batch(cams, T, starts, stride, touts)
        fus.sync()
        for k, cam in enumerate(cams):
            ref = _separate(sep, cam, light, tile_size=T, tile_start=starts[k], tile_stride=stride,
                            layout=N.VHX_LAYOUT_TILES)
            got = _host(touts[k])
            pad = ref["value"] == N.VHX_EMPTY  # padding and misses: shadowed 0 from the separate path's clear
            got["shadowed"] = np.where(pad & (got["shadowed"] == 7), 0, got["shadowed"])
            _assert_same(got, ref, f"tile set {k}")
    finally:
        sep.close()
        fus.close()


def test_fused_full_size_config5_frame():
    """The config-5 workload (3840x2160, scene S 1024^3 bd 4, light (S, S, S)) as a fused batch of two frames against
    the separate primary + shadow traces."""
    import torch
    size, W, H = 1024, 3840, 2160
    flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, size, 4, threads=16)
    light = (float(size),) * 3
    cam = vhx.glass_camera(size, W, H, target=(size / 2,) * 3)
    sep = vhx.Raytracer(0)
    fus = vhx.Raytracer(0)
    try:
        sep.upload(flat)
        fus.upload(flat)
        fus.set_shadow_light(light)
        ref = _separate(sep, cam, light)
        outs = [_outs(W * H) for _ in range(2)]
        torch.cuda.synchronize()
        fus.trace_primary_batch([cam, cam], outs)
        fus.sync()
        for k in range(2):
            _assert_same(_host(outs[k]), ref, f"config-5 frame {k}")
        assert (ref["shadowed"] == 1).sum() > 100000
    finally:
        sep.close()
        fus.close()


def test_fused_shadow_argument_errors(gpu):
    import torch
    gpu.upload(vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 64, 4))
    gpu.set_shadow_light((64.0, 64.0, 64.0))
    cam = vhx.glass_camera(64, 32, 32, target=(32.0,) * 3)
    o = _outs(32 * 32)
    del o["shadowed"]
    torch.cuda.synchronize()
    with pytest.raises(N.VhxError):
        gpu.trace_primary(cam, out=o)
    with pytest.raises(N.VhxError):
        gpu.set_shadow_light((float("nan"), 0.0, 0.0))
    gpu.set_shadow_light(None)
    gpu.trace_primary(cam, out=o)  # off again: the usual outputs suffice
    gpu.sync()
