"""vhx_trace_primary_batch: n whole frames traced as one pass ladder on one stream must equal n
vhx_trace_primary calls bit for bit, for every brick_dim, every pass schedule and queue order, distinct cameras in one
batch, and the headline 3840x2160 / 1024^3 frame against the committed golden digests (the oracle's frame).
"""
import json
import os

import numpy as np
import pytest

import voxelhex_amd as vhx
from tests.golden.make_frame_fixture import digest
from voxelhex_amd import _native as N

pytestmark = pytest.mark.gpu

FIELDS = ("value", "cell", "voxel", "impact", "normal", "depth", "rgba")
META = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "frames.json")))


def _outs(n, fields=FIELDS):
    import torch
    shapes = {"voxel": (n, 3), "impact": (n, 3), "normal": (n, 3)}
    dts = {"impact": torch.float32, "normal": torch.float32, "depth": torch.float32}
    # filled with a pattern the trace must overwrite everywhere
    return {f: torch.full(shapes.get(f, (n,)), 7, dtype=dts.get(f, torch.int32), device="cuda") for f in fields}


def _host(o):
    return {k: v.cpu().numpy().view(np.uint32) for k, v in o.items()}


def _orbit(size, W, H, n, step=0.05):
    return [vhx.glass_camera(size, W, H, angle=40.0 + k * step, target=(size / 2,) * 3) for k in range(n)]


def _check_batch(rt, cams, what, fields=FIELDS):
    import torch
    n = cams[0].width * cams[0].height
    outs = [_outs(n, fields) for _ in cams]
    torch.cuda.synchronize()
    rt.trace_primary_batch(cams, outs)
    rt.sync()
    got = [_host(o) for o in outs]
    for k, cam in enumerate(cams):
        ref = rt.trace_primary(cam, fields=fields)
        for f in fields:
            a, b = got[k][f], ref[f].view(np.uint32)
            bad = int(np.count_nonzero(a.reshape(-1) != b.reshape(-1)))
            assert bad == 0, f"{what}: frame {k} field {f} differs at {bad} entries"
    return got


@pytest.mark.parametrize("bd,size", [(1, 16), (2, 32), (4, 64), (8, 128), (16, 256), (32, 512)])
def test_batch_equals_single_frames_every_brick_dim(gpu, bd, size):
    gpu.upload(vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, size, bd))
    _check_batch(gpu, _orbit(size, 200, 136, 4), f"bd {bd}")


def test_batch_vs_oracle(gpu, oracle):
    flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 64, 4)
    gpu.upload(flat)
    cams = _orbit(64, 160, 120, 3, step=0.3)
    got = _check_batch(gpu, cams, "oracle case")
    for k, cam in enumerate(cams):
        ref = oracle.trace_primary(flat, cam, 0, 0, cam.width, cam.height, fields=FIELDS)
        for f in FIELDS:
            assert np.array_equal(got[k][f].reshape(-1), ref[f].view(np.uint32).reshape(-1)), (k, f)
    assert (got[0]["value"] != N.VHX_EMPTY).sum() > 1000


@pytest.mark.parametrize("tune", ["budgets=1,2,3,5,8,13", "budgets=4", "budgets=", "qorder=0", "qorder=8r",
                                  "qorder=m16", "qorder=32z", "rpw=0,16,8,4", "resume=0", "qsort=256",
                                  "qwaves=64;qxcd=0", "sparse=60,60,60", "p0lists=0", "qorder=16z", "qorder=128z",
                                  "scan_multi=1", "finter=0", "finter=0;qstate=1", "finter=0;p0lists=0"])
def test_batch_schedules_are_bit_identical(gpu, tune):
    flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 256, 4)
    rt = vhx.Raytracer(0, tune=tune)
    try:
        rt.upload(flat)
        _check_batch(rt, _orbit(256, 320, 180, 5, step=0.2), f"tune {tune}", fields=("value", "impact", "rgba"))
    finally:
        rt.close()


def test_batch_of_one_and_odd_sizes(gpu):
    gpu.upload(vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 64, 4))
    _check_batch(gpu, _orbit(64, 97, 33, 1), "one frame, 97x33")
    _check_batch(gpu, _orbit(64, 1, 1, 7), "1x1 frames")
    _check_batch(gpu, _orbit(64, 17, 250, 3), "17x250")


def test_batch_headline_frames_match_golden():
    """Three frames of the golden camera and two of other views in one batch of the headline workload: the golden
    frames' every field equals the committed digests, the others equal lone traces."""
    import torch
    m = META["c3_1024_bd4_3840x2160"]
    size, W, H = m["size"], m["width"], m["height"]
    flat = vhx.FlatTree.build_scene(m["scene"], size, m["brick_dim"], threads=min(16, os.cpu_count() or 1))
    rt = vhx.Raytracer(0)
    try:
        rt.upload(flat)
        gold = vhx.glass_camera(size, W, H, target=(size / 2,) * 3)
        other = _orbit(size, W, H, 2, step=0.01)
        cams = [gold, other[1], gold, gold, vhx.glass_camera(size, W, H, angle=41.0, target=(size / 2,) * 3)]
        outs = [_outs(W * H, FIELDS if k == 0 else ("rgba", "depth")) for k in range(len(cams))]
        torch.cuda.synchronize()
        rt.trace_primary_batch(cams, outs)
        rt.sync()
        for f in FIELDS:
            assert digest(_host(outs[0])[f]) == m["sha256"][f], f"golden frame field {f}"
        for k in (2, 3):
            for f in ("rgba", "depth"):
                assert digest(_host(outs[k])[f]) == m["sha256"][f], f"golden frame {k} field {f}"
        for k in (1, 4):
            ref = rt.trace_primary(cams[k], fields=("rgba", "depth"))
            for f in ("rgba", "depth"):
                assert np.array_equal(_host(outs[k])[f], ref[f].view(np.uint32)), (k, f)
    finally:
        rt.close()


@pytest.mark.parametrize("slots", [1, 4])
def test_batches_in_flight_on_shared_contexts(gpu, slots):
    """Two shared contexts, each submitting batches on its own stream without waiting: every frame equals a lone
    trace (the batch's queues, state and argument copies are per context). Five batches per context: with the
    staging ring on ("stage_slots=4") the ring wraps onto slots whose copies may not have run yet."""
    import torch
    flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 256, 4)
    owner = vhx.Raytracer(0)
    try:
        owner.upload(flat)
        other = owner.shared()
        for ctx in (owner, other):
            ctx.set_tuning(f"stage_slots={slots}")
        W, H = 480, 270
        cams = _orbit(256, W, H, 30, step=0.1)
        outs = [_outs(W * H, ("rgba", "depth")) for _ in cams]
        torch.cuda.synchronize()
        for b in range(10):  # even batches on the owner, odd ones on the other context, in flight together
            ctx = owner if b % 2 == 0 else other
            ctx.trace_primary_batch(cams[3 * b:3 * b + 3], outs[3 * b:3 * b + 3])
        owner.sync()
        other.sync()
        for k, cam in enumerate(cams):
            ref = owner.trace_primary(cam, fields=("rgba", "depth"))
            for f in ("rgba", "depth"):
                assert np.array_equal(_host(outs[k])[f], ref[f].view(np.uint32)), (k, f)
        other.close()
    finally:
        owner.close()


def test_batch_sees_updates_in_order(gpu):
    """A ranged write between two batches: the first batch's frames show the tree before it, the second's after it
    (stream-ordered, no host wait in between)."""
    import torch
    flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 64, 4)
    gpu.upload(flat)
    W, H = 128, 96
    cams = _orbit(64, W, H, 2, step=0.0)
    before = gpu.trace_primary(cams[0], fields=("rgba",))["rgba"].copy()
    outs_a = [_outs(W * H, ("rgba",)) for _ in cams]
    outs_b = [_outs(W * H, ("rgba",)) for _ in cams]
    torch.cuda.synchronize()
    gpu.trace_primary_batch(cams, outs_a)
    pal = np.asarray(flat.color_palette).copy()
    gpu.update_range(N.VHX_BUF_COLOR_PALETTE, 0, (pal ^ 0x00FFFFFF) | 0xFF000000)
    gpu.trace_primary_batch(cams, outs_b)
    gpu.sync()
    after = gpu.trace_primary(cams[0], fields=("rgba",))["rgba"]
    gpu.update_range(N.VHX_BUF_COLOR_PALETTE, 0, pal)
    assert not np.array_equal(before, after)
    for k in range(2):
        assert np.array_equal(_host(outs_a[k])["rgba"], before.view(np.uint32))
        assert np.array_equal(_host(outs_b[k])["rgba"], after.view(np.uint32))


def test_batch_argument_errors(gpu):
    import ctypes
    import torch
    flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 64, 4)
    gpu.upload(flat)
    lib = N.lib()
    a, b = vhx.glass_camera(64, 32, 32), vhx.glass_camera(64, 32, 16)
    o = _outs(32 * 32, ("rgba",))
    hs = (N.Hits * 2)(vhx.raytracing._hits_struct(o), vhx.raytracing._hits_struct(o))
    cs = (N.Camera * 2)(a, b)
    p = lambda x: ctypes.cast(x, ctypes.c_void_p)
    assert lib.vhx_trace_primary_batch(gpu._h, p(cs), 0, p(hs)) == N.VHX_E_INVALID_ARG  # no frames
    assert lib.vhx_trace_primary_batch(gpu._h, p(cs), 2, p(hs)) == N.VHX_E_INVALID_ARG  # sizes differ
    assert lib.vhx_trace_primary_batch(gpu._h, None, 1, p(hs)) == N.VHX_E_INVALID_ARG
    counted = dict(o, bytes=torch.zeros(32 * 32, dtype=torch.int32, device="cuda"))
    hb = (N.Hits * 1)(vhx.raytracing._hits_struct(counted))
    assert lib.vhx_trace_primary_batch(gpu._h, p(cs), 1, p(hb)) == N.VHX_E_INVALID_ARG  # byte counting
    with pytest.raises(ValueError):
        gpu.trace_primary_batch([a], [{"rgba": np.zeros(32 * 32, np.uint32)}])  # host outputs
    # a valid call after the refusals still works
    _check_batch(gpu, [a, a], "after errors", fields=("rgba",))


def _shadow_records(gpu, cams):
    import torch
    n = cams[0].width * cams[0].height
    outs = [_outs(n, ("value", "impact", "normal", "rgba")) for _ in cams]
    torch.cuda.synchronize()
    gpu.trace_primary_batch(cams, outs)
    gpu.sync()
    return outs


@pytest.mark.parametrize("W,H,nf", [(200, 136, 4), (97, 33, 3), (64, 64, 1), (1, 1, 5)])
def test_shadow_batch_equals_single_shadow_traces(gpu, W, H, nf):
    """vhx_trace_shadows_batch over nf frames' hit records equals one vhx_trace_shadows per frame: the shadowed flags
    and the darkened RGBA, bit for bit (the single shadow trace is pinned to the oracle's shadow pass elsewhere)."""
    import torch
    size = 256
    gpu.upload(vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, size, 4))
    cams = _orbit(size, W, H, nf, step=0.15)
    light = (float(size),) * 3
    recs = _shadow_records(gpu, cams)
    singles = []
    for r in recs:
        h = {k: v.clone() for k, v in r.items()}
        torch.cuda.synchronize()
        res = gpu.trace_shadows(light, h)
        gpu.sync()
        singles.append((res["shadowed"].cpu().numpy(), h["rgba"].cpu().numpy()))
    torch.cuda.synchronize()
    sh = gpu.trace_shadows_batch(light, recs)
    gpu.sync()
    for k in range(nf):
        assert np.array_equal(sh[k].cpu().numpy(), singles[k][0]), f"frame {k}: shadowed differs"
        assert np.array_equal(recs[k]["rgba"].cpu().numpy(), singles[k][1]), f"frame {k}: rgba differs"
    if W * H > 1000:
        assert sum(int(s.sum().item()) for s in sh) > 0, "no shadowed pixel: the case tests nothing"


def test_shadow_batch_argument_errors(gpu):
    import torch
    gpu.upload(vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 64, 4))
    recs = _shadow_records(gpu, _orbit(64, 32, 32, 2))
    with pytest.raises(ValueError):
        gpu.trace_shadows_batch((64.0,) * 3, [recs[0], {k: v[:100] for k, v in recs[1].items()}])
    # an output aliasing another frame's hit records is refused
    with pytest.raises(N.VhxError):
        gpu.trace_shadows_batch((64.0,) * 3, recs, shadowed_list=[recs[1]["value"], torch.empty_like(recs[0]["value"])])


@pytest.mark.parametrize("W,H,T,stride,starts", [(200, 136, 64, 3, (0, 1, 2)), (200, 136, 16, 5, (0, 4, 4, 9)),
                                                 (97, 33, 32, 2, (0, 1, 5)), (256, 256, 64, 1, (0, 0)),
                                                 (130, 70, 20, 2, (1, 0, 3))])
@pytest.mark.parametrize("tune", [None, "tlists=0", "budgets=4", "qstate=1", "resume=0", "finter=0"])
def test_tiles_batch_equals_single_tile_traces(W, H, T, stride, starts, tune):
    """vhx_trace_tiles_batch (a rank's tile sets of several frames, the multi-GPU split's batch): every frame equals
    the single TILES-layout trace of its camera and tile set bit for bit, padding entries included (both untouched),
    for sets of different sizes (a start past the last tile: no entries), tile sizes that are no multiple of 16, and the
    listed, flag-compacted and other pass schedules."""
    import torch
    rt = vhx.Raytracer(0, tune=tune)
    try:
        rt.upload(vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 64, 4))
        cams = _orbit(64, W, H, len(starts), step=0.3)
        ntiles = ((W + T - 1) // T) * ((H + T - 1) // T)
        sizes = [max(0, (ntiles - s + stride - 1) // stride) * T * T for s in starts]
        fields = ("value", "impact", "depth", "rgba")
        got = [_outs(max(1, n), fields) for n in sizes]
        ref = [_outs(max(1, n), fields) for n in sizes]
        torch.cuda.synchronize()
        rt.trace_tiles_batch(cams, T, starts, stride, got)
        for k, cam in enumerate(cams):
            if sizes[k]:
                rt.trace_primary(cam, tile_size=T, tile_start=starts[k], tile_stride=stride,
                                 layout=N.VHX_LAYOUT_TILES, out=ref[k])
        rt.sync()
        for k in range(len(cams)):
            a, b = _host(got[k]), _host(ref[k])
            for f in fields:
                assert np.array_equal(a[f], b[f]), f"frame {k} (start {starts[k]}) field {f}"
        assert sum((_host(g)["value"] != N.VHX_EMPTY).sum() for g in got) > 0
    finally:
        rt.close()


def test_tiles_batch_argument_errors(gpu):
    import torch
    gpu.upload(vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 64, 4))
    cams = _orbit(64, 64, 64, 2)
    o = [_outs(64 * 64, ("rgba",)) for _ in cams]
    with pytest.raises(ValueError):
        gpu.trace_tiles_batch(cams, 16, (0,), 1, o)  # one start per camera
    shared = {"rgba": o[0]["rgba"]}
    torch.cuda.synchronize()
    with pytest.raises(N.VhxError):
        gpu.trace_tiles_batch(cams, 16, (0, 0), 1, [shared, shared])  # both frames would write one array
    with pytest.raises(ValueError):
        gpu.trace_tiles_batch(cams, 16, (0, 1), 0, o)  # stride 0
    import ctypes
    cs = (N.Camera * 2)(*cams)
    st = (ctypes.c_uint32 * 2)(0, 1)
    # the library refuses the same through the C ABI (stride 0, tile size 0)
    assert N.lib().vhx_trace_tiles_batch(gpu._h, ctypes.cast(cs, ctypes.c_void_p), 2, 16, ctypes.cast(st, ctypes.c_void_p),
                                         0, None) == N.VHX_E_INVALID_ARG
    assert N.lib().vhx_trace_tiles_batch(gpu._h, ctypes.cast(cs, ctypes.c_void_p), 2, 0, ctypes.cast(st, ctypes.c_void_p),
                                         1, None) == N.VHX_E_INVALID_ARG
