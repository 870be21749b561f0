"""GPU parity: libvhx HIP kernels vs the CPU restatement (oracle) on the same inputs.

Bar (BASELINE.json north_star): integer fields (hit value, brick cell, hit voxel, rgba, byte counts) exact; depth,
impact and normal within |d| <= 1e-5 * max(1, |ref|). The kernels are expected to be bit-exact, so the
float comparison below checks bits first and reports the tolerance margin only if bits differ.
"""
import numpy as np
import pytest

import voxelhex_amd as vhx
from tests import kat_cases
from tests.test_oracle_kats import run_oracle
from voxelhex_amd import _native as N

pytestmark = pytest.mark.gpu

INT_FIELDS = ("value", "cell", "voxel", "rgba", "bytes")
FLOAT_FIELDS = ("impact", "normal", "depth")
TOL = 1e-5


def assert_same(got, ref, ctx=""):
    for k in ref:
        a, b = np.asarray(got[k]), np.asarray(ref[k])
        assert a.shape == b.shape, (k, a.shape, b.shape)
        if k in INT_FIELDS:
            bad = np.flatnonzero((a != b).reshape(a.shape[0], -1).any(axis=1))
            assert bad.size == 0, f"{ctx}: {k} differs at {bad.size} rays, first {bad[:5]}: {a[bad[:3]]} vs {b[bad[:3]]}"
        else:
            if np.array_equal(a.view(np.uint32), b.view(np.uint32)):
                continue
            fin = np.isfinite(b)
            same_inf = ~fin & (a == b)
            err = np.abs(a.astype(np.float64) - b.astype(np.float64))
            lim = TOL * np.maximum(1.0, np.abs(b.astype(np.float64)))
            ok = same_inf | (fin & (err <= lim)) | (np.isnan(a) & np.isnan(b))
            assert ok.all(), f"{ctx}: {k} beyond tolerance at {np.count_nonzero(~ok)} entries"


def rand_rays(rng, size, n, inside_frac=0.3):
    S = float(size)
    o = rng.uniform(-0.5 * S, 1.5 * S, (n, 3)).astype(np.float32)
    inside = rng.random(n) < inside_frac
    o[inside] = rng.uniform(0.0, S, (inside.sum(), 3)).astype(np.float32)
    tgt = rng.uniform(0.0, S, (n, 3)).astype(np.float32)
    d = tgt - o
    l = np.sqrt((d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2]).astype(np.float32)
    d = (d / l[:, None]).astype(np.float32)
    # axis-aligned and signed-zero directions exercise the inf/NaN paths of get_dda_scale_factors
    k = max(1, n // 50)
    d[:k] = np.array([0.0, -1.0, 0.0], np.float32)
    d[k:2 * k] = np.array([-0.0, 0.0, 1.0], np.float32)
    d[2 * k:3 * k] = np.array([0.6, -0.8, 0.0], np.float32)
    return o, d


@pytest.mark.parametrize("case", kat_cases.cases(), ids=lambda c: c.name)
def test_reference_kats_on_gpu(gpu, oracle, case):
    tree, rays = case.build()
    flat = tree.flatten()
    gpu.upload(flat)
    o = np.array([r[0] for r in rays], np.float32).reshape(-1, 3)
    d = np.array([r[1] for r in rays], np.float32).reshape(-1, 3)
    got = gpu.trace_rays(o, d, count_bytes=True)
    ref = oracle.trace_rays(flat, o, d, count_bytes=True)
    assert_same(got, ref, case.name)
    res = []
    for i in range(len(rays)):
        res.append(None if got["value"][i] == N.VHX_EMPTY else dict(
            entry=vhx.entry_from_value(got["value"][i], flat.color_palette, flat.data_palette),
            impact=got["impact"][i], normal=got["normal"][i]))
    assert case.check(res), f"{case.name} ({case.lines}) failed on the GPU"


def test_get_by_ray_api(gpu):
    """BoxTree.get_by_ray returns (entry, impact, normal) like src/raytracing/cpu.rs:296."""
    t = vhx.BoxTree(4, 1)
    t.insert((0, 3, 0), vhx.voxel_data(5))
    o = np.array([2.0, 2.0, -5.0], np.float32)
    hit = t.get_by_ray(vhx.Ray(vhx.V3c(*o), vhx.V3c(*kat_cases.normalized(np.array([0, 3, 0], np.float32) - o))))
    assert hit is not None and hit[0] == vhx.voxel_data(5)
    miss = t.get_by_ray(vhx.Ray(vhx.V3c(10.0, 10.0, 10.0), vhx.V3c(1.0, 0.0, 0.0)))
    assert miss is None


SCENE_TREES = [(N.VHX_SCENE_LATTICE_CUBE, 32, 8), (N.VHX_SCENE_LATTICE_CUBE, 32, 2), (N.VHX_SCENE_LATTICE_CUBE, 64, 1),
               (N.VHX_SCENE_LATTICE_CUBE, 256, 4), (N.VHX_SCENE_LATTICE_CUBE, 256, 16), (N.VHX_SCENE_LATTICE_CUBE, 128, 8),
               (N.VHX_SCENE_BENCH_REGION, 512, 8), (N.VHX_SCENE_HEIGHTFIELD, 256, 4), (N.VHX_SCENE_BOUNDARY, 128, 8)]


@pytest.mark.parametrize("scene,size,bd", SCENE_TREES)
def test_random_rays_vs_oracle(gpu, oracle, scene, size, bd):
    flat = vhx.FlatTree.build_scene(scene, size, bd)
    gpu.upload(flat)
    rng = np.random.default_rng(size * 131 + bd)
    o, d = rand_rays(rng, size, 20000)
    got = gpu.trace_rays(o, d, count_bytes=True)
    ref = oracle.trace_rays(flat, o, d, count_bytes=True)
    assert_same(got, ref, f"scene {scene} {size}/{bd}")
    assert (got["value"] != N.VHX_EMPTY).sum() > 100


def test_degenerate_directions_vs_oracle(gpu, oracle):
    """Rays whose distances are NaN or infinite (zero, NaN and infinite direction components, from inside and outside
    the tree): the reference loops until the iteration bound and reports a miss where such a ray stops making progress;
    so do the kernels, and a ray that runs past the bound inside a
    budgeted pass must not be resumed; the same result in every field, for every pass schedule."""
    flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 64, 4)
    gpu.upload(flat)
    nan, inf = np.float32("nan"), np.float32("inf")
    dirs = [(0, 0, 0), (nan, 0, 0), (nan, nan, nan), (0, nan, 1), (inf, 0, 0), (inf, inf, 0), (-inf, 1, 1),
            (1e-30, 0, 0), (0, -1e-30, 0), (1, 1, 1), (-0.0, -0.0, -1)]
    origins = [(32.5, 32.5, 32.5), (1.0, 63.0, 17.25), (-10.0, 30.0, 30.0), (30.0, 80.0, 30.0), (0.0, 0.0, 0.0)]
    o = np.array([oo for oo in origins for _ in dirs], np.float32)
    d = np.array([dd for _ in origins for dd in dirs], np.float32)
    fields = ("value", "cell", "voxel", "impact", "normal", "depth")
    ref = oracle.trace_rays(flat, o, d, fields=fields)
    try:
        for budgets in (DEFAULT_BUDGETS, (), (1, 2, 3)):
            gpu.set_pass_budgets(budgets)
            assert_same(gpu.trace_rays(o, d, fields=fields), ref, f"degenerate directions, budgets {budgets}")
    finally:
        gpu.set_pass_budgets(DEFAULT_BUDGETS)


def test_insert_built_tree_with_palettes(gpu, oracle):
    """Complex / informative / updated voxels and an explicitly simplified tree (Solid bricks, UniformLeaf)."""
    t = vhx.BoxTree(64, 4)
    rng = np.random.default_rng(3)
    for i in range(3000):
        p = rng.integers(0, 64, 3)
        k = i % 4
        e = (vhx.Albedo(int(p[0] * 4), int(p[1] * 4), int(p[2] * 4), 255) if k == 0 else
             int(1 + i % 7) if k == 1 else (vhx.Albedo(10, 20, 30, 255), 3) if k == 2 else vhx.Albedo.from_u32(0x11223344))
        t.insert(p, e)
    for x in range(16, 32):  # a solid 16^3 block, simplified into UniformLeaf/Solid bricks below
        for y in range(16, 32):
            for z in range(16, 32):
                t.insert((x, y, z), vhx.Albedo(200, 100, 50, 255))
    t.update((17, 17, 17), 9)
    for flat in (t.flatten(),):
        gpu.upload(flat)
        o, d = rand_rays(rng, 64, 20000)
        assert_same(gpu.trace_rays(o, d, count_bytes=True), oracle.trace_rays(flat, o, d, count_bytes=True), "insert")
    t.simplify(recursive=True)
    flat = t.flatten()
    assert (flat.node_type == N.VHX_NODE_UNIFORM_LEAF).any() or flat.solid_values.size > 0
    gpu.upload(flat)
    o, d = rand_rays(rng, 64, 20000)
    assert_same(gpu.trace_rays(o, d, count_bytes=True), oracle.trace_rays(flat, o, d, count_bytes=True), "simplified")


FRAMES = [(N.VHX_SCENE_LATTICE_CUBE, 32, 8, 256, 256), (N.VHX_SCENE_LATTICE_CUBE, 256, 4, 256, 256),
          (N.VHX_SCENE_LATTICE_CUBE, 256, 16, 192, 128), (N.VHX_SCENE_BENCH_REGION, 512, 8, 128, 128)]


@pytest.mark.parametrize("scene,size,bd,w,h", FRAMES)
def test_primary_frame_glass_vs_oracle(gpu, oracle, scene, size, bd, w, h):
    flat = vhx.FlatTree.build_scene(scene, size, bd)
    gpu.upload(flat)
    tgt = None if scene == N.VHX_SCENE_BENCH_REGION else (size / 2,) * 3
    cam = vhx.glass_camera(size, w, h, target=tgt)
    got = gpu.trace_primary(cam, count_bytes=True)
    ref = oracle.trace_primary(flat, cam, 0, 0, w, h, count_bytes=True)
    assert_same(got, ref, f"frame {size}/{bd}")
    assert (got["value"] != N.VHX_EMPTY).sum() > 100


def test_primary_frame_inverse_vp_vs_oracle(gpu, oracle):
    """examples/gpu_render.rs camera: Viewport(origin (0,100,0), dir (0,0,-10), frustum (10,10,1024), fov 50)."""
    flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 128, 8)
    gpu.upload(flat)
    vp = vhx.Viewport((150.0, 140.0, 170.0), tuple(kat_cases.normalized(np.array([-1.0, -0.8, -1.1], np.float32))),
                      (10.0, 10.0, 1024.0), 50.0)
    cam = vp.camera(200, 120)
    got = gpu.trace_primary(cam)
    ref = oracle.trace_primary(flat, cam, 0, 0, 200, 120)
    assert_same(got, ref, "inverse-vp")
    assert (got["value"] != N.VHX_EMPTY).sum() > 1000


@pytest.mark.parametrize("T,R", [(64, 3), (20, 2), (13, 4)])  # tile sizes need not be multiples of the 8x8 wave tile
def test_tiles_and_untile_match_framebuffer(gpu, T, R):
    import torch
    flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 64, 4)
    gpu.upload(flat)
    W, H = 200, 136
    cam = vhx.glass_camera(64, W, H, target=(32.0, 32.0, 32.0))
    full = gpu.trace_primary(cam, fields=("rgba",))["rgba"]
    ntiles = ((W + T - 1) // T) * ((H + T - 1) // T)
    per = (ntiles + R - 1) // R
    gathered = torch.zeros(R * per * T * T, dtype=torch.int32, device="cuda")
    for r in range(R):
        part = gpu.trace_primary(cam, tile_size=T, tile_start=r, tile_stride=R, layout=N.VHX_LAYOUT_TILES,
                                 fields=("rgba",))["rgba"]
        gathered[r * per * T * T: r * per * T * T + part.size] = torch.from_numpy(part.view(np.int32)).cuda()
    fb = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    gpu.untile_rgba(gathered.data_ptr(), R, per, T, W, H, fb.data_ptr())
    gpu.sync()
    assert np.array_equal(fb.cpu().numpy().view(np.uint32), full)


def test_update_range(gpu, oracle):
    """vhx_update_range (write_range_to_buffer, src/raytracing/bevy/streaming/mod.rs:344-370)."""
    t = vhx.BoxTree(64, 4)
    t.insert_scene(N.VHX_SCENE_LATTICE_CUBE)
    flat = t.flatten()
    gpu.upload(flat)
    rng = np.random.default_rng(5)
    o, d = rand_rays(rng, 64, 5000)
    before = gpu.trace_rays(o, d)
    vox = flat.voxels.copy()
    vox[: vox.size // 2] = N.VHX_EMPTY  # clear half of the bricks
    gpu.update_range(N.VHX_BUF_VOXELS, 0, vox[: vox.size // 2])
    after = gpu.trace_rays(o, d)
    flat.voxels[: vox.size // 2] = N.VHX_EMPTY  # same edit on the host copy, checked by the oracle
    assert_same(after, oracle.trace_rays(flat, o, d), "update_range")
    assert not np.array_equal(before["value"], after["value"])
    with pytest.raises(N.VhxError):
        gpu.update_range(N.VHX_BUF_VOXELS, vox.size - 4, np.zeros(8, np.uint32))


@pytest.mark.parametrize("scene,bd", [(N.VHX_SCENE_LATTICE_CUBE, 4), (N.VHX_SCENE_LATTICE_CUBE, 16),
                                      (N.VHX_SCENE_HEIGHTFIELD, 4)])
def test_full_size_frame_vs_oracle(gpu, oracle, scene, bd):
    """The bench frame (BASELINE config 3 geometry: 1024^3, 3840x2160, default schedule; scene S at brick_dim 4 is
    the bench workload): every pixel of the GPU frame equals the oracle's in every field, byte counts included, and
    the frame is identical run to run."""
    flat = vhx.FlatTree.build_scene(scene, 1024, bd)
    gpu.upload(flat)
    W, H = 3840, 2160
    cam = vhx.glass_camera(1024, W, H, target=(512.0, 512.0, 512.0))
    fields = ("value", "cell", "voxel", "impact", "normal", "depth", "rgba")
    ref = oracle.trace_primary(flat, cam, 0, 0, W, H, fields=fields, count_bytes=True)
    a = gpu.trace_primary(cam, fields=fields)  # the kernels bench.py times (no byte counting)
    assert_same(a, {k: ref[k] for k in fields}, "full frame")
    assert_same(gpu.trace_primary(cam, fields=fields), a, "idempotence")
    counted = gpu.trace_primary(cam, fields=(), count_bytes=True)
    assert np.array_equal(counted["bytes"], ref["bytes"]), "byte counts differ"
    assert (a["value"] != N.VHX_EMPTY).mean() > 0.1


def test_full_size_shadows_vs_oracle(gpu, oracle):
    """BASELINE config 5 at full size: shadow flags, darkened rgba and byte counts of the bench frame's 2.5 M shadow
    rays equal the oracle's."""
    flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 1024, 4)
    gpu.upload(flat)
    W, H = 3840, 2160
    cam = vhx.glass_camera(1024, W, H, target=(512.0, 512.0, 512.0))
    light = (1024.0,) * 3
    hits = gpu.trace_primary(cam, out=_device_hits(W * H))
    res = gpu.trace_shadows(light, hits, count_bytes=True)
    gpu.sync()
    ref_primary = oracle.trace_primary(flat, cam, 0, 0, W, H, fields=("value", "impact", "normal", "rgba"))
    ref = oracle.trace_shadows(flat, light, ref_primary)
    sh = res["shadowed"].cpu().numpy().view(np.uint32)
    assert np.array_equal(sh, ref["shadowed"]), f"shadow flags differ at {np.count_nonzero(sh != ref['shadowed'])}"
    assert np.array_equal(hits["rgba"].cpu().numpy().view(np.uint32), ref["rgba"])
    assert np.array_equal(res["bytes"].cpu().numpy().view(np.uint32), ref["bytes"])
    assert sh.sum() > 100000


DEFAULT_BUDGETS = (32, 128, 768)  # the library default (ctx.hpp)


@pytest.mark.parametrize("budgets", [(), (1,), (1, 2, 3), (1, 2, 3, 4), (4, 40), (8, 64, 512), (64,),
                                     (16, 64, 256, 1024), (1, 2, 4, 8, 16, 32), (24, 72, 216, 648), DEFAULT_BUDGETS])
def test_multipass_schedule_is_bit_identical(gpu, oracle, budgets):
    """The multi-pass scheduler (vhx_set_pass_budgets) abandons and re-traces rays; every schedule, down to a
    1-step first budget that requeues nearly every ray, must give the oracle's results (incl. byte counts)."""
    flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 256, 4)
    gpu.upload(flat)
    rng = np.random.default_rng(len(budgets) * 7 + sum(budgets))
    o, d = rand_rays(rng, 256, 20000)
    cam = vhx.glass_camera(256, 200, 136, target=(128.0, 128.0, 128.0))
    ref_rays = oracle.trace_rays(flat, o, d, count_bytes=True)
    ref_frame = oracle.trace_primary(flat, cam, 0, 0, 200, 136, count_bytes=True)
    try:
        gpu.set_pass_budgets(budgets)
        assert_same(gpu.trace_rays(o, d, count_bytes=True), ref_rays, f"rays {budgets}")
        assert_same(gpu.trace_primary(cam, count_bytes=True), ref_frame, f"frame {budgets}")
        # tile layout: queue indices map back through the tile numbering
        T, R = 64, 2
        full = ref_frame["rgba"].reshape(136, 200)
        for r in range(R):
            part = gpu.trace_primary(cam, tile_size=T, tile_start=r, tile_stride=R, layout=N.VHX_LAYOUT_TILES,
                                     fields=("rgba",))["rgba"].reshape(-1, T, T)
            tiles_x = (200 + T - 1) // T
            for j in range(part.shape[0]):
                tile = r + j * R
                tx, ty = (tile % tiles_x) * T, (tile // tiles_x) * T
                want = full[ty:ty + T, tx:tx + T]
                assert np.array_equal(part[j, :want.shape[0], :want.shape[1]], want), (budgets, tile)
    finally:
        gpu.set_pass_budgets(DEFAULT_BUDGETS)


SCHEDULER_TUNES = ["resume=0",                        # abandoned rays re-traced from scratch
                   "rpw=0,0;tw=7",                    # adaptive rays per wave, few waves
                   "rpw=0,3;tw=100000;qblock=64",     # one ray per wave, 1-wave workgroups
                   "qxcd=0;xcdg=0",                   # one counter, pass-0 blocks in dispatch order
                   "xcdg=3",                          # odd pass-0 XCD block runs
                   "qxcd=4",                          # shorter runs dealt over the XCDs
                   "qxcd=1;rpw=0,0;tw=7",             # ... single chunks, few adaptive waves
                   "sparse=64,64,64",                 # waves abandon as soon as one lane ends
                   "sparse=0",                        # no sparse-wave abandonment
                   "qxcd_all=1;qwavesm=300",          # every queue pass dealt over the XCDs
                   "qorder=16",                       # pass-0 queue in 16x16 tile order
                   "qorder=m8",                       # ... in Morton order of 8x8 tiles
                   "qorder=m32z",                     # ... every pixel in Morton order
                   "qorder=32r",                      # ... 32x32 tiles by rows
                   "qsort=0",                         # queue passes without the segment node sort
                   "qsort=256;rpw=0,0;tw=7",          # short sorted segments, few adaptive waves
                   "qsort=2048;resume=0"]             # the longest segments; re-traced rays (no state: no sort)


@pytest.mark.parametrize("tune", SCHEDULER_TUNES)
def test_scheduler_variants_are_bit_identical(oracle, tune):
    """Scheduler knobs (vhx_set_tuning: re-trace instead of resume, adaptive rays per wave, queue workgroup size, queue
    orders) change only the schedule: results and byte counts stay the oracle's."""
    rt = vhx.Raytracer(0, tune=tune)
    try:
        flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 256, 4)
        rt.upload(flat)
        rng = np.random.default_rng(11)
        o, d = rand_rays(rng, 256, 8000)
        cam = vhx.glass_camera(256, 160, 96, target=(128.0, 128.0, 128.0))
        ref_rays = oracle.trace_rays(flat, o, d, count_bytes=True)
        ref_frame = oracle.trace_primary(flat, cam, 0, 0, 160, 96, count_bytes=True)
        for budgets in ((2, 9, 30), (16,), ()):
            rt.set_pass_budgets(budgets)
            assert_same(rt.trace_rays(o, d, count_bytes=True), ref_rays, f"rays {tune} {budgets}")
            assert_same(rt.trace_primary(cam, count_bytes=True), ref_frame, f"frame {tune} {budgets}")
            full = ref_frame["rgba"].reshape(96, 160)
            for T, R in ((64, 2), (24, 3)):  # tile layout: the pixel stream maps back through the tile numbering
                tiles_x = (160 + T - 1) // T
                for r in range(R):
                    part = rt.trace_primary(cam, tile_size=T, tile_start=r, tile_stride=R, layout=N.VHX_LAYOUT_TILES,
                                            fields=("rgba",))["rgba"].reshape(-1, T, T)
                    for j in range(part.shape[0]):
                        tile = r + j * R
                        tx, ty = (tile % tiles_x) * T, (tile // tiles_x) * T
                        want = full[ty:ty + T, tx:tx + T]
                        assert np.array_equal(part[j, :want.shape[0], :want.shape[1]], want), (tune, budgets, T, tile)
    finally:
        rt.close()


def test_pass_budget_validation(gpu):
    for bad in ((0,), (5, 5), (9, 3), (1, 2, 3, 4, 5, 6, 7), (1 << 22,)):  # VHX_MAX_BUDGETS = 6
        with pytest.raises(N.VhxError):
            gpu.set_pass_budgets(bad)
    gpu.set_pass_budgets(DEFAULT_BUDGETS)


def test_adaptive_schedule_api(gpu):
    """vhx_set_pass_budgets fixes the schedule, vhx_set_adaptive_schedule restores the adaptive choice (a lone
    context: the lone-frame schedule {64}); vhx_get_pass_budgets reports the last trace's."""
    flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 64, 4)
    gpu.upload(flat)
    o, d = rand_rays(np.random.default_rng(5), 64, 5000)
    try:
        gpu.set_pass_budgets((8, 64))
        ref = gpu.trace_rays(o, d, fields=("value", "depth"))
        assert gpu.pass_budgets() == ((8, 64), "fixed")
        gpu.set_adaptive_schedule(True)
        got = gpu.trace_rays(o, d, fields=("value", "depth"))
        assert gpu.pass_budgets() == ((64,), "idle")
        assert_same(got, ref, "adaptive vs fixed schedule")
    finally:
        gpu.set_pass_budgets(DEFAULT_BUDGETS)


def _device_hits(n):
    import torch
    return {"value": torch.empty(n, dtype=torch.int32, device="cuda"),
            "impact": torch.empty((n, 3), dtype=torch.float32, device="cuda"),
            "normal": torch.empty((n, 3), dtype=torch.float32, device="cuda"),
            "rgba": torch.empty(n, dtype=torch.int32, device="cuda")}


SHADOW_CASES = [(N.VHX_SCENE_LATTICE_CUBE, 256, 4, 256, 192, ()), (N.VHX_SCENE_LATTICE_CUBE, 256, 4, 256, 192, (1,)),
                (N.VHX_SCENE_LATTICE_CUBE, 128, 8, 160, 120, (4, 40)), (N.VHX_SCENE_HEIGHTFIELD, 256, 4, 200, 150, ()),
                (N.VHX_SCENE_BENCH_REGION, 512, 8, 128, 128, DEFAULT_BUDGETS)]


@pytest.mark.parametrize("scene,size,bd,w,h,budgets", SHADOW_CASES)
def test_shadow_rays_vs_oracle(gpu, oracle, scene, size, bd, w, h, budgets):
    """vhx_trace_shadows (BASELINE config 5): shadow flags, darkened rgba and byte counts equal the oracle's on the
    same primary hits, for single- and multi-pass schedules."""
    flat = vhx.FlatTree.build_scene(scene, size, bd)
    gpu.upload(flat)
    tgt = None if scene == N.VHX_SCENE_BENCH_REGION else (size / 2,) * 3
    cam = vhx.glass_camera(size, w, h, target=tgt)
    light = (float(size),) * 3
    try:
        gpu.set_pass_budgets(budgets)
        hits = gpu.trace_primary(cam, out=_device_hits(w * h))
        res = gpu.trace_shadows(light, hits, count_bytes=True)
        gpu.sync()
        host = {k: v.cpu().numpy() for k, v in hits.items()}
        ref_primary = oracle.trace_primary(flat, cam, 0, 0, w, h, fields=("value", "impact", "normal", "rgba"))
        assert_same({k: host[k].view(np.uint32) if k in ("value", "rgba") else host[k] for k in ("value", "impact",
                     "normal")}, {k: ref_primary[k] for k in ("value", "impact", "normal")}, "primary")
        ref = oracle.trace_shadows(flat, light, ref_primary)
        sh = res["shadowed"].cpu().numpy().view(np.uint32)
        assert np.array_equal(sh, ref["shadowed"]), f"shadow flags differ at {np.count_nonzero(sh != ref['shadowed'])}"
        assert np.array_equal(host["rgba"].view(np.uint32), ref["rgba"])
        assert np.array_equal(res["bytes"].cpu().numpy().view(np.uint32), ref["bytes"])
        hit = ref_primary["value"] != N.VHX_EMPTY
        assert sh[~hit].sum() == 0
        if scene != N.VHX_SCENE_BENCH_REGION:
            assert 0 < sh[hit].sum() < hit.sum(), "expected both lit and shadowed hits"
    finally:
        gpu.set_pass_budgets(DEFAULT_BUDGETS)


def test_vox_model_frame_vs_oracle(gpu, oracle):
    """A tree imported from a .vox file (vhx_boxtree_load_vox; written by tests/test_vox.py's writer with rotated,
    translated models) traced on the GPU equals the oracle, incl. the simplified (Solid/UniformLeaf) parts."""
    from tests.test_vox import PALETTE, write_vox
    big = ((40, 24, 32), [(x, y, z, 1 + (x // 8 + (y // 8) * 5 + (z // 8) * 25) % 250 if x < 32 else 1 + (x * 7 + y) % 250)
                          for x in range(40) for y in range(24) for z in range(32)
                          if (x // 8 + y // 8 + z // 8) % 2 == 0 or x > 33])
    rod = ((3, 30, 3), [(x, y, z, 9) for x in range(3) for y in range(30) for z in range(3)])
    scene = [("T", {}, 1, [{}]), ("G", {}, [2, 4]),
             ("T", {}, 3, [{"_t": "0 0 0", "_r": "17"}]), ("S", {}, [(0, {})]),
             ("T", {}, 5, [{"_t": "30 -12 20"}]), ("S", {}, [(1, {})])]
    t = vhx.BoxTree.load_vox_bytes(write_vox([big, rod], PALETTE, scene), 4)
    flat = t.flatten()
    assert (flat.node_type == N.VHX_NODE_UNIFORM_LEAF).any() or flat.solid_values.size > 0
    gpu.upload(flat)
    S = float(flat.desc.boxtree_size)
    cam = vhx.glass_camera(int(S), 192, 128, target=(S / 4, S / 4, S / 4))
    got = gpu.trace_primary(cam, count_bytes=True)
    ref = oracle.trace_primary(flat, cam, 0, 0, 192, 128, count_bytes=True)
    assert_same(got, ref, "vox frame")
    assert (got["value"] != N.VHX_EMPTY).sum() > 500


def test_streamed_view_on_device_matches_mirror(gpu, oracle):
    """vhx_stream on a device context: after frames of ranged writes (nodes, children, voxels, solid values,
    palettes) and a view resize, the GPU traces the device view exactly like the oracle traces the host mirror,
    and like the full tree inside the streamed region."""
    from tests.test_streaming import FIELDS, _rays_in_box, _tree
    t = _tree(128, 8)
    flat = t.flatten()
    s = vhx.StreamingView(t, gpu, (40.0, 30.0, 50.0), 10.0)
    s.set_rates(16, 64, 10)
    s.set_viewport((40.0, 30.0, 50.0), 48.0)  # larger than the initial sizing: forces a resize
    stats, frames, resizes = s.upload_all()
    assert resizes >= 1 and frames > 2
    rng = np.random.default_rng(11)
    c = np.array((40.0, 30.0, 50.0), np.float32)
    lo, hi = np.maximum(c - 23, 0), np.minimum(c + 23, 128)
    o, d = _rays_in_box(rng, lo, hi, 20000)
    got = gpu.trace_rays(o, d, fields=FIELDS, count_bytes=True)
    mirror = oracle.trace_rays(s.view(), o, d, fields=FIELDS, count_bytes=True)
    assert_same(got, mirror, "device view vs host mirror")
    full = oracle.trace_rays(flat, o, d, fields=FIELDS)
    inside = (full["value"] != N.VHX_EMPTY) & np.all((full["impact"] >= lo) & (full["impact"] <= hi), axis=1)
    assert inside.sum() > 1000
    assert_same({k: got[k][inside] for k in FIELDS}, {k: full[k][inside] for k in FIELDS}, "streamed region")
    # move: slots are reused, the device follows the host mirror
    s.set_viewport((100.0, 100.0, 90.0), 48.0)
    s.upload_all()
    o, d = _rays_in_box(rng, np.array([80.0, 80.0, 70.0]), np.array([120.0, 120.0, 110.0]), 20000)
    assert_same(gpu.trace_rays(o, d, fields=FIELDS), oracle.trace_rays(s.view(), o, d, fields=FIELDS), "after move")
    s.close()


def test_tile_layout_padding_reads_zero_and_bytes_add_up(gpu):
    """Tile layout with host outputs: padding pixels past the frame edge read back as 0, so per-rank byte counts
    (the bench's roofline for N>1) add up to the whole frame's."""
    flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 64, 4)
    gpu.upload(flat)
    W, H, T, R = 200, 136, 64, 3
    cam = vhx.glass_camera(64, W, H, target=(32.0, 32.0, 32.0))
    whole = gpu.trace_primary(cam, fields=(), count_bytes=True)["bytes"].astype(np.uint64).sum()
    total = 0
    for r in range(R):
        b = gpu.trace_primary(cam, tile_size=T, tile_start=r, tile_stride=R, layout=N.VHX_LAYOUT_TILES,
                              fields=("value",), count_bytes=True)
        total += int(b["bytes"].astype(np.uint64).sum())
        tiles_x = (W + T - 1) // T
        v = b["value"].reshape(-1, T, T)
        for j in range(v.shape[0]):
            tile = r + j * R
            w = min(T, W - (tile % tiles_x) * T)
            h = min(T, H - (tile // tiles_x) * T)
            assert (v[j, h:, :] == 0).all() and (v[j, :, w:] == 0).all()
    assert total == int(whole)


def test_host_out_arrays_match_device_outputs(gpu):
    """trace_primary(out=...) with host arrays (copied back over PCIe into the caller's reused buffers) gives the
    device-output frame; undersized or mixed host/device out= dicts are refused before anything is written."""
    import torch
    flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 64, 4)
    gpu.upload(flat)
    W, H = 96, 64
    cam = vhx.glass_camera(64, W, H, target=(32.0, 32.0, 32.0))
    dev = gpu.trace_primary(cam, out={"rgba": torch.zeros(W * H, dtype=torch.int32, device="cuda"),
                                      "depth": torch.zeros(W * H, dtype=torch.float32, device="cuda")})
    gpu.sync()
    host = {"rgba": np.zeros(W * H, np.uint32), "depth": np.zeros(W * H, np.float32)}
    for _ in range(2):  # reused buffers
        gpu.trace_primary(cam, out=host)
        assert np.array_equal(host["rgba"], dev["rgba"].cpu().numpy().view(np.uint32))
        assert np.array_equal(host["depth"].view(np.uint32), dev["depth"].cpu().numpy().view(np.uint32))
    with pytest.raises(ValueError):
        gpu.trace_primary(cam, out={"rgba": np.zeros(W * H - 1, np.uint32)})
    with pytest.raises(ValueError):
        gpu.trace_primary(cam, out={"rgba": np.zeros(W * H, np.uint32), "depth": dev["depth"]})


def test_pass0_flags_at_ragged_frame_edges(oracle):
    """A frame whose width and height are not multiples of the 16x16 workgroup block, traced with a 1-step first
    budget (nearly every ray is abandoned and queued) on a fresh context (flags buffer sized exactly): lanes past the
    right and bottom frame edges must not write flags (they would alias the next row's left-edge pixels or run past
    the buffer), so every pixel, the left column included, equals the oracle."""
    flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 64, 4)
    W, H = 200, 136
    # zoomed onto the solid cube: every pixel, the left column included, hits geometry
    cam = vhx.glass_camera(64, W, H, target=(48.0, 48.0, 48.0), glass_width=0.6)
    ref = oracle.trace_primary(flat, cam, 0, 0, W, H, count_bytes=True)
    left = ref["value"].reshape(H, W)[:, :8]
    assert (left != N.VHX_EMPTY).mean() > 0.9
    for budgets in ((1,), (1, 2, 3)):
        rt = vhx.Raytracer(0)
        try:
            rt.upload(flat)
            rt.set_pass_budgets(budgets)
            assert_same(rt.trace_primary(cam, count_bytes=True), ref, f"ragged frame {budgets}")
        finally:
            rt.close()


@pytest.mark.parametrize("budgets", [(1,), DEFAULT_BUDGETS])
def test_sharded_framebuffer_multipass(gpu, oracle, budgets):
    """Framebuffer layout with a rank's tile subset (tile_start / tile_stride) under a multi-pass schedule: the rank
    writes exactly its own pixels (equal to the oracle's) and leaves every other pixel untouched, also after a
    whole-frame trace left its flags behind."""
    import torch
    flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 256, 4)
    gpu.upload(flat)
    W, H, T, R = 200, 136, 32, 3
    cam = vhx.glass_camera(256, W, H, target=(128.0, 128.0, 128.0))
    ref = oracle.trace_primary(flat, cam, 0, 0, W, H)
    try:
        gpu.set_pass_budgets(budgets)
        gpu.trace_primary(cam, fields=("value",))  # leaves this frame's pass-0 flags in the context
        tiles_x = (W + T - 1) // T
        for r in range(R):
            out = {"value": torch.full((W * H,), 0x5A5A5A5A, dtype=torch.int32, device="cuda"),
                   "rgba": torch.full((W * H,), 0x5A5A5A5A, dtype=torch.int32, device="cuda")}
            gpu.trace_primary(cam, tile_size=T, tile_start=r, tile_stride=R, out=out)
            gpu.sync()
            mine = np.zeros((H, W), bool)
            for tile in range(r, tiles_x * ((H + T - 1) // T), R):
                tx, ty = (tile % tiles_x) * T, (tile // tiles_x) * T
                mine[ty:ty + T, tx:tx + T] = True
            mine = mine.reshape(-1)
            for k in ("value", "rgba"):
                got = out[k].cpu().numpy().view(np.uint32)
                assert np.array_equal(got[mine], ref[k][mine]), (k, r, budgets)
                assert (got[~mine] == 0x5A5A5A5A).all(), (k, r, budgets, "foreign pixels written")
    finally:
        gpu.set_pass_budgets(DEFAULT_BUDGETS)


def test_shadow_outputs_must_not_alias_hits(gpu):
    """vhx_trace_shadows refuses outputs that overlap the hit records it reads (or each other)."""
    import torch
    flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 64, 4)
    gpu.upload(flat)
    W, H = 64, 48
    cam = vhx.glass_camera(64, W, H, target=(32.0, 32.0, 32.0))
    hits = gpu.trace_primary(cam, out=_device_hits(W * H))
    with pytest.raises(N.VhxError):
        gpu.trace_shadows((64.0,) * 3, hits, shadowed=hits["value"])
    with pytest.raises(N.VhxError):
        gpu.trace_shadows((64.0,) * 3, hits, shadowed=hits["rgba"])  # rgba is darkened in place: an output too
    with pytest.raises(N.VhxError):
        gpu.trace_shadows((64.0,) * 3, hits, shadowed=hits["impact"].view(-1)[5:5 + W * H].view(torch.int32))
    res = gpu.trace_shadows((64.0,) * 3, hits)
    gpu.sync()
    assert res["shadowed"].numel() == W * H
