"""Node MIP stand-ins on the GPU (vhx_set_node_mips; SURVEY.md 8f #4, the WGSL path's probe_MIP,
src/raytracing/bevy/viewport_render.wgsl:328-364, 438-454). Views cut below some depth (vhx_boxtree_flatten_lod) trace
the MIP brick of a node wherever an occupied child is absent; the oracle restates the same rule
(vhx_oracle_set_node_mips), so these frames are compared bit-exactly like the reference path. A full tree traces
identically with and without MIPs, and the reference-path kernels are not the MIP kernels (separate instantiations)."""
import numpy as np
import pytest

import voxelhex_amd as vhx
from voxelhex_amd import _native as N
from voxelhex_amd.boxtree import BoxTree
from tests.test_gpu_parity import DEFAULT_BUDGETS, _device_hits, assert_same, rand_rays

pytestmark = pytest.mark.gpu

SIZE, BD = 256, 4  # levels: root 256, 64, leaves 16 (4 * brick_dim)


@pytest.fixture(scope="module")
def mip_tree():
    tree = BoxTree(SIZE, BD)
    tree.insert_scene(N.VHX_SCENE_LATTICE_CUBE)
    tree.albedo_mip_map_resampling_strategy().switch_albedo_mip_maps(True)
    return tree, tree.flatten()


@pytest.fixture(scope="module")
def rt():
    r = vhx.Raytracer(0)
    yield r
    r.close()


@pytest.mark.parametrize("depth", [0, 1, None])
@pytest.mark.parametrize("budgets", [(), (1,), DEFAULT_BUDGETS])
def test_mip_lod_frame_vs_oracle(oracle, rt, mip_tree, depth, budgets):
    tree, full = mip_tree
    flat = full if depth is None else tree.flatten_lod(depth)
    W, H = 320, 200
    cam = vhx.glass_camera(SIZE, W, H, target=(SIZE / 2,) * 3)
    rt.upload(flat)
    try:
        rt.set_pass_budgets(budgets)
        rt.set_node_mips(flat.node_mips)
        got = rt.trace_primary(cam)
        with oracle.node_mips(flat.node_mips):
            ref = oracle.trace_primary(flat, cam, 0, 0, W, H)
        assert_same(got, ref, f"MIP frame depth {depth} budgets {budgets}")
        hit = ref["value"] != N.VHX_EMPTY
        assert hit.mean() > 0.2
        # explicit rays through the same view
        rng = np.random.default_rng(11)
        o, d = rand_rays(rng, SIZE, 4000)
        got_r = rt.trace_rays(o, d)
        with oracle.node_mips(flat.node_mips):
            ref_r = oracle.trace_rays(flat, o, d)
        assert_same(got_r, ref_r, f"MIP rays depth {depth}")
        if depth is None:  # every child present: MIPs change nothing
            rt.set_node_mips(None)
            assert_same(rt.trace_primary(cam), ref, "full tree without MIPs")
    finally:
        rt.set_node_mips(None)
        rt.set_pass_budgets(DEFAULT_BUDGETS)


def test_mip_lod_shadows_vs_oracle(oracle, rt, mip_tree):
    tree, _ = mip_tree
    flat = tree.flatten_lod(1)
    W, H = 256, 160
    cam = vhx.glass_camera(SIZE, W, H, target=(SIZE / 2,) * 3)
    light = (float(SIZE),) * 3
    rt.upload(flat)
    try:
        rt.set_node_mips(flat.node_mips)
        hits = rt.trace_primary(cam, out=_device_hits(W * H))
        res = rt.trace_shadows(light, hits)
        rt.sync()
        host = {k: v.cpu().numpy() for k, v in hits.items()}
        with oracle.node_mips(flat.node_mips):
            ref_p = oracle.trace_primary(flat, cam, 0, 0, W, H, fields=("value", "impact", "normal", "rgba"))
            ref = oracle.trace_shadows(flat, light, ref_p)
        assert np.array_equal(host["value"].view(np.uint32), ref_p["value"])
        sh = res["shadowed"].cpu().numpy().view(np.uint32)
        assert np.array_equal(sh, ref["shadowed"])
        assert np.array_equal(host["rgba"].view(np.uint32), ref["rgba"])
    finally:
        rt.set_node_mips(None)


def test_mip_lod_without_mips_is_the_reference_path(oracle, rt, mip_tree):
    """Without vhx_set_node_mips a cut view traces like the reference CPU path (a push into a missing child ends
    the ray as a miss), and the MIP mode refuses byte counting and bad descriptors."""
    tree, _ = mip_tree
    flat = tree.flatten_lod(1)
    W, H = 160, 100
    cam = vhx.glass_camera(SIZE, W, H, target=(SIZE / 2,) * 3)
    rt.upload(flat)
    assert_same(rt.trace_primary(cam, count_bytes=True), oracle.trace_primary(flat, cam, 0, 0, W, H, count_bytes=True),
                "cut view, MIPs off")
    rt.set_node_mips(flat.node_mips)
    try:
        with pytest.raises(N.VhxError):
            rt.trace_primary(cam, count_bytes=True)
        with pytest.raises(N.VhxError):
            rt.set_node_mips(flat.node_mips[:-1])  # count != node_count
        bad = flat.node_mips.copy()
        bad[0] = len(flat.voxels) // BD ** 3 + 5  # names no uploaded brick
        with pytest.raises(N.VhxError):
            rt.set_node_mips(bad)
    finally:
        rt.set_node_mips(None)


def test_mip_lod_trade_off(rt, mip_tree):
    """Measured trade-off of the LOD views (printed; docs/DESIGN_LOG.md §10b): pixels whose hit value differs from the full
    tree's and frame time, for each cut depth."""
    import time
    tree, full = mip_tree
    W, H = 1920, 1080
    cam = vhx.glass_camera(SIZE, W, H, target=(SIZE / 2,) * 3)
    rt.upload(full)
    exact = rt.trace_primary(cam, fields=("value",))

    def timed():
        rt.trace_primary(cam, fields=("value",))
        rt.sync()
        t0 = time.perf_counter()
        for _ in range(10):
            rt.trace_primary(cam, fields=("value",))
        rt.sync()
        return (time.perf_counter() - t0) / 10 * 1e3

    t_full = timed()
    for depth in (0, 1):
        flat = tree.flatten_lod(depth)
        rt.upload(flat)
        rt.set_node_mips(flat.node_mips)
        got = rt.trace_primary(cam, fields=("value",))
        t = timed()
        rt.set_node_mips(None)
        print(f"MIP LOD depth {depth}: {flat.node_type.size} nodes, {100 * np.mean(got['value'] != exact['value']):.2f} "
              f"% pixels differ, {t:.3f} ms/frame (host-synchronised) vs full tree {t_full:.3f}")


def test_mips_are_shared_by_frames_in_flight(oracle, mip_tree):
    """Contexts sharing the device tree (vhx_create_shared, frames in flight) trace with the owner's node MIPs; a new
    upload switches them off."""
    tree, _ = mip_tree
    flat = tree.flatten_lod(1)
    W, H = 160, 100
    cam = vhx.glass_camera(SIZE, W, H, target=(SIZE / 2,) * 3)
    owner = vhx.Raytracer(0)
    try:
        owner.upload(flat)
        owner.set_node_mips(flat.node_mips)
        sh = owner.shared()
        with oracle.node_mips(flat.node_mips):
            ref = oracle.trace_primary(flat, cam, 0, 0, W, H, fields=("value", "depth"))
        assert_same(sh.trace_primary(cam, fields=("value", "depth")), ref, "shared context with MIPs")
        with pytest.raises(N.VhxError):
            sh.set_node_mips(flat.node_mips)  # set through the owner
        again = tree.flatten_lod(1)  # a new tree object, so Raytracer.upload really uploads
        owner.upload(again)  # a new upload: MIPs off again
        assert_same(sh.trace_primary(cam, fields=("value", "depth")),
                    oracle.trace_primary(again, cam, 0, 0, W, H, fields=("value", "depth")), "after re-upload")
        sh.close()
    finally:
        owner.close()


@pytest.mark.parametrize("depth", [1, 2])
def test_headline_scale_mip_lod_frame_vs_oracle(oracle, rt, depth):
    """The bench's --mip-lod view of the headline tree (scene S 1024^3, brick_dim 4) from vhx_scene_build_lod (equal to
    the insert + MIP path, tests/test_scene_builder.py), a 960x540 glass frame bit-exact against the oracle."""
    S = 1024
    flat = vhx.FlatTree.build_scene_lod(N.VHX_SCENE_LATTICE_CUBE, S, 4, depth, threads=16)
    W, H = 960, 540
    cam = vhx.glass_camera(S, W, H, target=(S / 2,) * 3)
    rt.upload(flat)
    try:
        rt.set_node_mips(flat.node_mips)
        got = rt.trace_primary(cam)
        with oracle.node_mips(flat.node_mips):
            ref = oracle.trace_primary(flat, cam, 0, 0, W, H)
        assert_same(got, ref, f"1024^3 MIP frame depth {depth}")
        assert (ref["value"] != N.VHX_EMPTY).mean() > 0.2
    finally:
        rt.set_node_mips(None)
