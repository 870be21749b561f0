"""Streaming producer (vhx_stream <- BoxTreeGPUDataHandler + upload queue, src/raytracing/bevy/streaming/*.rs), host
side: the streamed view is checked by tracing it with the oracle against the oracle on the full tree.

Pinning: the reference has no streaming tests (only a hash test, streaming/types.rs:126-140); the property checked
here is the one the reference's design promises — inside the uploaded region the view renders what the tree renders.
"""
import numpy as np
import pytest

import voxelhex_amd as vhx
from voxelhex_amd import _native as N
from tests.test_gpu_parity import assert_same

FIELDS = ("value", "cell", "voxel", "impact", "normal", "depth")


def _tree(size=64, bd=4, scene=N.VHX_SCENE_LATTICE_CUBE):
    t = vhx.BoxTree(size, bd)
    t.insert_scene(scene)
    return t


def _rays_in_box(rng, lo, hi, n):
    o = rng.uniform(lo, hi, (n, 3)).astype(np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d /= np.sqrt((d * d).sum(1, keepdims=True)).astype(np.float32)
    return o, d.astype(np.float32)


def test_view_covering_the_tree_renders_like_the_tree(oracle):
    t = _tree()
    S = 64.0
    s = vhx.StreamingView(t, None, (S / 2, S / 2, S / 2), 2 * S)
    stats, frames, resizes = s.upload_all()
    assert stats["pending"] == 0 and stats["nodes_resident"] > 1 and stats["bricks_resident"] > 1
    rng = np.random.default_rng(1)
    o = rng.uniform(-0.5 * S, 1.5 * S, (4000, 3)).astype(np.float32)
    tgt = rng.uniform(0, S, (4000, 3)).astype(np.float32)
    d = tgt - o
    d = (d / np.sqrt((d * d).sum(1, keepdims=True))).astype(np.float32)
    full = oracle.trace_rays(t.flatten(), o, d, fields=FIELDS)
    view = oracle.trace_rays(s.view(), o, d, fields=FIELDS)
    assert_same(view, full, "full view")
    assert (full["value"] != N.VHX_EMPTY).sum() > 500


@pytest.mark.parametrize("size,bd,center,dist", [(64, 4, (10.0, 12.0, 9.0), 24.0), (128, 2, (40.0, 20.0, 50.0), 20.0),
                                                  (128, 8, (100.0, 90.0, 110.0), 60.0)])
def test_partial_view_matches_inside_the_region(oracle, size, bd, center, dist):
    t = _tree(size, bd)
    s = vhx.StreamingView(t, None, center, dist)
    s.set_rates(8, 16, 10)  # several frames of uploads
    stats, frames, resizes = s.upload_all()
    assert frames > 1 and stats["pending"] == 0
    c = np.array(center, np.float32)
    lo, hi = np.maximum(c - dist / 2 + 1, 0), np.minimum(c + dist / 2 - 1, size)
    rng = np.random.default_rng(bd)
    o, d = _rays_in_box(rng, lo, hi, 6000)
    full = oracle.trace_rays(t.flatten(), o, d, fields=FIELDS)
    view = oracle.trace_rays(s.view(), o, d, fields=FIELDS)
    hit = full["value"] != N.VHX_EMPTY
    inside = hit & np.all((full["impact"] >= lo) & (full["impact"] <= hi), axis=1)
    assert inside.sum() > 200
    assert_same({k: v[inside] for k, v in view.items()}, {k: v[inside] for k, v in full.items()}, "in region")


def test_viewport_moves_evict_and_refill(oracle):
    """Moving the viewport across the tree with a small view reuses node and brick slots (eviction); each new
    region renders like the tree once its uploads are done."""
    t = _tree(128, 8)
    s = vhx.StreamingView(t, None, (16.0, 16.0, 16.0), 24.0)
    s.upload_all()
    cap0 = None
    rng = np.random.default_rng(7)
    for c in [(16.0, 16.0, 16.0), (40.0, 16.0, 16.0), (40.0, 40.0, 20.0), (100.0, 100.0, 100.0), (20.0, 60.0, 16.0)]:
        s.set_viewport(c, 24.0)
        stats, frames, resizes = s.upload_all()
        cap0 = cap0 or (stats["nodes_in_view"], stats["bricks_in_view"])
        c = np.array(c, np.float32)
        lo, hi = np.maximum(c - 11, 0), np.minimum(c + 11, 128)
        o, d = _rays_in_box(rng, lo, hi, 3000)
        full = oracle.trace_rays(t.flatten(), o, d, fields=FIELDS)
        view = oracle.trace_rays(s.view(), o, d, fields=FIELDS)
        inside = (full["value"] != N.VHX_EMPTY) & np.all((full["impact"] >= lo) & (full["impact"] <= hi), axis=1)
        assert_same({k: v[inside] for k, v in view.items()}, {k: v[inside] for k, v in full.items()}, f"at {c}")
    # the view stayed bounded: slots were reused rather than the capacity growing without limit
    assert stats["bricks_resident"] <= stats["bricks_in_view"]
    assert stats["bricks_in_view"] < t.flatten().desc.brick_count + stats["nodes_in_view"]


def test_reload_and_small_capacity_growth(oracle):
    t = _tree(16, 1)
    s = vhx.StreamingView(t, None, (8.0, 8.0, 8.0), 2.0)  # a tiny view: capacity must grow
    s.set_rates(64, 1024, 64)  # single-voxel bricks: a higher brick rate than the reference's default 50
    s.set_viewport((8.0, 8.0, 8.0), 50.0)
    stats, frames, resizes = s.upload_all()
    assert resizes >= 1 and stats["pending"] == 0
    s.reload()
    stats2, frames2, _ = s.upload_all()
    assert stats2["pending"] == 0
    rng = np.random.default_rng(3)
    o, d = _rays_in_box(rng, np.zeros(3), np.full(3, 16.0), 3000)
    assert_same(oracle.trace_rays(s.view(), o, d, fields=FIELDS), oracle.trace_rays(t.flatten(), o, d, fields=FIELDS),
                "reloaded full view")


def _edit(t, rng, size):
    """Inserts into empty space (new nodes and bricks), updates of existing voxels (changed bricks) and a small block
    insert (insert_at_lod). A block that covers a node's six faces would make it occluded, and the upload walk never
    descends into an occluded node (upload_queue.rs:528-531; its MIP stands in for it in the reference, and MIPs are
    off by default): the view would then miss that node's inside, in the reference as here."""
    for _ in range(60):
        x, y, z = (int(v) for v in rng.integers(0, size, 3))
        t.insert((x, y, z), vhx.Albedo(int(rng.integers(1, 255)), 40, 200, 255))
    for _ in range(40):
        x, y, z = (int(v) for v in rng.integers(0, size, 3))
        t.update((x, y, z), vhx.Albedo(250, int(rng.integers(1, 255)), 10, 255))
    x, y, z = (int(v) for v in rng.integers(0, size - 8, 3))
    t.insert_at_lod((x - x % 2, y - y % 2, z - z % 2), 2, vhx.Albedo(9, 9, 250, 255))


@pytest.mark.parametrize("size,bd,dist", [(64, 4, 128.0), (128, 8, 256.0), (32, 2, 64.0)])
def test_tree_changes_propagate_into_the_stream(oracle, size, bd, dist):
    """handle_tree_updates (src/raytracing/bevy/streaming/mod.rs:35-286): after the view is complete, edits of the
    tree are queued by its update trigger and re-uploaded by the next frames, so the view renders the edited tree."""
    t = _tree(size, bd)
    S = float(size)
    s = vhx.StreamingView(t, None, (S / 2, S / 2, S / 2), dist)
    s.upload_all()
    rng = np.random.default_rng(size + bd)
    o = rng.uniform(-0.5 * S, 1.5 * S, (5000, 3)).astype(np.float32)
    tgt = rng.uniform(0, S, (5000, 3)).astype(np.float32)
    d = tgt - o
    d = (d / np.sqrt((d * d).sum(1, keepdims=True))).astype(np.float32)
    for rnd in range(2):
        before = oracle.trace_rays(t.flatten(), o, d, fields=FIELDS)
        _edit(t, rng, size)
        stats, frames, _ = s.upload_all()
        assert stats["pending"] == 0 and frames >= 1
        full = oracle.trace_rays(t.flatten(), o, d, fields=FIELDS)
        assert not np.array_equal(before["value"], full["value"])  # the edits are visible
        assert_same(oracle.trace_rays(s.view(), o, d, fields=FIELDS), full, f"edited tree, round {rnd}")


def test_tree_changes_are_queued_only_while_streamed():
    t = _tree(64, 4)
    t.insert((3, 3, 3), vhx.Albedo(1, 2, 3, 255))  # no stream yet: nothing is queued
    s = vhx.StreamingView(t, None, (32.0, 32.0, 32.0), 128.0)
    s.upload_all()
    t.insert((5, 5, 5), vhx.Albedo(1, 2, 3, 255))
    assert s.upload()[0]["pending"] >= 0
    s.close()
    t.insert((7, 7, 7), vhx.Albedo(1, 2, 3, 255))  # the stream is gone: not queued (nothing would pop it)


def _mip_stream(ctx):
    t = _tree(256, 4)
    t.albedo_mip_map_resampling_strategy().switch_albedo_mip_maps(True)
    s = vhx.StreamingView(t, ctx, (60.0, 50.0, 70.0), 40.0)
    s.set_rates(16, 64, 10)
    stats, frames, resizes = s.upload_all()
    assert stats["pending"] == 0
    return t, s


def test_streamed_mips_stand_in_outside_the_region(oracle):
    """With the tree's MIP maps on, the stream writes node MIPs (cache.rs:435-453) into its MIP slots: traced with
    them, rays leaving the resident region hit MIP stand-ins instead of missing, and the region itself is unchanged."""
    t, s = _mip_stream(None)
    mips = s.node_mips()
    view = s.view()
    assert len(mips) == view.desc.node_count and (mips != N.VHX_EMPTY).sum() > 3
    rng = np.random.default_rng(5)
    o, d = _rays_in_box(rng, np.array([0.0, 0.0, 0.0]), np.array([256.0, 256.0, 256.0]), 6000)
    base = oracle.trace_rays(view, o, d, fields=FIELDS)
    with oracle.node_mips(mips):
        lod = oracle.trace_rays(view, o, d, fields=FIELDS)
    gained = (lod["value"] != N.VHX_EMPTY) & (base["value"] == N.VHX_EMPTY)
    lo, hi = np.array([41.0, 31.0, 51.0]), np.array([79.0, 69.0, 89.0])
    oi, di = _rays_in_box(rng, lo, hi, 6000)
    with oracle.node_mips(mips):
        lod_in = oracle.trace_rays(view, oi, di, fields=FIELDS)
    full = oracle.trace_rays(t.flatten(), oi, di, fields=FIELDS)
    inside = (full["value"] != N.VHX_EMPTY) & np.all((full["impact"] >= lo) & (full["impact"] <= hi), axis=1)
    assert inside.sum() > 200
    assert_same({k: v[inside] for k, v in lod_in.items()}, {k: v[inside] for k, v in full.items()}, "region, MIPs")
    assert gained.sum() > 100, "MIP stand-ins should catch rays the partial view misses"
    # without MIP maps the stream leaves node_mips pointing at bare slots, which no trace reads
    t2 = _tree(64, 4)
    s2 = vhx.StreamingView(t2, None, (20.0, 20.0, 20.0), 16.0)
    s2.upload_all()
    assert len(s2.node_mips()) == s2.view().desc.node_count


def _view_arrays(s):
    import ctypes
    d = s.view().desc
    n3 = d.brick_dim ** 3
    out = {}
    for name, n, dt in (("node_type", d.node_count, np.uint32), ("node_ocbits", d.node_count, np.uint64),
                        ("node_children", d.node_count * 64, np.uint32), ("voxels", d.brick_count * n3, np.uint32),
                        ("solid_values", d.solid_count, np.uint32), ("color_palette", d.color_count, np.uint32),
                        ("data_palette", d.data_count, np.uint32)):
        ptr = getattr(d, name)
        nb = n * np.dtype(dt).itemsize
        out[name] = np.frombuffer((ctypes.c_uint8 * nb).from_address(ptr), dt).copy() if n and ptr else np.zeros(0, dt)
    return out


@pytest.mark.parametrize("batch", [2, 5])
def test_batched_uploads_equal_single_uploads(batch):
    """vhx_stream_upload_frames(K) decides exactly what K vhx_stream_upload calls decide (the reference's per-frame
    rates, tree changes first): after every batch the view mirror equals that of a twin stream uploaded frame by frame,
    through viewport moves, capacity growth and tree edits between batches."""
    size, S = 64, 64.0
    ta, tb = _tree(size, 4), _tree(size, 4)
    a = vhx.StreamingView(ta, None, (S / 2, S / 2, S / 2), S / 4)
    b = vhx.StreamingView(tb, None, (S / 2, S / 2, S / 2), S / 4)
    for s in (a, b):
        s.set_rates(8, 32, 10)
    rng_a, rng_b = np.random.default_rng(5), np.random.default_rng(5)
    for step in range(12):
        if step in (4, 9):
            _edit(ta, rng_a, size)
            _edit(tb, rng_b, size)
        if step == 6:
            for s in (a, b):
                s.set_viewport((0.6 * S, 0.5 * S, 0.5 * S), S)
        _, grow_a = a.upload(frames=batch)
        grow_b = False
        for _ in range(batch):
            _, g = b.upload()
            grow_b = grow_b or g
            if g:
                break  # a capacity stop ends the batch too
        assert grow_a == grow_b, step
        if grow_a:
            a.resize()
            b.resize()
        va, vb = _view_arrays(a), _view_arrays(b)
        for k in va:
            assert np.array_equal(va[k], vb[k]), f"batch {batch} step {step}: {k} differs"
    a.close()
    b.close()


@pytest.mark.parametrize("size,bd,dist,step", [(256, 4, 64.0, 3.0), (128, 2, 20.0, 5.0), (128, 8, 60.0, 7.0),
                                               (64, 1, 16.0, 2.5), (256, 4, 40.0, 31.0)])
def test_incremental_view_set_equals_full_rebuild(size, bd, dist, step):
    """After every viewport move (small steps along an orbit, and jumps across node boundaries) the view set the
    incremental rebuild keeps equals the set a full rebuild at that viewport makes (vhx_stream_view_set_check), and
    most moves are incremental."""
    t = _tree(size, bd)
    S = float(size)
    s = vhx.StreamingView(t, None, (S / 2, S / 2, S / 2), dist)
    s.set_rates(25, 50, 10)
    s.upload()
    rng = np.random.default_rng(size + bd)
    for k in range(40):
        a = 2.0 * np.pi * k * step / (4.0 * S)
        c = (S / 2 + 0.3 * S * np.cos(a), S / 2 + (rng.uniform(-1, 1) if k % 3 == 0 else 0.0), S / 2 + 0.3 * S * np.sin(a))
        if k % 13 == 12:
            c = tuple(rng.uniform(-0.1 * S, 1.1 * S, 3))  # a jump (partly outside the tree)
        s.set_viewport(c, dist)
        if s.upload()[1]:
            s.resize()  # the view grew (re_evaluate_view_size): re-create it, as a renderer does
        same, full, inc = s.view_set_check()
        assert same, f"move {k} to {c}: incremental view set differs from a full rebuild"
    assert inc >= 10, (full, inc)


def test_incremental_view_set_with_tree_edits():
    """Tree edits between moves (queued changes force the next rebuild to be full); the set stays equal to a full
    rebuild's."""
    t = _tree(256, 4)
    s = vhx.StreamingView(t, None, (128.0, 128.0, 128.0), 48.0)
    s.upload()
    for k in range(12):
        s.set_viewport((128.0 + 5 * k, 128.0, 120.0 - 4 * k), 48.0)
        if k % 4 == 1:
            t.insert((120 + k, 40, 140), vhx.Albedo(10, 20, 30, 255))
        if s.upload()[1]:
            s.resize()
        same, _, _ = s.view_set_check()
        assert same, f"move {k}"


def test_incremental_view_set_with_edits_inside_the_view():
    """a move and an edit in the same upload. The move's rebuild runs before the upload applies
    the queued edit, so an incremental walk would start from masks of the tree before it. Edits inside the current
    include box that subdivide a node (one voxel of another colour in a filled region) or collapse one (a whole
    aligned cube overwritten, then simplified) must leave the set equal to a full rebuild's, and the upload
    converges (nothing pending)."""
    t = _tree(256, 4)
    s = vhx.StreamingView(t, None, (128.0, 128.0, 128.0), 48.0)
    s.upload()
    for k in range(16):
        c = (128.0 + 3 * k, 128.0 - 2 * k, 120.0 + 2 * k)
        s.set_viewport(c, 48.0)
        p = tuple(int(v) + 4 for v in c)
        if k % 3 == 0:
            t.insert(p, vhx.Albedo(200, 10 + k, 30, 255))  # subdivides the leaf around p
        elif k % 3 == 1:
            q = tuple((v // 16) * 16 for v in p)
            t.insert_at_lod(q, 16, vhx.Albedo(40, 50, 60 + k, 255))  # one aligned 16^3 cube, uniform content
            t.simplify(True)
        if s.upload()[1]:
            s.resize()
        same, _, _ = s.view_set_check()
        assert same, f"move {k}"
    stats, _, _ = s.upload_all()
    assert stats["pending"] == 0
    assert s.view_set_check()[0]
