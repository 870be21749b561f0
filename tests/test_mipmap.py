"""MIP maps of the host BoxTree (src/boxtree/mipmap.rs, iterate.rs:349-560) against the reference's own KATs
(`mod mipmap_tests`, src/boxtree/tests.rs:877-1330), transcribed with the same trees, inserts and expected colours.
CPU only: MIP generation is host code in the reference as well."""
import math
import os

import numpy as np
import pytest

from voxelhex_amd.boxtree import Albedo, BoxTree, MIPResamplingMethods

BOX_NODE_CHILDREN_COUNT = 64
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

red = Albedo.from_u32(0xFF0000FF)
green = Albedo.from_u32(0x00FF00FF)
blue = Albedo.from_u32(0x0000FFFF)


def _rust_as_u32(f):
    return int(f)  # positive finite values: `as u32` truncates


def mix2():  # tests.rs:883-889: ((255^2 / 2).sqrt() as u32) in r and g
    v = _rust_as_u32(math.sqrt(np_f32(255.0) ** 2 / np_f32(2.0)))
    return Albedo.from_u32((v << 16) | (v << 24) | 0xFF)


def mix3():  # tests.rs:1170-1177: ((255^2 / 3).sqrt() as u32) in r, g and b
    v = _rust_as_u32(np_f32(math.sqrt(np_f32(np_f32(255.0) ** 2 / np_f32(3.0)))))
    return Albedo.from_u32((v << 8) | (v << 16) | (v << 24) | 0xFF)


def np_f32(x):
    return float(np.float32(x))


SIX = [((0, 0, 0), red), ((0, 0, 1), green), ((0, 1, 0), red), ((0, 1, 1), green), ((1, 0, 0), red),
       ((1, 0, 1), green)]


def _root_mip(tree, sectant, pos):
    return tree.albedo_mip_map_resampling_strategy().sample_root_mip(sectant, pos)


def test_mixed_mip_lvl1():  # tests.rs:880-923
    tree = BoxTree(4, 1)
    tree.auto_simplify = False
    tree.albedo_mip_map_resampling_strategy().switch_albedo_mip_maps(True).set_method_at(
        1, MIPResamplingMethods.BoxFilter)
    for p, c in SIX:
        tree.insert(p, c)
    e = _root_mip(tree, BOX_NODE_CHILDREN_COUNT, (0, 0, 0))
    assert e.albedo() is not None
    assert e.albedo() == mix2()


def test_mixed_mip_lvl1_where_dim_is_32():  # tests.rs:925-968
    tree = BoxTree(128, 32)
    tree.auto_simplify = False
    tree.albedo_mip_map_resampling_strategy().switch_albedo_mip_maps(True).set_method_at(
        1, MIPResamplingMethods.BoxFilter)
    for p, c in [((126, 126, 126), red), ((126, 126, 127), green), ((126, 127, 126), red), ((126, 127, 127), green),
                 ((127, 126, 126), red), ((127, 126, 127), green)]:
        tree.insert(p, c)
    e = _root_mip(tree, BOX_NODE_CHILDREN_COUNT, (31, 31, 31))
    assert e.albedo() == mix2()


@pytest.mark.parametrize("mixed", [False, True])
def test_mip_lvl2_where_dim_is_2(mixed):  # tests.rs:970-1040 (solid) and 1042-1120 (mixed)
    tree = BoxTree(8, 2)
    tree.auto_simplify = False
    tree.albedo_mip_map_resampling_strategy().switch_albedo_mip_maps(True).set_method_at(
        1, MIPResamplingMethods.BoxFilter)
    for p, c in SIX:
        tree.insert(p, c if mixed else red)
    e = _root_mip(tree, BOX_NODE_CHILDREN_COUNT, (0, 0, 0))
    assert e.albedo() == (mix2() if mixed else red)
    for pos in [(0, 0, 1), (0, 1, 0), (0, 1, 1), (1, 0, 0), (1, 0, 1), (1, 1, 0), (1, 1, 1)]:
        assert _root_mip(tree, BOX_NODE_CHILDREN_COUNT, pos).albedo() is None


def _lvl2_dim4_inserts(tree):
    for p, c in SIX + [((16, 0, 0), red), ((16, 0, 1), green), ((16, 1, 0), blue), ((16, 1, 1), green),
                       ((17, 1, 0), red), ((17, 0, 1), blue)]:
        tree.insert(p, c)


def _check_lvl2_dim4(tree):
    assert _root_mip(tree, 0, (0, 0, 0)).albedo() == mix2()
    assert _root_mip(tree, 1, (0, 0, 0)).albedo() == mix3()
    assert _root_mip(tree, BOX_NODE_CHILDREN_COUNT, (0, 0, 0)).albedo() == mix2()
    assert _root_mip(tree, BOX_NODE_CHILDREN_COUNT, (1, 0, 0)).albedo() == mix3()


def test_mixed_mip_lvl2_where_dim_is_4():  # tests.rs:1122-1234
    tree = BoxTree(64, 4)
    tree.auto_simplify = False
    tree.albedo_mip_map_resampling_strategy().switch_albedo_mip_maps(True).set_method_at(
        1, MIPResamplingMethods.BoxFilter).set_method_at(2, MIPResamplingMethods.BoxFilter)
    _lvl2_dim4_inserts(tree)
    _check_lvl2_dim4(tree)


def test_mixed_mip_regeneration_lvl2_where_dim_is_4():  # tests.rs:1236-1330
    tree = BoxTree(64, 4)
    tree.auto_simplify = False
    _lvl2_dim4_inserts(tree)
    for pos in [(0, 0, 0), (1, 0, 0)]:
        assert _root_mip(tree, BOX_NODE_CHILDREN_COUNT, pos).albedo() is None  # MIPs are off by default
    tree.albedo_mip_map_resampling_strategy().switch_albedo_mip_maps(True).set_method_at(
        1, MIPResamplingMethods.BoxFilter).set_method_at(2, MIPResamplingMethods.BoxFilter).recalculate_mips()
    _check_lvl2_dim4(tree)


def test_incremental_mips_equal_recalculated():
    """MIPs kept up to date by inserts equal the MIPs recalculated from scratch (default strategy, BoxFilter
    levels): the incremental update_mip of every insert and recalculate_mips build the same bricks."""
    a = BoxTree(64, 4)
    b = BoxTree(64, 4)
    a.auto_simplify = b.auto_simplify = False
    a.albedo_mip_map_resampling_strategy().switch_albedo_mip_maps(True).set_method_at(
        1, MIPResamplingMethods.BoxFilter)
    rng = np.random.default_rng(7)
    cols = [red, green, blue, Albedo(10, 200, 30, 255)]
    pts = rng.integers(0, 64, size=(300, 3))
    for i, p in enumerate(pts):
        a.insert(tuple(p), cols[i % 4])
        b.insert(tuple(p), cols[i % 4])
    b.albedo_mip_map_resampling_strategy().switch_albedo_mip_maps(True).set_method_at(
        1, MIPResamplingMethods.BoxFilter).recalculate_mips()
    fa, fb = a.flatten(), b.flatten()
    assert np.array_equal(fa.node_mips, fb.node_mips)
    for s in list(range(64)) + [64]:
        for pos in [(0, 0, 0), (3, 1, 2), (2, 3, 3)]:
            assert _root_mip(a, s, pos) == _root_mip(b, s, pos)


def test_flatten_lod_cuts_children_and_keeps_mips():
    tree = BoxTree(64, 4)
    tree.auto_simplify = False
    _lvl2_dim4_inserts(tree)
    tree.albedo_mip_map_resampling_strategy().switch_albedo_mip_maps(True)
    full, cut = tree.flatten(), tree.flatten_lod(0)
    assert len(full.node_mips) == len(full.node_type) > 1
    assert len(cut.node_type) == len(cut.node_mips) == 1  # only the root
    assert np.all(cut.node_children == 0xFFFFFFFF)
    assert cut.node_ocbits[0] == full.node_ocbits[0]
    assert cut.node_mips[0] != 0xFFFFFFFF


def _scene_tree(size, bd, lod_enable=True):
    from voxelhex_amd import _native as N
    tree = BoxTree(size, bd)
    tree.insert_scene(N.VHX_SCENE_LATTICE_CUBE)
    if lod_enable:
        tree.albedo_mip_map_resampling_strategy().switch_albedo_mip_maps(True)
    return tree


def test_oracle_mips_on_a_full_tree_change_nothing(oracle):
    """With every child present no MIP stand-in fires: MIP-enabled traces equal the reference path."""
    import voxelhex_amd as vhx
    tree = _scene_tree(64, 4)
    flat = tree.flatten()
    assert len(flat.node_mips) == len(flat.node_type)
    cam = vhx.glass_camera(64, 96, 64, target=(32.0,) * 3)
    ref = oracle.trace_primary(flat, cam, 0, 0, 96, 64, count_bytes=True)
    with oracle.node_mips(flat.node_mips):
        got = oracle.trace_primary(flat, cam, 0, 0, 96, 64, count_bytes=True)
    for k in ref:
        assert np.array_equal(ref[k].view(np.uint32) if ref[k].dtype == np.float32 else ref[k],
                              got[k].view(np.uint32) if got[k].dtype == np.float32 else got[k]), k


def test_oracle_lod_cut_renders_from_mips(oracle):
    """A view cut below the root: without MIPs the rays that would enter a missing child miss (the reference CPU path
    cannot go there); with MIPs they hit the root's MIP brick, whose cells carry MIP colours."""
    import voxelhex_amd as vhx
    tree = _scene_tree(64, 4)
    full, cut = tree.flatten(), tree.flatten_lod(0)
    cam = vhx.glass_camera(64, 96, 64, target=(32.0,) * 3)
    exact = oracle.trace_primary(full, cam, 0, 0, 96, 64, fields=("value",))
    bare = oracle.trace_primary(cut, cam, 0, 0, 96, 64, fields=("value",))
    with oracle.node_mips(cut.node_mips):
        lod = oracle.trace_primary(cut, cam, 0, 0, 96, 64, fields=("value", "cell", "voxel", "depth"))
    hit_exact = exact["value"] != 0xFFFFFFFF
    assert not (bare["value"] != 0xFFFFFFFF).any()
    hit_lod = lod["value"] != 0xFFFFFFFF
    assert hit_lod.sum() > 0.5 * hit_exact.sum()
    # every MIP hit names a cell of the root's MIP brick: voxel = a multiple of the MIP cell edge (64 / 4)
    assert (lod["voxel"][hit_lod] % 16 == 0).all()
    assert set(np.unique(lod["value"][hit_lod])) <= set(cut.voxels.tolist()) | set(cut.solid_values.tolist())


def test_mips_follow_lod_inserts():
    """insert_at_lod with MIPs on (every node on the insert's path updates its MIP, insert.rs:494): large and
    unaligned blocks keep the MIP bricks in bounds, the root's MIP shows the inserted colours, and a leaf filled
    whole (a UniformLeaf) has no MIP of its own (mipmap.rs:71-77: its content is its MIP)."""
    tree = BoxTree(64, 4)
    tree.auto_simplify = True
    tree.albedo_mip_map_resampling_strategy().switch_albedo_mip_maps(True)
    tree.insert_at_lod((0, 0, 0), 16, red)
    tree.insert_at_lod((10, 20, 30), 24, green)
    tree.insert_at_lod((60, 60, 60), 8, blue)

    def root_colours():
        cells = [_root_mip(tree, BOX_NODE_CHILDREN_COUNT, (x, y, z)).albedo()
                 for x in range(4) for y in range(4) for z in range(4)]
        return {c for c in cells if c is not None}

    assert root_colours()
    assert tree.node_info((1, 1, 1))["content"] == "UniformLeaf"
    assert _root_mip(tree, 0, (0, 0, 0)).albedo() is None
    tree.albedo_mip_map_resampling_strategy().recalculate_mips()
    assert root_colours()


def _py_round(x):  # Rust f32::round (half away from zero) for non-negative values
    return int(np.floor(np.float32(x) + np.float32(0.5))) if x >= 0 else -int(np.floor(-x + 0.5))


def _posterize(colours, thr):
    """Python restatement of MIPResamplingMethods::Posterize (iterate.rs:507-557) with groups in first-seen order."""
    groups = []  # [sum of squares (r, g, b, a), count]
    f32 = np.float32
    for c in colours:
        col = (c.r, c.g, c.b, c.a)
        for g in groups:
            poster = [_py_round(float(np.sqrt(f32(_py_round(float(f32(s) / f32(g[1]))))))) for s in g[0]]
            d = [(p - v) % 2 ** 32 for p, v in zip(poster, col)]
            length = float(np.sqrt(f32(sum((x * x) % 2 ** 32 for x in d) % 2 ** 32)))
            if length < float(f32(thr) * f32(255.0)):
                g[0] = [s + v * v for s, v in zip(g[0], col)]
                g[1] += 1
                break
        else:
            groups.append([[v * v for v in col], 1])
    best = 0
    for i in range(1, len(groups)):
        if groups[i][1] >= groups[best][1]:
            best = i
    s, n = groups[best]
    out = [min(255, _py_round(float(np.sqrt(f32(_py_round(float(f32(x) / f32(n)))))))) for x in s]
    return Albedo(*out)


def test_point_filter_and_posterize_without_ties():
    """PointFilter takes the most frequent colour, Posterize the average of the largest group of similar colours
    (iterate.rs:484-557); checked on a leaf root (tree 4, brick_dim 1: MIP level 2 samples its 4^3 voxels) against a
    Python restatement, with colour counts that leave no tie (the reference's HashMap order is then irrelevant)."""
    near_red = [Albedo(250, 0, 0, 255), Albedo(245, 5, 0, 255)]
    voxels = [((0, 0, 0), red), ((1, 0, 0), near_red[0]), ((2, 0, 0), near_red[1]), ((3, 0, 0), near_red[0]),
              ((0, 1, 0), green), ((1, 1, 0), green), ((0, 0, 1), blue)]
    order = sorted(voxels, key=lambda e: (e[0][0], e[0][1], e[0][2]))  # the sampler's x, y, z loop order
    for method, expect in ((MIPResamplingMethods.PointFilter, near_red[0]),
                           (MIPResamplingMethods.Posterize(0.1), _posterize([c for _, c in order], 0.1))):
        tree = BoxTree(4, 1)
        tree.auto_simplify = False
        tree.albedo_mip_map_resampling_strategy().set_method_at(2, method).set_color_similarity_thr_at(2, 0.0)
        for p, c in voxels:
            tree.insert(p, c)
        tree.albedo_mip_map_resampling_strategy().switch_albedo_mip_maps(True)
        got = _root_mip(tree, BOX_NODE_CHILDREN_COUNT, (0, 0, 0)).albedo()
        assert got == expect, (method, got, expect)


_SHORTCUT_CASES = {
    # name: (tree size, brick_dim, scene or None for random inserts, level-2 method)
    "scene64_bd4_box": (64, 4, 1, "box"),
    "scene256_bd4_box": (256, 4, 1, "box"),
    "scene32_bd2_box": (32, 2, 1, "box"),         # a leaf MIP cell spans 2x2x2 bricks
    "scene128_bd8_point": (128, 8, 1, "point"),
    "random64_bd4_posterize": (64, 4, None, "posterize"),
    "random64_bd4_pointbd": (64, 4, None, "pointbd"),
}


def _shortcut_tree_digest(name):
    """sha256 over the MIP-enabled tree's flattened buffers (node MIPs, voxels incl. the MIP bricks, palettes)."""
    import hashlib
    size, bd, scene, method = _SHORTCUT_CASES[name]
    tree = BoxTree(size, bd)
    tree.auto_simplify = False
    if scene is None:
        rng = np.random.default_rng(size + bd)
        cols = [Albedo(int(r), int(g), int(b), 255) for r, g, b in rng.integers(0, 256, size=(24, 3))]
        for i, p in enumerate(rng.integers(0, size, size=(700, 3))):
            tree.insert(tuple(int(v) for v in p), cols[i % len(cols)])
    else:
        from voxelhex_amd import _native as N
        tree.insert_scene(scene)
    m = {"box": MIPResamplingMethods.BoxFilter, "point": MIPResamplingMethods.PointFilter,
         "pointbd": MIPResamplingMethods.PointFilterBD, "posterize": MIPResamplingMethods.Posterize(0.08)}[method]
    tree.albedo_mip_map_resampling_strategy().set_method_at(2, m).switch_albedo_mip_maps(True)
    f = tree.flatten()
    h = hashlib.sha256()
    for a in (f.node_mips, f.voxels, f.solid_values, f.color_palette, f.node_type, f.node_children):
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def test_recalculate_mips_shortcuts_equal_the_direct_restatement():
    """recalculate_mips' leaf resampling in integer arithmetic (BoxTree::leaf_value) and its memoised palette matching
    (mip_palette_match) build the same MIP bricks and palette as the direct restatement (get_internal per sample, a full
    palette scan per store), selected by vhx_boxtree_set_mip_options(direct=1); several leaf samplers, brick dims
    2/4/8, and a single leaf-resampling worker against the default pool."""
    from voxelhex_amd import _native as N
    names = sorted(_SHORTCUT_CASES)
    shortcut = [_shortcut_tree_digest(n) for n in names]
    assert N.lib().vhx_boxtree_set_mip_options(1, 1) == 0
    try:
        generic = [_shortcut_tree_digest(n) for n in names]
    finally:
        assert N.lib().vhx_boxtree_set_mip_options(0, 0) == 0
    assert N.lib().vhx_boxtree_set_mip_options(0, -1) == N.VHX_E_INVALID_ARG
    assert generic == shortcut
