"""Tree-builder known-answer tests transcribed from the reference (src/boxtree/update/tests.rs): insert / get /
update / insert_at_lod / auto-simplify behaviour of the C++ BoxTree restatement that builds every KAT tree and the
streaming mirror. Tests that need `clear` are not transcribed (clear is not restated, docs/DESIGN_LOG.md §10).

Each test cites the reference lines it follows; values, positions and expected counts are the reference's.
"""
import math

import pytest

import voxelhex_amd as vhx
from voxelhex_amd import BoxTreeEntry as E

A = vhx.Albedo.from_u32  # impl From<u32> for Albedo (src/boxtree/detail.rs:72-85), 0xRRGGBBAA
RED, GREEN, BLUE = A(0xFF0000FF), A(0x00FF00FF), A(0x0000FFFF)


def rround(x):
    """f32::round (half away from zero), as in impl From<V3c<f32>> for V3c<u32> (vector.rs:345-355)."""
    return int(math.floor(x + 0.5)) if x >= 0 else -int(math.floor(-x + 0.5))


def sectant_offset(s, scale):
    """V3c::<u32>::from(SECTANT_OFFSET_LUT[s] * scale) (src/spatial/lut.rs:4-24: (s&3, (s>>2)&3, s>>4) / 4)."""
    return tuple(rround(c / 4.0 * scale) for c in (s & 3, (s >> 2) & 3, s >> 4))


def tree(size, bd, auto_simplify=None):
    t = vhx.BoxTree(size, bd)
    if auto_simplify is not None:
        t.auto_simplify = auto_simplify
    return t


def count_hits(t, rng, expect):
    hits = 0
    for x in range(rng):
        for y in range(rng):
            for z in range(rng):
                h = t.get((x, y, z))
                if h != E.Empty():
                    assert h == expect, ((x, y, z), h)
                    hits += 1
    return hits


def test_simplest_insert_and_get():  # update/tests.rs:9-18
    t = tree(4, 1, False)
    red = A(0xFF000001)
    t.insert((0, 0, 0), red)
    assert t.get((0, 0, 0)) == E.Visual(red)


@pytest.mark.parametrize("size,bd,far", [(4, 1, False), (8, 2, True)])
def test_simple_insert_and_get(size, bd, far):  # update/tests.rs:20-47 (dim 1), 113-141 (dim 2)
    t = tree(size, bd, False)
    t.insert((1, 0, 0), RED)
    t.insert((0, 1, 0), GREEN)
    t.insert((0, 0, 1), BLUE)
    assert t.get((1, 0, 0)) == E.Visual(RED)
    assert t.get((0, 1, 0)) == E.Visual(GREEN)
    assert t.get((0, 0, 1)) == E.Visual(BLUE)
    if not far:
        assert t.get((1, 1, 1)) == E.Empty()
    else:
        t.insert((3, 0, 0), RED)
        t.insert((0, 3, 0), GREEN)
        t.insert((0, 0, 3), BLUE)
        assert t.get((3, 0, 0)) == E.Visual(RED)
        assert t.get((0, 3, 0)) == E.Visual(GREEN)
        assert t.get((0, 0, 3)) == E.Visual(BLUE)
    t.insert((1, 0, 0), GREEN)  # overwrite
    assert t.get((1, 0, 0)) == E.Visual(GREEN)
    assert t.get((0, 1, 0)) == E.Visual(GREEN)
    assert t.get((0, 0, 1)) == E.Visual(BLUE)
    if not far:
        assert t.get((1, 1, 1)) == E.Empty()


def test_insert_empty():  # update/tests.rs:49-55
    t = tree(4, 1, False)
    t.insert((0, 0, 0), E.Empty())
    assert t.get((0, 0, 0)) == E.Empty()


def test_complex_insert_and_get():  # update/tests.rs:57-111
    t = tree(4, 1, False)
    t.insert((1, 0, 0), (RED, 3))
    t.insert((0, 1, 0), (GREEN, 1))
    t.insert((0, 0, 1), vhx.voxel_data(2))
    assert t.get((1, 0, 0)) == E.Complex(RED, 3)
    assert t.get((0, 1, 0)) == E.Complex(GREEN, 1)
    assert t.get((0, 0, 1)) == vhx.voxel_data(2)
    assert t.get((1, 1, 1)) == E.Empty()
    t.insert((1, 0, 0), vhx.voxel_data(3))  # overwrite
    assert t.get((1, 0, 0)) == vhx.voxel_data(3)
    assert t.get((0, 1, 0)) == E.Complex(GREEN, 1)
    assert t.get((0, 0, 1)) == vhx.voxel_data(2)
    assert t.get((1, 1, 1)) == E.Empty()


@pytest.mark.parametrize("size,bd", [(16, 1), (8, 2)])
def test_insert_at_lod(size, bd):  # update/tests.rs:143-192 (dim 1), 194-243 (dim 2)
    t = tree(size, bd, False)
    t.insert_at_lod((0, 0, 0), 2, RED)
    for p in [(x, y, z) for x in (0, 1) for y in (0, 1) for z in (0, 1)]:
        assert t.get(p) == E.Visual(RED), p
    t.insert_at_lod((0, 0, 0), 4, GREEN)
    assert count_hits(t, 4, E.Visual(GREEN)) == 64


def test_update_color():  # update/tests.rs:359-371
    t = tree(4, 1, False)
    t.insert((0, 0, 0), (RED, 3))
    assert t.get((0, 0, 0)) == E.Complex(RED, 3)
    t.update((0, 0, 0), GREEN)
    assert t.get((0, 0, 0)) == E.Complex(GREEN, 3)


def test_update_data():  # update/tests.rs:373-386
    t = tree(4, 1, False)
    t.insert((0, 0, 0), (RED, 3))
    t.update((0, 0, 0), E.Informative(4))
    assert t.get((0, 0, 0)) == E.Complex(RED, 4)


def test_update_empty():  # update/tests.rs:388-399
    t = tree(4, 1, False)
    t.insert((0, 0, 0), (RED, 3))
    t.update((0, 0, 0), E.Empty())
    assert t.get((0, 0, 0)) == E.Complex(RED, 3)


def test_uniform_solid_leaf_separated_by_insert_where_dim_is_1():  # update/tests.rs:437-466
    t = tree(4, 1)
    orig = A(0xFFFF00FF)
    for s in range(64):
        t.insert(sectant_offset(s, 1.0), orig)
    assert t.get((0, 0, 0)) == E.Visual(orig)
    t.insert((0, 0, 0), A(0xFFFF00FF))
    assert t.get((0, 0, 0)) == E.Visual(A(0xFFFF00FF))
    for s in range(1, 64):
        assert t.get(sectant_offset(s, 1.0)) == E.Visual(orig)


def test_uniform_solid_leaf_separated_by_insert_where_dim_is_4():  # update/tests.rs:515-563
    t = tree(16, 4)
    base = 0xFFFF00AA
    for s in range(64):
        sp = sectant_offset(s, 16.0)
        for x in range(4):
            for y in range(4):
                for z in range(4):
                    t.insert((sp[0] + x, sp[1] + y, sp[2] + z), A(base + s))
    assert t.get((0, 0, 0)) == E.Visual(A(base))
    mod = A(0x000000FF)
    t.insert((0, 0, 0), mod)
    assert t.get((0, 0, 0)) == E.Visual(mod)
    for s in range(64):
        sp = sectant_offset(s, 16.0)
        for x in range(4):
            for y in range(4):
                for z in range(4):
                    if (x, y, z, s) == (0, 0, 0, 0):
                        continue
                    assert t.get((sp[0] + x, sp[1] + y, sp[2] + z)) == E.Visual(A(base + s))


def test_simple_uniform_parted_brick_leaf_overwrites_separated_by_insert_where_dim_is_2():  # tests.rs:635-661
    t = tree(8, 2)
    base = 0xF00000FF
    for s in range(64):
        t.insert_at_lod(sectant_offset(s, 2.0), 2, A(base + 2 * s))
    assert t.get((0, 0, 0)) == E.Visual(A(base))
    mod = A(0x000000FF)
    t.insert((0, 0, 0), mod)
    assert t.get((0, 0, 0)) == E.Visual(mod)


def test_simple_uniform_parted_brick_leaf_separated_by_insert_where_dim_is_2():  # update/tests.rs:663-712
    t = tree(8, 2)
    base = 0xF00000FF
    for s in range(64):
        t.insert_at_lod(sectant_offset(s, 8.0), 2, A(base + 2 * s))
    assert t.get((0, 0, 0)) == E.Visual(A(base))
    mod = A(0x000000FF)
    t.insert((0, 0, 0), mod)
    assert t.get((0, 0, 0)) == E.Visual(mod)
    for x in range(2):
        for y in range(2):
            for z in range(2):
                for s in range(64):
                    sp = sectant_offset(s, 8.0)
                    p = (sp[0] + x, sp[1] + y, sp[2] + z)
                    want = mod if (x, y, z, s) == (0, 0, 0, 0) else A(base + 2 * s)
                    assert t.get(p) == E.Visual(want), (p, s)


def test_simple_uniform_parted_brick_leaf_separated_by_insert_where_dim_is_4():  # update/tests.rs:714-789
    t = tree(16, 4)

    def col(x, y, z):
        return vhx.Albedo(x - x % 2, y - y % 2, z - z % 2, 255)

    for s in range(64):
        sp = sectant_offset(s, 16.0)
        for x in range(4):
            for y in range(4):
                for z in range(4):
                    p = (sp[0] + x, sp[1] + y, sp[2] + z)
                    t.insert(p, col(x, y, z))
                    assert t.get(p) == E.Visual(col(x, y, z)), p
    assert t.get((0, 0, 0)) == E.Visual(A(0x000000FF))
    mod = A(0xFF0000FF)
    t.insert((1, 1, 1), mod)
    assert t.get((1, 1, 1)) == E.Visual(mod)
    assert t.get((0, 0, 0)) == E.Visual(A(0x000000FF))
    for s in range(64):
        sp = sectant_offset(s, 16.0)
        for x in range(4):
            for y in range(4):
                for z in range(4):
                    p = (sp[0] + x, sp[1] + y, sp[2] + z)
                    want = mod if (x, y, z, s) == (1, 1, 1, 0) else col(x, y, z)
                    assert t.get(p) == E.Visual(want), p


@pytest.mark.parametrize("size,bd,pos,lod,rng,hits", [
    (16, 4, (1, 1, 1), 4, 4, 27),   # update/tests.rs:791-829: one brick at most, 3x3x3 from (1,1,1)
    (16, 1, (2, 2, 2), 3, 8, 8),    # 831-861
    (16, 1, (3, 3, 3), 3, 8, 1),    # 863-894: the position is a brick corner, one voxel
    (16, 4, (1, 1, 1), 3, 8, 27),   # 896-927
])
def test_insert_at_lod_unaligned(size, bd, pos, lod, rng, hits):
    t = tree(size, bd, False)
    t.insert_at_lod(pos, lod, RED)
    assert t.get(pos) == E.Visual(RED)
    assert count_hits(t, rng, E.Visual(RED)) == hits


def test_insert_at_lod_with_simplify():  # update/tests.rs:929-983
    t = tree(16, 1)
    t.insert_at_lod((4, 0, 0), 2, RED)
    for p in [(x, y, z) for x in (4, 5) for y in (0, 1) for z in (0, 1)]:
        assert t.get(p) == E.Visual(RED), p
    t.insert_at_lod((0, 0, 0), 4, GREEN)
    hits = count_hits(t, 4, E.Visual(GREEN))
    for x in (4, 5):
        for y in (0, 1):
            for z in (0, 1):
                h = t.get((x, y, z))
                if h != E.Empty():
                    assert h == E.Visual(RED)
                    hits += 1
    assert hits == 64 + 8


@pytest.mark.parametrize("size,bd", [(4, 1), (8, 2)])
def test_simplifyable_insert_and_get(size, bd):  # update/tests.rs:985-1014 (dim 1), 1016-1045 (dim 2)
    t = tree(size, bd)
    for x in range(size):
        for y in range(size):
            for z in range(size):
                t.insert((x, y, z), RED)
    t.insert((0, 0, 0), GREEN)  # breaks the simplified node back into parts
    assert t.get((0, 0, 0)) == E.Visual(GREEN)
    for x in range(1, size):
        for y in range(1, size):
            for z in range(1, size):
                assert t.get((x, y, z)) == E.Visual(RED)


@pytest.mark.parametrize("insert_lod", [True, False])
def test_set_small_part_of_large_node(insert_lod):  # update/tests.rs:1110-1125, 1127-1140 (the insert halves)
    t = tree(128, 8)
    if insert_lod:
        t.insert_at_lod((33, 33, 33), 2, RED)
        assert t.get((33, 33, 33)) == E.Visual(RED)
    else:
        t.insert((31, 31, 31), RED)
        assert t.get((31, 31, 31)) == E.Visual(RED)


def test_overwrite_whole_nodes_where_dim_is_4():  # update/tests.rs:1684-1739
    t = tree(16, 4)
    t.insert_at_lod((0, 0, 0), 8, RED)
    assert count_hits(t, 8, E.Visual(RED)) == 512
    t.insert_at_lod((0, 0, 0), 5, BLUE)
    red = blue = 0
    for x in range(8):
        for y in range(8):
            for z in range(8):
                h = t.get((x, y, z))
                assert h != E.Empty()
                red += h == E.Visual(RED)
                blue += h == E.Visual(BLUE)
    assert (red, blue) == (512 - 64, 64)


def test_edge_case_boxtree_set():  # update/tests.rs:1741-1755
    t = tree(16, 1)
    for x in range(6, 16):
        for y in range(6, 16):
            for z in range(6, 16):
                t.insert((x, y, z), A(x + y + z))
                assert t.get((x, y, z)) == E.Visual(A(x + y + z))


def test_case_inserting_empty():  # update/tests.rs:1757-1769: Albedo::zero() is transparent, nothing is stored
    t = tree(4, 1)
    t.insert((3, 0, 0), vhx.Albedo(0, 0, 0, 0))
    assert t.get((3, 0, 0)) == E.Empty()
