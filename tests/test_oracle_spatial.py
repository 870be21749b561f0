"""Oracle pinned against the reference's spatial known-answer tests and LUT tables.

src/spatial/tests.rs:23-128, src/spatial/raytracing/tests.rs:35-312, src/spatial/math/tests.rs:26-65,
src/raytracing/tests.rs:812-902 (NodeStack), LUT values of src/spatial/lut.rs:4-161 (tests/golden/luts.json).
"""
import json
import os

import numpy as np
import pytest

from tests.kat_cases import normalized

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "luts.json")


def test_luts_match_reference_tables(oracle):
    g = json.load(open(GOLDEN))
    off, step, occ = oracle.luts()
    assert np.array_equal(off, np.array(g["sectant_offset"], np.float32))
    assert np.array_equal(step, np.array(g["sectant_step_result"], np.uint8))
    assert np.array_equal(occ, np.array([int(v) for v in g["ray_to_node_occupancy_bitmask"]], np.uint64))


def test_hash_region(oracle):  # src/spatial/tests.rs:23-30
    assert oracle.offset_sectant((0, 0, 0), 12.0) == 0
    assert oracle.offset_sectant((3, 0, 0), 12.0) == 1
    assert oracle.offset_sectant((0, 3, 0), 12.0) == 4
    assert oracle.offset_sectant((0, 0, 3), 12.0) == 16
    assert oracle.offset_sectant((10, 10, 10), 12.0) == 63


def test_step_sectant(oracle):  # src/spatial/tests.rs:32-67
    s = oracle.offset_sectant((0, 10, 0), 40.0)
    assert s == 4
    assert oracle.step_sectant(s, (1, 0, 0)) == 5
    assert oracle.step_sectant(s, (0, -1, 0)) == 0
    assert oracle.step_sectant(s, (0, 1, 0)) == 8
    assert oracle.step_sectant(s, (1, 1, 0)) == 9
    assert oracle.step_sectant(s, (1, 1, 1)) == 25
    s = oracle.offset_sectant((0, 0, 0), 40.0)
    assert oracle.step_sectant(s, (-1, 0, 0)) - 64 == 3
    assert oracle.step_sectant(s, (0, -1, 0)) - 64 == 12
    assert oracle.step_sectant(s, (0, 0, -1)) - 64 == 48
    assert oracle.step_sectant(s, (-1, -1, -1)) - 64 == 63


@pytest.mark.parametrize("off,size,expected", [
    ((0, 0, 0), 4.0, 0), ((0, 0, 2), 4.0, 32), ((3, 3, 3), 4.0, 63),  # tests.rs:103-108
    ((0, 0, 0), 10.0, 0), ((0, 0, 5), 10.0, 32), ((5, 5, 5), 10.0, 42), ((9, 9, 9), 10.0, 63),  # 110-116
    ((0, 0, 0), 2.0, 0), ((1, 0, 0), 2.0, 2), ((0, 1, 0), 2.0, 8), ((1, 1, 0), 2.0, 10), ((0, 0, 1), 2.0, 32),
    ((1, 0, 1), 2.0, 34), ((0, 1, 1), 2.0, 40), ((1, 1, 1), 2.0, 42),  # 118-128
    ((-1, 0, 0), 4.0, 0), ((-1, 2, 0), 4.0, 7),  # saturating `as u8` of a negative flat index / partial sum
])
def test_offset_sectant(oracle, off, size, expected):
    assert oracle.offset_sectant(off, size) == expected


def test_cube_contains_ray(oracle):  # src/spatial/raytracing/tests.rs:123-222
    cube = ((0, 0, 0), 4.0)
    assert oracle.intersect_ray(*cube, (2, 5, 2), (0, -1, 0)) is not None
    assert oracle.intersect_ray(*cube, (2, -5, 2), (0, 1, 0)) is not None
    assert oracle.intersect_ray(*cube, (2, 5, 2), (0, 1, 0)) is None
    assert oracle.intersect_ray(*cube, (-1, -1, -1), normalized((1, 1, 1))) is not None
    o = np.array([4, -1, 4], np.float32)
    assert oracle.intersect_ray(*cube, o, normalized(np.array([4.055] * 3, np.float32) - o)) is None
    assert oracle.intersect_ray(*cube, (-1, -1, -1), normalized((1, 100, 1))) is None


def test_intersect_edge_cases(oracle):  # src/spatial/raytracing/tests.rs:224-312
    assert oracle.intersect_ray((0, 0, 0), 8.0, (8, 4, 5), (-0.842701, -0.24077171, -0.48154342)) == 0.0
    assert oracle.intersect_ray((0, 0, 0), 16.0, (5, 8, 5), (-0.48507127, -0.7276069, -0.48507127)) == "inside"
    t = oracle.intersect_ray((0, 2, 0), 2.0, (6, 7, 6), (-0.6154574, -0.49236596, -0.6154574))
    assert isinstance(t, float) and t > 0.0


def test_intersect_distance(oracle):  # src/spatial/math/tests.rs:26-51
    o = np.array([8.965594, 10.0, -4.4292345], np.float32)
    d = np.array([-0.5082971, -0.72216684, 0.46915793], np.float32)
    t = oracle.intersect_ray((2, 0, 0), 2.0, o, d)
    assert abs(t - 11.077772) < 0.001
    assert abs(float(o[1] + d[1] * np.float32(t)) - 2.0) < 0.001


@pytest.mark.parametrize("p,n", [((1, 1, 2), (0, 0, 1)), ((1, 2, 1), (0, 1, 0)), ((2, 1, 1), (1, 0, 0)),
                                 ((1, 1, 0), (0, 0, -1)), ((1, 0, 1), (0, -1, 0)), ((0, 1, 1), (-1, 0, 0))])
def test_impact_normal(oracle, p, n):  # src/spatial/math/tests.rs:53-65
    assert tuple(oracle.impact_normal((0, 0, 0), 2.0, p)) == n


def test_hash_direction(oracle):  # math/mod.rs:48-52: add-then-compare, x=1, z=2, y=4
    assert oracle.hash_direction((1, 0, 0)) == 7
    assert oracle.hash_direction((-1, 0, 0)) == 6
    assert oracle.hash_direction((0, -1, 0)) == 3
    assert oracle.hash_direction((0, 0, -1)) == 5
    assert oracle.hash_direction((-0.5, -0.5, -0.7)) == 0


def test_nodestack_ring(oracle):  # src/raytracing/tests.rs:816-851: SIZE=3, push 4 overwrites the oldest
    push, pop, last = (lambda v: v), -1, -2
    r = oracle.nodestack(3, [1, 2, 3, 4, last, pop, last, pop, last, pop, pop])
    assert r[4:] == [4, 4, 3, 3, 2, 2, None]
    r = oracle.nodestack(3, [10, 20, 30, last, 40, last])  # 854-867
    assert r[3] == 30 and r[5] == 40
    r = oracle.nodestack(3, [5, 15, 25, pop, pop, pop, pop])  # 887-901
    assert r[3:] == [25, 15, 5, None]


def test_closed_form_step_rule_matches_reference_lut():
    """The GPU evaluates SECTANT_STEP_RESULT_LUT in closed form (voxelhex_amd/csrc/trace.hpp step_sectant_i)."""
    g = np.array(json.load(open(GOLDEN))["sectant_step_result"]).reshape(64, 3, 3, 3)
    for s in range(64):
        sx, sy, sz = s & 3, (s >> 2) & 3, s >> 4
        for dx in (-1, 0, 1):
            for dy in (-1, 0, 1):
                for dz in (-1, 0, 1):
                    x, y, z = sx + dx, sy + dy, sz + dz
                    out = not (0 <= x <= 3 and 0 <= y <= 3 and 0 <= z <= 3)
                    assert g[s, dx + 1, dy + 1, dz + 1] == (64 if out else 0) + (x & 3) + (y & 3) * 4 + (z & 3) * 16


def test_closed_form_occupancy_rule_matches_reference_lut():
    """RAY_TO_NODE_OCCUPANCY_BITMASK_LUT as evaluated by trace.hpp occ_lut (per-axis 4-bit masks)."""
    g = [int(v) for v in json.load(open(GOLDEN))["ray_to_node_occupancy_bitmask"]]
    for s in range(64):
        sx, sy, sz = s & 3, (s >> 2) & 3, s >> 4
        for o in range(8):
            mx = (0xF << sx) & 0xF if o & 1 else 0xF >> (3 - sx)
            my = (0xF << sy) & 0xF if o & 4 else 0xF >> (3 - sy)
            mz = (0xF << sz) & 0xF if o & 2 else 0xF >> (3 - sz)
            row16 = sum((mx << (4 * y)) for y in range(4) if (my >> y) & 1)
            m = sum((row16 << (16 * z)) for z in range(4) if (mz >> z) & 1)
            assert m == g[s * 8 + o]
