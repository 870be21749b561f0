"""Known-answer tests of the reference raytracer, transcribed from VoxelHex src/raytracing/tests.rs:140-809.

Each case builds its tree with the same insert calls as the reference test (through the C++ BoxTree restatement),
casts the same rays and states the reference's assertion. The reference draws some origins / fills with
rand::thread_rng() (unseeded); here they are drawn from a seeded numpy generator over the same ranges.
"""
import numpy as np

from voxelhex_amd import Albedo, BoxTree, BoxTreeEntry, voxel_data
from voxelhex_amd import _native as N

f32 = np.float32


def normalized(v):
    v = np.asarray(v, f32)
    l = f32(np.sqrt(f32(f32(v[0] * v[0]) + f32(v[1] * v[1])) + f32(v[2] * v[2])))
    return np.array([v[0] / l, v[1] / l, v[2] / l], f32)


def ray_to(target, origin):
    o = np.asarray(origin, f32)
    return o, normalized(np.asarray(target, f32) - o)


class Case:
    def __init__(self, name, lines, build, rays, check):
        self.name, self.lines, self.build, self.rays, self.check = name, lines, build, rays, check

    def __repr__(self):
        return self.name


def _rand_plane(size, bd, seed):
    """test_get_by_ray_from_outside(_where_dim_is_2): random z=1 plane of data 5 (tests.rs:140-182)."""
    rng = np.random.default_rng(seed)
    tree = BoxTree(size, bd)
    filled = []
    for x in range(1, 4):
        for y in range(1, 4):
            if 10 > rng.integers(0, 20):
                tree.insert((x, y, 1), voxel_data(5))
                filled.append((x, y, 1))
    rays = [ray_to(p, rng.integers(8, 16, size=3).astype(f32)) for p in filled]
    return tree, rays


def _rand_cube(seed, edge):
    """test_get_by_ray_from_edge / from_inside: random 3^3 cube of data 5 in a (16,1) tree (tests.rs:196-247)."""
    rng = np.random.default_rng(seed)
    tree = BoxTree(16, 1)
    filled = []
    for x in range(1, 4):
        for y in range(1, 4):
            for z in range(1, 4):
                if 10 > rng.integers(0, 20):
                    tree.insert((x, y, z), voxel_data(5))
                    filled.append((x, y, z))
    rays = []
    for p in filled:
        if edge:
            o = np.array([rng.integers(0, 8), rng.integers(0, 8), 8], f32)
            rays.append(ray_to(np.array(p, f32) + f32(0.1), o))
        else:
            rays.append(ray_to(p, rng.integers(8, 16, size=3).astype(f32)))
    return tree, rays


def _ramp(mixed=False):
    """Diagonal ramp of tests.rs:251-275 / 315-339 / 485-509."""
    tree = BoxTree(4, 1)
    tree.insert((3, 0, 0), Albedo.from_u32(0))
    tree.insert((3, 3, 0), Albedo.from_u32(1))
    tree.insert((0, 3, 0), Albedo.from_u32(2))
    for y in range(4):
        if mixed:
            tree.insert((0, y, y), Albedo.from_u32(3))
            tree.insert((1, y, y), Albedo.from_u32(4))
            tree.insert((2, y, y), voxel_data(5))
            tree.insert((3, y, y), Albedo.from_u32(6))
        else:
            for x in range(4):
                tree.insert((x, y, y), Albedo.from_u32(3))
    return tree


def _floor(size=4, bd=1, extent=4):
    tree = BoxTree(size, bd)
    for x in range(extent):
        for z in range(extent):
            tree.insert((x, 0, z), voxel_data(5))
    return tree


def _hit5(results):
    return all(r is not None and r["entry"] == voxel_data(5) for r in results)


def _some(results):
    return all(r is not None for r in results)


def cases(seed=0):
    cs = []
    cs.append(Case("from_outside", "tests.rs:140-160", lambda: _rand_plane(4, 1, seed), None, _hit5))
    cs.append(Case("from_outside_where_dim_is_2", "tests.rs:162-182", lambda: _rand_plane(8, 2, seed + 1), None,
                   _hit5))
    cs.append(Case("from_edge", "tests.rs:196-221", lambda: _rand_cube(seed + 2, True), None, _hit5))
    cs.append(Case("from_inside", "tests.rs:223-247", lambda: _rand_cube(seed + 3, False), None, _hit5))

    def unreachable():
        return _ramp(), [(np.array([10.0, 10.0, -5.0], f32), np.array([-0.66739213, -0.6657588, 0.333696], f32))]
    cs.append(Case("edge_case_unreachable", "tests.rs:249-290", unreachable, None, lambda r: True))

    def empty_line():
        t = BoxTree(4, 1)
        t.insert((2, 1, 1), Albedo.from_u32(3))
        return t, [(np.array([8.965594, 10.0, -4.4292345], f32), np.array([-0.5082971, -0.72216684, 0.46915793], f32))]
    cs.append(Case("edge_case_empty_line_in_middle", "tests.rs:292-311", empty_line, None, _some))

    def zero_advance():
        return _ramp(), [(np.array([8.930992, 10.0, -4.498597], f32), np.array([-0.4687217, -0.772969, 0.42757326], f32))]
    cs.append(Case("edge_case_zero_advance", "tests.rs:313-354", zero_advance, None, _some))

    def behind():
        t = BoxTree(4, 1)
        t.insert((0, 3, 0), voxel_data(5))
        return t, [ray_to((0.0, 3.0, 0.0), (2.0, 2.0, -5.0))]
    cs.append(Case("edge_case_ray_behind_boxtree", "tests.rs:356-371", behind, None, _hit5))

    def overlapping():
        t = BoxTree(4, 1)
        t.insert((0, 0, 0), voxel_data(5))
        t.insert((1, 0, 0), Albedo.from_u32(6))
        return t, [(np.array([2.0, 4.0, -2.0], f32), np.array([-0.23184556, -0.79392403, 0.5620785], f32))]
    cs.append(Case("edge_case_overlapping_voxels", "tests.rs:373-398", overlapping, None,
                   lambda r: r[0] is not None and r[0]["entry"] == BoxTreeEntry.Visual(Albedo.from_u32(6))))

    def edge_raycast():
        return _floor(), [(np.array([2.0, 4.0, -2.0], f32), np.array([-0.47839317, -0.71670955, 0.50741255], f32))]
    cs.append(Case("edge_case_edge_raycast", "tests.rs:400-425", edge_raycast, None,
                   lambda r: r[0] is None or r[0]["entry"] == voxel_data(5)))

    def voxel_corner():
        return _floor(), [(np.array([2.0, 4.0, -2.0], f32), np.array([-0.27100056, -0.7961219, 0.54106253], f32))]
    cs.append(Case("edge_case_voxel_corner", "tests.rs:427-453", voxel_corner, None, _hit5))

    def bottom_edge():
        return _floor(), [(np.array([2.0, 4.0, -2.0], f32), np.array([-0.379010856, -0.822795153, 0.423507959], f32))]
    cs.append(Case("edge_case_bottom_edge", "tests.rs:455-481", bottom_edge, None, _hit5))

    def loop_stuck():
        return _ramp(mixed=True), [(np.array([0.024999974, 10.0, 0.0], f32),
                                    np.array([-0.0030831057, -0.98595166, 0.16700225], f32))]
    cs.append(Case("edge_case_loop_stuck", "tests.rs:483-524", loop_stuck, None, lambda r: True))

    def brick_undetected():
        return _floor(16, 4), [(np.array([-1.0716193, 8.0, -7.927902], f32),
                                np.array([0.18699232, -0.6052176, 0.7737865], f32))]
    cs.append(Case("edge_case_brick_undetected", "tests.rs:526-559", brick_undetected, None, _hit5))

    def detailed_brick_undetected():
        t = BoxTree(8, 2)
        for x in range(8):
            for y in range(8):
                for z in range(8):
                    t.insert((x, y, z), voxel_data(5))
        return t, [(np.array([15.8443775, 16.0, 2.226141], f32), np.array([-0.7984906, -0.60134345, 0.028264323], f32))]
    cs.append(Case("edge_case_detailed_brick_undetected", "tests.rs:561-591", detailed_brick_undetected, None, _hit5))

    def z_edge():
        t = BoxTree(8, 2)
        for x in range(1, 8):
            for y in range(1, 8):
                for z in range(1, 8):
                    t.insert((x, y, z), Albedo.from_u32(z))
        return t, [(np.array([11.92238, 16.0, -10.670372], f32), np.array([-0.30062392, -0.6361918, 0.7105529], f32))]
    cs.append(Case("edge_case_detailed_brick_z_edge_error", "tests.rs:593-624", z_edge, None,
                   lambda r: r[0] is not None and r[0]["entry"] == BoxTreeEntry.Visual(Albedo.from_u32(1))
                   and tuple(float(v) for v in r[0]["normal"]) == (0.0, 0.0, -1.0)))

    def deep_stack():
        t = BoxTree(1024, 1)
        target = (1023, 1023, 1023)
        t.insert((0, 0, 0), Albedo.from_u32(0x000000EE))
        t.insert(target, Albedo.from_u32(0x000000FF))
        o = np.array([0.0, 5.0, -1.0], f32)
        return t, [(o, normalized(np.array(target, f32) + f32(0.5) - o))]
    cs.append(Case("edge_case_deep_stack", "tests.rs:626-651", deep_stack, None,
                   lambda r: r[0] is not None and r[0]["entry"] == BoxTreeEntry.Visual(Albedo.from_u32(0xFF))))

    def traversal_error():
        t = BoxTree(8, 2)
        t.insert((0, 0, 0), Albedo.from_u32(0x000000FF))
        return t, [(np.array([23.84362, 32.0, -21.342018], f32), np.array([-0.51286834, -0.70695364, 0.48701409], f32))]

    def traversal_ok(r):
        if r[0] is None or r[0]["entry"] != BoxTreeEntry.Visual(Albedo.from_u32(0xFF)):
            return False
        n = np.asarray(r[0]["normal"], f32)
        return float(np.sqrt(np.float32(n @ n))) < 1.1
    cs.append(Case("edge_case_brick_traversal_error", "tests.rs:653-681", traversal_error, None, traversal_ok))

    def boundary():
        t = BoxTree(128, 8)
        t.insert_scene(N.VHX_SCENE_BOUNDARY)
        return t, [(np.array([191.60886, 256.0, -169.77057], f32), np.array([-0.38838777, -0.49688956, 0.7760514], f32))]
    cs.append(Case("edge_case_brick_boundary_error", "tests.rs:683-725", boundary, None, _some))

    def cube_flaps():
        t = BoxTree(64, 1)
        t.insert_scene(N.VHX_SCENE_CUBE)
        return t, [(np.array([47.898006, 64.0, -42.44739], f32), np.array([-0.42279032, -0.4016629, 0.8123516], f32))]
    cs.append(Case("edge_case_cube_flaps", "tests.rs:727-766", cube_flaps, None, lambda r: r[0] is None))

    def context_bleed():
        t = BoxTree(64, 1)
        t.insert_scene(N.VHX_SCENE_LATTICE)
        return t, [(np.array([47.898006, 64.0, -42.44739], f32), np.array([-0.49263135, -0.49703234, 0.714334], f32))]
    cs.append(Case("edge_case_context_bleed", "tests.rs:768-809", context_bleed, None, _some))
    return cs


def build(case):
    tree, rays = case.build()
    return tree, rays
