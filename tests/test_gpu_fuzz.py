"""Randomised trees against the oracle, every brick_dim the kernels are built for (1, 2, 4, 8, 16, 32).

Each case builds a BoxTree through the reference API (BoxTree::insert / insert_at_lod / update / simplify,
voxelhex_amd/csrc/boxtree.cpp restating src/boxtree/update/*.rs): scattered single voxels of both kinds of content
(albedo and data), solid boxes inserted at a level of detail (Solid bricks and UniformLeaf nodes after a simplify),
overwrites, then traces explicit rays (30 % starting inside the tree, axis-aligned and signed-zero directions
included) and a glass frame from a random viewpoint, under the default schedule and under a one-step first budget
(every ray resumed from saved state many times). Every field, byte counts included, must equal the oracle's
(tests/test_gpu_parity.py assert_same: integers exact, floats bit-exact or within 1e-5)."""
import numpy as np
import pytest

import voxelhex_amd as vhx
from tests.test_gpu_parity import assert_same, rand_rays

pytestmark = pytest.mark.gpu

CASES = [(0, 16, 1), (1, 64, 1), (2, 32, 2), (3, 128, 2), (4, 64, 4), (5, 256, 4), (6, 128, 8), (7, 256, 16),
         (8, 128, 32), (9, 512, 32)]


def random_tree(seed, size, bd):
    rng = np.random.default_rng(seed)
    t = vhx.BoxTree(size, bd)
    # clustered scatter: a few centres, voxels around them (dense bricks next to sparse ones)
    centres = rng.integers(0, size, (4, 3))
    n = min(4000, size * size * 2)
    for i in range(n):
        c = centres[i % 4]
        p = np.clip(c + rng.normal(0, size / 8, 3).astype(np.int64), 0, size - 1)
        k = rng.integers(0, 3)
        e = (vhx.Albedo(int(rng.integers(0, 256)), int(rng.integers(0, 256)), int(rng.integers(0, 256)), 255)
             if k == 0 else int(rng.integers(1, 50)) if k == 1 else
             (vhx.Albedo(int(rng.integers(0, 256)), 7, 9, 255), int(rng.integers(1, 9))))
        t.insert(p, e)
    # solid boxes at a level of detail (power-of-two sizes, aligned like the reference requires)
    for _ in range(3):
        s = int(2 ** rng.integers(0, max(1, int(np.log2(size)) - 1)))
        p = (rng.integers(0, size // s, 3) * s).astype(np.int64)
        t.insert_at_lod(p, s, vhx.Albedo(int(rng.integers(0, 256)), 40, 200, 255))
    for _ in range(200):
        p = rng.integers(0, size, 3)
        t.update(p, int(rng.integers(1, 50)))
    if seed % 2 == 0:
        t.simplify(recursive=True)
    return t, rng


@pytest.mark.parametrize("seed,size,bd", CASES)
def test_random_tree_vs_oracle(gpu, oracle, seed, size, bd):
    t, rng = random_tree(seed, size, bd)
    flat = t.flatten()
    gpu.upload(flat)
    o, d = rand_rays(rng, size, 12000)
    ref = oracle.trace_rays(flat, o, d, count_bytes=True)
    for budgets in (None, (1, 3, 9)):
        if budgets is not None:
            gpu.set_pass_budgets(budgets)
        assert_same(gpu.trace_rays(o, d, count_bytes=True), ref, f"rays seed {seed} bd {bd} budgets {budgets}")
    gpu.set_adaptive_schedule(True)
    W, H = 160, 96
    cam = vhx.glass_camera(size, W, H, angle=float(rng.uniform(0, 6.3)), radius=float(rng.uniform(0.3, 2.0)) * size,
                           target=tuple(float(v) for v in rng.uniform(0, size, 3)))
    fields = ("value", "cell", "voxel", "impact", "normal", "depth", "rgba")
    ref_f = oracle.trace_primary(flat, cam, 0, 0, W, H, count_bytes=True, fields=fields)
    got_f = gpu.trace_primary(cam, count_bytes=True, fields=fields)
    assert_same(got_f, ref_f, f"frame seed {seed} bd {bd}")
