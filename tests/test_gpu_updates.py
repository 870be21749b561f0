"""Ranged writes into an uploaded tree (vhx_update_range / vhx_update_ranges; the reference's write_range_to_buffer,
src/raytracing/bevy/streaming/mod.rs:344-370, issued per range of a streaming::upload frame, 420-635).

The writes are stream-ordered (no host synchronisation) and refresh the derived device state selectively: node headers
of the written nodes, bitmaps of the written bricks, the child records of the written nodes and of the nodes holding
written bricks (brick_dim <= 4), everything after a palette write. Each test edits the host arrays the oracle reads the
same way and compares traces; the sources are overwritten right after the call (they are staged before it returns).
"""
import numpy as np
import pytest

import voxelhex_amd as vhx
from voxelhex_amd import _native as N
from tests.test_gpu_parity import assert_same, rand_rays

pytestmark = pytest.mark.gpu


def _tree(size=64, bd=4):
    t = vhx.BoxTree(size, bd)
    t.insert_scene(N.VHX_SCENE_LATTICE_CUBE)
    return t.flatten()


def _frame(rt, oracle, flat, what):
    S = float(flat.desc.boxtree_size)
    cam = vhx.glass_camera(int(S), 160, 96, target=(S / 2, S / 2, S / 2))
    assert_same(rt.trace_primary(cam, count_bytes=True), oracle.trace_primary(flat, cam, 0, 0, 160, 96,
                                                                              count_bytes=True), what)


@pytest.mark.parametrize("bd", [4, 8])
def test_update_ranges_batch(oracle, bd):
    size = 64 if bd == 4 else 128  # BoxTree sizes are brick_dim * 4^k
    flat = _tree(size, bd)
    rt = vhx.Raytracer(0)
    try:
        rt.upload(flat)
        rng = np.random.default_rng(bd)
        o, d = rand_rays(rng, size, 6000)
        n3 = bd ** 3
        nb = flat.desc.brick_count
        nn = flat.desc.node_count
        writes = []
        # voxels of a few bricks only (their holders' child records must follow without a node write)
        for b in rng.choice(nb, size=min(6, nb), replace=False):
            v = flat.voxels[b * n3:(b + 1) * n3].copy()
            v[rng.random(n3) < 0.5] = N.VHX_EMPTY
            flat.voxels[b * n3:(b + 1) * n3] = v
            writes.append((N.VHX_BUF_VOXELS, int(b) * n3, v))
        # children entries of one leaf node: a brick dropped
        leaves = np.flatnonzero(flat.node_type == N.VHX_NODE_LEAF)
        if leaves.size:
            k = int(leaves[len(leaves) // 2])
            ch = flat.node_children[k * 64:(k + 1) * 64].copy()
            ch[rng.random(64) < 0.3] = N.VHX_EMPTY
            flat.node_children[k * 64:(k + 1) * 64] = ch
            writes.append((N.VHX_BUF_NODE_CHILDREN, k * 64, ch))
        # occupancy bits of two nodes (pop decisions) and one node type
        for k in (1 % nn, nn // 2):
            ob = flat.node_ocbits[k:k + 1].copy()
            ob[0] &= np.uint64(0x0F0F0F0F0F0F0F0F)
            flat.node_ocbits[k:k + 1] = ob
            writes.append((N.VHX_BUF_NODE_OCBITS, k, ob))
        if leaves.size > 1:
            k = int(leaves[0])
            ty = np.array([N.VHX_NODE_NOTHING], np.uint32)
            flat.node_type[k:k + 1] = ty
            writes.append((N.VHX_BUF_NODE_TYPE, k, ty))
        rt.update_ranges(writes)
        for _, _, v in writes:  # the sources were staged before the call returned
            v[...] = 0
        assert_same(rt.trace_rays(o, d, count_bytes=True), oracle.trace_rays(flat, o, d, count_bytes=True),
                    f"batch bd{bd}")
        _frame(rt, oracle, flat, f"batch frame bd{bd}")
        # a palette write: a colour made transparent empties its cells everywhere
        if flat.desc.color_count:
            col = flat.color_palette[:1].copy()
            col[0] &= np.uint32(0x00FFFFFF)
            flat.color_palette[:1] = col
            rt.update_ranges([(N.VHX_BUF_COLOR_PALETTE, 0, col)])
            col[...] = 0xFFFFFFFF
            assert_same(rt.trace_rays(o, d, count_bytes=True), oracle.trace_rays(flat, o, d, count_bytes=True),
                        f"palette bd{bd}")
        # consecutive single-range writes, no synchronisation between them
        for b in range(min(nb, 40)):
            v = np.full(n3, N.VHX_EMPTY, np.uint32)
            flat.voxels[b * n3:(b + 1) * n3] = v
            rt.update_range(N.VHX_BUF_VOXELS, b * n3, v)
        _frame(rt, oracle, flat, f"single writes bd{bd}")
        # validation: nothing is written when one range of a batch is out of bounds
        before = rt.trace_rays(o, d)
        bad = [(N.VHX_BUF_VOXELS, 0, np.zeros(n3, np.uint32)), (N.VHX_BUF_VOXELS, flat.voxels.size - 2,
                                                                np.zeros(4, np.uint32))]
        with pytest.raises(N.VhxError):
            rt.update_ranges(bad)
        assert_same(rt.trace_rays(o, d), before, "failed batch wrote nothing")
    finally:
        rt.close()


def test_update_ranges_large_and_many(oracle):
    """A batch of 3000 small ranges plus one range of several MB (pieces of 16 KiB), twice, on the bench tree size."""
    flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 256, 4)
    rt = vhx.Raytracer(0)
    try:
        rt.upload(flat)
        rng = np.random.default_rng(3)
        n3 = 64
        for rep in range(2):
            writes = []
            for b in rng.choice(flat.desc.brick_count, size=3000, replace=False):
                v = flat.voxels[b * n3:(b + 1) * n3].copy()
                v[rng.random(n3) < 0.2] = N.VHX_EMPTY
                flat.voxels[b * n3:(b + 1) * n3] = v
                writes.append((N.VHX_BUF_VOXELS, int(b) * n3, v))
            lo = int(rng.integers(0, flat.desc.brick_count // 2)) * n3
            big = flat.voxels[lo:lo + (1 << 20)].copy()
            big[rng.random(big.size) < 0.1] = N.VHX_EMPTY
            flat.voxels[lo:lo + big.size] = big
            writes.append((N.VHX_BUF_VOXELS, lo, big))
            rt.update_ranges(writes)
            _frame(rt, oracle, flat, f"large batch {rep}")
    finally:
        rt.close()
