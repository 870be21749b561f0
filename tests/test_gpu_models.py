"""Frames at the BASELINE configs' own resolutions and on the reference's real model, GPU against the oracle.

* Config 2: 1920x1080 primary rays on the 256^3 trees (brick_dim 4 and 16), glass camera aimed at the
  tree centre, every hit field and the byte counts.
* Config 3 on the reference's own asset: the gingerbread house (whisp/assets/models/gingerbread_house_by_kirra_luan.vox)
  imported by vhx_boxtree_load_vox at brick_dim 8 (a 2048^3 tree). The GPU box has no reference checkout, so the tree
  travels as a derived fixture (tests/golden/gingerbread_bd8.npz, made by tests/golden/make_vox_fixture.py and checked
  against the asset by tests/test_vox.py where the checkout exists).
"""
import os

import numpy as np
import pytest

import voxelhex_amd as vhx
from voxelhex_amd import _native as N
from tests._arraytree import ArrayTree
from tests.test_gpu_parity import assert_same

pytestmark = pytest.mark.gpu

GINGERBREAD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "gingerbread_bd8.npz")


@pytest.mark.parametrize("bd", [4, 16])
def test_config2_1080p_frame_vs_oracle(gpu, oracle, bd):
    flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 256, bd)
    gpu.upload(flat)
    cam = vhx.glass_camera(256, 1920, 1080, target=(128.0, 128.0, 128.0))
    got = gpu.trace_primary(cam, count_bytes=True)
    ref = oracle.trace_primary(flat, cam, 0, 0, 1920, 1080, count_bytes=True)
    assert_same(got, ref, f"config 2, 1920x1080, 256^3 bd{bd}")
    assert (got["value"] != N.VHX_EMPTY).mean() > 0.1


@pytest.mark.parametrize("W,H,radius,target", [(1920, 1080, 0.7, (0.25, 0.125, 0.25)),
                                                (3840, 2160, 1.0, (0.5, 700 / 2048, 0.1875))])
def test_gingerbread_model_frame_vs_oracle(gpu, oracle, W, H, radius, target):
    tree = ArrayTree(GINGERBREAD)
    assert tree.brick_dim == 8 and tree.boxtree_size == 2048
    gpu.upload(tree)
    S = float(tree.boxtree_size)
    # glass camera of benches/performance.rs at 40 rad, closer than the default 2S (the house fills the lower third of
    # the 2048^3 cube: x 0..2048, y 0..2040, z 0..768)
    cam = vhx.glass_camera(int(S), W, H, radius=radius * S, target=tuple(t * S for t in target))
    fields = ("value", "cell", "voxel", "impact", "normal", "depth", "rgba")
    got = gpu.trace_primary(cam, fields=fields, count_bytes=True)
    ref = oracle.trace_primary(tree, cam, 0, 0, W, H, fields=fields, count_bytes=True)
    assert_same(got, ref, f"gingerbread {W}x{H}")
    assert (got["value"] != N.VHX_EMPTY).mean() > 0.05
