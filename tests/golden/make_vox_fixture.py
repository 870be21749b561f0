"""Derived test input for the GPU: the tree BoxTree::load_vox_file (restated in voxelhex_amd/csrc/vox.cpp) builds from
the reference's own model asset whisp/assets/models/gingerbread_house_by_kirra_luan.vox (brick_dim 8, a 2048^3 tree),
flattened and stored as compressed arrays, so that the GPU box (which has no /root/reference) can trace the reference's
real model against the oracle. The source file's SHA-256 is recorded; tests/test_vox.py rebuilds the tree from the
asset when the reference checkout is present and checks it equals this fixture.

usage: python tests/golden/make_vox_fixture.py  ->  tests/golden/gingerbread_bd8.npz
"""
import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
SRC = "/root/reference/whisp/assets/models/gingerbread_house_by_kirra_luan.vox"
OUT = os.path.join(ROOT, "tests", "golden", "gingerbread_bd8.npz")
FIELDS = ("node_type", "node_ocbits", "node_children", "voxels", "solid_values", "color_palette", "data_palette")


def build(path=SRC, brick_dim=8):
    import voxelhex_amd as vhx
    flat = vhx.BoxTree.load_vox_file(path, brick_dim).flatten()
    arrays = {k: np.array(getattr(flat, k), copy=True) for k in FIELDS}
    arrays["sizes"] = np.array([flat.desc.boxtree_size, flat.desc.brick_dim], np.uint32)
    return arrays


def main():
    arrays = build()
    sha = hashlib.sha256(open(SRC, "rb").read()).hexdigest()
    np.savez_compressed(OUT, source_sha256=np.array(sha), **arrays)
    print(OUT, os.path.getsize(OUT), "bytes; source", sha)


if __name__ == "__main__":
    main()
