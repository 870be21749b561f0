"""A flattened tree held in numpy arrays (a derived fixture under tests/golden/) with the vhx_tree_desc that libvhx
(vhx_upload_tree) and the oracle read, like voxelhex_amd.FlatTree. Test infrastructure."""
import numpy as np

from voxelhex_amd import _native as N

FIELDS = ("node_type", "node_ocbits", "node_children", "voxels", "solid_values", "color_palette", "data_palette")
DTYPES = {"node_ocbits": np.uint64}


class ArrayTree:
    def __init__(self, npz_path):
        z = np.load(npz_path)  # no pickles: allow_pickle stays False
        self.arrays = {k: np.ascontiguousarray(z[k], DTYPES.get(k, np.uint32)) for k in FIELDS}
        size, bd = (int(v) for v in z["sizes"])
        a = self.arrays
        d = N.TreeDesc()
        d.boxtree_size, d.brick_dim = size, bd
        d.node_count = a["node_type"].size
        d.brick_count = a["voxels"].size // (bd ** 3)
        d.solid_count, d.color_count, d.data_count = (a["solid_values"].size, a["color_palette"].size,
                                                      a["data_palette"].size)
        for k in FIELDS:
            setattr(d, k, a[k].ctypes.data if a[k].size else None)
        self.desc = d
        self.source_sha256 = str(z["source_sha256"]) if "source_sha256" in z else None

    @property
    def boxtree_size(self):
        return self.desc.boxtree_size

    @property
    def brick_dim(self):
        return self.desc.brick_dim

    def nbytes(self):
        return sum(v.nbytes for v in self.arrays.values())
