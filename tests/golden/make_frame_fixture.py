"""Golden frames: the oracle's hit buffers for the BASELINE geometries, committed as SHA-256 digests
of every field of the full frames plus a 64x64 crop of value / depth / rgba around the frame centre.

The oracle (oracle/vhx_oracle.c) is the generator; it is pinned to the reference by the reference's own KATs
(tests/test_oracle_kats.py, tests/test_oracle_spatial.py). These fixtures freeze its frames so that the oracle itself
cannot drift unnoticed (tests/test_golden_frames.py recomputes the small ones on the CPU) and so that the GPU frames
can be checked against committed data without running the oracle (tests/test_gpu_golden.py).

Run in the build container:  python tests/golden/make_frame_fixture.py
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

FIELDS = ("value", "cell", "voxel", "impact", "normal", "depth", "rgba")
CROP = 64
# name: (scene, tree size, brick_dim, width, height) -- BASELINE configs 1, 2 and 3 (SURVEY.md 8d mapping)
CASES = {
    "c1_32_bd8_256x256": (1, 32, 8, 256, 256),
    "c1_32_bd2_256x256": (1, 32, 2, 256, 256),
    "c2_256_bd4_1920x1080": (1, 256, 4, 1920, 1080),
    "c2_256_bd16_1920x1080": (1, 256, 16, 1920, 1080),
    "c3_1024_bd4_3840x2160": (1, 1024, 4, 3840, 2160),
}
# node-MIP views: the scene inserted into a host BoxTree with MIP maps on, flattened down to a depth
# (vhx_boxtree_flatten_lod) and traced with the MIP stand-ins -- pins the host MIP generation and the stand-in rule
# name: (scene, tree size, brick_dim, width, height, depth)
MIP_CASES = {
    "mip_lod0_64_bd4_256x256": (1, 64, 4, 256, 256, 0),
    "mip_lod1_256_bd4_480x270": (1, 256, 4, 480, 270, 1),
}


def digest(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def frame(oracle, scene, size, bd, W, H):
    import voxelhex_amd as vhx
    flat = vhx.FlatTree.build_scene(scene, size, bd)
    cam = vhx.glass_camera(size, W, H, target=(size / 2,) * 3)
    return flat, cam, oracle.trace_primary(flat, cam, 0, 0, W, H, fields=FIELDS)


def mip_view(scene, size, bd, depth):
    from voxelhex_amd.boxtree import BoxTree
    tree = BoxTree(size, bd)
    tree.insert_scene(scene)
    tree.albedo_mip_map_resampling_strategy().switch_albedo_mip_maps(True)
    return tree.flatten_lod(depth)


def mip_frame(oracle, scene, size, bd, W, H, depth):
    import voxelhex_amd as vhx
    flat = mip_view(scene, size, bd, depth)
    cam = vhx.glass_camera(size, W, H, target=(size / 2,) * 3)
    with oracle.node_mips(flat.node_mips):
        return flat, cam, oracle.trace_primary(flat, cam, 0, 0, W, H, fields=FIELDS)


def crop(a, W, H):
    x0, y0 = (W - CROP) // 2, (H - CROP) // 2
    img = a.reshape(H, W, *a.shape[1:])
    return img[y0:y0 + CROP, x0:x0 + CROP].reshape(CROP * CROP, *a.shape[1:])


def main():
    from tests._oracle import Oracle
    oracle = Oracle()
    meta, crops = {}, {}
    for name, case in list(CASES.items()) + list(MIP_CASES.items()):
        scene, size, bd, W, H = case[:5]
        _, _, f = frame(oracle, *case[:5]) if name in CASES else mip_frame(oracle, *case)
        meta[name] = {"scene": scene, "size": size, "brick_dim": bd, "width": W, "height": H,
                      "camera": "glass_camera(size, W, H, target=(size/2,)*3)",
                      "sha256": {k: digest(f[k]) for k in FIELDS},
                      "hits": int((f["value"] != 0xFFFFFFFF).sum())}
        if name in MIP_CASES:
            meta[name]["mip_lod_depth"] = case[5]
        for k in ("value", "depth", "rgba"):
            crops[f"{name}__{k}"] = crop(f[k], W, H)
        print(name, meta[name]["hits"], flush=True)
    json.dump(meta, open(os.path.join(HERE, "frames.json"), "w"), indent=1, sort_keys=True)
    np.savez_compressed(os.path.join(HERE, "frame_crops.npz"), **crops)


if __name__ == "__main__":
    main()
