"""Fraction of the 3840x2160 headline frame (scene S 1024^3, brick_dim 4, glass camera) whose hit value differs between
the exact path and the MIP stand-in views of vhx_scene_build_lod at depths 1 and 2 (docs/DESIGN_LOG.md §10b)."""
import numpy as np
import voxelhex_amd as vhx
from voxelhex_amd import _native as N

S, W, H = 1024, 3840, 2160
cam = vhx.glass_camera(S, W, H, target=(S / 2,) * 3)
rt = vhx.Raytracer(0)
rt.upload(vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, S, 4, threads=16))
exact = rt.trace_primary(cam)["value"].copy()
print("exact hit fraction", round(float((exact != N.VHX_EMPTY).mean()), 4), flush=True)
for depth in (1, 2):
    flat = vhx.FlatTree.build_scene_lod(N.VHX_SCENE_LATTICE_CUBE, S, 4, depth, threads=16)
    rt.upload(flat)
    rt.set_node_mips(flat.node_mips)
    v = rt.trace_primary(cam)["value"]
    rt.set_node_mips(None)
    hit_e, hit_l = exact != N.VHX_EMPTY, v != N.VHX_EMPTY
    print(f"depth {depth}: nodes {flat.node_type.size}, pixels with a different value {float((v != exact).mean()):.4f}, "
          f"hit/miss differs {float((hit_e != hit_l).mean()):.4f}", flush=True)
rt.close()
