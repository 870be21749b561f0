"""Diagnostic input: per-ray step counts of the bench frame (oracle, off-box) and the pixel lists the probes use.
usage: make_tail_pixels.py OUT.npz  ->  steps (per pixel), top64 (64 longest, longest first), tail (>256 steps),
t64 (>64 steps), and shuffled copies of the last two."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import voxelhex_amd as vhx
from voxelhex_amd import _native as N
from tests._oracle import ORACLE_LIB

W, H = 3840, 2160
flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 1024, 4)
cam = vhx.glass_camera(1024, W, H, target=(512.0, 512.0, 512.0))
lib = ctypes.CDLL(ORACLE_LIB)
steps = np.zeros(W * H, np.uint32)
rc = lib.vhx_oracle_ray_steps(ctypes.byref(flat.desc), ctypes.byref(cam), 0, 0, W, H,
                              steps.ctypes.data_as(ctypes.c_void_p), 0)
assert rc == 0
rng = np.random.default_rng(0)
order = np.argsort(-steps.astype(np.int64), kind="stable")
tail = np.nonzero(steps > 256)[0].astype(np.int64)
t64 = np.nonzero(steps > 64)[0].astype(np.int64)
np.savez_compressed(sys.argv[1], steps=steps.astype(np.uint16), top64=order[:64], tail=tail, tail_shuf=rng.permutation(tail), t64=t64,
         t64_shuf=rng.permutation(t64))
print("max steps", steps.max(), "tail>256", len(tail), "tail>64", len(t64), "mean", steps.mean())
