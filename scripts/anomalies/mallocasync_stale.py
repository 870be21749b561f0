"""Runs the hipMallocAsync staging probe (mallocasync_stale.hip) on the HIP runtime torch loads, like libvhx under
Python. usage: mallocasync_stale.py MODE CALLS"""
import ctypes, os, sys
import torch  # noqa: F401  (its HIP runtime first, as voxelhex_amd._native does)
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libmallocasync_stale.so"))
sys.exit(lib.anomaly_run(int(sys.argv[1]), int(sys.argv[2])))
