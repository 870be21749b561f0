"""voxelhex_amd — MI355X-native drop-in for VoxelHex's `src/raytracing` module.

Host side (BoxTree data model and flattening) and the HIP kernels for gfx950 both live in libvhx.so
(C ABI: include/vhx.h, include/vhx_boxtree.h); this package mirrors the reference's Rust API on top of it.
"""
from .boxtree import (Albedo, BoxTree, BoxTreeEntry, FlatTree, InvalidBrickDimension, InvalidPosition, InvalidSize,
                      InvalidStructure, OctreeError, V3c, entry_from_value, voxel_data)
from .raytracing import BoxTreeGPUHost, BoxTreeGPUView, Ray, Raytracer, Viewport, default_raytracer, glass_camera
from .streaming import StreamingView
from . import _native as native

__all__ = [
    "Albedo", "BoxTree", "BoxTreeEntry", "FlatTree", "OctreeError", "InvalidSize", "InvalidBrickDimension",
    "InvalidStructure", "InvalidPosition", "V3c", "entry_from_value", "voxel_data", "Ray", "Raytracer", "Viewport",
    "BoxTreeGPUHost", "BoxTreeGPUView", "default_raytracer", "glass_camera", "native",
]
