"""Host-side BoxTree API, mirroring VoxelHex's `voxelhex::boxtree` (src/boxtree/mod.rs, src/boxtree/types.rs).

The tree itself lives in libvhx (C++ restatement of the reference's insert/get/simplify, include/vhx_boxtree.h);
this module keeps the reference's names, argument meaning and error behaviour:

    BoxTree(size, brick_dim)             BoxTree::new            -> raises OctreeError.InvalidSize / ...
    tree.insert(pos, entry)              BoxTree::insert         -> raises OctreeError.InvalidPosition
    tree.insert_at_lod(pos, size, entry) BoxTree::insert_at_lod
    tree.update(pos, entry)              BoxTree::update
    tree.get(pos) -> BoxTreeEntry        BoxTree::get
    tree.get_by_ray(ray)                 BoxTree::get_by_ray (src/raytracing/cpu.rs:296), traced on the GPU
"""
from dataclasses import dataclass
import ctypes

import numpy as np

from . import _native as N


class OctreeError(Exception):
    """OctreeError (src/boxtree/types.rs:9-21)."""


class InvalidSize(OctreeError):
    pass


class InvalidBrickDimension(OctreeError):
    pass


class InvalidStructure(OctreeError):
    pass


class InvalidPosition(OctreeError):
    pass


_TREE_ERRORS = {
    N.VHX_E_TREE_INVALID_SIZE: InvalidSize,
    N.VHX_E_TREE_INVALID_BRICK_DIMENSION: InvalidBrickDimension,
    N.VHX_E_TREE_INVALID_STRUCTURE: InvalidStructure,
    N.VHX_E_TREE_INVALID_POSITION: InvalidPosition,
}


def _tree_check(rc, what=""):
    if rc == N.VHX_OK:
        return
    if rc in _TREE_ERRORS:
        raise _TREE_ERRORS[rc](what)
    raise N.VhxError(rc, what)


@dataclass(frozen=True)
class V3c:
    x: float
    y: float
    z: float

    def __iter__(self):
        return iter((self.x, self.y, self.z))


@dataclass(frozen=True)
class Albedo:
    """Albedo (src/boxtree/types.rs:103-109)."""
    r: int = 0
    g: int = 0
    b: int = 0
    a: int = 0

    @staticmethod
    def from_u32(value):
        """impl From<u32> for Albedo (src/boxtree/detail.rs:72-85): 0xRRGGBBAA."""
        value &= 0xFFFFFFFF
        return Albedo((value >> 24) & 0xFF, (value >> 16) & 0xFF, (value >> 8) & 0xFF, value & 0xFF)

    @staticmethod
    def from_packed(p):
        return Albedo(p & 0xFF, (p >> 8) & 0xFF, (p >> 16) & 0xFF, (p >> 24) & 0xFF)

    def packed(self):
        """r | g<<8 | b<<16 | a<<24, the palette encoding of include/vhx.h."""
        return (self.r & 0xFF) | ((self.g & 0xFF) << 8) | ((self.b & 0xFF) << 16) | ((self.a & 0xFF) << 24)

    def is_transparent(self):
        return self.a == 0


@dataclass(frozen=True)
class BoxTreeEntry:
    """BoxTreeEntry<u32> (src/boxtree/types.rs:25-37): kind in {Empty, Visual, Informative, Complex}."""
    kind: str = "Empty"
    albedo_: Albedo = None
    data_: int = None

    @staticmethod
    def Empty():
        return BoxTreeEntry("Empty")

    @staticmethod
    def Visual(albedo):
        return BoxTreeEntry("Visual", albedo, None)

    @staticmethod
    def Informative(data):
        return BoxTreeEntry("Informative", None, int(data))

    @staticmethod
    def Complex(albedo, data):
        return BoxTreeEntry("Complex", albedo, int(data))

    def albedo(self):
        return self.albedo_ if self.kind in ("Visual", "Complex") else None

    def data(self):
        return self.data_ if self.kind in ("Informative", "Complex") else None

    def is_none(self):
        """BoxTreeEntry::is_none (src/boxtree/mod.rs:99-106)."""
        if self.kind == "Empty":
            return True
        if self.kind == "Visual":
            return self.albedo_.is_transparent()
        if self.kind == "Informative":
            return self.data_ == 0
        return self.albedo_.is_transparent() and self.data_ == 0

    def is_some(self):
        return not self.is_none()


class MIPResamplingMethods:
    """MIPResamplingMethods (src/boxtree/types.rs:113-149) as (code, threshold) pairs for set_method_at."""
    BoxFilter = (0, 0.0)
    PointFilter = (1, 0.0)
    PointFilterBD = (2, 0.0)

    @staticmethod
    def Posterize(thr):
        return (3, float(thr))

    @staticmethod
    def PosterizeBD(thr):
        return (4, float(thr))


class StrategyUpdater:
    """StrategyUpdater (src/boxtree/mipmap.rs:458-668): chainable MIP-map settings of a BoxTree."""

    def __init__(self, tree):
        self._t = tree

    def switch_albedo_mip_maps(self, enabled):
        N.check(N.lib().vhx_boxtree_switch_mips(self._t._h, int(bool(enabled))))
        self._t._version += 1
        return self

    def set_method_at(self, mip_level, method):
        code, thr = method
        N.check(N.lib().vhx_boxtree_set_mip_method(self._t._h, int(mip_level), code, thr))
        return self

    def set_color_similarity_thr_at(self, mip_level, similarity_thr):
        N.check(N.lib().vhx_boxtree_set_mip_color_threshold(self._t._h, int(mip_level), float(similarity_thr)))
        return self

    def recalculate_mips(self):
        N.check(N.lib().vhx_boxtree_recalculate_mips(self._t._h))
        self._t._version += 1
        return self

    def sample_root_mip(self, sectant, position):
        x, y, z = _pos(position)
        k, a, d = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        N.check(N.lib().vhx_boxtree_sample_root_mip(self._t._h, int(sectant), x, y, z, ctypes.byref(k),
                                                    ctypes.byref(a), ctypes.byref(d)))
        return _entry_of(k.value, a.value, d.value)


def _entry_of(kind, albedo, data):
    if kind == N.VHX_ENTRY_EMPTY:
        return BoxTreeEntry.Empty()
    if kind == N.VHX_ENTRY_VISUAL:
        return BoxTreeEntry.Visual(Albedo.from_packed(albedo))
    if kind == N.VHX_ENTRY_INFORMATIVE:
        return BoxTreeEntry.Informative(data)
    return BoxTreeEntry.Complex(Albedo.from_packed(albedo), data)


def voxel_data(data=None):
    """The reference's voxel_data! macro (src/boxtree/mod.rs:65-72)."""
    return BoxTreeEntry.Empty() if data is None else BoxTreeEntry.Informative(data)


def _entry(e):
    """Into<BoxTreeEntry>: Albedo -> Visual, int -> Informative, (Albedo, int) -> Complex."""
    if isinstance(e, BoxTreeEntry):
        return e
    if isinstance(e, Albedo):
        return BoxTreeEntry.Visual(e)
    if isinstance(e, tuple) and len(e) == 2:
        return BoxTreeEntry.Complex(e[0], e[1])
    if isinstance(e, (int, np.integer)):
        return BoxTreeEntry.Informative(int(e))
    raise TypeError(f"cannot convert {e!r} into a BoxTreeEntry")


def _entry_args(e):
    e = _entry(e)
    kinds = {"Empty": N.VHX_ENTRY_EMPTY, "Visual": N.VHX_ENTRY_VISUAL, "Informative": N.VHX_ENTRY_INFORMATIVE,
             "Complex": N.VHX_ENTRY_COMPLEX}
    alb = e.albedo_.packed() if e.albedo_ is not None else 0
    dat = (e.data_ or 0) & 0xFFFFFFFF
    return kinds[e.kind], alb, dat


def entry_from_value(value, color_palette, data_palette):
    """NodeContent::pix_get_ref (src/boxtree/node.rs:335-373) for a PaletteIndexValues."""
    value = int(value)
    ci, di = value & 0xFFFF, (value >> 16) & 0xFFFF
    cn, dn = ci == 0xFFFF, di == 0xFFFF
    if cn and dn:
        return BoxTreeEntry.Empty()
    alb = Albedo.from_packed(int(color_palette[ci])) if not cn and ci < len(color_palette) else None
    dat = int(data_palette[di]) if not dn and di < len(data_palette) else None
    if dn:
        return BoxTreeEntry.Visual(alb)
    if cn:
        return BoxTreeEntry.Informative(dat)
    return BoxTreeEntry.Complex(alb, dat)


def _pos(p):
    x, y, z = (int(v) for v in p)
    if min(x, y, z) < 0:
        raise InvalidPosition(f"{(x, y, z)}")
    return x, y, z


class _OwnedBuffer:
    """Buffer-protocol view of libvhx-owned memory that keeps its owner alive."""

    def __init__(self, owner, ptr, nbytes):
        self._owner = owner
        self._mem = (ctypes.c_char * nbytes).from_address(ptr)

    @property
    def __array_interface__(self):
        return {"shape": (len(self._mem),), "typestr": "|u1", "data": (ctypes.addressof(self._mem), False),
                "version": 3}


class FlatTree:
    """Flattened tree (vhx_tree_desc) owned by libvhx; arrays are zero-copy numpy views."""

    def __init__(self, handle):
        self._h = ctypes.c_void_p(handle)
        self.desc = N.TreeDesc()
        N.check(N.lib().vhx_flat_desc(self._h, ctypes.byref(self.desc)))
        d = self.desc
        n3 = d.brick_dim ** 3

        def arr(ptr, n, dt):
            if n == 0 or not ptr:
                return np.zeros(0, dt)
            # a view whose base chain holds this FlatTree, so the buffers outlive any temporary owner
            return np.asarray(_OwnedBuffer(self, ptr, n * np.dtype(dt).itemsize)).view(dt)

        self.node_type = arr(d.node_type, d.node_count, np.uint32)
        self.node_ocbits = arr(d.node_ocbits, d.node_count, np.uint64)
        self.node_children = arr(d.node_children, d.node_count * 64, np.uint32)
        self.voxels = arr(d.voxels, d.brick_count * n3, np.uint32)
        self.solid_values = arr(d.solid_values, d.solid_count, np.uint32)
        self.color_palette = arr(d.color_palette, d.color_count, np.uint32)
        self.data_palette = arr(d.data_palette, d.data_count, np.uint32)
        mp, mc = ctypes.c_void_p(), ctypes.c_uint32()
        N.check(N.lib().vhx_flat_node_mips(self._h, ctypes.byref(mp), ctypes.byref(mc)))
        # per node: its MIP brick descriptor (empty unless the tree was flattened with MIPs)
        self.node_mips = arr(mp.value, mc.value, np.uint32)

    @property
    def boxtree_size(self):
        return self.desc.boxtree_size

    @property
    def brick_dim(self):
        return self.desc.brick_dim

    def nbytes(self):
        return sum(a.nbytes for a in (self.node_type, self.node_ocbits, self.node_children, self.voxels,
                                      self.solid_values, self.color_palette, self.data_palette))

    @classmethod
    def _from_handle(cls, h):
        t = cls.__new__(cls)
        t._h = h
        t._version = 0
        t._flat = None
        t._flat_version = -1
        return t

    @classmethod
    def from_scene(cls, scene, size, brick_dim, seed=0x5EED, threads=0):
        """The tree insert_scene builds, from the bulk builder's image (vhx_scene_build_tree: seconds at 1024^3 where the
        insert loop takes minutes); occlusion bits and MIP maps are not restored (include/vhx_boxtree.h)."""
        h = ctypes.c_void_p()
        _tree_check(N.lib().vhx_scene_build_tree(scene, size, brick_dim, seed, threads, ctypes.byref(h)),
                    f"scene {scene} size {size} brick_dim {brick_dim}")
        return cls._from_handle(h)

    @classmethod
    def load_vox_file(cls, filename, brick_dimension):
        """BoxTree::load_vox_file (src/convert/magicavoxel.rs:234-265): MagicaVoxel .vox import (C++,
        voxelhex_amd/csrc/vox.cpp). Raises VhxError for unreadable / unsupported files, InvalidPosition for voxels
        outside the tree (the reference panics)."""
        h = ctypes.c_void_p()
        _tree_check(N.lib().vhx_boxtree_load_vox(str(filename).encode(), brick_dimension, ctypes.byref(h)),
                    f"{filename}")
        return cls._from_handle(h)

    @classmethod
    def load_vox_bytes(cls, data, brick_dimension):
        """load_vox_file over an in-memory .vox image."""
        buf = (ctypes.c_uint8 * len(data)).from_buffer_copy(bytes(data))
        h = ctypes.c_void_p()
        _tree_check(N.lib().vhx_boxtree_load_vox_memory(buf, len(data), brick_dimension, ctypes.byref(h)),
                    "vox bytes")
        return cls._from_handle(h)

    def __del__(self):
        if getattr(self, "_h", None) and self._h.value:
            N.lib().vhx_flat_free(self._h)
            self._h = ctypes.c_void_p(None)

    @staticmethod
    def build_scene(scene, size, brick_dim, seed=0x5EED, threads=0):
        """Bulk-builds the canonical tree that inserting `scene` voxel by voxel would produce."""
        h = ctypes.c_void_p()
        _tree_check(N.lib().vhx_scene_build(scene, size, brick_dim, seed, threads, ctypes.byref(h)),
                    f"scene {scene} size {size} brick_dim {brick_dim}")
        return FlatTree(h.value)

    @staticmethod
    def build_scene_lod(scene, size, brick_dim, max_depth, seed=0x5EED, threads=0):
        """build_scene with the default MIP maps switched on and flattened like BoxTree.flatten_lod(max_depth): the
        image the insert loop + switch_albedo_mip_maps(True) + flatten_lod would give, without the insert loop."""
        h = ctypes.c_void_p()
        _tree_check(N.lib().vhx_scene_build_lod(scene, size, brick_dim, seed, threads, int(max_depth), ctypes.byref(h)),
                    f"scene {scene} size {size} brick_dim {brick_dim}")
        return FlatTree(h.value)


class BoxTree:
    """BoxTree<u32> (src/boxtree/types.rs:219-255) backed by libvhx."""

    ROOT_NODE_KEY = 0

    def __init__(self, size, brick_dimension):
        h = ctypes.c_void_p()
        _tree_check(N.lib().vhx_boxtree_new(size, brick_dimension, ctypes.byref(h)),
                    f"size {size} brick_dim {brick_dimension}")
        self._h = h
        self._version = 0
        self._flat = None
        self._flat_version = -1

    @classmethod
    def _from_handle(cls, h):
        t = cls.__new__(cls)
        t._h = h
        t._version = 0
        t._flat = None
        t._flat_version = -1
        return t

    @classmethod
    def from_scene(cls, scene, size, brick_dim, seed=0x5EED, threads=0):
        """The tree insert_scene builds, from the bulk builder's image (vhx_scene_build_tree: seconds at 1024^3 where the
        insert loop takes minutes); occlusion bits and MIP maps are not restored (include/vhx_boxtree.h)."""
        h = ctypes.c_void_p()
        _tree_check(N.lib().vhx_scene_build_tree(scene, size, brick_dim, seed, threads, ctypes.byref(h)),
                    f"scene {scene} size {size} brick_dim {brick_dim}")
        return cls._from_handle(h)

    @classmethod
    def load_vox_file(cls, filename, brick_dimension):
        """BoxTree::load_vox_file (src/convert/magicavoxel.rs:234-265): MagicaVoxel .vox import (C++,
        voxelhex_amd/csrc/vox.cpp). Raises VhxError for unreadable / unsupported files, InvalidPosition for voxels
        outside the tree (the reference panics)."""
        h = ctypes.c_void_p()
        _tree_check(N.lib().vhx_boxtree_load_vox(str(filename).encode(), brick_dimension, ctypes.byref(h)),
                    f"{filename}")
        return cls._from_handle(h)

    @classmethod
    def load_vox_bytes(cls, data, brick_dimension):
        """load_vox_file over an in-memory .vox image."""
        buf = (ctypes.c_uint8 * len(data)).from_buffer_copy(bytes(data))
        h = ctypes.c_void_p()
        _tree_check(N.lib().vhx_boxtree_load_vox_memory(buf, len(data), brick_dimension, ctypes.byref(h)),
                    "vox bytes")
        return cls._from_handle(h)

    def __del__(self):
        if getattr(self, "_h", None) and self._h.value:
            N.lib().vhx_boxtree_free(self._h)
            self._h = ctypes.c_void_p(None)

    # -- reference API -------------------------------------------------------------------------------------------
    @property
    def auto_simplify(self):
        return self._auto_simplify if hasattr(self, "_auto_simplify") else True

    @auto_simplify.setter
    def auto_simplify(self, v):
        self._auto_simplify = bool(v)
        N.check(N.lib().vhx_boxtree_set_auto_simplify(self._h, int(bool(v))))

    def insert(self, position, data):
        x, y, z = _pos(position)
        _tree_check(N.lib().vhx_boxtree_insert(self._h, x, y, z, *_entry_args(data)), f"{(x, y, z)}")
        self._version += 1

    def insert_at_lod(self, position, insert_size, data):
        x, y, z = _pos(position)
        _tree_check(N.lib().vhx_boxtree_insert_at_lod(self._h, x, y, z, insert_size, *_entry_args(data)),
                    f"{(x, y, z)}")
        self._version += 1

    def update(self, position, data):
        x, y, z = _pos(position)
        _tree_check(N.lib().vhx_boxtree_update(self._h, x, y, z, *_entry_args(data)), f"{(x, y, z)}")
        self._version += 1

    def get(self, position):
        x, y, z = _pos(position)
        k, a, d = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        N.check(N.lib().vhx_boxtree_get(self._h, x, y, z, ctypes.byref(k), ctypes.byref(a), ctypes.byref(d)))
        return _entry_of(k.value, a.value, d.value)

    def albedo_mip_map_resampling_strategy(self):
        """BoxTree::albedo_mip_map_resampling_strategy (src/boxtree/mod.rs:241-243)."""
        return StrategyUpdater(self)

    def simplify(self, recursive=True):
        N.check(N.lib().vhx_boxtree_simplify(self._h, int(recursive)))
        self._version += 1

    def node_info(self, position):
        """The deepest node containing `position` (get_node_internal): key, content, occupied and occlusion bits."""
        key, content, occ, occl = ctypes.c_uint64(), ctypes.c_uint32(), ctypes.c_uint64(), ctypes.c_uint32()
        _tree_check(N.lib().vhx_boxtree_node_info(self._h, *[float(v) for v in position], ctypes.byref(key),
                                                  ctypes.byref(content), ctypes.byref(occ), ctypes.byref(occl)),
                    f"{position}")
        return {"key": key.value, "content": ("Nothing", "Internal", "Leaf", "UniformLeaf")[content.value],
                "occupied_bits": occ.value, "occlusion_bits": occl.value}

    def info(self):
        a = (ctypes.c_uint32 * 5)()
        N.check(N.lib().vhx_boxtree_info(self._h, ctypes.byref(a)))
        return dict(size=a[0], brick_dim=a[1], nodes=a[2], colors=a[3], data=a[4])

    def get_size(self):
        return self.info()["size"]

    def insert_scene(self, scene, seed=0x5EED):
        """Runs the reference insert loop of a procedural scene (vhx_scene_insert)."""
        N.check(N.lib().vhx_scene_insert(self._h, scene, seed))
        self._version += 1

    # -- flattening ------------------------------------------------------------------------------------------------
    def flatten(self):
        """Full-residency flattened image of the tree (cached until the tree changes)."""
        if self._flat is None or self._flat_version != self._version:
            h = ctypes.c_void_p()
            N.check(N.lib().vhx_boxtree_flatten(self._h, ctypes.byref(h)))
            self._flat = FlatTree(h.value)
            self._flat_version = self._version
        return self._flat

    def flatten_lod(self, max_depth):
        """Flattened image with node MIPs and only the nodes down to `max_depth` (root = 0): the deeper nodes are left
        out, their parents' MIPs stand in for them in a MIP-enabled trace (vhx_boxtree_flatten_lod)."""
        h = ctypes.c_void_p()
        N.check(N.lib().vhx_boxtree_flatten_lod(self._h, int(max_depth), ctypes.byref(h)))
        return FlatTree(h.value)

    # -- raytracing (src/raytracing/cpu.rs:296) ----------------------------------------------------------------
    def get_by_ray(self, ray, device=None):
        """Closest hit of `ray`: (BoxTreeEntry, impact_point, impact_normal) or None. Runs on the GPU."""
        from .raytracing import default_raytracer
        rt = default_raytracer(device)
        rt.upload(self.flatten())
        hits = rt.trace_rays(np.array([list(ray.origin)], np.float32), np.array([list(ray.direction)], np.float32))
        if hits["value"][0] == N.VHX_EMPTY:
            return None
        flat = self.flatten()
        entry = entry_from_value(hits["value"][0], flat.color_palette, flat.data_palette)
        return entry, V3c(*map(float, hits["impact"][0])), V3c(*map(float, hits["normal"][0]))
