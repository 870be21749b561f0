"""ctypes bindings of libvhx.so (include/vhx.h, include/vhx_boxtree.h).

The library is built in-tree by voxelhex_amd/_build.py (or __graft_entry__.build()). There is no fallback: if the
library is missing, importing the GPU path raises immediately.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# VHX_LIB: an alternative build of libvhx (A/B probes of kernel variants); the in-tree build by default
LIB_PATH = os.environ.get("VHX_LIB") or os.path.join(_HERE, "_lib", "libvhx.so")

c_u32 = ctypes.c_uint32
c_u64 = ctypes.c_uint64
c_int = ctypes.c_int
c_f32 = ctypes.c_float
c_void_p = ctypes.c_void_p
P = ctypes.POINTER

VHX_OK = 0
VHX_E_INVALID_ARG = -1
VHX_E_HIP = -2
VHX_E_CAPACITY = -3
VHX_E_NO_DEVICE = -4
VHX_E_STATE = -5
VHX_E_RCCL = -6
VHX_MGPU_ID_BYTES = 128
VHX_MGPU_MAX_INFLIGHT = 16
VHX_MGPU_MAX_ROOT_SLOTS = 4
VHX_MAX_BUDGETS = 6
VHX_E_TREE_INVALID_SIZE = -10
VHX_E_TREE_INVALID_BRICK_DIMENSION = -11
VHX_E_TREE_INVALID_STRUCTURE = -12
VHX_E_TREE_INVALID_POSITION = -13
VHX_E_VOX_FORMAT = -14
VHX_E_VOX_IO = -15

VHX_EMPTY = 0xFFFFFFFF
VHX_SOLID_BIT = 0x80000000
VHX_NODE_NOTHING, VHX_NODE_INTERNAL, VHX_NODE_LEAF, VHX_NODE_UNIFORM_LEAF = 0, 1, 2, 3
VHX_ENTRY_EMPTY, VHX_ENTRY_VISUAL, VHX_ENTRY_INFORMATIVE, VHX_ENTRY_COMPLEX = 0, 1, 2, 3
VHX_RAY_INVERSE_VP, VHX_RAY_GLASS = 0, 1
VHX_LAYOUT_FRAMEBUFFER, VHX_LAYOUT_TILES = 0, 1
VHX_SCENE_LATTICE_CUBE, VHX_SCENE_BENCH_REGION, VHX_SCENE_LATTICE = 1, 2, 3
VHX_SCENE_CUBE, VHX_SCENE_BOUNDARY, VHX_SCENE_HEIGHTFIELD = 4, 5, 6
VHX_BUF_NODE_TYPE, VHX_BUF_NODE_OCBITS, VHX_BUF_NODE_CHILDREN, VHX_BUF_VOXELS = 0, 1, 2, 3
VHX_BUF_SOLID_VALUES, VHX_BUF_COLOR_PALETTE, VHX_BUF_DATA_PALETTE = 4, 5, 6
VHX_DERIVED_NODE_HDR, VHX_DERIVED_BRICK_OCC = 0, 1


class TreeDesc(ctypes.Structure):
    _fields_ = [
        ("boxtree_size", c_u32), ("brick_dim", c_u32), ("node_count", c_u32), ("brick_count", c_u32),
        ("solid_count", c_u32), ("color_count", c_u32), ("data_count", c_u32), ("reserved0", c_u32),
        ("node_type", c_void_p), ("node_ocbits", c_void_p), ("node_children", c_void_p), ("voxels", c_void_p),
        ("solid_values", c_void_p), ("color_palette", c_void_p), ("data_palette", c_void_p),
    ]


class Range(ctypes.Structure):
    _fields_ = [("buffer_id", ctypes.c_int32), ("reserved0", c_u32), ("elem_offset", c_u64), ("elem_count", c_u64),
                ("src", c_void_p)]


class Camera(ctypes.Structure):
    _fields_ = [
        ("ray_model", c_u32), ("width", c_u32), ("height", c_u32), ("reserved0", c_u32),
        ("origin", c_f32 * 3), ("glass_bottom_left", c_f32 * 3), ("glass_right", c_f32 * 3),
        ("glass_up", c_f32 * 3), ("pixel_width", c_f32), ("pixel_height", c_f32),
        ("inv_view_proj", c_f32 * 16),
    ]


class TilePlan(ctypes.Structure):
    _fields_ = [(n, c_u32) for n in ("tiles_x", "tiles_y", "tiles", "slots", "tiles_per_slot", "first_slot",
                                     "slot_count", "reserved")]


class Hits(ctypes.Structure):
    _fields_ = [
        ("value", c_void_p), ("cell", c_void_p), ("voxel", c_void_p), ("impact", c_void_p),
        ("normal", c_void_p), ("depth", c_void_p), ("rgba", c_void_p), ("bytes", c_void_p),
        ("shadowed", c_void_p),  # ABI 6
    ]


class ShadowFrame(ctypes.Structure):  # vhx_shadow_frame
    _fields_ = [("value", c_void_p), ("impact", c_void_p), ("normal", c_void_p), ("shadowed", c_void_p),
                ("rgba", c_void_p)]


# (name, restype, argtypes) — one line per symbol declared in include/*.h
SIGNATURES = [
    ("vhx_abi_version", c_u32, []),
    ("vhx_device_count", c_int, [P(c_int)]),
    ("vhx_device_error", ctypes.c_char_p, []),
    ("vhx_create", c_int, [c_int, P(c_void_p)]),
    ("vhx_create_shared", c_int, [c_void_p, P(c_void_p)]),
    ("vhx_destroy", None, [c_void_p]),
    ("vhx_last_error", ctypes.c_char_p, [c_void_p]),
    ("vhx_set_stream", c_int, [c_void_p, c_void_p]),
    ("vhx_get_stream", c_int, [c_void_p, P(c_void_p)]),
    ("vhx_sync", c_int, [c_void_p, P(c_f32)]),
    ("vhx_set_pass_budgets", c_int, [c_void_p, P(c_u32), c_u32]),
    ("vhx_set_adaptive_schedule", c_int, [c_void_p, c_int]),
    ("vhx_get_pass_budgets", c_int, [c_void_p, P(c_u32), P(c_u32), P(c_int)]),
    ("vhx_set_tuning", c_int, [c_void_p, ctypes.c_char_p]),
    ("vhx_upload_tree", c_int, [c_void_p, P(TreeDesc)]),
    ("vhx_upload_tree_device", c_int, [c_void_p, P(TreeDesc)]),
    ("vhx_set_node_mips", c_int, [c_void_p, c_void_p, c_u32]),
    ("vhx_update_range", c_int, [c_void_p, c_int, c_u64, c_u64, c_void_p]),
    ("vhx_update_ranges", c_int, [c_void_p, c_void_p, c_u32]),
    ("vhx_set_depth_prepass", c_int, [c_void_p, c_int, ctypes.c_float]),
    ("vhx_set_shadow_light", c_int, [c_void_p, c_void_p]),
    ("vhx_read_derived", c_int, [c_void_p, c_int, c_u64, c_u64, c_void_p]),
    ("vhx_tree_device_bytes", c_int, [c_void_p, P(c_u64)]),
    ("vhx_trace_primary", c_int, [c_void_p, P(Camera), c_u32, c_u32, c_u32, c_u32, P(Hits), c_int]),
    ("vhx_trace_primary_batch", c_int, [c_void_p, c_void_p, c_u32, c_void_p]),
    ("vhx_trace_tiles_batch", c_int, [c_void_p, c_void_p, c_u32, c_u32, c_void_p, c_u32, c_void_p]),
    ("vhx_profile_counters", c_int, [c_void_p, P(c_u64), c_u32, c_int]),
    ("vhx_chain_profile", c_int, [c_void_p, c_void_p, P(c_u32), c_u32, P(c_u64)]),
    ("vhx_tail_info", c_int, [c_void_p, P(c_u32), P(c_u32), P(c_u32)]),
    ("vhx_trace_rays", c_int, [c_void_p, c_void_p, c_u64, P(Hits), c_int]),
    ("vhx_trace_shadows", c_int, [c_void_p, P(c_f32), c_u64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                  c_void_p]),
    ("vhx_trace_shadows_batch", c_int, [c_void_p, P(c_f32), c_u32, c_u64, c_void_p]),
    ("vhx_untile_rgba", c_int, [c_void_p, c_void_p, c_u32, c_u32, c_u32, c_u32, c_u32, c_void_p, c_int]),
    ("vhx_untile_frame", c_int, [c_void_p, c_void_p, c_u32, c_u32, c_u32, c_u32, c_u32, c_u32, c_void_p, c_void_p]),
    ("vhx_mgpu_unique_id", c_int, [c_void_p]),
    ("vhx_mgpu_create", c_int, [c_void_p, c_void_p, c_int, c_int, c_u32, P(c_void_p)]),
    ("vhx_mgpu_create_from_comm", c_int, [c_void_p, c_void_p, c_u32, P(c_void_p)]),
    ("vhx_mgpu_broadcast_tree", c_int, [c_void_p, P(TreeDesc)]),
    ("vhx_mgpu_set_overlap", c_int, [c_void_p, c_int]),
    ("vhx_mgpu_set_frames_in_flight", c_int, [c_void_p, c_u32]),
    ("vhx_mgpu_render", c_int, [c_void_p, P(Camera), c_void_p, c_void_p]),
    ("vhx_mgpu_render_batch", c_int, [c_void_p, c_void_p, c_u32, c_void_p, c_void_p]),
    ("vhx_mgpu_sync", c_int, [c_void_p, P(c_f32)]),
    ("vhx_mgpu_info", c_int, [c_void_p, c_u32, c_u32, P(c_int), P(c_int), P(c_u64)]),
    ("vhx_mgpu_set_root_slots", c_int, [c_void_p, c_u32]),
    ("vhx_mgpu_set_planes", c_int, [c_void_p, c_u32]),
    ("vhx_mgpu_frame_bytes", c_int, [c_void_p, c_u32, c_u32, P(c_u64)]),
    ("vhx_mgpu_balance", c_int, [c_void_p, P(Camera), c_u32, P(c_u32), P(c_f32), P(c_f32)]),
    ("vhx_mgpu_tile_plan", c_int, [c_u32, c_u32, c_u32, c_u32, c_u32, c_u32, P(TilePlan)]),
    ("vhx_mgpu_measure", c_int, [c_void_p, P(Camera), c_u32, P(c_f32), P(c_f32)]),
    ("vhx_mgpu_destroy", None, [c_void_p]),
    ("vhx_boxtree_new", c_int, [c_u32, c_u32, P(c_void_p)]),
    ("vhx_boxtree_set_mip_options", c_int, [c_int, c_int]),
    ("vhx_boxtree_free", None, [c_void_p]),
    ("vhx_boxtree_set_auto_simplify", c_int, [c_void_p, c_int]),
    ("vhx_boxtree_insert", c_int, [c_void_p, c_u32, c_u32, c_u32, c_u32, c_u32, c_u32]),
    ("vhx_boxtree_insert_at_lod", c_int, [c_void_p, c_u32, c_u32, c_u32, c_u32, c_u32, c_u32, c_u32]),
    ("vhx_boxtree_update", c_int, [c_void_p, c_u32, c_u32, c_u32, c_u32, c_u32, c_u32]),
    ("vhx_boxtree_get", c_int, [c_void_p, c_u32, c_u32, c_u32, P(c_u32), P(c_u32), P(c_u32)]),
    ("vhx_boxtree_simplify", c_int, [c_void_p, c_int]),
    ("vhx_boxtree_info", c_int, [c_void_p, P(c_u32 * 5)]),
    ("vhx_scene_insert", c_int, [c_void_p, c_u32, c_u64]),
    ("vhx_boxtree_flatten", c_int, [c_void_p, P(c_void_p)]),
    ("vhx_stream_create", c_int, [c_void_p, c_void_p, P(c_f32), c_f32, P(c_void_p)]),
    ("vhx_stream_destroy", None, [c_void_p]),
    ("vhx_stream_set_rates", c_int, [c_void_p, c_u32, c_u32, c_u32]),
    ("vhx_stream_set_viewport", c_int, [c_void_p, P(c_f32), c_f32]),
    ("vhx_stream_upload", c_int, [c_void_p, c_void_p]),
    ("vhx_stream_upload_frames", c_int, [c_void_p, c_u32, c_void_p]),
    ("vhx_stream_resize", c_int, [c_void_p]),
    ("vhx_stream_reload", c_int, [c_void_p]),
    ("vhx_stream_view_set_check", c_int, [c_void_p, P(ctypes.c_uint64), P(ctypes.c_uint64)]),
    ("vhx_stream_view", c_int, [c_void_p, P(TreeDesc)]),
    ("vhx_stream_node_mips", c_int, [c_void_p, P(c_void_p), P(c_u32)]),
    ("vhx_boxtree_node_info", c_int, [c_void_p, c_f32, c_f32, c_f32, P(c_u64), P(c_u32), P(c_u64), P(c_u32)]),
    ("vhx_boxtree_load_vox", c_int, [ctypes.c_char_p, c_u32, P(c_void_p)]),
    ("vhx_boxtree_load_vox_memory", c_int, [c_void_p, c_u64, c_u32, P(c_void_p)]),
    ("vhx_vox_tree_size", c_u32, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, c_u32]),
    ("vhx_vox_rotation", c_int, [ctypes.c_uint8, P(ctypes.c_int32 * 9)]),
    ("vhx_scene_build", c_int, [c_u32, c_u32, c_u32, c_u64, c_int, P(c_void_p)]),
    ("vhx_scene_build_lod", c_int, [c_u32, c_u32, c_u32, c_u64, c_int, c_u32, P(c_void_p)]),
    ("vhx_scene_build_tree", c_int, [c_u32, c_u32, c_u32, c_u64, c_int, P(c_void_p)]),
    ("vhx_flat_desc", c_int, [c_void_p, P(TreeDesc)]),
    ("vhx_boxtree_switch_mips", c_int, [c_void_p, c_int]),
    ("vhx_boxtree_set_mip_method", c_int, [c_void_p, c_u32, c_u32, c_f32]),
    ("vhx_boxtree_set_mip_color_threshold", c_int, [c_void_p, c_u32, c_f32]),
    ("vhx_boxtree_recalculate_mips", c_int, [c_void_p]),
    ("vhx_boxtree_sample_root_mip", c_int, [c_void_p, c_u32, c_u32, c_u32, c_u32, P(c_u32), P(c_u32), P(c_u32)]),
    ("vhx_boxtree_flatten_lod", c_int, [c_void_p, c_u32, P(c_void_p)]),
    ("vhx_flat_node_mips", c_int, [c_void_p, P(c_void_p), P(c_u32)]),
    ("vhx_flat_free", None, [c_void_p]),
]

_lib = None


def lib():
    """Loads libvhx.so (raises if it has not been built — there is no CPU fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
        try:
            # torch ships its own HIP runtime (libamdhip64.so.7); loading it first makes libvhx bind to the same
            # runtime instance, so torch streams, events and device pointers are valid in libvhx calls
            import torch  # noqa: F401
        except ImportError:
            pass
        l = ctypes.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            f = getattr(l, name)
            f.restype = res
            f.argtypes = args
        _lib = l
    return _lib


class VhxError(RuntimeError):
    def __init__(self, code, msg=""):
        super().__init__(f"libvhx error {code}: {msg}")
        self.code = code


def check(code, ctx=None):
    if code != VHX_OK:
        msg = ""
        if ctx:
            m = lib().vhx_last_error(ctx)
            msg = m.decode() if m else ""
        raise VhxError(code, msg)
    return code
