"""GPU raytracing API: the MI355X replacement of VoxelHex's `src/raytracing` module.

    Ray                      voxelhex::raytracing::Ray (src/spatial/raytracing/mod.rs:8-22)
    Raytracer                a libvhx context: one device, the tree resident in HBM (BoxTreeGPUHost + view,
                             src/raytracing/bevy/mod.rs:164-180, src/raytracing/bevy/view.rs:36-137)
    Raytracer.trace_rays     BoxTree::get_by_ray over a batch (src/raytracing/cpu.rs:296)
    Raytracer.trace_primary  one frame of per-pixel primary rays (VhxRenderNode::run,
                             src/raytracing/bevy/pipeline/mod.rs:96-155, with the CPU frame semantics of
                             examples/gpu_render.rs:196-257)
    Viewport                 src/raytracing/bevy/types.rs:60-88 with update_matrices (src/raytracing/bevy/view.rs:211-239)
    glass_camera             the pinhole camera of benches/performance.rs:29-61

Every call goes through the HIP kernels of libvhx; there is no CPU path here.
"""
import ctypes
from dataclasses import dataclass, field
import math

import numpy as np

from . import _native as N
from .boxtree import V3c, FlatTree

f32 = np.float32
_libm = ctypes.CDLL("libm.so.6")
_libm.sinf.restype = ctypes.c_float
_libm.sinf.argtypes = [ctypes.c_float]
_libm.cosf.restype = ctypes.c_float
_libm.cosf.argtypes = [ctypes.c_float]
_libm.tanf.restype = ctypes.c_float
_libm.tanf.argtypes = [ctypes.c_float]


@dataclass
class Ray:
    origin: V3c
    direction: V3c

    def is_valid(self):
        d = np.array(list(self.direction), f32)
        return abs(f32(1) - _len(d)) < f32(0.000001)


# ---------------------------------------------------------------------------------------------- f32 V3c helpers
def _v(*a):
    return np.array(a, f32)


def _len(v):
    """V3c::length (src/spatial/math/vector.rs:71-73): sqrt((x*x + y*y) + z*z) in f32."""
    return f32(np.sqrt(f32(f32(v[0] * v[0]) + f32(v[1] * v[1])) + f32(v[2] * v[2])))


def _normalized(v):
    """V3c::normalized: v / length (three f32 divisions)."""
    l = _len(v)
    return np.array([v[0] / l, v[1] / l, v[2] / l], f32)


def _cross(a, b):
    """V3c::cross (src/spatial/math/vector.rs:196-202)."""
    return np.array([f32(a[1] * b[2]) - f32(a[2] * b[1]), f32(a[2] * b[0]) - f32(a[0] * b[2]),
                     f32(a[0] * b[1]) - f32(a[1] * b[0])], f32)


def glass_camera(tree_size, width, height, angle=40.0, radius=None, target=None, glass_width=4.0,
                 glass_height=None, fov=3.0):
    """Pinhole 'glass' camera of benches/performance.rs:32-61.

    The reference bench renders 128x128 rays through a 4x4 glass at distance 3 from a camera at
    (sin(40) R, R, cos(40) R), R = 2*tree_size, aimed at (0,0,0). Defaults keep that geometry; `target` re-aims it
    (SURVEY.md 8d aims at the tree centre) and glass_height defaults to 4*height/width so pixels stay square.
    Arithmetic is f32 in the reference's op order; sin/cos come from libm's sinf/cosf like Rust's f32::sin.
    """
    S = f32(tree_size)
    R = f32(2.0) * S if radius is None else f32(radius)
    a = f32(angle)
    origin = _v(f32(_libm.sinf(a)) * R, R, f32(_libm.cosf(a)) * R)
    tgt = _v(0, 0, 0) if target is None else np.array(target, f32)
    direction = _normalized(tgt - origin)
    up = _v(0, 1, 0)
    right = _normalized(_cross(up, direction))
    gw = f32(glass_width)
    gh = f32(glass_width * height / width) if glass_height is None else f32(glass_height)
    pw = f32(gw / f32(width))
    ph = f32(gh / f32(height))
    bl = ((origin + direction * f32(fov)) - up * f32(gh / f32(2))) - right * f32(gw / f32(2))
    cam = N.Camera()
    cam.ray_model = N.VHX_RAY_GLASS
    cam.width, cam.height = width, height
    cam.origin[:] = [float(v) for v in origin]
    cam.glass_bottom_left[:] = [float(v) for v in bl]
    cam.glass_right[:] = [float(v) for v in right]
    cam.glass_up[:] = [float(v) for v in up]
    cam.pixel_width = float(pw)
    cam.pixel_height = float(ph)
    return cam


@dataclass
class Viewport:
    """Viewport (src/raytracing/bevy/types.rs:60-88)."""
    origin: tuple
    direction: tuple
    frustum: tuple
    fov: float
    view_matrix: np.ndarray = field(default_factory=lambda: np.eye(4, dtype=f32))
    projection_matrix: np.ndarray = field(default_factory=lambda: np.eye(4, dtype=f32))
    inverse_view_projection_matrix: np.ndarray = field(default_factory=lambda: np.eye(4, dtype=f32))

    def update_matrices(self, resolution):
        """Viewport::update_matrices (src/raytracing/bevy/view.rs:211-239); matrices stored column-major like glam.

        look_at_rh and perspective_rh follow glam 0.29's formulas in f32; the inverse is computed in f64 and
        rounded (glam's cofactor order is not restated: parity for this matrix is unpinned)."""
        fwd = np.array(self.direction, f32)
        right = _normalized(_cross(fwd, _v(0, 1, 0)))
        up = _normalized(_cross(right, fwd))
        eye = np.array(self.origin, f32)
        center = eye + fwd
        f = _normalized(center - eye)
        s = _normalized(_cross(f, up))
        u = _cross(s, f)
        view = np.zeros((4, 4), f32)  # [col][row]
        view[0] = [s[0], u[0], -f[0], 0]
        view[1] = [s[1], u[1], -f[1], 0]
        view[2] = [s[2], u[2], -f[2], 0]
        view[3] = [-np.dot(eye, s), -np.dot(eye, u), np.dot(eye, f), 1]
        aspect = f32(resolution[0]) / f32(resolution[1])
        fov_r = f32(math.radians(self.fov))
        near = f32(self.frustum[1]) / f32(2.0) / f32(_libm.tanf(fov_r / f32(2.0)))
        far = f32(self.frustum[2])
        half = f32(0.5) * fov_r
        h = f32(_libm.cosf(half)) / f32(_libm.sinf(half))
        w = h / aspect
        r = far / (near - far)
        proj = np.zeros((4, 4), f32)
        proj[0] = [w, 0, 0, 0]
        proj[1] = [0, h, 0, 0]
        proj[2] = [0, 0, r, -1]
        proj[3] = [0, 0, r * near, 0]
        # column-major storage: M[col][row]; math matrix = storage.T
        vp = (proj.T.astype(np.float64) @ view.T.astype(np.float64))
        self.view_matrix, self.projection_matrix = view, proj
        self.inverse_view_projection_matrix = np.linalg.inv(vp).T.astype(f32)

    def camera(self, width, height):
        self.update_matrices((width, height))
        cam = N.Camera()
        cam.ray_model = N.VHX_RAY_INVERSE_VP
        cam.width, cam.height = width, height
        cam.origin[:] = [float(v) for v in self.origin]
        cam.inv_view_proj[:] = [float(v) for v in self.inverse_view_projection_matrix.reshape(-1)]
        return cam


HIT_FIELDS = (("value", np.uint32, 1), ("cell", np.uint32, 1), ("voxel", np.uint32, 3), ("impact", np.float32, 3),
              ("normal", np.float32, 3), ("depth", np.float32, 1), ("rgba", np.uint32, 1), ("bytes", np.uint32, 1),
              ("shadowed", np.uint32, 1))


def _hits_struct(arrays):
    h = N.Hits()
    for name, _, _ in HIT_FIELDS:
        a = arrays.get(name)
        setattr(h, name, None if a is None else _ptr(a))
    return h


def _on_device(arrays):
    """1 when every array of an out= dict is a GPU tensor, 0 when every one is host memory (numpy / CPU tensor)."""
    dev = {bool(getattr(a, "is_cuda", False)) for a in arrays.values() if a is not None}
    if len(dev) > 1:
        raise ValueError("out= mixes device and host arrays")
    return 1 if dev == {True} else 0


def _ptr(a):
    if hasattr(a, "data_ptr"):  # torch tensor (device or host)
        return a.data_ptr()
    return a.ctypes.data


class Raytracer:
    """A libvhx context on one HIP device with a tree resident in HBM."""

    def __init__(self, device=0, tune=None):
        """tune: a vhx_set_tuning spec ("key=value;..."), scheduling knobs of experiments (results never change)."""
        lib = N.lib()
        n = ctypes.c_int()
        rc = lib.vhx_device_count(ctypes.byref(n))
        if rc != N.VHX_OK:
            raise N.VhxError(rc, "vhx_device_count: " + (lib.vhx_device_error() or b"").decode())
        if n.value == 0:
            raise RuntimeError("voxelhex_amd: no HIP device is visible (the raytracer has no CPU fallback)")
        h = ctypes.c_void_p()
        N.check(lib.vhx_create(device, ctypes.byref(h)))
        self._h = h
        self.device = device
        self._tree = None
        if tune:
            self.set_tuning(tune)

    def set_tuning(self, spec):
        """vhx_set_tuning: scheduling knobs as "key=value;..." (include/vhx.h); a dict is joined the same way."""
        if isinstance(spec, dict):
            spec = ";".join(f"{k}={v}" for k, v in spec.items())
        self._check(N.lib().vhx_set_tuning(self._h, spec.encode()))

    def shared(self):
        """vhx_create_shared: another context (its own stream, queues and outputs) tracing this context's tree."""
        if self._tree is None:
            raise RuntimeError("upload a tree before sharing it")
        rt = Raytracer.__new__(Raytracer)
        h = ctypes.c_void_p()
        self._check(N.lib().vhx_create_shared(self._h, ctypes.byref(h)))
        rt._h, rt.device, rt._tree = h, self.device, self._tree
        return rt

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            N.lib().vhx_destroy(self._h)
            self._h = ctypes.c_void_p(None)

    def __del__(self):
        try:
            self.close()
        except (TypeError, AttributeError):  # interpreter shutdown: module globals already torn down
            pass

    def _check(self, rc):
        return N.check(rc, self._h)

    def upload(self, flat: FlatTree):
        if self._tree is flat:
            return
        self._check(N.lib().vhx_upload_tree(self._h, ctypes.byref(flat.desc)))
        self._tree = flat

    def update_range(self, buffer_id, elem_offset, values):
        values = np.ascontiguousarray(values)
        self._check(N.lib().vhx_update_range(self._h, buffer_id, elem_offset, values.size, values.ctypes.data))

    def update_ranges(self, writes):
        """vhx_update_ranges: writes = [(buffer_id, elem_offset, values), ...] in one staged copy + scatter."""
        keep = [np.ascontiguousarray(v) for _, _, v in writes]
        rs = (N.Range * max(1, len(writes)))()
        for r, (bid, off, _), v in zip(rs, writes, keep):
            r.buffer_id, r.elem_offset, r.elem_count, r.src = bid, off, v.size, v.ctypes.data
        self._check(N.lib().vhx_update_ranges(self._h, ctypes.cast(rs, ctypes.c_void_p), len(writes)))

    def read_derived(self, which, offset, count):
        dt = np.uint32 if which == N.VHX_DERIVED_NODE_HDR else np.uint64
        k = 4 if which == N.VHX_DERIVED_NODE_HDR else 1
        a = np.empty(count * k, dt)
        self._check(N.lib().vhx_read_derived(self._h, which, offset, count, a.ctypes.data))
        return a.reshape(count, k) if k > 1 else a

    def device_bytes(self):
        b = ctypes.c_uint64()
        self._check(N.lib().vhx_tree_device_bytes(self._h, ctypes.byref(b)))
        return b.value

    def set_stream(self, stream_ptr):
        self._check(N.lib().vhx_set_stream(self._h, ctypes.c_void_p(stream_ptr)))

    def stream(self):
        """The context's hipStream_t (vhx_get_stream): the one set by set_stream, else its own (created now if
        needed); wrap it with torch.cuda.ExternalStream to order torch work and events with the traces."""
        s = ctypes.c_void_p()
        self._check(N.lib().vhx_get_stream(self._h, ctypes.byref(s)))
        return s.value

    def set_node_mips(self, node_mips):
        """vhx_set_node_mips: node MIPs stand in for occupied but absent children (the WGSL path's probe_MIP);
        None disables them. `node_mips` is FlatTree.node_mips of the uploaded tree."""
        if node_mips is None:
            self._check(N.lib().vhx_set_node_mips(self._h, None, 0))
            self._mips = None
            return
        self._mips = np.ascontiguousarray(node_mips, np.uint32)
        self._check(N.lib().vhx_set_node_mips(self._h, self._mips.ctypes.data, len(self._mips)))

    def set_depth_prepass(self, enable=True, margin=0.0):
        """vhx_set_depth_prepass: the opt-in half-resolution depth-prepass fast mode (not the reference's semantics)."""
        self._check(N.lib().vhx_set_depth_prepass(self._h, 1 if enable else 0, float(margin)))

    def set_shadow_light(self, light=None):
        """vhx_set_shadow_light: fused hard shadows (config 5) in trace_primary / trace_primary_batch /
        trace_tiles_batch, whose outputs then need value, impact, normal and shadowed; None turns them off."""
        lt = None if light is None else (ctypes.c_float * 3)(*[float(v) for v in light])
        self._check(N.lib().vhx_set_shadow_light(self._h, lt))

    def set_pass_budgets(self, budgets):
        """Step budgets of the multi-pass ray scheduler (vhx_set_pass_budgets); () = one unbounded pass."""
        b = (ctypes.c_uint32 * max(1, len(budgets)))(*budgets)
        self._check(N.lib().vhx_set_pass_budgets(self._h, b, len(budgets)))

    def set_adaptive_schedule(self, on=True):
        """Restores (or ends) the adaptive choice between the frames-in-flight and the lone-frame schedule."""
        self._check(N.lib().vhx_set_adaptive_schedule(self._h, 1 if on else 0))

    def tail_info(self):
        """vhx_tail_info: (pixels the next lone frame traces early, (width, height) they were recorded for)."""
        n, w, h = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        self._check(N.lib().vhx_tail_info(self._h, ctypes.byref(n), ctypes.byref(w), ctypes.byref(h)))
        return n.value, (w.value, h.value)

    def pass_budgets(self):
        """(budgets of the last trace, schedule): schedule "busy" (frames in flight), "idle" (lone frame) or "fixed"."""
        b = (ctypes.c_uint32 * N.VHX_MAX_BUDGETS)()
        n, sched = ctypes.c_uint32(), ctypes.c_int()
        self._check(N.lib().vhx_get_pass_budgets(self._h, b, ctypes.byref(n), ctypes.byref(sched)))
        return tuple(b[:n.value]), {1: "busy", 0: "idle"}.get(sched.value, "fixed")

    def sync(self):
        ms = ctypes.c_float()
        self._check(N.lib().vhx_sync(self._h, ctypes.byref(ms)))
        return ms.value

    def trace_rays(self, origins, directions, fields=("value", "cell", "voxel", "impact", "normal", "depth", "rgba"),
                   count_bytes=False):
        """Traces rays given as (n,3) f32 origins and directions on the host; returns numpy hit arrays."""
        o = np.ascontiguousarray(origins, f32).reshape(-1, 3)
        d = np.ascontiguousarray(directions, f32).reshape(-1, 3)
        n = o.shape[0]
        rays = np.ascontiguousarray(np.concatenate([o, d], axis=1), f32)
        fields = tuple(fields) + (("bytes",) if count_bytes else ())
        out = {name: np.empty((n, k) if k > 1 else (n,), dt) for name, dt, k in HIT_FIELDS if name in fields}
        hs = _hits_struct(out)
        self._check(N.lib().vhx_trace_rays(self._h, rays.ctypes.data, n, ctypes.byref(hs), 0))
        return out

    def trace_primary(self, cam, tile_size=0, tile_start=0, tile_stride=1, layout=N.VHX_LAYOUT_FRAMEBUFFER,
                      fields=("value", "cell", "voxel", "impact", "normal", "depth", "rgba"), count_bytes=False,
                      out=None):
        """Traces one frame (or this rank's tiles). With out=dict of device tensors nothing is copied back; with
        out=dict of host arrays (numpy or CPU tensors, reused across frames) the results are copied into them."""
        if layout == N.VHX_LAYOUT_FRAMEBUFFER:
            n = cam.width * cam.height
        else:
            T = tile_size
            ntiles = ((cam.width + T - 1) // T) * ((cam.height + T - 1) // T)
            n = max(0, (ntiles - tile_start + tile_stride - 1) // tile_stride) * T * T
        if out is not None:
            for name, dt, k in HIT_FIELDS:
                a = out.get(name)
                nbytes = None if a is None else (a.numel() * a.element_size() if hasattr(a, "numel") else a.nbytes)
                if nbytes is not None and nbytes < n * k * 4:
                    raise ValueError(f"out[{name!r}] holds {nbytes} bytes, the trace writes {n * k * 4}")
            hs = _hits_struct(out)
            self._check(N.lib().vhx_trace_primary(self._h, ctypes.byref(cam), tile_size, tile_start, tile_stride,
                                                  layout, ctypes.byref(hs), _on_device(out)))
            return out
        fields = tuple(fields) + (("bytes",) if count_bytes else ())
        alloc = np.empty if layout == N.VHX_LAYOUT_FRAMEBUFFER else np.zeros  # tiles past the frame edge stay 0
        res = {name: alloc((n, k) if k > 1 else (n,), dt) for name, dt, k in HIT_FIELDS if name in fields}
        hs = _hits_struct(res)
        self._check(N.lib().vhx_trace_primary(self._h, ctypes.byref(cam), tile_size, tile_start, tile_stride, layout,
                                              ctypes.byref(hs), 0))
        return res

    def trace_primary_batch(self, cams, outs):
        """vhx_trace_primary_batch: whole frames cams[k] -> outs[k] (dicts of device tensors, framebuffer layout) as one
        pass ladder on this context's stream; results equal one trace_primary per frame."""
        if len(cams) != len(outs) or not cams:
            raise ValueError("trace_primary_batch: one output dict per camera")
        n = cams[0].width * cams[0].height
        for out in outs:
            if _on_device(out) != 1:
                raise ValueError("trace_primary_batch writes device tensors")
            for name, dt, k in HIT_FIELDS:
                a = out.get(name)
                if a is not None and a.numel() * a.element_size() < n * k * 4:
                    raise ValueError(f"out[{name!r}] holds {a.numel() * a.element_size()} bytes, a frame needs {n * k * 4}")
        cs = (N.Camera * len(cams))(*cams)
        hs = (N.Hits * len(outs))(*[_hits_struct(o) for o in outs])
        self._check(N.lib().vhx_trace_primary_batch(self._h, ctypes.cast(cs, ctypes.c_void_p), len(cams),
                                                    ctypes.cast(hs, ctypes.c_void_p)))
        return outs

    def trace_tiles_batch(self, cams, tile_size, tile_starts, tile_stride, outs):
        """vhx_trace_tiles_batch: frame k = the tile set tile_starts[k], +tile_stride, ... of cams[k] (tile layout) into
        outs[k] (dicts of device tensors) as one pass ladder; equal to one trace_primary(layout=TILES) per frame."""
        if len(cams) != len(outs) or len(cams) != len(tile_starts) or not cams:
            raise ValueError("trace_tiles_batch: one output dict and one tile start per camera")
        T = tile_size
        if T < 1 or tile_stride < 1:
            raise ValueError("trace_tiles_batch: tile_size and tile_stride must be >= 1")
        ntiles = ((cams[0].width + T - 1) // T) * ((cams[0].height + T - 1) // T)
        for st, out in zip(tile_starts, outs):
            if _on_device(out) != 1:
                raise ValueError("trace_tiles_batch writes device tensors")
            n = max(0, (ntiles - st + tile_stride - 1) // tile_stride) * T * T
            for name, dt, k in HIT_FIELDS:
                a = out.get(name)
                if a is not None and a.numel() * a.element_size() < n * k * 4:
                    raise ValueError(f"out[{name!r}] holds {a.numel() * a.element_size()} bytes, the set needs {n * k * 4}")
        cs = (N.Camera * len(cams))(*cams)
        st = (ctypes.c_uint32 * len(cams))(*[int(v) for v in tile_starts])
        hs = (N.Hits * len(outs))(*[_hits_struct(o) for o in outs])
        self._check(N.lib().vhx_trace_tiles_batch(self._h, ctypes.cast(cs, ctypes.c_void_p), len(cams), T,
                                                  ctypes.cast(st, ctypes.c_void_p), tile_stride,
                                                  ctypes.cast(hs, ctypes.c_void_p)))
        return outs

    def trace_shadows_batch(self, light, hits_list, shadowed_list=None, darken=True):
        """vhx_trace_shadows_batch: the hard shadows of several frames' device-resident hit records (dicts like
        trace_shadows' `hits`, the same record count each) as one pass ladder; returns the int32 `shadowed` tensors.
        Equal to one trace_shadows per frame."""
        import torch
        if not hits_list:
            raise ValueError("trace_shadows_batch: no frames")
        n = hits_list[0]["value"].numel()
        if any(h["value"].numel() != n for h in hits_list):
            raise ValueError("trace_shadows_batch: every frame needs the same record count")
        for h in hits_list:
            if _on_device(h) != 1:
                raise ValueError("trace_shadows_batch reads device tensors")
        if shadowed_list is None:
            shadowed_list = [torch.empty(n, dtype=torch.int32, device=h["value"].device) for h in hits_list]
        if len(shadowed_list) != len(hits_list):
            raise ValueError("trace_shadows_batch: one shadowed tensor per frame")

        def need(a, words, what):
            # the library trusts n for every array of every frame: a short tensor would be read or written past its end
            if a is None or not hasattr(a, "numel") or not a.is_cuda or a.numel() * a.element_size() < 4 * words:
                raise ValueError(f"trace_shadows_batch: {what} must be a device tensor of at least {4 * words} bytes")

        for k, h in enumerate(hits_list):
            need(h["value"], n, f"frame {k} value")
            need(h["impact"], 3 * n, f"frame {k} impact")
            need(h["normal"], 3 * n, f"frame {k} normal")
            need(shadowed_list[k], n, f"frame {k} shadowed")
            if darken and h.get("rgba") is not None:
                need(h["rgba"], n, f"frame {k} rgba")
        fr = (N.ShadowFrame * len(hits_list))()
        for k, h in enumerate(hits_list):
            rgba = h.get("rgba") if darken else None
            fr[k] = N.ShadowFrame(_ptr(h["value"]), _ptr(h["impact"]), _ptr(h["normal"]), _ptr(shadowed_list[k]),
                                  None if rgba is None else _ptr(rgba))
        lt = (ctypes.c_float * 3)(*[float(v) for v in light])
        self._check(N.lib().vhx_trace_shadows_batch(self._h, lt, len(hits_list), n, ctypes.cast(fr, ctypes.c_void_p)))
        return shadowed_list

    def trace_shadows(self, light, hits, shadowed=None, darken=True, count_bytes=False):
        """Hard shadow rays (vhx_trace_shadows) for the device-resident hit records `hits` of a previous trace
        (dict of torch tensors with value, impact, normal and optionally rgba). Returns a dict with the int32
        `shadowed` flags (and `bytes`); hits["rgba"] is darkened in place when darken."""
        import torch
        n = hits["value"].numel()
        if shadowed is None:
            shadowed = torch.empty(n, dtype=torch.int32, device=hits["value"].device)
        res = {"shadowed": shadowed}
        if count_bytes:
            res["bytes"] = torch.empty(n, dtype=torch.int32, device=hits["value"].device)
        lt = (ctypes.c_float * 3)(*[float(v) for v in light])
        rgba = hits.get("rgba") if darken else None
        self._check(N.lib().vhx_trace_shadows(
            self._h, lt, n, ctypes.c_void_p(_ptr(hits["value"])), ctypes.c_void_p(_ptr(hits["impact"])),
            ctypes.c_void_p(_ptr(hits["normal"])), ctypes.c_void_p(_ptr(shadowed)),
            ctypes.c_void_p(None if rgba is None else _ptr(rgba)),
            ctypes.c_void_p(_ptr(res["bytes"]) if count_bytes else None)))
        return res

    def untile_frame(self, gathered_dev_ptr, planes, ranks, tiles_per_rank, tile_size, width, height, rgba_dev_ptr,
                     depth_dev_ptr=None):
        """vhx_untile_frame: rank-major [RGBA plane | depth plane] tile buffers -> device framebuffers."""
        self._check(N.lib().vhx_untile_frame(self._h, ctypes.c_void_p(gathered_dev_ptr), planes, ranks,
                                             tiles_per_rank, tile_size, width, height, ctypes.c_void_p(rgba_dev_ptr),
                                             ctypes.c_void_p(depth_dev_ptr)))

    def untile_rgba(self, gathered_dev_ptr, ranks, tiles_per_rank, tile_size, width, height, fb_dev_ptr):
        self._check(N.lib().vhx_untile_rgba(self._h, ctypes.c_void_p(gathered_dev_ptr), ranks, tiles_per_rank,
                                            tile_size, width, height, ctypes.c_void_p(fb_dev_ptr), 1))


_default = {}


def default_raytracer(device=None):
    dev = 0 if device is None else device
    if dev not in _default:
        _default[dev] = Raytracer(dev)
    return _default[dev]


class BoxTreeGPUHost:
    """BoxTreeGPUHost (src/raytracing/bevy/types.rs:91-103): owns the tree and renders views of it on a GPU."""

    def __init__(self, tree, device=0):
        self.tree = tree
        self.raytracer = Raytracer(device)

    def create_new_view(self, viewport, resolution):
        return BoxTreeGPUView(self, viewport, resolution)


class BoxTreeGPUView:
    """A view (src/raytracing/bevy/types.rs:134-180): viewport + output resolution, rendered to RGBA8."""

    def __init__(self, host, viewport, resolution):
        self.host, self.viewport, self.resolution = host, viewport, tuple(resolution)

    def render(self, fields=("rgba", "depth")):
        flat = self.host.tree.flatten() if hasattr(self.host.tree, "flatten") else self.host.tree
        self.host.raytracer.upload(flat)
        w, h = self.resolution
        res = self.host.raytracer.trace_primary(self.viewport.camera(w, h), fields=fields)
        if "rgba" in res:
            res["image"] = res["rgba"].view(np.uint8).reshape(h, w, 4)
        return res
