"""Streaming view of a BoxTree on the GPU (vhx_stream, include/vhx_stream.h).

Mirrors the reference's BoxTreeGPUDataHandler (src/raytracing/bevy/streaming/*.rs): a device buffer set with a bounded
number of node and brick slots, filled around the viewport a few nodes/bricks per frame with ranged writes. A
Raytracer that hosts a stream traces the streamed view.
"""
import ctypes

import numpy as np

from . import _native as N

STAT_FIELDS = ("bytes_written", "bricks_written", "nodes_written", "nodes_resident", "bricks_resident",
               "nodes_in_view", "bricks_in_view", "nodes_to_see", "pending")


class StreamStats(ctypes.Structure):
    _fields_ = [(f, ctypes.c_uint64) for f in STAT_FIELDS]


class ViewDesc:
    """Host mirror of the device view, usable wherever a FlatTree's `desc` is read (e.g. the test oracle)."""

    def __init__(self, stream, desc):
        self._stream = stream  # the arrays live in the stream
        self.desc = desc


class StreamingView:
    """A streamed view (vhx_stream). raytracer=None keeps it on the host (vhx_stream_view only)."""

    def __init__(self, tree, raytracer, origin, view_distance):
        self.tree = tree
        self.raytracer = raytracer
        h = ctypes.c_void_p()
        ctx = raytracer._h if raytracer is not None else None
        o = (ctypes.c_float * 3)(*[float(v) for v in origin])
        N.check(N.lib().vhx_stream_create(tree._h, ctx, o, float(view_distance), ctypes.byref(h)), ctx)
        self._h = h
        if raytracer is not None:
            raytracer._tree = self  # the context now holds the streamed view

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            N.lib().vhx_stream_destroy(self._h)
            self._h = ctypes.c_void_p(None)

    def __del__(self):
        try:
            self.close()
        except (TypeError, AttributeError):  # interpreter shutdown
            pass

    def _ctx(self):
        return self.raytracer._h if self.raytracer is not None else None

    def set_rates(self, node_uploads_per_frame=25, brick_uploads_per_frame=50, brick_unload_search_perimeter=10):
        N.check(N.lib().vhx_stream_set_rates(self._h, node_uploads_per_frame, brick_uploads_per_frame,
                                             brick_unload_search_perimeter))

    def set_viewport(self, origin, view_distance):
        o = (ctypes.c_float * 3)(*[float(v) for v in origin])
        N.check(N.lib().vhx_stream_set_viewport(self._h, o, float(view_distance)))

    def upload(self, frames=1):
        """One frame of uploads (frames > 1: that many frames' uploads written as one batch,
        vhx_stream_upload_frames); returns (stats dict, needs_resize)."""
        st = StreamStats()
        if frames == 1:
            rc = N.lib().vhx_stream_upload(self._h, ctypes.byref(st))
        else:
            rc = N.lib().vhx_stream_upload_frames(self._h, frames, ctypes.byref(st))
        if rc not in (N.VHX_OK, N.VHX_E_CAPACITY):
            N.check(rc, self._ctx())
        return {f: getattr(st, f) for f in STAT_FIELDS}, rc == N.VHX_E_CAPACITY

    def resize(self):
        N.check(N.lib().vhx_stream_resize(self._h), self._ctx())

    def reload(self):
        N.check(N.lib().vhx_stream_reload(self._h))

    def view_set_check(self):
        """vhx_stream_view_set_check: (equal to a full rebuild, full rebuilds, incremental rebuilds)."""
        f, i = ctypes.c_uint64(), ctypes.c_uint64()
        rc = N.lib().vhx_stream_view_set_check(self._h, ctypes.byref(f), ctypes.byref(i))
        if rc not in (N.VHX_OK, N.VHX_E_STATE):
            N.check(rc)
        return rc == N.VHX_OK, f.value, i.value

    def upload_all(self, max_frames=100000):
        """Uploads frame by frame (resizing when the view is too small) until nothing is pending."""
        frames = resizes = 0
        stats = None
        while frames < max_frames:
            stats, grow = self.upload()
            frames += 1
            if grow:
                self.resize()
                resizes += 1
                continue
            if stats["pending"] == 0:
                break
        return stats, frames, resizes

    def node_mips(self):
        """Copy of the view's node MIP descriptors (vhx_stream_node_mips)."""
        ptr, cnt = ctypes.c_void_p(), ctypes.c_uint32()
        N.check(N.lib().vhx_stream_node_mips(self._h, ctypes.byref(ptr), ctypes.byref(cnt)))
        if not cnt.value:
            return np.zeros(0, np.uint32)
        return np.ctypeslib.as_array((ctypes.c_uint32 * cnt.value).from_address(ptr.value)).copy()

    def view(self):
        d = N.TreeDesc()
        N.check(N.lib().vhx_stream_view(self._h, ctypes.byref(d)))
        return ViewDesc(self, d)
