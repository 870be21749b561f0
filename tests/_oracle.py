"""ctypes loader of oracle/_build/liboracle.so — the CPU restatement used as the checker (test infrastructure)."""
import contextlib
import ctypes
import os

import numpy as np

from voxelhex_amd import _native as N
from voxelhex_amd.raytracing import HIT_FIELDS, _hits_struct

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# VHX_ORACLE_LIB: another build of the same source (scripts/asan_cpu.sh builds it with the sanitizers)
ORACLE_LIB = os.environ.get("VHX_ORACLE_LIB") or os.path.join(ROOT, "oracle", "_build", "liboracle.so")


class Oracle:
    def __init__(self):
        l = ctypes.CDLL(ORACLE_LIB)
        P = ctypes.POINTER
        l.vhx_oracle_trace_rays.argtypes = [P(N.TreeDesc), ctypes.c_void_p, ctypes.c_uint64, P(N.Hits), ctypes.c_int]
        l.vhx_oracle_trace_primary.argtypes = [P(N.TreeDesc), P(N.Camera), ctypes.c_uint32, ctypes.c_uint32,
                                               ctypes.c_uint32, ctypes.c_uint32, P(N.Hits), ctypes.c_int]
        l.vhx_oracle_trace_shadows.argtypes = [P(N.TreeDesc), ctypes.c_void_p, ctypes.c_uint64] + \
            [ctypes.c_void_p] * 6 + [ctypes.c_int]
        l.vhx_oracle_luts.argtypes = [ctypes.c_void_p] * 3
        l.vhx_oracle_luts.restype = None
        l.vhx_oracle_offset_sectant.argtypes = [ctypes.c_void_p, ctypes.c_float]
        l.vhx_oracle_offset_sectant.restype = ctypes.c_uint32
        l.vhx_oracle_step_sectant.argtypes = [ctypes.c_uint32, ctypes.c_void_p]
        l.vhx_oracle_step_sectant.restype = ctypes.c_uint32
        l.vhx_oracle_hash_direction.argtypes = [ctypes.c_void_p]
        l.vhx_oracle_hash_direction.restype = ctypes.c_uint32
        l.vhx_oracle_intersect_ray.argtypes = [ctypes.c_void_p, ctypes.c_float, ctypes.c_void_p, ctypes.c_void_p]
        l.vhx_oracle_cube_impact_normal.argtypes = [ctypes.c_void_p, ctypes.c_float, ctypes.c_void_p, ctypes.c_void_p]
        l.vhx_oracle_cube_impact_normal.restype = None
        l.vhx_oracle_nodestack_run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
        self.lib = l

    # -- traversal ----------------------------------------------------------------------------------------------
    @contextlib.contextmanager
    def node_mips(self, mips):
        """Traces inside the block use the node MIP stand-ins of `mips` (vhx_oracle_set_node_mips)."""
        arr = np.ascontiguousarray(mips, np.uint32)
        self.lib.vhx_oracle_set_node_mips.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
        self.lib.vhx_oracle_set_node_mips.restype = None
        self.lib.vhx_oracle_set_node_mips(arr.ctypes.data, len(arr))
        try:
            yield
        finally:
            self.lib.vhx_oracle_set_node_mips(None, 0)

    def trace_rays(self, flat, origins, directions, threads=0, count_bytes=False,
                   fields=("value", "cell", "voxel", "impact", "normal", "depth", "rgba")):
        o = np.ascontiguousarray(origins, np.float32).reshape(-1, 3)
        d = np.ascontiguousarray(directions, np.float32).reshape(-1, 3)
        rays = np.ascontiguousarray(np.concatenate([o, d], axis=1), np.float32)
        n = o.shape[0]
        fields = tuple(fields) + (("bytes",) if count_bytes else ())
        out = {nm: np.empty((n, k) if k > 1 else (n,), dt) for nm, dt, k in HIT_FIELDS if nm in fields}
        hs = _hits_struct(out)
        assert self.lib.vhx_oracle_trace_rays(ctypes.byref(flat.desc), rays.ctypes.data, n, ctypes.byref(hs),
                                              threads) == 0
        return out

    def trace_primary(self, flat, cam, x0, y0, w, h, threads=0, count_bytes=False,
                      fields=("value", "cell", "voxel", "impact", "normal", "depth", "rgba")):
        n = w * h
        fields = tuple(fields) + (("bytes",) if count_bytes else ())
        out = {nm: np.empty((n, k) if k > 1 else (n,), dt) for nm, dt, k in HIT_FIELDS if nm in fields}
        hs = _hits_struct(out)
        assert self.lib.vhx_oracle_trace_primary(ctypes.byref(flat.desc), ctypes.byref(cam), x0, y0, w, h,
                                                 ctypes.byref(hs), threads) == 0
        return out

    def trace_shadows(self, flat, light, hits, threads=0):
        """Shadow flags, darkened rgba and bytes for host hit records (value, impact, normal, rgba)."""
        n = hits["value"].shape[0]
        lt = np.asarray(light, np.float32)
        value = np.ascontiguousarray(hits["value"], np.uint32)
        imp = np.ascontiguousarray(hits["impact"], np.float32)
        nrm = np.ascontiguousarray(hits["normal"], np.float32)
        sh = np.empty(n, np.uint32)
        rgba = np.array(hits["rgba"], np.uint32, copy=True)
        by = np.empty(n, np.uint32)
        assert self.lib.vhx_oracle_trace_shadows(ctypes.byref(flat.desc), lt.ctypes.data, n, value.ctypes.data,
                                                 imp.ctypes.data, nrm.ctypes.data, sh.ctypes.data, rgba.ctypes.data,
                                                 by.ctypes.data, threads) == 0
        return {"shadowed": sh, "rgba": rgba, "bytes": by}

    # -- primitives -----------------------------------------------------------------------------------------------
    def luts(self):
        off = np.zeros(64 * 3, np.float32)
        step = np.zeros(64 * 27, np.uint8)
        occ = np.zeros(64 * 8, np.uint64)
        self.lib.vhx_oracle_luts(off.ctypes.data, step.ctypes.data, occ.ctypes.data)
        return off.reshape(64, 3), step, occ

    def offset_sectant(self, off, size):
        a = np.array(off, np.float32)
        return self.lib.vhx_oracle_offset_sectant(a.ctypes.data, size)

    def step_sectant(self, s, step):
        a = np.array(step, np.float32)
        return self.lib.vhx_oracle_step_sectant(s, a.ctypes.data)

    def hash_direction(self, d):
        a = np.array(d, np.float32)
        return self.lib.vhx_oracle_hash_direction(a.ctypes.data)

    def intersect_ray(self, cmin, csize, origin, direction):
        c = np.array(cmin, np.float32)
        r = np.array(list(origin) + list(direction), np.float32)
        t = ctypes.c_float(0)
        k = self.lib.vhx_oracle_intersect_ray(c.ctypes.data, csize, r.ctypes.data, ctypes.byref(t))
        return None if k == 0 else ("inside" if k == 1 else float(np.float32(t.value)))

    def impact_normal(self, cmin, csize, p):
        c = np.array(cmin, np.float32)
        pp = np.array(p, np.float32)
        n = np.zeros(3, np.float32)
        self.lib.vhx_oracle_cube_impact_normal(c.ctypes.data, csize, pp.ctypes.data, n.ctypes.data)
        return n

    def nodestack(self, size, ops):
        a = np.array(ops, np.int32)
        r = np.zeros(len(ops), np.int32)
        assert self.lib.vhx_oracle_nodestack_run(size, a.ctypes.data, len(ops), r.ctypes.data) == 0
        return [None if v == np.iinfo(np.int32).min else int(v) for v in r]
