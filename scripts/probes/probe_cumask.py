"""Probe: does a CU partition let a lone frame's longest rays run beside the rest of the frame
without the contention that undid round 4's ahead stream?

The bench frame's rays are traced as explicit ray batches (vhx_trace_rays: the same traversal, 1-D ray order; the
timings compare the partition against the same path without it, not against vhx_trace_primary). The longest rays are
picked by their algorithmic byte counts (count_bytes, a proxy of their step counts). Streams come from
hipExtStreamCreateWithCUMask (libamdhip64 via ctypes) and are handed to libvhx contexts with vhx_set_stream.

Per configuration: the whole frame on one unmasked stream; the frame minus the top-N rays on a stream masked to the
other CUs while the top-N rays run on a stream holding `k` CUs (mask bits chosen three ways), both submitted at once,
timed from the first submit to both streams' completion (device events on a third, unmasked stream joined by waits).
usage: probe_cumask.py [--size 1024] [--top 256,1024,4096] [--cus 8,16,32]"""
import argparse
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import voxelhex_amd as vhx  # noqa: E402
from voxelhex_amd import _native as N  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--size", type=int, default=1024)
ap.add_argument("--width", type=int, default=3840)
ap.add_argument("--height", type=int, default=2160)
ap.add_argument("--top", default="256,1024,4096")
ap.add_argument("--cus", default="8,16,32")
ap.add_argument("--reps", type=int, default=5)
a = ap.parse_args()

hip = ctypes.CDLL("libamdhip64.so")
hip.hipExtStreamCreateWithCUMask.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32,
                                             ctypes.POINTER(ctypes.c_uint32)]
hip.hipExtStreamCreateWithCUMask.restype = ctypes.c_int


def masked_stream(bits, ncu):
    words = (ctypes.c_uint32 * ((ncu + 31) // 32))()
    for b in bits:
        words[b // 32] |= 1 << (b % 32)
    s = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), len(words), words)
    assert rc == 0, f"hipExtStreamCreateWithCUMask rc={rc}"
    return s.value


S, W, H = a.size, a.width, a.height
flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, S, 4, threads=16)
rt = vhx.Raytracer(0)
rt.upload(flat)
cam = vhx.glass_camera(S, W, H, target=(S / 2,) * 3)
ncu = torch.cuda.get_device_properties(0).multi_processor_count
by = rt.trace_primary(cam, fields=(), count_bytes=True)["bytes"].astype(np.int64)
# the glass camera's rays (benches/performance.rs:54-61), in f32 like the kernel (timing probe: exactness not needed)
x = np.arange(W, dtype=np.float32)[None, :].repeat(H, 0).reshape(-1)
y = (H - 1 - np.arange(H, dtype=np.float32))[:, None].repeat(W, 1).reshape(-1)
bl, r, u = (np.array(v, np.float32) for v in (cam.glass_bottom_left, cam.glass_right, cam.glass_up))
gp = bl[None] + r[None] * (x[:, None] * np.float32(cam.pixel_width)) + u[None] * (y[:, None] * np.float32(cam.pixel_height))
o = np.array(cam.origin, np.float32)[None].repeat(W * H, 0)
d = gp - o
d = (d / np.sqrt((d * d).sum(1, keepdims=True))).astype(np.float32)
rays = np.ascontiguousarray(np.concatenate([o, d], 1).astype(np.float32))
order = np.argsort(-by, kind="stable")
dev = torch.device("cuda", 0)
all_rays = torch.from_numpy(rays).to(dev)


def outs(n):
    return {"rgba": torch.empty(n, dtype=torch.int32, device=dev), "depth": torch.empty(n, dtype=torch.float32, device=dev)}


def trace(ctx, rays_dev, out):
    hs = vhx.raytracing._hits_struct(out)
    ctx._check(N.lib().vhx_trace_rays(ctx._h, ctypes.c_void_p(rays_dev.data_ptr()), rays_dev.shape[0],
                                      ctypes.byref(hs), 1))


main, side = rt.shared(), rt.shared()
for c in (main, side):
    c.set_pass_budgets((64,))  # the lone-frame schedule on both, whatever else is in flight
base_out = outs(W * H)
torch.cuda.synchronize()


def timed(fn, reps):
    ts = []
    for _ in range(reps + 1):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        torch.cuda.synchronize()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return float(np.median(ts[1:]))


full_stream = masked_stream(range(ncu), ncu)
main.set_stream(full_stream)
t_full = timed(lambda: trace(main, all_rays, base_out), a.reps)
print(f"whole frame as a ray batch on all {ncu} CUs: {t_full:.3f} ms (lone vhx_trace_primary ~1.22 ms)", flush=True)
for top in (int(v) for v in a.top.split(",")):
    idx_top = np.sort(order[:top])
    idx_rest = np.sort(order[top:])
    r_top = all_rays[torch.from_numpy(idx_top).to(dev)].contiguous()
    r_rest = all_rays[torch.from_numpy(idx_rest).to(dev)].contiguous()
    o_top, o_rest = outs(top), outs(len(idx_rest))
    side.set_stream(full_stream)
    t_top_alone = timed(lambda: trace(side, r_top, o_top), a.reps)
    t_rest_alone = timed(lambda: trace(main, r_rest, o_rest), a.reps)
    print(f"top {top}: alone on all CUs {t_top_alone:.3f} ms; the rest alone {t_rest_alone:.3f} ms", flush=True)
    for k in (int(v) for v in a.cus.split(",")):
        for name, bits in (("low bits", list(range(k))), ("strided", list(range(0, ncu, ncu // k))[:k]),
                           ("per-8 runs", [b for b in range(ncu) if (b % 32) < k // 8][:k])):
            rest_bits = [b for b in range(ncu) if b not in set(bits)]
            s_side, s_main = masked_stream(bits, ncu), masked_stream(rest_bits, ncu)
            side.set_stream(s_side)
            main.set_stream(s_main)

            def both():
                trace(side, r_top, o_top)
                trace(main, r_rest, o_rest)
            t_both = timed(both, a.reps)
            t_side = timed(lambda: trace(side, r_top, o_top), 2)
            print(f"  top {top} on {k} CUs ({name}) beside the rest on {ncu - k}: {t_both:.3f} ms "
                  f"(top alone on its {k} CUs {t_side:.3f} ms)", flush=True)
            side.set_stream(full_stream)
            main.set_stream(full_stream)
main.close()
side.close()
rt.close()
