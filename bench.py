"""Headline benchmark: primary Mrays/s at 3840x2160 on a 1024^3 brick tree (BASELINE.json `metric`).

One step = one frame: every pixel's primary ray traced with get_by_ray semantics (src/raytracing/cpu.rs:296-458)
through the HIP kernel, shaded to RGBA8 + f32 depth in HBM. With N GPUs (torchrun, one process per GPU, RCCL) the
frame is split into 64x64 screen tiles dealt round-robin over the ranks; each rank traces its tiles into a
contiguous buffer, rank 0 gathers the RGBA tiles over RCCL and scatters them into the framebuffer. Weak scaling:
the camera's field of view is fixed and the resolution grows with N so every rank keeps 3840x2160 rays
(N=4 is config 4's 7680x4320 frame; N=2 5432x3056, N=8 10864x6112).

Workload: the reference's lattice+cube scene S (examples/gpu_render.rs:57-82) at 1024^3
with brick_dim 4 (1024 is not a valid size for brick_dim 8, src/boxtree/mod.rs:188-202; the 1024^3 .vox model is not
in the reference checkout), glass camera of benches/performance.rs on radius 2S at 40 rad aimed at the centre.

Also printed: roofline (algorithmic bytes per launch, counted by the instrumented kernel, / measured kernel time vs
8 TB/s; `traffic` = the PMC-measured memory-side read bytes of the same launch from profiles/, see
scripts/pmc_traffic.py), and cpu_baseline: the CPU restatement of the reference raytracer (oracle/) on the host
cores over the same frame.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE = json.load(open(os.path.join(ROOT, "BASELINE.json")))
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--size", type=int, default=1024)
    p.add_argument("--brick-dim", type=int, default=4)
    p.add_argument("--width", type=int, default=3840, help="per-rank-equivalent frame width (N=1 frame)")
    p.add_argument("--height", type=int, default=2160)
    p.add_argument("--scene", type=int, default=1, help="VHX_SCENE_* (1 = lattice+cube scene S)")
    p.add_argument("--vox", default=None, help="trace a MagicaVoxel model instead (BoxTree::load_vox_file, bd = "
                                              "--brick-dim; tree size from the model)")
    p.add_argument("--tile", type=int, default=64)
    p.add_argument("--shadows", action="store_true",
                   help="config 5: each step = primary frame + one hard-shadow ray per hit toward (S,S,S)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-roofline", action="store_true")
    p.add_argument("--no-overlap", action="store_true",
                   help="N>1: gather each frame before tracing the next (default: frame k's gather overlaps k+1)")
    return p.parse_args()


def frame_size(w, h, world):
    """Weak scaling: same field of view, w*h rays per rank (dimensions rounded to multiples of 8)."""
    if world == 1:
        return w, h
    f = world ** 0.5
    return int(round(w * f / 8.0)) * 8, int(round(h * f / 8.0)) * 8


TRAFFIC_FILE = os.path.join(ROOT, "profiles", "traffic.json")


def pmc_traffic(workload):
    """Memory-side read bytes per launch for this workload, from the committed PMC summary (or None)."""
    try:
        d = json.load(open(TRAFFIC_FILE))
    except (OSError, ValueError):
        return None
    e = d.get(workload)
    return None if e is None else e


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    import voxelhex_amd as vhx
    from voxelhex_amd import _native as N
    from voxelhex_amd import multigpu as M

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal of the multi-GPU path on a single GPU: VHX_BENCH_REHEARSAL=1 puts every rank on cuda:0 and gathers
    # over gloo through host memory (RCCL needs one GPU per rank); timings from such a run are not scaling numbers
    rehearsal = world > 1 and os.environ.get("VHX_BENCH_REHEARSAL") == "1"
    if rehearsal:
        local = 0
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(local)
        if rehearsal:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    t0 = time.time()
    if args.vox:
        flat = vhx.BoxTree.load_vox_file(args.vox, args.brick_dim).flatten()
        args.size = int(flat.desc.boxtree_size)
    else:
        flat = vhx.FlatTree.build_scene(args.scene, args.size, args.brick_dim, threads=min(16, os.cpu_count() or 1))
    build_s = time.time() - t0
    rt = vhx.Raytracer(local)
    # one dedicated (non-null) stream shared by libvhx and torch: the kernel, the torch events that time it and
    # the RCCL gather are ordered on it
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    rt.set_stream(stream.cuda_stream)
    t0 = time.time()
    rt.upload(flat)
    upload_s = time.time() - t0

    (W, H), T = frame_size(args.width, args.height, world), args.tile
    c = args.size / 2.0
    cam = vhx.glass_camera(args.size, W, H, target=(c, c, c))
    if world == 1:
        n_out = W * H
        trace_kw = dict(tile_size=0, tile_start=0, tile_stride=1, layout=N.VHX_LAYOUT_FRAMEBUFFER)
        tiles_per_rank = 0
    else:
        tiles_per_rank = M.tiles_per_rank(W, H, T, world)
        n_out = tiles_per_rank * T * T
        trace_kw = dict(tile_size=T, tile_start=rank, tile_stride=world, layout=N.VHX_LAYOUT_TILES)
    rgba = torch.zeros(n_out, dtype=torch.int32, device=dev)
    depth = torch.zeros(n_out, dtype=torch.float32, device=dev)
    out = {"rgba": rgba, "depth": depth}
    light = (float(args.size),) * 3  # ambient_light_position, src/raytracing/bevy/view.rs:81-85
    if args.shadows:
        # -1 = VHX_EMPTY: tile padding past the frame edge is never written and casts no shadow ray
        out.update(value=torch.full((n_out,), -1, dtype=torch.int32, device=dev),
                   impact=torch.zeros((n_out, 3), dtype=torch.float32, device=dev),
                   normal=torch.zeros((n_out, 3), dtype=torch.float32, device=dev))
        shadowed = torch.zeros(n_out, dtype=torch.int32, device=dev)
    pipe = None
    if world > 1:
        framebuffer = torch.zeros(W * H, dtype=torch.int32, device=dev) if rank == 0 else None

        def untile(gathered, slot):
            rt.untile_rgba(gathered.data_ptr(), world, tiles_per_rank, T, W, H, framebuffer.data_ptr())

        # double-buffered: frame k's RCCL gather to rank 0 (and the untile there) overlaps frame k+1's trace
        pipe = M.GatherPipeline(n_out, world, rank, dist, dev, untile, overlap=not args.no_overlap,
                                host_staging=rehearsal)

    ev = []

    def step(timed):
        if pipe is not None:
            out["rgba"] = pipe.out_buffer()
        if timed:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
        rt.trace_primary(cam, out=out, **trace_kw)
        if args.shadows:
            rt.trace_shadows(light, out, shadowed=shadowed)
        if timed:
            e1.record(stream)
            ev.append((e0, e1))
        if pipe is not None:
            pipe.submit()

    for _ in range(args.warmup):
        step(False)
    if pipe is not None:
        pipe.drain()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    if pipe is not None:
        pipe.drain()  # the last frame's gather and untile are inside the timed region
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if rehearsal else dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    kernel_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))

    scene_tag = f"vox:{os.path.basename(args.vox)}" if args.vox else f"S{args.scene}"
    workload = f"primary {W}x{H} {scene_tag} {args.size}^3 bd{args.brick_dim} ranks{world}"
    total_rays = W * H
    n_shadow = 0
    if args.shadows:
        workload += " +shadows"
        n_shadow = int((out["value"] != -1).sum().item())  # shadow rays this rank traced per frame
        if world > 1:
            ts = torch.tensor([n_shadow], dtype=torch.int64, device="cpu" if rehearsal else dev)
            dist.all_reduce(ts)
            n_shadow = int(ts.item())
        total_rays += n_shadow
    mrays = total_rays * args.steps / elapsed / 1e6
    ms_per_step = elapsed * 1e3 / args.steps

    # ---- multi-GPU check (untimed): the gathered, untiled frame equals rank 0 tracing the whole frame alone -------
    mgpu = None
    if world > 1 and rank == 0:
        whole = rt.trace_primary(cam, fields=("rgba",))["rgba"]
        got = framebuffer.cpu().numpy().view(np.uint32)
        mgpu = {"frame_equal": bool(np.array_equal(got, whole)), "pixels": int(whole.size)}

    # ---- roofline: algorithmic bytes of this rank's launch (instrumented kernel, untimed) -------------------------
    roof = None
    if not args.no_roofline and not args.shadows:
        res = rt.trace_primary(cam, fields=(), count_bytes=True, **trace_kw)
        tree_bytes = float(res["bytes"].astype(np.float64).sum())
        my_rays = W * H if world == 1 else M.rank_rays(W, H, T, rank, world)
        out_bytes = 8.0 * my_rays  # rgba8 + f32 depth per ray
        launch_bytes = tree_bytes + out_bytes
        achieved = launch_bytes / (kernel_ms * 1e-3) / 1e9
        tr = pmc_traffic(workload)
        roof = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 5),
                "traffic": None if tr is None else tr["read_bytes_per_launch"],
                "traffic_source": None if tr is None else tr["source"],
                "kernel": "vhx_trace_primary launch = k_trace_primary (pass 0, step budget) + k_trace_queue "
                          "(the rays over budget, resumed from their saved state), timed together with HIP events "
                          "on the trace stream",
                "kernel_ms": round(kernel_ms, 4),
                "algorithmic_bytes_per_launch": launch_bytes, "tree_bytes_per_ray": round(tree_bytes / max(1, my_rays), 2)}

    # ---- CPU baseline: the oracle (reference semantics) on the host cores, rank 0 at N=1 only ----------------------
    cpu = None
    if world == 1 and rank == 0 and not args.no_cpu_baseline and not args.shadows:
        from tests._oracle import Oracle
        orc = Oracle()
        cores = max(1, min(16, len(os.sched_getaffinity(0))))
        orc.trace_primary(flat, cam, 0, 0, W, 16, threads=cores, fields=("rgba",))  # warm
        ts = []
        for _ in range(3):  # three full frames (about 15 s of CPU work on 16 cores), the median reported
            t0 = time.perf_counter()
            orc.trace_primary(flat, cam, 0, 0, W, H, threads=cores, fields=("rgba", "depth"))
            ts.append(time.perf_counter() - t0)
        cpu_s = sorted(ts)[1]
        cpu = {"value": round(W * H / cpu_s / 1e6, 4), "unit": "Mrays/s", "cores": cores, "kind": "port",
               "sample": f"median of 3 full {W}x{H} frames, same tree and camera, OpenMP dynamic over pixels, "
                         f"{cpu_s:.2f} s per frame"}

    if rank == 0:
        metric = BASELINE["metric"]
        if args.shadows:
            metric = "primary + hard-shadow Mrays/s (BASELINE config 5)"
        line = {
            "metric": metric, "value": round(mrays, 3), "unit": "Mrays/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "model file" if args.vox else "synthetic",
            "config": {"workload": f"primary rays {W}x{H}, {args.size}^3 "
                                   + (f".vox model {os.path.basename(args.vox)}" if args.vox
                                      else "procedural scene S (lattice+cube)")
                                   + f", brick_dim {args.brick_dim}, glass camera"
                                   + (f", {W * H // world} rays per rank" if world > 1 else ""),
                       "workload_key": workload,
                       "shadow_rays_per_frame": n_shadow if args.shadows else None,
                       "tree_size": args.size, "brick_dim": args.brick_dim, "width": W, "height": H,
                       "scene": args.scene, "tile": T if world > 1 else None,
                       "parallelism": (f"screen-tile split x{world} + " + (
                           "gloo gather (single-GPU rehearsal)" if rehearsal else
                           "RCCL gather" + ("" if args.no_overlap else ", overlapped with the next frame's trace")))
                       if world > 1 else "single GPU",
                       "tree_nodes": int(flat.desc.node_count), "tree_bricks": int(flat.desc.brick_count),
                       "tree_gb": round(flat.nbytes() / 1e9, 3), "build_s": round(build_s, 2),
                       "upload_s": round(upload_s, 2)},
            "roofline": roof, "cpu_baseline": cpu,
        }
        if mgpu is not None:
            line["multi_gpu_check"] = mgpu
        if cpu:
            line["gpu_over_cpu"] = round(mrays / cpu["value"], 2)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    rt.close()


if __name__ == "__main__":
    main()
