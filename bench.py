"""Headline benchmark: primary Mrays/s at 3840x2160 on a 1024^3 brick tree (BASELINE.json `metric`).

One step = one frame: every pixel's primary ray traced with get_by_ray semantics (src/raytracing/cpu.rs:296-458)
through the HIP kernel, shaded to RGBA8 + f32 depth in HBM.

Multi-GPU (torchrun, one process per GPU): the split lives behind the C ABI (vhx_mgpu_*, include/vhx.h): libvhx owns
an RCCL communicator (its id travels over a gloo process group, which also carries the barriers and the max-over-ranks
timing), rank 0 builds the tree and ncclBroadcasts it to the other GPUs, and every frame each rank traces its 64x64
screen tiles (dealt round-robin, rank 0's share balanced by vhx_mgpu_balance before the warm-up), point-to-point RCCL
transfers bring RGBA8 + f32 depth to rank 0, rank 0 untiles them into its framebuffers; frame k's transfers overlap
the next frames' traces. Scaling modes (--scaling):
  auto   (default) N = 1: the headline 3840x2160 frame; N > 1: BASELINE config 4, a fixed 7680x4320 frame (strong)
  strong the 7680x4320 config-4 frame at every N (N = 1 included)
  weak   the field of view fixed, W*H grown with N so that every rank keeps 3840x2160 rays
--mgpu torch keeps the previous torch.distributed gather (and VHX_BENCH_REHEARSAL=1 rehearses it with two ranks on
one GPU over gloo; RCCL needs one GPU per rank).

Workload: the reference's lattice+cube scene S (examples/gpu_render.rs:57-82) at 1024^3
with brick_dim 4 (1024 is not a valid size for brick_dim 8, src/boxtree/mod.rs:188-202; the 1024^3 .vox model is not
in the reference checkout), glass camera of benches/performance.rs on radius 2S at 40 rad aimed at the centre.

Also printed: roofline (algorithmic bytes per launch, counted by the instrumented kernel, / measured kernel time vs
8 TB/s; `traffic` = the memory-side read bytes of the same launch, measured in this run by a `rocprofv3 --pmc
FETCH_SIZE` child run of the same workload (N = 1; --no-pmc, or a failed child run, falls back to the committed
profiles/traffic.json figure), and cpu_baseline: the CPU restatement of the reference raytracer (oracle/) on the host
cores over the same frame (all cores available to the process and 1 core, 1 warm-up + median of 5).
"""
import argparse
import csv
import glob
import json
import os
import shutil
import signal
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE = json.load(open(os.path.join(ROOT, "BASELINE.json")))
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=None,
                   help="GPUs (ranks) of the run, default 1. Under torchrun (WORLD_SIZE set) it must equal WORLD_SIZE; "
                        "without it and N > 1 this process starts the N rank processes itself (launch_ranks) and "
                        "relays rank 0's line")
    p.add_argument("--print-launch", action="store_true",
                   help="N > 1 without WORLD_SIZE: print the rank processes that would be started (command and "
                        "environment) as one JSON line and exit, starting nothing")
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--size", type=int, default=1024)
    p.add_argument("--brick-dim", type=int, default=4)
    p.add_argument("--width", type=int, default=None, help="frame width (default: by --scaling)")
    p.add_argument("--height", type=int, default=None)
    p.add_argument("--scaling", choices=("auto", "weak", "strong"), default="auto",
                   help="auto: N=1 3840x2160, N>1 config 4 (7680x4320 fixed); strong: 7680x4320 at every N; weak: "
                        "3840x2160 rays per rank")
    p.add_argument("--mgpu", choices=("vhx", "torch"), default="vhx",
                   help="N>1 data path: vhx = RCCL behind the C ABI (vhx_mgpu_*), torch = torch.distributed gather")
    p.add_argument("--scene", type=int, default=1, help="VHX_SCENE_* (1 = lattice+cube scene S)")
    p.add_argument("--vox", default=None, help="trace a MagicaVoxel model instead (BoxTree::load_vox_file, bd = "
                                              "--brick-dim; tree size from the model)")
    p.add_argument("--tile", type=int, default=64)
    p.add_argument("--shadows", action="store_true",
                   help="config 5: each step = primary frame + one hard-shadow ray per hit toward (S,S,S)")
    p.add_argument("--shadow-mode", choices=("fused", "separate"), default="separate",
                   help="--shadows: 'separate' = vhx_trace_primary then vhx_trace_shadows (_batch) on the same stream; "
                        "'fused' = the shadow rays run in the primary trace (vhx_set_shadow_light: a lane goes on with "
                        "its hit's shadow ray), bit-identical and measured 4-5 %% slower (DESIGN.md §8.1)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-roofline", action="store_true")
    p.add_argument("--no-frame-check", action="store_true",
                   help="skip the untimed check of the in-flight frames (frames_equal / golden_match)")
    p.add_argument("--no-isolated", action="store_true",
                   help="skip the isolated (one frame at a time) launches after the timed region: the PMC child's "
                        "counters then cover the timed frames' schedule only")
    p.add_argument("--no-pmc", action="store_true",
                   help="skip the rocprofv3 FETCH_SIZE child run (roofline.traffic from profiles/traffic.json)")
    p.add_argument("--inflight", type=int, default=None,
                   help="contexts in flight per GPU: F contexts sharing the tree (vhx_create_shared), each on its own "
                        "stream, frame (or batch) i traced by context i %% F, so a latency-bound long-ray tail overlaps the "
                        "next frame's pass 0 (1 = one at a time). Default with batches 3 (the hardware queues left at "
                        "the process default), without 20 frames in flight with GPU_MAX_HW_QUEUES raised to F + 4 so "
                        "that every frame's stream has a hardware queue of its own")
    p.add_argument("--batch", type=int, default=None, metavar="K",
                   help="frames per vhx_trace_primary_batch call (one pass ladder over K frames on one stream); 0 = one "
                        "vhx_trace_primary per frame. Default 7 (on 3 contexts) for one-GPU primary frames without --inflight "
                        "(docs/DESIGN_LOG.md §16.1: 7 frames x 3 contexts was the fastest split of the driver's 20-frame window), "
                        "else 0")
    p.add_argument("--orbit", type=float, default=0.0,
                   help="moving camera: frame k (warm-up included) views from angle 40 + k*ORBIT rad on the glass "
                        "camera's circle (0 = the reference bench's static camera); the roofline bytes are then the "
                        "mean of the first, middle and last timed views")
    p.add_argument("--depth-prepass", type=float, default=None, metavar="MARGIN",
                   help="opt-in approximate mode (vhx_set_depth_prepass, not the reference semantics): a half-resolution "
                        "depth prepass, full-resolution rays start at the min of 4 texels minus MARGIN")
    p.add_argument("--budgets", default=None, metavar="B1,B2,...",
                   help="step budgets of the pass schedule (vhx_set_pass_budgets; \"\" = one pass); default: the library's adaptive choice ({32, 128, 768} with frames in flight, {24, 72, 216, 648} for shadow traces, {64} for a lone frame), one pass with --mip-lod (its rays are short: 0.092 against 0.136 ms per depth-1 frame, profiles/r02/mips/headline/budgets)")
    p.add_argument("--mip-lod", type=int, default=None, metavar="DEPTH",
                   help="opt-in MIP stand-in mode (not the reference path): the scene inserted into a host BoxTree with "
                        "MIP maps on, flattened down to DEPTH (vhx_boxtree_flatten_lod) and traced with its node MIPs "
                        "(vhx_set_node_mips); N = 1, no roofline / CPU leg (keep --size <= 256: O(size^3) inserts)")
    p.add_argument("--no-overlap", action="store_true",
                   help="N>1: gather each frame before tracing the next (default: frame k's gather overlaps k+1)")
    p.add_argument("--tune", default=None, metavar="SPEC",
                   help="scheduling knobs of every context (vhx_set_tuning \"key=value;...\", include/vhx.h; results "
                        "never change): experiments only")
    p.add_argument("--planes", type=int, choices=(1, 2), default=1,
                   help="N>1 (vhx_mgpu): planes each rank sends to rank 0 in the timed frames: 1 = RGBA8 (the reference's "
                        "display output, the rgba8unorm view texture of src/raytracing/bevy/view.rs:269-289), 2 = RGBA8 + "
                        "f32 depth; the untimed multi-GPU check runs both")
    p.add_argument("--no-extra", action="store_true",
                   help="skip the untimed-region extras of an N = 1 line: the `lone` (one frame at a time) and `orbit` "
                        "(distinct cameras in flight) sub-objects")
    p.add_argument("--root-slots", type=int, default=0,
                   help="N>1 (vhx_mgpu): rank 0's share of the tile slots (R of R+N-1); 0 (default) = measured before "
                        "the warm-up by vhx_mgpu_balance (untimed)")
    return p.parse_args()


CONFIG4 = (7680, 4320)  # BASELINE config 4 frame
HEADLINE = (3840, 2160)  # BASELINE metric / config 3 frame


def frame_size(args, world):
    """(W, H, scaling label). Weak scaling keeps the field of view and W*H/N = 3840*2160 (dimensions rounded to
    multiples of 8); strong scaling keeps the frame."""
    mode = args.scaling
    if mode == "auto":
        mode = "strong" if world > 1 else "single"
    if args.width and args.height:
        return args.width, args.height, ("weak" if mode == "weak" else "strong")
    if mode == "single":  # one GPU, the fixed headline frame: no scaling is measured
        return HEADLINE[0], HEADLINE[1], "none"
    if mode == "strong":
        return CONFIG4[0], CONFIG4[1], "strong"
    w, h = HEADLINE
    if world == 1:
        return w, h, "weak"
    f = world ** 0.5
    return int(round(w * f / 8.0)) * 8, int(round(h * f / 8.0)) * 8, "weak"


def cpu_cores():
    """Cores this process may run on: the affinity set, capped by a cgroup CPU quota when there is one (a GPU box
    shows the whole machine's CPUs but grants each job a share)."""
    n = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = max(1, int(-(-int(q) // int(per))))
    except (OSError, ValueError):
        pass
    return (min(n, quota) if quota else n), n, quota


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


TRAFFIC_FILE = os.path.join(ROOT, "profiles", "traffic.json")


def pmc_traffic(workload):
    """Memory-side read bytes per launch for this workload, from the committed PMC summary (or None)."""
    try:
        d = json.load(open(TRAFFIC_FILE))
    except (OSError, ValueError):
        return None
    e = d.get(workload)
    return None if e is None else e


FRAME_KERNELS = ("k_trace_primary<false", "k_trace_primary_batch<", "k_trace_queue<false", "k_count_flags", "k_scan_counts", "k_emit_flags",
                 "k_gather_chunks", "k_put_queue_args")


def parse_pmc_dir(d, blocks_per_frame=None):
    """Per-frame figures from rocprofv3 counter_collection CSVs under `d` (see measure_traffic), or None. A pass-0
    dispatch is one frame; a batch's pass-0 dispatch (k_trace_primary_batch) is Grid_Size / (256 x blocks_per_frame)
    frames."""
    tot, per_kernel, frames, batch_frames = {}, {}, set(), {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            n = row["Kernel_Name"].replace("void ", "")
            if not n.startswith(FRAME_KERNELS):
                continue
            c, v = row["Counter_Name"], float(row["Counter_Value"])
            tot[c] = tot.get(c, 0.0) + v
            k = per_kernel.setdefault(n.split("<")[0], {})
            k[c] = k.get(c, 0.0) + v
            if n.startswith("k_trace_primary<false"):
                frames.add(row["Dispatch_Id"])
            elif n.startswith("k_trace_primary_batch<") and blocks_per_frame:
                # the list order pads a frame to whole 64x64 tiles (< 1 % more workgroups): nearest whole frame count
                batch_frames[row["Dispatch_Id"]] = round(int(row["Grid_Size"]) / (256 * blocks_per_frame))
    if not (frames or batch_frames) or "FETCH_SIZE" not in tot:
        return None
    nf = len(frames) + sum(batch_frames.values())
    lanes = {k: round(v["SQ_THREAD_CYCLES_VALU"] / max(1.0, v["SQ_ACTIVE_INST_VALU"]), 2)
             for k, v in per_kernel.items() if "trace" in k and "SQ_ACTIVE_INST_VALU" in v}
    return {"bytes": tot["FETCH_SIZE"] * 1024.0 * 2.0 / nf, "frames": nf,
            "valu": tot.get("SQ_INSTS_VALU", 0.0) / nf,
            "useful": tot.get("SQ_THREAD_CYCLES_VALU", 0.0) / (64.0 * max(1.0, tot.get("SQ_ACTIVE_INST_VALU", 0.0))),
            "lanes": lanes}


def measure_traffic(busy_only=False, tune=None, blocks_per_frame=None):
    """Memory-side read bytes per frame, measured now: this bench (same arguments, 5 timed + 1 warm-up frames, no
    roofline / CPU leg) under `rocprofv3 --pmc FETCH_SIZE --kernel-trace` as a child process, FETCH_SIZE summed over
    the frame kernels and divided by the pass-0 dispatches, x1024 B and x2 (gfx950: FETCH_SIZE derives from
    TCC_EA0_RDREQ and reads half the bytes; /opt/skills/guides/MI355X_MICROARCH.md, HBM section; Infinity-Cache hits
    included, an upper bound of HBM bytes). The same pass (one --pmc run: 3 TCC + 3 SQ counters) collects
    SQ_INSTS_VALU, SQ_THREAD_CYCLES_VALU and SQ_ACTIVE_INST_VALU for the issue side. Returns a dict (bytes,
    valu, active lanes per VALU instruction per trace kernel, frames) or None (no profiler, a failure or 120 s).
    busy_only: every frame of the child runs the frames-in-flight schedule (vhx_set_tuning "adaptive=0", after any
    --tune of this run), the schedule of the timed frames; otherwise its setup frames (one per context, each alone)
    would run the lone-frame schedule and their counters would mix into the per-frame figures."""
    rp = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(rp):
        return None
    d = tempfile.mkdtemp(prefix="vhx_pmc_", dir="/tmp")
    counters = ["FETCH_SIZE", "SQ_INSTS_VALU", "SQ_THREAD_CYCLES_VALU", "SQ_ACTIVE_INST_VALU"]
    cmd = ([rp, "--pmc"] + counters + ["--kernel-trace", "-f", "csv", "-d", d, "-o", "pmc", "--", sys.executable,
                                       os.path.abspath(__file__)] + sys.argv[1:] +
           ["--steps", "5", "--warmup", "1", "--no-cpu-baseline", "--no-roofline", "--no-pmc",
            "--no-frame-check", "--no-extra", "--no-isolated"] +
           (["--tune", (tune + ";" if tune else "") + "adaptive=0"] if busy_only else []))
    env = dict(os.environ, TMPDIR="/tmp")
    env.pop("VHX_BENCH_MGPU1", None)  # the child times the single-GPU path only
    try:
        proc = subprocess.Popen(cmd, cwd="/tmp", env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                                start_new_session=True)
        try:
            rc = proc.wait(timeout=120)
        except subprocess.TimeoutExpired:
            os.killpg(proc.pid, signal.SIGKILL)
            proc.wait()
            return None
        if rc != 0:
            return None
        return parse_pmc_dir(d, blocks_per_frame)
    except (OSError, ValueError, KeyError):
        return None
    finally:
        shutil.rmtree(d, ignore_errors=True)


def cpu_baseline(flat, cam, W, H, threads_all, light=None):
    """The oracle (reference semantics, oracle/) on the host cores over the bench frame: all cores available to the
    process (OpenMP, dynamic over pixels), 1 warm-up + median of 5 full frames; and 1 core, 1 warm-up + median of 5
    frames of the same view at a quarter of the resolution per axis (a uniform 1/16 sample of the frame's rays, about
    0.4 s each, so that the default bench still finishes in minutes). With a light (config 5) each frame is the
    primary frame plus the oracle's hard-shadow pass over its hits."""
    from tests._oracle import Oracle
    orc = Oracle()
    fields = ("rgba", "depth", "value", "impact", "normal") if light is not None else ("rgba", "depth")

    rays = {}

    def frame(w, h, c, threads):
        hits = orc.trace_primary(flat, c, 0, 0, w, h, threads=threads, fields=fields)
        rays[(w, h)] = w * h
        if light is not None:
            orc.trace_shadows(flat, light, hits, threads=threads)
            rays[(w, h)] += int((hits["value"] != 0xFFFFFFFF).sum())  # one shadow ray per hit

    def timed(w, h, c, threads):
        frame(w, h, c, threads)  # warm-up
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            frame(w, h, c, threads)
            ts.append(time.perf_counter() - t0)
        return sorted(ts)[2]

    import voxelhex_amd as vhx
    t_all = timed(W, H, cam, threads_all)
    w1, h1 = max(1, W // 4), max(1, H // 4)
    c1 = vhx.glass_camera(int(flat.desc.boxtree_size), w1, h1, target=(flat.desc.boxtree_size / 2.0,) * 3)
    t_one = timed(w1, h1, c1, 1)
    return t_all, t_one, (w1, h1), rays[(W, H)], rays[(w1, h1)]


GOLDEN = os.path.join(ROOT, "tests", "golden", "frames.json")
GOLDEN_FIELDS = ("value", "cell", "voxel", "impact", "normal", "depth", "rgba")


def golden_case(args, W, H):
    """The tests/golden/frames.json entry of this workload (the oracle's frame, SHA-256 per field), or None: the
    reference-path frame of a procedural scene with the golden camera (glass_camera(size, W, H, target=centre))."""
    if args.vox or args.orbit or args.depth_prepass is not None or args.mip_lod is not None:
        return None
    try:
        meta = json.load(open(GOLDEN))
    except (OSError, ValueError):
        return None
    for name, m in meta.items():
        if (m.get("scene"), m.get("size"), m.get("brick_dim"), m.get("width"), m.get("height")) == \
                (args.scene, args.size, args.brick_dim, W, H) and not name.startswith("mip"):
            return name, m
    return None


def check_frames(args, rt, rts, outs, last_cam, light, W, H, dev):
    """Untimed check of the timed configuration: context f's last frame (RGBA8 + f32 depth, and the shadow flags
    with --shadows) is compared bit for bit with the owner context tracing the same camera alone, one frame at a time;
    when the workload is a golden case every field of that lone frame and the RGBA / depth of every in-flight frame
    are compared with the committed SHA-256 digests."""
    import hashlib

    import torch

    def sha(a):
        return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()

    gc = golden_case(args, W, H)
    torch.cuda.synchronize(dev)
    got = {f: {k: outs[f][k].cpu().numpy().view(np.uint32).copy()
               for k in (("rgba", "depth", "shadowed") if args.shadows else ("rgba", "depth"))}
           for f in sorted(last_cam)}
    refs, mism = {}, []
    for f in sorted(last_cam):
        cam = last_cam[f]
        key = id(cam)
        if key not in refs:
            if args.shadows:
                n = W * H
                o = {"rgba": torch.zeros(n, dtype=torch.int32, device=dev),
                     "depth": torch.zeros(n, dtype=torch.float32, device=dev),
                     "value": torch.full((n,), -1, dtype=torch.int32, device=dev),
                     "impact": torch.zeros((n, 3), dtype=torch.float32, device=dev),
                     "normal": torch.zeros((n, 3), dtype=torch.float32, device=dev),
                     "shadowed": torch.zeros(n, dtype=torch.int32, device=dev)}
                rt.trace_primary(cam, out=o)
                rt.trace_shadows(light, o, shadowed=o["shadowed"])
                rt.sync()
                refs[key] = {k: o[k].cpu().numpy().view(np.uint32).copy() for k in ("rgba", "depth", "shadowed")}
            else:
                fr = rt.trace_primary(cam, fields=GOLDEN_FIELDS if gc else ("rgba", "depth"))
                refs[key] = {k: v.view(np.uint32) for k, v in fr.items()}
        ref = refs[key]
        for k, a in got[f].items():
            if not np.array_equal(a, ref[k]):
                mism.append({"context": f, "field": k, "pixels": int((a != ref[k]).sum())})
    res = {"contexts": len(got), "frames_equal": not mism, "mismatches": mism[:8],
           "basis": "last frame of each of the F contexts in flight vs the owner context tracing the same camera "
                    "alone (bit-exact, " + ("RGBA8 + depth + shadow flags" if args.shadows else "RGBA8 + depth") + ")",
           "golden_match": None}
    if gc is not None and not args.shadows:
        name, m = gc
        lone = refs[next(iter(refs))]
        bad = [k for k in GOLDEN_FIELDS if sha(lone[k]) != m["sha256"][k]]
        bad += [f"context{f}.{k}" for f in got for k in ("rgba", "depth") if sha(got[f][k]) != m["sha256"][k]]
        res.update(golden_match=not bad, golden_case=name, golden_mismatch=bad,
                   golden_basis="tests/golden/frames.json (the oracle's frame, SHA-256 per field): every field of the "
                                "lone frame, RGBA / depth of every in-flight frame")
    return res


def visible_gpus():
    """GPUs a rank process would see, counted in a child process (torch.cuda.device_count reads the device list
    without initialising HIP; the child keeps even that out of the launcher). -1 if the count failed."""
    try:
        r = subprocess.run([sys.executable, "-c", "import torch; print(torch.cuda.device_count())"],
                           capture_output=True, text=True, timeout=600)
        return int(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else -1
    except (OSError, ValueError, IndexError, subprocess.TimeoutExpired):
        return -1


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_plan(n, argv, port):
    """The N rank processes of `bench.py --gpus N`: this script with the same arguments, one process per GPU, with the
    environment torchrun would give them (RANK, LOCAL_RANK, WORLD_SIZE, LOCAL_WORLD_SIZE, MASTER_ADDR/PORT on
    127.0.0.1)."""
    cmd = [sys.executable, os.path.abspath(__file__)] + list(argv)
    plan = []
    for r in range(n):
        env = {"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(n), "LOCAL_WORLD_SIZE": str(n),
               "GROUP_RANK": "0", "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
               "HSA_ENABLE_IPC_MODE_LEGACY": "0", "VHX_BENCH_LAUNCHED": "1"}
        plan.append({"rank": r, "cmd": cmd, "env": env})
    return plan


def launch_ranks(args):
    """`python bench.py --gpus N` (N > 1) with no WORLD_SIZE in the environment: this process is only the launcher.
    It imports neither torch nor libvhx and touches no GPU: it counts the visible GPUs in a child process, fails with
    a message (exit 2) if there are fewer than N, starts N rank processes of this script (rank_plan) in sessions of
    their own, and exits with 0 once all N exit 0 -- rank 0 prints the JSON line straight to the shared stdout --
    or, as soon as one rank fails, stops the others and exits with that rank's status. One-GPU runs never come here,
    so `--gpus N` can never print a one-GPU line."""
    n = args.gpus
    argv = [a for a in sys.argv[1:] if a != "--print-launch"]
    port = free_port()
    plan = rank_plan(n, argv, port)
    if args.print_launch:
        print(json.dumps({"launcher": "bench.py", "world": n, "master": f"127.0.0.1:{port}", "ranks": plan,
                          "torch_imported": "torch" in sys.modules,
                          "vhx_imported": any(m.startswith("voxelhex_amd") for m in sys.modules)}), flush=True)
        return 0
    if os.environ.get("VHX_BENCH_SKIP_DEVICE_CHECK") != "1":
        have = visible_gpus()
        if have < n:
            print(f"bench.py --gpus {n}: {n} GPUs requested, "
                  + (f"{have} visible" if have >= 0 else "the device count failed")
                  + " -- refusing to run (no line is printed for fewer GPUs than requested)", file=sys.stderr,
                  flush=True)
            return 2
    procs = []
    for p in plan:
        procs.append(subprocess.Popen(p["cmd"], env=dict(os.environ, **p["env"]), start_new_session=True))

    def stop_all(sig=signal.SIGTERM):
        for q in procs:
            if q.poll() is None:
                try:
                    os.killpg(q.pid, sig)
                except OSError:
                    pass

    def on_signal(signum, _frame):
        stop_all(signal.SIGTERM)
        raise SystemExit(128 + signum)

    signal.signal(signal.SIGTERM, on_signal)
    signal.signal(signal.SIGINT, on_signal)
    rc = 0
    live = set(range(n))
    while live:
        for r in sorted(live):
            s = procs[r].poll()
            if s is None:
                continue
            live.discard(r)
            if s != 0 and rc == 0:
                rc = s if s > 0 else 128 - s
                print(f"bench.py --gpus {n}: rank {r} exited with status {s}; stopping the other ranks",
                      file=sys.stderr, flush=True)
                stop_all(signal.SIGTERM)
                deadline = time.time() + 15
                while time.time() < deadline and any(q.poll() is None for q in procs):
                    time.sleep(0.1)
                stop_all(signal.SIGKILL)
        time.sleep(0.05)
    for q in procs:
        q.wait()
    return rc


def scaling_n1(args):
    """The scaling curve's N = 1 point: the N > 1 default workload -- BASELINE config 4, the
    7680x4320 frame (--scaling strong) -- run by the N > 1 ranks' own code (vhx_mgpu on a one-rank RCCL communicator,
    VHX_BENCH_MGPU1, frames in flight, the tiles untiled into rank 0's framebuffer) as a child process of this bench
    (its own hardware queues, like every rank of an N > 1 run), 20 timed frames after 5 warm-up frames. Returns the
    sub-object for the line; value(N) / (N x this value) is then like-for-like strong scaling."""
    cmd = [sys.executable, os.path.abspath(__file__), "--scaling", "strong", "--steps", "20", "--warmup", "5",
           "--size", str(args.size), "--brick-dim", str(args.brick_dim), "--scene", str(args.scene),
           "--tile", str(args.tile), "--planes", str(args.planes), "--no-cpu-baseline", "--no-roofline", "--no-pmc",
           "--no-extra", "--no-isolated"]
    env = dict(os.environ, VHX_BENCH_MGPU1="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()),
               RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    env.pop("GPU_MAX_HW_QUEUES", None)  # the child raises it for its frames in flight, as an N > 1 rank does
    t0 = time.time()
    try:
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240, start_new_session=True)
    except subprocess.TimeoutExpired:
        return {"error": "timed out after 240 s"}
    line = None
    for ln in r.stdout.splitlines():
        if ln.startswith("{"):
            try:
                line = json.loads(ln)
            except ValueError:
                pass
    if r.returncode != 0 or line is None:
        return {"error": f"exit {r.returncode}", "stderr_tail": r.stderr[-400:]}
    return {"value": line["value"], "unit": line["unit"], "ms_per_step": line["ms_per_step"], "steps": line["steps"],
            "warmup": line["warmup"], "workload": line["config"]["workload"], "parallelism": line["config"]["parallelism"],
            "frames_in_flight": line.get("frames_in_flight"), "frame_equal": (line.get("multi_gpu_check") or {}).get(
                "frame_equal"), "mgpu_fallback": line.get("mgpu_fallback"), "child_wall_s": round(time.time() - t0, 1),
            "basis": "N = 1 point of the multi-GPU curve: the workload every N > 1 run of this bench times (BASELINE "
                     "config 4, strong scaling) through the same rank code (vhx_mgpu, one-rank RCCL communicator, tile "
                     "layout + untile), run as a child process of this bench; scaling at N = value(N) / (N x this)"}


def hw_queues(frames):
    """Hardware queues for F frames in flight: HIP maps streams onto GPU_MAX_HW_QUEUES hardware queues per process (4
    by default) round-robin, and the default stream holds one, so with the default four frames in flight two frames
    share a queue and run one after the other (bench frame: 0.93 ms per frame at F = 4 against 0.70 with five queues;
    0.66 at F = 8 with nine or more). Read by the HIP runtime at initialisation: set before torch is imported. The
    frames' streams, the gather stream (N > 1) and the default stream each get their own queue (at most 32)."""
    want = min(32, frames + 4)
    try:
        cur = int(os.environ.get("GPU_MAX_HW_QUEUES", "4"))
    except ValueError:
        cur = 4
    if cur < want:
        os.environ["GPU_MAX_HW_QUEUES"] = str(want)
    return int(os.environ.get("GPU_MAX_HW_QUEUES", "4"))


def main():
    args = parse()
    if args.tune in ("", "-"):
        args.tune = None  # "-": the library defaults (scripts that loop over specs)
    if "WORLD_SIZE" not in os.environ:
        if args.gpus is not None and args.gpus > 1:
            sys.exit(launch_ranks(args))
        if args.gpus is not None and args.gpus < 1:
            raise SystemExit(f"bench.py --gpus {args.gpus}: at least one GPU")
    elif args.gpus is not None and args.gpus != int(os.environ["WORLD_SIZE"]):
        raise SystemExit(f"bench.py --gpus {args.gpus} under a launcher with WORLD_SIZE={os.environ['WORLD_SIZE']}: "
                         "the two must agree")
    echo = os.environ.get("VHX_BENCH_RANK_ECHO")
    if echo is not None and os.environ.get("VHX_BENCH_LAUNCHED") == "1":
        # launcher self-test (tests/test_bench_launch.py): the rank reports its environment and exits before torch
        keys = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")
        print(json.dumps({"rank_echo": {k: os.environ.get(k) for k in keys}, "argv": sys.argv[1:]}), flush=True)
        sys.exit(3 if echo == "fail" + os.environ.get("RANK", "") else 0)
    if args.batch is None:
        # batches wherever they are the faster line: one GPU, primary rays on the exact path, and no explicit
        # --inflight (which asks for that many per-frame contexts). Config 5 (--shadows) keeps twenty per-frame
        # contexts: its batches (vhx_trace_shadows_batch, --batch K) measured 1.31 against 1.17-1.23 ms per frame
        # (docs/DESIGN_LOG.md §16.3), 1.08 against 0.99-1.00 ms in round 6 (profiles/r06/shadows/); fused shadows
        # batch (7 x 3)
        # The multi-GPU ranks (vhx_mgpu) batch too: each rank's tile sets of K frames as one vhx_trace_tiles_batch
        # (vhx_mgpu_render_batch) -- a rank's share of a config-4 frame is half a headline frame, and traced one frame
        # at a time it ran at 55 % of the whole frame's rate (scripts/probes/probe_tiles.py)
        world_env = int(os.environ.get("WORLD_SIZE", "1"))
        single = world_env == 1 and os.environ.get("VHX_BENCH_MGPU1") != "1"
        mgpu_path = (world_env > 1 or os.environ.get("VHX_BENCH_MGPU1") == "1") and args.mgpu == "vhx" and \
            os.environ.get("VHX_BENCH_REHEARSAL") != "1"
        args.batch = 7 if ((single or mgpu_path) and args.inflight is None and
                           (not args.shadows or args.shadow_mode == "fused") and
                           args.depth_prepass is None and args.mip_lod is None) else 0
        if args.batch:
            args.inflight = 3
    if args.inflight is None:
        args.inflight = 2 if args.batch else 20
    if args.batch and int(os.environ.get("WORLD_SIZE", "1")) == 1 and os.environ.get("VHX_BENCH_MGPU1") != "1":
        # one stream per batch in flight: the box's default hardware queues (GPU_MAX_HW_QUEUES unset: 4) suffice for
        # three contexts (the default stream holds one queue); more contexts get a queue each
        queues = hw_queues(args.inflight) if args.inflight > 3 else int(os.environ.get("GPU_MAX_HW_QUEUES", "4"))
    else:
        # per-frame contexts, or a multi-GPU rank's batch contexts plus its communication stream: a queue each
        queues = hw_queues(max(1, args.inflight))
    import torch
    import torch.distributed as dist

    import voxelhex_amd as vhx
    from voxelhex_amd import _native as N
    from voxelhex_amd import multigpu as M

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal of the torch multi-GPU path on a single GPU: VHX_BENCH_REHEARSAL=1 puts every rank on cuda:0 and
    # gathers over gloo through host memory (RCCL needs one GPU per rank); timings from such a run are not scaling
    rehearsal = world > 1 and os.environ.get("VHX_BENCH_REHEARSAL") == "1"
    # VHX_BENCH_MGPU1=1 (diagnostics): the vhx_mgpu data path on a one-rank communicator, so that a one-GPU box runs
    # every step of the multi-GPU bench path (gloo setup, RCCL id exchange, tree broadcast, frames in flight, gather,
    # untile, frame check) that the N > 1 runs take
    force1 = world == 1 and os.environ.get("VHX_BENCH_MGPU1") == "1"
    use_vhx_mgpu = (world > 1 or force1) and args.mgpu == "vhx" and not rehearsal
    if rehearsal:
        local = 0
    elif world > 1 and torch.cuda.device_count() < world:
        raise SystemExit(f"bench.py rank {rank}: WORLD_SIZE={world} needs {world} visible GPUs, "
                         f"{torch.cuda.device_count()} visible")
    if force1:
        for k, v in (("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", "29533"), ("RANK", "0"), ("WORLD_SIZE", "1")):
            os.environ.setdefault(k, v)
    if world > 1 or force1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(local)
        if rehearsal or use_vhx_mgpu:
            # gloo: barriers, the max-over-ranks timing and the RCCL id exchange; the frame data moves over RCCL
            # inside libvhx (vhx_mgpu) or, in the rehearsal, over gloo through host memory
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    rt = vhx.Raytracer(local, tune=args.tune)
    # the context's own stream, shared with torch (ExternalStream): the kernels and the events that time them are
    # ordered on it. Every frame in flight traces on its context's own stream; those streams are created back to back
    # so that each gets a hardware queue of its own (GPU_MAX_HW_QUEUES = 4; streams share queues round-robin in
    # creation order, and extra streams created in between made two frames share a queue: 0.91 against 0.70 ms/frame)
    stream = torch.cuda.ExternalStream(rt.stream(), device=dev)
    torch.cuda.set_stream(stream)
    F = max(1, args.inflight)
    if world > 1 and not use_vhx_mgpu:
        F = 1  # the torch gather pipeline keeps one frame per rank in flight

    mg = None
    mgpu_fallback = None
    if use_vhx_mgpu:
        # RCCL behind the ABI; if it cannot start on every rank (no loadable RCCL, communicator init failed), all ranks
        # fall back together to the torch.distributed gather (RCCL via torch), and the line says so
        uid = None
        if rank == 0:
            try:
                uid = M.mgpu_unique_id()
            except Exception as e:  # noqa: BLE001 (reported in the line)
                mgpu_fallback = f"vhx_mgpu_unique_id: {e}"
        obj = [uid]
        dist.broadcast_object_list(obj, src=0)
        ok = obj[0] is not None
        if ok:
            try:
                mg = M.MgpuRenderer(rt, obj[0], world, rank, tile_size=args.tile, overlap=not args.no_overlap)
                mg.set_frames_in_flight(min(F, N.VHX_MGPU_MAX_INFLIGHT))
            except Exception as e:  # noqa: BLE001
                mgpu_fallback = f"vhx_mgpu on rank {rank}: {e}"
                mg = None
        flag = torch.tensor([1 if mg is not None else 0], dtype=torch.int32)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        if int(flag.item()) == 0:
            if mg is not None:
                mg.close()
                mg = None
            fb = [mgpu_fallback]
            dist.broadcast_object_list(fb, src=0)
            mgpu_fallback = mgpu_fallback or fb[0] or "vhx_mgpu failed on another rank"
            use_vhx_mgpu = False
            dist.destroy_process_group()
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
            F = 1
        else:
            # collective (the ranks agree on the plane count over the communicator): only once every rank has its
            # renderer, so that no rank waits in it for one that fell back
            mg.set_planes(args.planes)

    # the tree: built on the host (rank 0 only when it is broadcast over RCCL), uploaded to HBM
    t0 = time.time()
    flat = None
    if args.mip_lod is not None:
        if world > 1 or args.shadows:
            raise SystemExit("--mip-lod is a one-GPU primary-ray mode")
        args.no_roofline = args.no_cpu_baseline = args.no_pmc = True
        # the buffers of insert_scene + switch_albedo_mip_maps(True) + flatten_lod (tests/test_scene_builder.py)
        flat = vhx.FlatTree.build_scene_lod(args.scene, args.size, args.brick_dim, args.mip_lod,
                                            threads=min(16, os.cpu_count() or 1))
    elif args.vox:
        if mg is None or rank == 0:
            flat = vhx.BoxTree.load_vox_file(args.vox, args.brick_dim).flatten()
    elif mg is None or rank == 0:
        flat = vhx.FlatTree.build_scene(args.scene, args.size, args.brick_dim, threads=min(16, os.cpu_count() or 1))
    build_s = time.time() - t0
    t0 = time.time()
    if mg is not None:
        mg.broadcast_tree(flat if rank == 0 else None)
    else:
        rt.upload(flat)
        if args.mip_lod is not None:
            rt.set_node_mips(flat.node_mips)  # shared contexts trace with the owner's MIPs
    upload_s = time.time() - t0
    tree_info = None
    if rank == 0:
        tree_info = dict(tree_nodes=int(flat.desc.node_count), tree_bricks=int(flat.desc.brick_count),
                         tree_gb=round(flat.nbytes() / 1e9, 3), size=int(flat.desc.boxtree_size))
    if args.vox:
        obj = [tree_info["size"] if rank == 0 else None]
        if world > 1:
            dist.broadcast_object_list(obj, src=0)
        args.size = obj[0]

    W, H, scaling = frame_size(args, world)
    T = args.tile
    c = args.size / 2.0
    cam = vhx.glass_camera(args.size, W, H, target=(c, c, c))
    cams = [cam]
    if args.orbit:
        cams = [vhx.glass_camera(args.size, W, H, angle=40.0 + k * args.orbit, target=(c, c, c))
                for k in range(args.warmup + args.steps)]
    light = (float(args.size),) * 3  # ambient_light_position, src/raytracing/bevy/view.rs:81-85
    if world == 1:
        n_out = W * H
        trace_kw = dict(tile_size=0, tile_start=0, tile_stride=1, layout=N.VHX_LAYOUT_FRAMEBUFFER)
        tiles_per_rank = 0
    else:
        tiles_per_rank = M.tiles_per_rank(W, H, T, world)
        n_out = tiles_per_rank * T * T
        trace_kw = dict(tile_size=T, tile_start=rank, tile_stride=world, layout=N.VHX_LAYOUT_TILES)
    if args.shadows and mg is not None:
        raise SystemExit("--shadows with N > 1 needs --mgpu torch")
    fb_rgba = fb_depth = None
    if mg is not None and rank == 0:
        fb_rgba = torch.zeros(W * H, dtype=torch.int32, device=dev)
        fb_depth = torch.zeros(W * H, dtype=torch.float32, device=dev) if args.planes == 2 else None
    # frames in flight (single-GPU and torch paths; vhx_mgpu keeps its own): F contexts sharing the tree, F streams,
    # F output sets
    if args.depth_prepass is not None:
        rt.set_depth_prepass(True, args.depth_prepass)  # shared contexts inherit it
    rts, streams, outs = [rt], [stream], []
    if mg is None:
        for _ in range(F - 1):
            r = rt.shared()
            if args.tune:
                r.set_tuning(args.tune)
            rts.append(r)
            streams.append(torch.cuda.ExternalStream(r.stream(), device=dev))
    # the pass schedule of every context (vhx_mgpu re-copies the owner context's settings to its frames' contexts)
    budgets = args.budgets if args.budgets is not None else ("" if args.mip_lod is not None else None)
    if budgets is not None:
        for r in rts:
            r.set_pass_budgets(tuple(int(b) for b in budgets.split(",") if b.strip()))
    fused = args.shadows and args.shadow_mode == "fused"
    if fused:  # config 5 in the primary trace: every timed trace casts its hits' shadow rays
        for r in rts:
            r.set_shadow_light(light)
    K = args.batch if ((mg is None and world == 1) or mg is not None) else 0
    if args.batch and not K:
        raise SystemExit("--batch needs one GPU or the vhx_mgpu path (not --mgpu torch)")
    fbs_rgba = fbs_depth = None
    if mg is not None and rank == 0:
        # a batch's frames land in K framebuffers (frame 0 of every batch in fb_rgba / fb_depth)
        fbs_rgba = [fb_rgba] + [torch.zeros(W * H, dtype=torch.int32, device=dev) for _ in range(max(1, K) - 1)]
        if fb_depth is not None:
            fbs_depth = [fb_depth] + [torch.zeros(W * H, dtype=torch.float32, device=dev) for _ in range(max(1, K) - 1)]
    for _ in range(len(rts) * max(1, K) if mg is None else 1):  # batch mode: K output sets per context, outs[f * K + j]
        o = {"rgba": torch.zeros(n_out, dtype=torch.int32, device=dev),
             "depth": torch.zeros(n_out, dtype=torch.float32, device=dev)}
        if args.shadows:
            # -1 = VHX_EMPTY: tile padding past the frame edge is never written and casts no shadow ray
            o.update(value=torch.full((n_out,), -1, dtype=torch.int32, device=dev),
                     impact=torch.zeros((n_out, 3), dtype=torch.float32, device=dev),
                     normal=torch.zeros((n_out, 3), dtype=torch.float32, device=dev),
                     shadowed=torch.zeros(n_out, dtype=torch.int32, device=dev))
        outs.append(o)
    out = outs[0]
    torch.cuda.synchronize(dev)  # the zero fills run on torch's stream: complete before the context streams write
    pipe = None
    framebuffer = None
    if world > 1 and mg is None:
        framebuffer = torch.zeros(W * H, dtype=torch.int32, device=dev) if rank == 0 else None

        def untile(gathered, slot):
            rt.untile_rgba(gathered.data_ptr(), world, tiles_per_rank, T, W, H, framebuffer.data_ptr())

        # double-buffered: frame k's gather to rank 0 (and the untile there) overlaps frame k+1's trace
        pipe = M.GatherPipeline(n_out, world, rank, dist, dev, untile, overlap=not args.no_overlap,
                                host_staging=rehearsal)

    ev = []
    frame = [0]
    last_cam = {}  # context -> camera of its last frame (the frame check after the timed region)
    NOEV = os.environ.get("VHX_BENCH_NOEV") == "1"

    def step(timed):
        f = frame[0] % len(rts)
        cam_k = cams[frame[0] % len(cams)]
        frame[0] += 1
        r, s_, o = rts[f], streams[f], outs[f]
        last_cam[f] = cam_k
        if timed and mg is None and not NOEV:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s_)
        if mg is not None:
            mg.render(cam_k, fb_rgba, fb_depth)  # this rank's tiles -> sends to rank 0 -> untile on rank 0
        else:
            if pipe is not None:
                o["rgba"] = pipe.out_buffer()
            r.trace_primary(cam_k, out=o, **trace_kw)
            if args.shadows and not fused:
                r.trace_shadows(light, o, shadowed=o["shadowed"])
        if timed and mg is None and not NOEV:
            e1.record(s_)  # the launch on its own stream (the gather runs on the communication stream)
            ev.append((e0, e1))
        if pipe is not None:
            pipe.submit()

    batch_i = [0]

    def submit_batch(nf, timed):
        """One vhx_trace_primary_batch of the next nf frames on context batch_i % F (vhx_mgpu: one
        vhx_mgpu_render_batch, its contexts taken in turn by the library)."""
        f = batch_i[0] % len(rts)
        batch_i[0] += 1
        r, s_ = rts[f], streams[f]
        cams_b = [cams[(frame[0] + j) % len(cams)] for j in range(nf)]
        frame[0] += nf
        if mg is not None:
            mg.render_batch(cams_b, None if fbs_rgba is None else fbs_rgba[:nf],
                            None if fbs_depth is None else fbs_depth[:nf])
            return
        for j in range(nf):
            last_cam[f * K + j] = cams_b[j]
        if timed and not NOEV:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s_)
        r.trace_primary_batch(cams_b, outs[f * K:f * K + nf])
        if args.shadows and not fused:  # config 5: the batch's shadow rays, one more pass ladder on the same stream
            ob = outs[f * K:f * K + nf]
            r.trace_shadows_batch(light, ob, shadowed_list=[o["shadowed"] for o in ob])
        if timed and not NOEV:
            e1.record(s_)
            ev.append((e0, e1, nf))

    def run(n, timed):
        """n frames: one step each, or batches of K."""
        if K:
            while n > 0:
                submit_batch(min(K, n), timed)
                n -= min(K, n)
        else:
            for _ in range(n):
                step(timed)

    def drain():
        if pipe is not None:
            pipe.drain()
        if mg is not None:
            mg.sync()
        torch.cuda.synchronize(dev)

    # setup (not a step): one untimed frame (batch mode: one batch of K frames) per context allocates its queues and
    # state buffers, so that no allocation (hipMalloc synchronises the device) falls into the timed region when F
    # exceeds the warm-up count
    for _ in range(len(rts) if mg is None else (F if K else 1)):
        run(max(1, K), False)
    drain()
    split = None
    if mg is not None:
        # rank 0's share of the tiles (untimed): a link-bound split moves tiles to rank 0, whose parts cross no link
        if args.root_slots > 0:
            mg.set_root_slots(args.root_slots)
            split = {"root_slots": args.root_slots, "source": "--root-slots"}
        else:
            R, a, g = mg.balance(cam, frames=4)
            split = {"root_slots": R, "rank0_trace_ms_one_slot": round(a, 4), "transfer_ms_one_slot": round(g, 4),
                     "source": "vhx_mgpu_balance"}
            if K and world > 1:
                # vhx_mgpu_balance models the split from single frames, whose per-slot trace is about twice a batched
                # one's: with batches, time the candidate shares directly instead (untimed region, every
                # rank the same R; 3 batches per candidate, the first one a warm-up) and keep the fastest
                cand = {}
                for r_try in range(1, N.VHX_MGPU_MAX_ROOT_SLOTS + 1):
                    mg.set_root_slots(r_try)
                    run(K, False)
                    drain()
                    dist.barrier()
                    tc0 = time.perf_counter()
                    run(2 * K, False)
                    drain()
                    dist.barrier()
                    tt = torch.tensor([time.perf_counter() - tc0], dtype=torch.float64)
                    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
                    cand[r_try] = round(float(tt.item()) * 1e3 / (2 * K), 4)
                R = min(cand, key=lambda r_: (cand[r_] * (1.0 if r_ == 1 else 1.02), r_))  # R > 1 must win by 2 %
                mg.set_root_slots(R)
                split.update(root_slots=R, source="batched search (ms per frame by R; vhx_mgpu_balance's pick "
                                                  f"was {split['root_slots']})", candidates_ms_per_frame=cand)
        # the buffers of the chosen split are allocated outside the timed region (every batch context's)
        for _ in range(F if K else 1):
            run(max(1, K), False)
        drain()
    frame[0] = 0
    batch_i[0] = 0
    run(args.warmup, False)
    drain()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    run(args.steps, True)
    submit_s = time.perf_counter() - t0  # host time to submit the K steps (the GPU runs behind it)
    drain()  # the last frame's gather and untile are inside the timed region
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64)
        if not (rehearsal or use_vhx_mgpu):
            tt = tt.to(dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    # ---- frame check (untimed, N = 1): the last frame of every context in flight equals one context tracing the
    # same camera alone, and the committed golden digests where the workload is a golden case
    # the schedule the timed frames ran (adaptive by default: the frames-in-flight one once other contexts' frames are
    # in flight; vhx_get_pass_budgets), read before the untimed frames below
    sched_timed = None if mg is not None else rts[-1].pass_budgets()
    if fused:
        # the owner context traces the untimed reference frames, the isolated launches and the byte counts the separate
        # way (vhx_trace_primary + vhx_trace_shadows): the frame check then compares fused with separate shadows
        rt.set_shadow_light(None)
    frames_check = None
    if mg is None and world == 1 and not args.no_frame_check:
        frames_check = check_frames(args, rt, rts, outs, last_cam, light, W, H, dev)

    # per-launch duration: with frames in flight (HIP events on each launch's stream, over the timed region); the
    # isolated launch (one frame at a time, libvhx's own events) after it
    if ev:  # per frame: a batch's device time over its frames
        kernel_ms = float(np.mean([e[0].elapsed_time(e[1]) / (e[2] if len(e) > 2 else 1) for e in ev]))
    iso, iso_wall = [], []
    for _ in range(0 if args.no_isolated else 5):
        tw0 = time.perf_counter()
        if mg is not None:
            mg.render(cam, fb_rgba, fb_depth)
            iso.append(mg.sync())
        else:
            if args.shadows:  # the primary frame and its shadow rays, between events on the context's stream
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                rt.trace_primary(cam, out=out, **trace_kw)
                rt.trace_shadows(light, out, shadowed=out["shadowed"])
                e1.record(stream)
                rt.sync()
                iso.append(e0.elapsed_time(e1))
            else:
                rt.trace_primary(cam, out=out, **trace_kw)
                iso.append(rt.sync())
        iso_wall.append(time.perf_counter() - tw0)
    kernel_ms_isolated = float(np.median(iso)) if iso else None
    sched_iso = None if mg is not None else rt.pass_budgets()
    # ---- extras of an N = 1 line (untimed region): the lone frame -- the reference's call shape,
    # one dispatch per frame (VhxRenderNode::run, src/raytracing/bevy/pipeline/mod.rs:96-155) -- and distinct cameras
    # in flight (an orbiting view, every frame a different camera)
    lone = orbit = None
    if mg is None and world == 1 and not args.shadows and not args.no_extra and iso:
        lone = {"ms": round(kernel_ms_isolated, 4), "mrays_per_s": round(W * H / kernel_ms_isolated / 1e3, 3),
                "wall_ms": round(float(np.median(iso_wall)) * 1e3, 4), "frames": len(iso),
                "schedule": None if sched_iso is None else {"budgets": list(sched_iso[0]), "choice": sched_iso[1]},
                "basis": "one frame at a time on one context (submit, synchronise): median of 5 device times between "
                         "libvhx's events around the launch (ms) and of the host wall time of submit + synchronise "
                         "(wall_ms); the bench camera, after the timed frames"}
        if not args.orbit and len(rts) > 1:
            ko, wo, rad = 20, 5, 0.01
            ocams = [vhx.glass_camera(args.size, W, H, angle=40.0 + k * rad, target=(c, c, c)) for k in range(wo + ko)]
            seen = {}
            torch.cuda.synchronize(dev)
            to0 = None
            if K:  # batches of K distinct cameras, the warm-up frames first
                cams_o, kk, bi = ocams, 0, 0
                while kk < wo + ko:
                    nf = min(K, (wo if kk < wo else wo + ko) - kk)
                    if kk == wo:
                        torch.cuda.synchronize(dev)
                        to0 = time.perf_counter()
                    f = bi % len(rts)
                    bi += 1
                    rts[f].trace_primary_batch(cams_o[kk:kk + nf], outs[f * K:f * K + nf])
                    for j in range(nf):
                        seen[f * K + j] = cams_o[kk + j]
                    kk += nf
            for k in range(0 if K else wo + ko):
                if k == wo:
                    torch.cuda.synchronize(dev)
                    to0 = time.perf_counter()
                f = k % len(rts)
                rts[f].trace_primary(ocams[k], out=outs[f], **trace_kw)
                seen[f] = ocams[k]
            torch.cuda.synchronize(dev)
            o_el = time.perf_counter() - to0
            # two contexts' last orbit frames against one context tracing the same camera alone
            o_eq = True
            for f in sorted(seen)[:2]:
                ref = rt.trace_primary(seen[f], fields=("rgba", "depth"))
                for k2 in ("rgba", "depth"):
                    o_eq = o_eq and bool(np.array_equal(outs[f][k2].cpu().numpy().view(np.uint32),
                                                        ref[k2].view(np.uint32)))
            orbit = {"ms_per_frame": round(o_el * 1e3 / ko, 4), "mrays_per_s": round(W * H * ko / o_el / 1e6, 3),
                     "frames": ko, "warmup": wo, "rad_per_frame": rad, "frames_in_flight": len(rts),
                     "frames_equal": o_eq,
                     "basis": f"{ko} timed frames after {wo} warm-up frames, frame k viewing from 40 + {rad}k rad (every "
                              "frame a distinct camera), submitted like the timed steps and timed between "
                              "synchronisations; the last frames of two contexts compared with a lone trace"}
    if not ev:
        kernel_ms = kernel_ms_isolated

    scene_tag = f"vox:{os.path.basename(args.vox)}" if args.vox else f"S{args.scene}"
    workload = f"primary {W}x{H} {scene_tag} {args.size}^3 bd{args.brick_dim} ranks{world}" + (
        f" orbit{args.orbit}" if args.orbit else "") + (
        f" prepass{args.depth_prepass}" if args.depth_prepass is not None else "") + (
        f" mip-lod{args.mip_lod}" if args.mip_lod is not None else "")
    total_rays = W * H
    n_shadow = 0
    if args.shadows:
        workload += " +shadows"
        n_shadow = int((outs[0]["value"] != -1).sum().item())  # shadow rays this rank traced per frame
        if world > 1:
            ts = torch.tensor([n_shadow], dtype=torch.int64)
            if not rehearsal:
                ts = ts.to(dev)
            dist.all_reduce(ts)
            n_shadow = int(ts.item())
        total_rays += n_shadow
    mrays = total_rays * args.steps / elapsed / 1e6
    ms_per_step = elapsed * 1e3 / args.steps

    # ---- multi-GPU per-rank figures (untimed, after the timed region): every rank's trace and transfer device time
    # at the split that was timed, frames one at a time (vhx_mgpu_measure), to test DESIGN.md §7's model ---------------
    if mg is not None:
        tr_ms, tx_ms = mg.measure(cam, frames=4)
        per_rank = [None] * world
        dist.all_gather_object(per_rank, {"rank": rank, "trace_ms": round(tr_ms, 4), "transfer_ms": round(tx_ms, 4),
                                          "rays": int(mg.rays(W, H))})
        if split is not None:
            split["planes"] = args.planes
            split["bytes_into_rank0_per_frame"] = int(mg.frame_bytes(W, H))
            split["per_rank"] = per_rank
            split["per_rank_basis"] = ("vhx_mgpu_measure at the timed split, 4 frames one at a time (median): trace = "
                                       "the rank's tile slots, transfer = rank 0 its receives / ranks >= 1 their send")

    # ---- multi-GPU check (untimed): the gathered, untiled frame equals rank 0 tracing the whole frame alone -------
    mgpu = None
    if world > 1 or mg is not None:
        whole = None
        if rank == 0:
            whole = rt.trace_primary(cam, fields=("rgba", "depth") if mg is not None else ("rgba",))
            got = (fb_rgba if mg is not None else framebuffer).cpu().numpy().view(np.uint32)
            eq = bool(np.array_equal(got, whole["rgba"]))
            fields = ["rgba"]
            if fb_depth is not None:
                eq = eq and bool(np.array_equal(fb_depth.cpu().numpy().view(np.uint32), whole["depth"].view(np.uint32)))
                fields.append("depth")
            nfb = 1
            if fbs_rgba is not None and not args.orbit:  # the other framebuffers of the timed batches
                for k in range(1, len(fbs_rgba)):
                    eq = eq and bool(np.array_equal(fbs_rgba[k].cpu().numpy().view(np.uint32), whole["rgba"]))
                    if fbs_depth is not None:
                        eq = eq and bool(np.array_equal(fbs_depth[k].cpu().numpy().view(np.uint32),
                                                        whole["depth"].view(np.uint32)))
                nfb = len(fbs_rgba)
            mgpu = {"frame_equal": eq, "fields": fields, "pixels": int(W * H), "framebuffers": nfb,
                    "basis": "the gathered, untiled frames of the timed configuration (every framebuffer of a batch) "
                             "vs rank 0 tracing the frame alone"}
        if mg is not None and args.planes == 1:
            # the two-plane transfer too (collective on every rank): RGBA8 + depth gathered and untiled
            mg.set_planes(2)
            fbd2 = torch.zeros(W * H, dtype=torch.float32, device=dev) if rank == 0 else None
            mg.render(cam, fb_rgba, fbd2)
            mg.sync()
            if rank == 0:
                eq2 = bool(np.array_equal(fb_rgba.cpu().numpy().view(np.uint32), whole["rgba"])) and \
                    bool(np.array_equal(fbd2.cpu().numpy().view(np.uint32), whole["depth"].view(np.uint32)))
                mgpu["two_plane_frame_equal"] = eq2
            mg.set_planes(1)

    # ---- roofline: algorithmic bytes of this rank's launch (instrumented kernel, untimed) -------------------------
    roof = None
    shadow_bytes = None
    if not args.no_roofline:
        views = [cam] if len(cams) == 1 else [cams[args.warmup], cams[args.warmup + args.steps // 2], cams[-1]]
        tree_bytes = float(np.mean([rt.trace_primary(v, fields=(), count_bytes=True, **trace_kw)["bytes"]
                                    .astype(np.float64).sum() for v in views]))
        my_rays = W * H if world == 1 else M.rank_rays(W, H, T, rank, world)
        out_bytes = 8.0 * my_rays  # rgba8 + f32 depth per ray
        launch_bytes = tree_bytes + out_bytes
        if args.shadows:
            # config 5: the primary pass also writes the hit records the shadow rays start from (value, impact, normal:
            # 28 B per ray); each shadow ray reads its record (28 B), walks the tree (its counted bytes), writes its flag
            # (4 B) and darkens the pixel (rgba read + write, 8 B); the hit compaction reads every value (4 B per ray)
            sv = []
            for v in views:
                o = {"rgba": out["rgba"], "depth": out["depth"], "value": out["value"], "impact": out["impact"],
                     "normal": out["normal"]}
                rt.trace_primary(v, out=o, **trace_kw)
                sv.append(rt.trace_shadows(light, o, shadowed=out["shadowed"], count_bytes=True)["bytes"]
                          .to(torch.float64).sum().item())
            n_sh = int((out["value"] != -1).sum().item())
            shadow_bytes = float(np.mean(sv))
            launch_bytes += shadow_bytes + 28.0 * my_rays + 4.0 * my_rays + (28.0 + 4.0 + 8.0) * n_sh
        # chip-level: a launch's bytes per frame period (F frames in flight overlap: each launch's own duration
        # includes the time it shares the GPU with its neighbours)
        period_ms = ms_per_step if world == 1 else (kernel_ms_isolated or kernel_ms)
        achieved = launch_bytes / (period_ms * 1e-3) / 1e9
        tr = pmc_traffic(workload)
        measured = None
        if world == 1 and rank == 0 and not args.no_pmc and mg is None:
            # the timed frames run the frames-in-flight schedule whenever F > 1 and the schedule is adaptive
            measured = measure_traffic(busy_only=F > 1 and budgets is None and not K, tune=args.tune,
                                       blocks_per_frame=((W + 15) // 16) * ((H + 15) // 16))
        roof = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 5),
                "basis": ("algorithmic bytes of one frame's launch / the frame period (wall time per frame with "
                          + (f"batches of {K} frames on {F} contexts in flight)" if K else f"{F} frames in flight)"))
                         if world == 1 else
                         "algorithmic bytes of rank 0's launch / its isolated launch duration",
                "achieved_per_launch": round(launch_bytes / (kernel_ms * 1e-3) / 1e9, 2),
                "achieved_isolated_launch": None if not kernel_ms_isolated else
                round(launch_bytes / (kernel_ms_isolated * 1e-3) / 1e9, 2),
                "traffic": measured["bytes"] if measured else (None if tr is None else tr["read_bytes_per_launch"]),
                "traffic_source": (f"measured in this run: rocprofv3 --pmc FETCH_SIZE child run of this workload "
                                   f"(x1024 B, x2 gfx950), frame kernels / frames ({measured['frames']})"
                                   + ("; every child frame on the timed frames' schedule (frames in flight)"
                                      if F > 1 and budgets is None else "")) if measured else
                                  (None if tr is None else tr["source"] + " (committed profile)"),
                "traffic_committed": None if tr is None else tr["read_bytes_per_launch"],
                "kernel": "vhx_trace_primary launch = k_trace_primary (pass 0, step budget) + k_trace_queue "
                          "(the rays over budget, resumed from their saved state), timed together with HIP events "
                          "on the trace stream" + (" (N>1: rank 0's tile set; the gather runs on the communication "
                                                   "stream)" if world > 1 else ""),
                "kernel_ms": round(kernel_ms, 4),
                "kernel_ms_isolated": None if kernel_ms_isolated is None else round(kernel_ms_isolated, 4),
                "frames_in_flight": F,
                "algorithmic_bytes_per_launch": launch_bytes, "tree_bytes_per_ray": round(tree_bytes / max(1, my_rays), 2)}
        if args.shadows:
            roof["shadow_tree_bytes_per_shadow_ray"] = round(shadow_bytes / max(1, n_sh), 2)
            roof["kernel"] = ("primary frame with its hard-shadow rays fused into the same passes (vhx_set_shadow_light: "
                              "a lane goes on with its hit's shadow ray; leftovers ride the queue passes)" if fused else
                              "primary frame (vhx_trace_primary) + its hard-shadow rays (vhx_trace_shadows: hit "
                              "compaction, then the shadow queue passes), timed together on the trace stream")
        iss = None
        if measured and measured["valu"] > 0:
            iss = {"valu_wave_instructions_per_frame": measured["valu"], "useful_lane_frac": round(measured["useful"], 4),
                   "active_lanes_per_valu": measured["lanes"], "peak_valu_wave_instructions_per_s": 1024 * 2.4e9 / 2,
                   "source": "measured in this run: rocprofv3 --pmc SQ_INSTS_VALU, SQ_THREAD_CYCLES_VALU / "
                             f"SQ_ACTIVE_INST_VALU (same child run), frame kernels / frames ({measured['frames']})"
                             + ("; every child frame on the timed frames' schedule (frames in flight)"
                                if F > 1 and budgets is None else "")}
        elif tr is not None and "issue" in tr:
            iss = dict(tr["issue"], source=tr["issue"]["source"] + " (committed profile)")
        if iss is not None:
            # issue side (the traversal is bound by SIMD issue and divergence, not bytes): VALU wave-instructions of
            # a frame per frame period against 1024 SIMDs x 2.4 GHz / 2 cycles, and the share of those slots' lanes
            # doing useful work
            valu_rate = iss["valu_wave_instructions_per_frame"] / (period_ms * 1e-3) / 1e9
            peak_rate = iss["peak_valu_wave_instructions_per_s"] / 1e9
            roof["issue"] = {"bound": "valu issue", "achieved": round(valu_rate, 1), "peak": round(peak_rate, 1),
                             "unit": "G wave64 VALU instr/s", "frac": round(valu_rate / peak_rate, 4),
                             "useful_lane_frac": iss["useful_lane_frac"],
                             "useful_lane_ops_frac": round(valu_rate / peak_rate * iss["useful_lane_frac"], 4),
                             "active_lanes_per_valu": iss["active_lanes_per_valu"],
                             "valu_wave_instructions_per_frame": iss["valu_wave_instructions_per_frame"],
                             "source": iss["source"]}

    # ---- CPU baseline: the oracle (reference semantics) on the host cores, rank 0 at N=1 only ----------------------
    cpu = None
    if world == 1 and rank == 0 and not args.no_cpu_baseline:
        cores, affinity, quota = cpu_cores()
        t_all, t_one, (w1, h1), r_all, r_one = cpu_baseline(flat, cam, W, H, cores, light if args.shadows else None)
        cpu = {"value": round(r_all / t_all / 1e6, 4), "unit": "Mrays/s", "cores": cores, "kind": "port",
               "value_1core": round(r_one / t_one / 1e6, 4),
               "nproc": os.cpu_count(), "affinity_cpus": affinity, "cgroup_cpu_quota": quota,
               "cpu_model": cpu_model(),
               "sample": f"all {cores} cores: 1 warm-up + median of 5 full {W}x{H} frames ({t_all:.2f} s per frame); "
                         f"1 core: 1 warm-up + median of 5 {w1}x{h1} frames of the same view ({t_one:.2f} s each); "
                         f"same tree and camera, OpenMP dynamic over pixels"
                         + (f"; each frame = primary rays + the oracle's shadow pass over its hits ({r_all} rays in the "
                            f"full frame)" if args.shadows else "")}

    scal = None
    if (world == 1 and mg is None and not args.no_extra and not args.shadows and not args.vox and not args.orbit
            and args.mip_lod is None and args.depth_prepass is None and args.scaling == "auto" and not args.width):
        scal = scaling_n1(args)

    if rank == 0:
        metric = BASELINE["metric"]
        if args.shadows:
            metric = "primary + hard-shadow Mrays/s (BASELINE config 5)"
        if world > 1 or mg is not None:
            par = f"screen-tile split x{world} + " + (
                "gloo gather (single-GPU rehearsal)" if rehearsal else
                ("RCCL point-to-point transfers of RGBA8 + depth to rank 0 behind the C ABI (vhx_mgpu), tree "
                 "ncclBroadcast from rank 0"
                 if mg is not None else "RCCL gather via torch.distributed")
                + ("" if args.no_overlap else ", overlapped with the next frame's trace"))
        else:
            par = "single GPU"
        cfg4 = (W, H) == CONFIG4
        line = {
            "metric": metric, "value": round(mrays, 3), "unit": "Mrays/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True, "scaling": scaling, "vs_baseline": None, "dtype": "f32",
            "frames_in_flight": F * max(1, K), "contexts_in_flight": F, "batch": K or None,
            "gpu_max_hw_queues": queues,
            "host_submit_ms_per_step": round(submit_s * 1e3 / args.steps, 4),
            "pass_budgets": args.budgets if args.budgets is not None else ("one pass" if args.mip_lod is not None
                                                                           else "library default (adaptive)"),
            "schedule": None if sched_timed is None else {
                "timed_frames": {"budgets": list(sched_timed[0]), "choice": sched_timed[1]},
                "isolated_frames": None if sched_iso is None else {"budgets": list(sched_iso[0]),
                                                                   "choice": sched_iso[1]}},
            "data": "model file" if args.vox else "synthetic",
            "config": {"workload": ("BASELINE config 4: " if cfg4 else "") + f"primary rays {W}x{H}, {args.size}^3 "
                                   + (f".vox model {os.path.basename(args.vox)}" if args.vox
                                      else "procedural scene S (lattice+cube)")
                                   + f", brick_dim {args.brick_dim}, glass camera"
                                   + (f" orbiting {args.orbit} rad per frame" if args.orbit else "")
                                   + (f", APPROXIMATE depth-prepass mode (margin {args.depth_prepass}; not the "
                                      "reference semantics)" if args.depth_prepass is not None else "")
                                   + (f", MIP stand-in mode: the view holds nodes down to depth {args.mip_lod}, node "
                                      "MIPs below (not the reference CPU semantics)" if args.mip_lod is not None else "")
                                   + (f", {T}x{T} tiles round-robin over {world} ranks" if world > 1 else ""),
                       "workload_key": workload,
                       "shadow_rays_per_frame": n_shadow if args.shadows else None,
                       "shadow_mode": args.shadow_mode if args.shadows else None,
                       "camera_orbit_rad_per_frame": args.orbit, "tree_size": args.size, "brick_dim": args.brick_dim, "width": W, "height": H,
                       "scene": args.scene, "tile": T if world > 1 else None, "parallelism": par,
                       **{k: v for k, v in tree_info.items() if k != "size"}, "build_s": round(build_s, 2), "upload_s": round(upload_s, 2)},
            "roofline": roof, "cpu_baseline": cpu,
        }
        if frames_check is not None:
            line.update(frames_equal=frames_check["frames_equal"], golden_match=frames_check["golden_match"],
                        frames_check=frames_check)
        if lone is not None:
            line["lone"] = lone
        if orbit is not None:
            line["orbit"] = orbit
        if scal is not None:
            line["scaling_n1"] = scal
        if world > 1 and cfg4:
            line["scaling_basis"] = ("strong scaling of BASELINE config 4 (7680x4320); its N = 1 point is the "
                                     "`scaling_n1` object of the N = 1 line (same workload, same rank code)")
        if args.tune:
            line["tune"] = args.tune
        if mgpu is not None:
            line["multi_gpu_check"] = mgpu
        if mgpu_fallback:
            line["mgpu_fallback"] = mgpu_fallback
        if split is not None:
            line["mgpu_split"] = split
        if cpu:
            line["gpu_over_cpu"] = round(mrays / cpu["value"], 2)
        print(json.dumps(line), flush=True)
    if mg is not None:
        mg.close()
    if dist.is_initialized():
        dist.destroy_process_group()
    for r in rts[1:]:
        r.close()
    rt.close()


if __name__ == "__main__":
    main()
