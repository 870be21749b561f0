"""Per-pass PMC figures of the bench frame from a gpu_profile.sh directory: every counter of every pmc*_counter_collection
.csv summed per pass of the multi-pass schedule and divided by the frames of that run. A frame's dispatches are told
apart by their hardware queue (each context of the frames in flight submits on its own): on one queue, a
k_trace_primary<false..> dispatch opens a frame (pass 0) and the k_trace_queue<false..> dispatches after it are passes
1, 2, ...
Derived per pass: active lanes per VALU instruction (SQ_THREAD_CYCLES_VALU / SQ_ACTIVE_INST_VALU), VALU and SALU
wave-instructions per frame, the fraction of wave cycles spent issuing / waiting on dependencies / waiting on memory
(SQ_ACTIVE_INST_ANY, SQ_WAIT_INST_ANY, SQ_WAIT_ANY over SQ_WAVE_CYCLES; quad-cycle units cancel) and the memory-side
reads (FETCH_SIZE x 1024 B x 2, the gfx950 correction of scripts/pmc_frame.py).
--inflight-only (round 4): only frames that ran the frames-in-flight schedule (the most passes
seen) and come after the first SKIP frames of the run (--skip SKIP: the setup frames that allocate the contexts and the
warm-up), so that the lone frames of the run (the setup's first frame, the isolated frames after the timed region) do
not mix into the per-pass figures.
--primary-passes P (config 5, bench.py --shadows): a frame's dispatches after its first P are the shadow trace's passes
(vhx_trace_shadows on the same stream); they are labelled "shadow pass p - P".
Batches (bench.py --batch, vhx_trace_primary_batch): a k_trace_primary_batch dispatch opens a group of K frames (K =
its grid / (256 x --frame-blocks, default 32400 = 3840x2160 in 16x16 blocks), rounded: the list order pads a frame to
whole tiles); its passes' sums are divided by the frames of the kept groups, and SKIP counts groups.
usage: pmc_passes.py PROFILE_DIR [OUT_TXT] [--inflight-only] [--skip SKIP] [--primary-passes P] [--frame-blocks B]"""
import csv
import glob
import os
import sys
from collections import defaultdict

args = [a for a in sys.argv[1:] if not a.startswith("--")]
inflight_only = "--inflight-only" in sys.argv
skip = int(sys.argv[sys.argv.index("--skip") + 1]) if "--skip" in sys.argv else 0
if "--skip" in sys.argv:
    args.remove(str(skip))
prim = int(sys.argv[sys.argv.index("--primary-passes") + 1]) if "--primary-passes" in sys.argv else None
if prim is not None:
    args.remove(str(prim))
fblocks = int(sys.argv[sys.argv.index("--frame-blocks") + 1]) if "--frame-blocks" in sys.argv else 32400
if "--frame-blocks" in sys.argv:
    args.remove(str(fblocks))
d = args[0]
sums = defaultdict(lambda: defaultdict(float))  # (run, pass) -> counter -> total
runs = {}  # run -> (counter names, frames)
for path in sorted(glob.glob(os.path.join(d, "pmc*_counter_collection.csv"))):
    run = os.path.basename(path).split("_")[0]
    disp, names = {}, set()
    for r in csv.DictReader(open(path)):  # one row per (dispatch, counter)
        e = disp.setdefault(int(r["Dispatch_Id"]),
                            {"name": r["Kernel_Name"].replace("void ", ""), "queue": r["Queue_Id"], "c": defaultdict(float),
                             "grid": int(r["Grid_Size"])})
        e["c"][r["Counter_Name"]] += float(r["Counter_Value"])
        names.add(r["Counter_Name"])
    # per frame (or batch: a group of K frames, in dispatch order of its pass 0): its dispatches by pass; queue -> group
    frames, weight, open_frame = [], [], {}
    for k in sorted(disp):
        e = disp[k]
        if e["name"].startswith(("k_trace_primary<false", "k_trace_primary_batch<")):
            open_frame[e["queue"]] = len(frames)
            frames.append([e])
            weight.append(max(1, round(e["grid"] / (256 * fblocks))) if "batch" in e["name"] else 1)
        elif e["name"].startswith("k_trace_queue<false") and e["queue"] in open_frame:
            frames[open_frame[e["queue"]]].append(e)
    most = max((len(f) for f in frames), default=0)
    keep = [i for i, f in enumerate(frames) if i >= skip and (not inflight_only or len(f) == most)]
    for i in keep:
        for p, e in enumerate(frames[i]):
            for c, v in e["c"].items():
                sums[(run, p)][c] += v
    runs[run] = (names, sum(weight[i] for i in keep))

passes = sorted({p for (_, p) in sums})


def per_frame(p, c):
    for run, (names, nf) in runs.items():
        if c in names and nf:
            return sums[(run, p)][c] / nf
    return None


lines = [f"per-pass PMC figures per frame, {os.path.basename(os.path.normpath(d))}"
         + (f" (frames-in-flight schedule only, first {skip} frames skipped)" if inflight_only or skip else "")
         + " (frames per pmc run: "
         + ", ".join(f"{run} {nf}" for run, (_, nf) in runs.items()) + ")"]
for p in passes:
    valu, salu = per_frame(p, "SQ_INSTS_VALU"), per_frame(p, "SQ_INSTS_SALU")
    tc, ai = per_frame(p, "SQ_THREAD_CYCLES_VALU"), per_frame(p, "SQ_ACTIVE_INST_VALU")
    wc, waves = per_frame(p, "SQ_WAVE_CYCLES"), per_frame(p, "SQ_WAVES")
    act, wi, wa = per_frame(p, "SQ_ACTIVE_INST_ANY"), per_frame(p, "SQ_WAIT_INST_ANY"), per_frame(p, "SQ_WAIT_ANY")
    fetch = per_frame(p, "FETCH_SIZE")
    hit, miss = per_frame(p, "TCC_HIT_sum"), per_frame(p, "TCC_MISS_sum")
    parts = [f"pass {p}:" if prim is None or p < prim else f"shadow pass {p - prim}:"]
    if waves is not None:
        parts.append(f"waves {waves:.0f}")
    if valu is not None:
        parts.append(f"VALU {valu / 1e6:.1f} M")
    if salu is not None:
        parts.append(f"SALU {salu / 1e6:.1f} M")
    if tc and ai:
        parts.append(f"lanes/VALU {tc / ai:.1f}")
    if wc:
        parts.append(f"issuing {act / wc:.0%}, dependency waits {wi / wc:.0%}, memory waits {wa / wc:.0%} of wave cycles")
    if fetch is not None:
        parts.append(f"reads {fetch * 2048 / 1e6:.1f} MB")
    if hit is not None and miss is not None and hit + miss > 0:
        parts.append(f"L2 hit rate {hit / (hit + miss):.1%} of {(hit + miss) / 1e6:.1f} M requests")
    lines.append("  " + "  ".join(parts))
txt = "\n".join(lines)
print(txt)
if len(args) > 1:
    open(args[1], "w").write(txt + "\n")
