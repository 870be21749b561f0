"""Frame timing from a rocprofv3 kernel trace of bench.py (gpu_profile.sh ks_kernel_trace.csv): for the timed frames
(the pass-0 dispatches after the setup and warm-up ones), the span from the first timed pass-0 start to the last
frame-kernel end divided by the frame count (the frame period, to compare with bench's ms_per_step), and the mean
per-frame sum of kernel durations by kernel (with frames in flight the kernels of different frames overlap, so these
sums exceed the period), and per kernel class the BUSY time: the union of its dispatches' [start, end) intervals
over the timed span (the time at least one dispatch of that class ran), per frame and as a fraction of the span, so that
overlapping frames are not double counted; "any frame kernel" is the union over all classes.
usage: trace_frames.py KERNEL_TRACE_CSV SKIP STEPS [FRAME_BLOCKS]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
skip, steps = int(sys.argv[2]), int(sys.argv[3])
frame_k = ("k_trace_primary<false", "k_trace_primary_batch<", "k_trace_queue<false", "k_count_flags", "k_scan_counts",
           "k_emit_flags", "k_gather_chunks", "k_put_queue_args", "k_scan_sums")
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].replace("void ", ""),
             int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0)) for r in rows)
# pass-0 dispatches with the frames each opens: 1, or a batch's K (grid / (256 x FRAME_BLOCKS), FRAME_BLOCKS = 32400
# for 3840x2160, rounded: the list order pads a frame to whole tiles); SKIP and STEPS count frames
fb = int(sys.argv[4]) if len(sys.argv) > 4 else 32400
p0 = [(k[0], max(1, round(k[3] / (256 * fb))) if "batch" in k[2] else 1) for k in ks
      if k[2].startswith(("k_trace_primary<false", "k_trace_primary_batch<"))]
cum, t0, t_last_start = 0, None, None
for start, w in p0:
    if t0 is None and cum >= skip:
        t0 = start
    if cum >= skip + steps:
        t_last_start = start
        break
    cum += w
ks = [k[:3] for k in ks]
sel = [k for k in ks if k[2].startswith(frame_k) and k[0] >= t0 and (t_last_start is None or k[0] < t_last_start)]
end = max(k[1] for k in sel)
print(f"timed frames {steps}: span {(end - t0) / 1e6:.4f} ms, period {(end - t0) / 1e6 / steps:.4f} ms/frame")
dur = defaultdict(float)
for s, e, n in sel:
    dur[n.split("(")[0]] += (e - s) / 1e6
for n, v in sorted(dur.items(), key=lambda x: -x[1]):
    print(f"  {n:32s} {v / steps:.4f} ms per frame (summed over its dispatches)")


def union(iv):
    tot, cs, ce = 0, None, None
    for a, b in sorted(iv):
        if cs is None or a > ce:
            if cs is not None:
                tot += ce - cs
            cs, ce = a, b
        else:
            ce = max(ce, b)
    return tot + (ce - cs if cs is not None else 0)


span = end - t0
classes = defaultdict(list)
for s_, e_, n in sel:
    k = n.split("(")[0]
    classes["trace (pass 0 + queue passes)" if "trace" in k else "compaction (count/scan/emit/gather/args/sums)"].append((s_, e_))
    classes[k].append((s_, e_))
classes["any frame kernel"] = [(s_, e_) for s_, e_, _ in sel]
print("busy time (union of dispatch intervals) per frame:")
for n, iv in sorted(classes.items(), key=lambda x: -union(x[1])):
    u = union(iv)
    print(f"  {n:40s} {u / 1e6 / steps:.4f} ms per frame, {u / span:6.1%} of the span")
