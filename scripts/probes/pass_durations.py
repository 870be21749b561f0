"""Mean dispatch duration of every pass of a frame from a rocprofv3 kernel trace (ks_kernel_trace.csv of
scripts/gpu_profile.sh): per stream, dispatches in order; a k_trace_primary* dispatch starts a primary frame, a
k_count_flags<true> starts its shadow trace; the k_trace_queue dispatches after either are its passes 1.. (primary) or
0.. (shadow). Frames in flight overlap, so a duration includes the time a pass shares the GPU with other frames.
usage: pass_durations.py ks_kernel_trace.csv [--skip N]   (N = first frames per stream skipped)"""
import csv
import sys
from collections import defaultdict

path = sys.argv[1]
skip = int(sys.argv[sys.argv.index("--skip") + 1]) if "--skip" in sys.argv else 1
rows = list(csv.DictReader(open(path)))
by_stream = defaultdict(list)
for r in rows:
    by_stream[(r["Queue_Id"], r["Stream_Id"])].append(r)
acc = defaultdict(list)
for key, rs in by_stream.items():
    rs.sort(key=lambda r: int(r["Start_Timestamp"]))
    frame, mode, p = -1, None, 0
    for r in rs:
        n = r["Kernel_Name"].removeprefix("void ")
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
        if n.startswith("k_trace_primary"):
            frame, mode, p = frame + 1, "primary", 1
            if frame >= skip:
                acc[("primary", 0)].append(d)
        elif n.startswith("k_count_flags<true>"):
            mode, p = "shadow", 0
        elif n.startswith("k_trace_queue") and mode and frame >= skip:
            acc[(mode, p)].append(d)
            p += 1
        elif n.startswith("k_trace_queue"):
            p += 1
for (mode, p), ds in sorted(acc.items()):
    print(f"{mode:8s} pass {p}: {len(ds):4d} dispatches, mean {sum(ds) / len(ds):.4f} ms, max {max(ds):.4f} ms")
