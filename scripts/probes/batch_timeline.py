"""Timeline of a frame batch (vhx_trace_primary_batch) from a rocprofv3 kernel trace: per batch (one
k_trace_primary_batch dispatch and the dispatches on its queue up to the next one), every kernel with its start offset
and duration, and the idle time between consecutive dispatches (the GPU runs nothing of the batch then: with one
context in flight, nothing at all). Prints one batch in full and the mean per kernel over the batches after --skip.
usage: batch_timeline.py ks_kernel_trace.csv|ks_results.db [--skip N] [--show I]   (.db: rocprofv3's default rocpd
output, its `kernels` view)"""
import csv
import sys
from collections import defaultdict

if sys.argv[1].endswith(".db"):
    import sqlite3
    con = sqlite3.connect(sys.argv[1])
    rows = [{"Kernel_Name": n, "Start_Timestamp": a, "End_Timestamp": b, "Queue_Id": str(q)}
            for n, a, b, q in con.execute("select name, start, end, queue_id from kernels")]
else:
    rows = list(csv.DictReader(open(sys.argv[1])))
skip = int(sys.argv[sys.argv.index("--skip") + 1]) if "--skip" in sys.argv else 2
show = int(sys.argv[sys.argv.index("--show") + 1]) if "--show" in sys.argv else skip
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].removeprefix("void ").split("(")[0],
             r["Queue_Id"]) for r in rows)
starts = [i for i, k in enumerate(ks) if k[2].startswith("k_trace_primary_batch")]
batches = []
for j, i in enumerate(starts):
    q = ks[i][3]
    end = starts[j + 1] if j + 1 < len(starts) else len(ks)
    batches.append([k for k in ks[i:end] if k[3] == q and k[2].startswith("k_")])
tot, gaps, spans = defaultdict(float), [], []
for b, ds in enumerate(batches):
    t0 = ds[0][0]
    if b == show:
        print(f"batch {b}: {len(ds)} dispatches")
        prev = t0
        for s, e, n, _ in ds:
            print(f"  +{(s - t0) / 1e6:8.4f} ms  {((e - s) / 1e6):8.4f} ms  gap {((s - prev) / 1e6):7.4f}  {n}")
            prev = e
    if b < skip or b == len(batches) - 1:
        continue
    spans.append((ds[-1][1] - t0) / 1e6)
    g = 0.0
    prev = t0
    for s, e, n, _ in ds:
        tot[n] += (e - s) / 1e6
        g += max(0, s - prev) / 1e6
        prev = max(prev, e)
    gaps.append(g)
nb = len(spans)
if nb:
    print(f"batches {nb}: span {sum(spans) / nb:.4f} ms, idle between dispatches {sum(gaps) / nb:.4f} ms")
    for n, v in sorted(tot.items(), key=lambda x: -x[1]):
        print(f"  {n:36s} {v / nb:.4f} ms per batch")
