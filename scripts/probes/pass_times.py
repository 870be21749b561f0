"""Per-kernel durations of the last traced frame in a rocprofv3 kernel trace (multi-pass schedule diagnostics)."""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# frames start with a pass-0 kernel (k_trace_primary); print the last frame's kernels
starts = [i for i, r in enumerate(rows) if "k_trace_primary" in r["Kernel_Name"]]
last = rows[starts[-1]:]
t0 = int(last[0]["Start_Timestamp"])
for r in last:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(")[0].replace("void ", "")
    print(f"  {name:32s} start {(s - t0) / 1e3:8.1f} us  dur {(e - s) / 1e3:8.1f} us")
print(f"  frame {(int(last[-1]['End_Timestamp']) - t0) / 1e3:.1f} us")
