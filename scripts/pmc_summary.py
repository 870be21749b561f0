"""Summarises rocprofv3 counter_collection CSVs of the primary-ray kernel (mean per dispatch)."""
import csv
import glob
import os
import sys
from collections import defaultdict


def summary(d, kernel_sub="k_trace_p"):
    vals = defaultdict(list)
    for f in sorted(glob.glob(os.path.join(d, "p*_counter_collection.csv"))):
        per = defaultdict(float)
        for row in csv.DictReader(open(f)):
            if kernel_sub not in row["Kernel_Name"] or "true" in row["Kernel_Name"]:
                continue
            per[(row["Dispatch_Id"], row["Counter_Name"])] += float(row["Counter_Value"])
        for (disp, name), v in per.items():
            vals[name].append(v)
    return {k: sum(v) / len(v) for k, v in vals.items()}


if __name__ == "__main__":
    for d in sys.argv[1:]:
        s = summary(d)
        print(d)
        for k in sorted(s):
            print(f"  {k:32s} {s[k]:.4g}")
        if "SQ_WAVE_CYCLES" in s:
            wc = s["SQ_WAVE_CYCLES"]
            print("  derived: wait_any %.2f wait_inst %.2f active %.2f of wave-cycles" % (
                s["SQ_WAIT_ANY"] / wc, s["SQ_WAIT_INST_ANY"] / wc, s["SQ_ACTIVE_INST_ANY"] / wc))
            print("  avg active threads per VALU inst: %.1f" % (s["SQ_THREAD_CYCLES_VALU"] / s["SQ_ACTIVE_INST_VALU"]))
        if "TCC_HIT_sum" in s:
            print("  L2 hit rate %.3f" % (s["TCC_HIT_sum"] / (s["TCC_HIT_sum"] + s["TCC_MISS_sum"])))
