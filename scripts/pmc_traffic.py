"""Memory-side read traffic per vhx_trace_primary launch from rocprofv3 PMC runs of bench.py.

Recipe (/opt/skills/guides/MI355X_MICROARCH.md, HBM section): FETCH_SIZE (KB) is derived from the L2 memory-side
request counter TCC_EA0_RDREQ and on gfx950 reports half the bytes of a read, so bytes = FETCH_SIZE * 1024 * 2.
Each counter is collected in its own --pmc pass (beside --kernel-trace only). Infinity-Cache hits are counted, so
this is L2-miss traffic, an upper bound of HBM bytes. One launch = the k_trace_primary<false,..> dispatch of a
frame plus the k_trace_queue<false,..> dispatch that follows it.

usage: pmc_traffic.py PMC_DIR WORKLOAD_KEY OUT_JSON
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def per_dispatch(d, counter):
    vals = defaultdict(float)
    names = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row["Counter_Name"] != counter:
                continue
            k = int(row["Dispatch_Id"])
            vals[k] += float(row["Counter_Value"])
            names[k] = row["Kernel_Name"]
    return vals, names


def per_launch(vals, names):
    """Sums pass-0 + queue-pass dispatches of the timed (non-counting) trace kernels into launches."""
    launches, cur = [], None
    for k in sorted(vals):
        n = names[k]
        if "<false" not in n:
            continue
        if n.startswith("void k_trace_primary") or n.startswith("k_trace_primary"):
            if cur is not None:
                launches.append(cur)
            cur = vals[k]
        elif "k_trace_queue" in n and cur is not None:
            cur += vals[k]
    if cur is not None:
        launches.append(cur)
    return launches


def main():
    d, key, out = sys.argv[1], sys.argv[2], sys.argv[3]
    fetch, names = per_dispatch(d, "FETCH_SIZE")
    lf = per_launch(fetch, names)
    rd, names2 = per_dispatch(d, "TCC_EA0_RDREQ_sum")
    lr = per_launch(rd, names2)
    if not lf:
        sys.exit("no FETCH_SIZE samples for the trace kernels")
    lf = sorted(lf)[len(lf) // 2]  # median launch
    entry = {"read_bytes_per_launch": lf * 1024.0 * 2.0, "fetch_size_kb": lf, "gfx950_correction": 2.0,
             "tcc_ea0_rdreq_per_launch": sorted(lr)[len(lr) // 2] if lr else None,
             "source": f"rocprofv3 --pmc FETCH_SIZE (x1024 B, x2 gfx950), median launch; {os.path.basename(d.rstrip('/'))}"}
    try:
        allv = json.load(open(out))
    except (OSError, ValueError):
        allv = {}
    allv[key] = entry
    json.dump(allv, open(out, "w"), indent=1, sort_keys=True)
    print(key, json.dumps(entry))


if __name__ == "__main__":
    main()
