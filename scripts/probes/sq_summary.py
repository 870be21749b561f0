"""Summarises SQ counter CSVs (rocprofv3 --pmc) per kernel name: the last dispatch of each kernel, counters of all
passes merged. usage: sq_summary.py DIR PREFIX"""
import collections, csv, glob, sys
d, pre = sys.argv[1], sys.argv[2]
res = collections.defaultdict(dict)
for f in sorted(glob.glob(f"{d}/{pre}_p*_counter_collection.csv")):
    rows = list(csv.DictReader(open(f)))
    agg = collections.defaultdict(float)
    last = {}
    for r in rows:
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if "trace" not in k:
            continue
        agg[(k, r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        last[k] = max(last.get(k, 0), int(r["Dispatch_Id"]))
    for (k, did, c), v in agg.items():
        if int(did) == last[k]:
            res[k][c] = v
for k, cs in res.items():
    print(k)
    for c in sorted(cs):
        print(f"   {c:24s} {cs[c]:16.0f}")
