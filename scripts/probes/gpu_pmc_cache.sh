#!/bin/bash
# Cache hit rates of the trace kernels on the bench frame: L2 (TCC) hits/misses and vector-L1 (TCP) accesses vs the
# requests it forwards to L2. One PMC pass (4 TCC + 2 TCP counters) beside --kernel-trace only.
cd "$GRAFT_REPO_ROOT" || exit 1
R="$GRAFT_REPO_ROOT"; D="$R/gpurun_out/pmc_cache"; mkdir -p "$D"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum --kernel-trace -f csv -d "$D" -o c -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-roofline > "$D/c.log" 2>&1; rc=$?
echo "pmc rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$D/c.log"; exit $rc; }
cd "$R" && python3 - "$D/c_counter_collection.csv" <<'PY'
import csv, collections, sys
agg = collections.defaultdict(float); last = {}
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].split("(")[0].replace("void ", "")
    if "trace" not in k: continue
    agg[(k, r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    last[k] = max(last.get(k, 0), int(r["Dispatch_Id"]))
for k in last:
    c = {cn: v for (kk, d, cn), v in agg.items() if kk == k and int(d) == last[k]}
    hit, miss, req = c.get("TCC_HIT_sum", 0), c.get("TCC_MISS_sum", 0), c.get("TCC_REQ_sum", 0)
    tcp, tcp2 = c.get("TCP_TOTAL_CACHE_ACCESSES_sum", 0), c.get("TCP_TCC_READ_REQ_sum", 0)
    print(k, {n: int(v) for n, v in c.items()}, f"L2 hit {hit / max(1, hit + miss):.3f}", f"L1 hit {1 - tcp2 / max(1, tcp):.3f}")
PY
