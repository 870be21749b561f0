#!/bin/bash
# Round 5: sparse-wave abandonment in the budgeted queue passes (pass 1 runs 18.8 lanes per VALU instruction)
# in the batch default; two rounds, one box.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05m; mkdir -p $O
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pmc --no-extra"
for round in 1 2; do
  for v in "|" "|sparse=12,8" "|sparse=12,16" "|sparse=12,16,16,16" "|sparse=12,24,24,24" "|sparse=12,8,8,8" "|sparse=12,32"; do
    cfg=${v%%|*}; tune=${v#*|}
    f=$O/r${round}_$(echo "x$cfg$tune" | tr -c 'a-zA-Z0-9\n' '_').log
    timeout -k 10 200 $B $cfg ${tune:+--tune "$tune"} > $f 2>&1 || { echo "bench failed: $v"; tail -20 $f; exit 1; }
    python - "$f" "${cfg:-batch 7x3} ${tune:-default} r$round" <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(l)
print(f"{sys.argv[2]:48s} {d['ms_per_step']:.4f} ms/frame {d['value']:.0f} Mrays/s frames_equal {d.get('frames_equal')} golden {d.get('golden_match')}")
PY
  done
done
