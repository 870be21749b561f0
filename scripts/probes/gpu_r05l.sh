#!/bin/bash
# Round 5: XCD-dealt chunks for every queue pass in the batch default (pass 1 waits on memory 67 % of its cycles
# there, prof_r05_final): qxcd_all / run length; two rounds, one box.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05l; mkdir -p $O
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pmc --no-extra"
for round in 1 2; do
  for v in "|" "|qxcd_all=1" "|qxcd_all=1;qxcd=4" "|qxcd_all=1;qxcd=64" "|qxcd=0" "--batch 0|" "--batch 0|qxcd_all=1"; do
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
