#!/bin/bash
# Round 5: unequal batches on the 3 contexts (--batch-sizes): do contexts whose pass ladders are out of step (one in
# its issue-bound pass 0 while another is in its memory-bound queue passes) beat three equal batches in lockstep?
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05w; mkdir -p $O
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pmc --no-extra"
for round in 1 2; do
  for v in "" "10,6,4" "9,7,4" "8,7,5" "12,5,3" "6,7,7" "11,9"; do
    f=$O/r${round}_$(echo "x$v" | tr -c 'a-zA-Z0-9\n' '_').log
    timeout -k 10 200 $B ${v:+--batch-sizes $v} > $f 2>&1 || { echo "bench failed: $v"; tail -20 $f; exit 1; }
    python - "$f" "sizes ${v:-7 x 3} r$round" <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(l)
print(f"{sys.argv[2]:24s} {d['ms_per_step']:.4f} ms/frame {d['value']:.0f} Mrays/s frames_equal {d.get('frames_equal')} golden {d.get('golden_match')}")
PY
  done
done
