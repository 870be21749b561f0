#!/bin/bash
# Same-box A/B of source trees (git worktrees of earlier commits with their own built libvhx, e.g. scratch/wt_<sha>):
# the default bench of each tree in TREES ("|"-separated, "." = this tree) with BENCH_ARGS, REPS times in alternation.
# Every GPU step under its own time limit; stops at the first failure. usage: TAG=x TREES="scratch/wt_abc|." gpu_ab_trees.sh
cd "$GRAFT_REPO_ROOT" || exit 1
D="$GRAFT_REPO_ROOT/gpurun_out/${TAG:-abt}"; mkdir -p "$D"
IFS='|' read -ra S <<< "${TREES:-.}"
for rep in $(seq 1 ${REPS:-2}); do
  for k in "${!S[@]}"; do
    tr=${S[$k]}
    (cd "$GRAFT_REPO_ROOT/$tr" && timeout -k 10 300 python3 bench.py --steps ${STEPS:-100} --warmup 10 --no-cpu-baseline --no-extra --no-pmc $BENCH_ARGS) > $D/t${k}_$rep.log 2>&1 || { echo "bench in $tr failed"; tail -5 $D/t${k}_$rep.log; exit 1; }
    python3 - "$D/t${k}_$rep.log" "$tr" <<'PY'
import json, sys
ln = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
d = json.loads(ln)
print(f"{sys.argv[2]:24s} {d['ms_per_step']:.4f} ms/step {d['value']:.0f} Mrays/s frames_equal={d.get('frames_equal')} golden={d.get('golden_match')}")
PY
  done
done
