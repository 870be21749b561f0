#!/bin/bash
# Round 5: (1) the lone frame in the tile order with pass-0 lists (qorder on both schedules) against the idle
# schedule's output order; (2) batch sizes x contexts at the box's 4 hardware queues.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05i; mkdir -p $O
summ() {
  python - "$1" "$2" <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(l)
lone = d.get("lone") or {}
orb = d.get("orbit") or {}
print(f"{sys.argv[2]:36s} {d['ms_per_step']:.4f} ms/frame {d['value']:.0f} Mrays/s frames_equal {d.get('frames_equal')} golden {d.get('golden_match')} lone {lone.get('ms')} orbit {orb.get('ms_per_frame')}")
PY
}
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pmc"
for round in 1 2; do
  for tune in "" "qorder=64z" "qorder=16z"; do
    f=$O/lone_r${round}_$(echo "x$tune" | tr -c 'a-zA-Z0-9\n' '_').log
    timeout -k 10 200 $B ${tune:+--tune "$tune"} > $f 2>&1 || { echo "bench failed: $tune"; tail -20 $f; exit 1; }
    summ $f "20 contexts ${tune:-default} r$round"
  done
done
for round in 1 2; do
  for cfg in "--batch 5 --inflight 4" "--batch 6 --inflight 4" "--batch 7 --inflight 3" "--batch 8 --inflight 3" "--batch 10 --inflight 3" "--batch 5 --inflight 3" "--batch 4 --inflight 5"; do
    f=$O/batch_r${round}_$(echo "$cfg" | tr -c 'a-zA-Z0-9\n' '_').log
    timeout -k 10 200 $B --no-extra $cfg > $f 2>&1 || { echo "bench failed: $cfg"; tail -20 $f; exit 1; }
    summ $f "$cfg r$round"
  done
done
