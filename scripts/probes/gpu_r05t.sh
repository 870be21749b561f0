#!/bin/bash
# Round 5: the lone frame's tail pass with chunks strided over the queue (tstride=1: a wave's rays come from all over
# the frame, so the few longest rays land in different waves), with and without the node sort; the batch tests first.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05t; mkdir -p $O
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_batch.py -m gpu > $O/pytest_batch.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest_batch.log; exit 1; }
tail -1 $O/pytest_batch.log
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pmc"
for round in 1 2; do
  for tune in "" "tstride=1" "tstride=1;qsort=0" "qsort=0"; do
    f=$O/r${round}_$(echo "x$tune" | tr -c 'a-zA-Z0-9\n' '_').log
    timeout -k 10 200 $B ${tune:+--tune "$tune"} > $f 2>&1 || { echo "bench failed: $tune"; tail -20 $f; exit 1; }
    python - "$f" "${tune:-default} r$round" <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(l)
lone = d.get("lone") or {}
orb = d.get("orbit") or {}
print(f"{sys.argv[2]:28s} {d['ms_per_step']:.4f} ms/frame frames_equal {d.get('frames_equal')} golden {d.get('golden_match')} lone {lone.get('ms')} orbit {orb.get('ms_per_frame')}")
PY
  done
done
