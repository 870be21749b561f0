#!/bin/bash
# Round 5: vhx_trace_shadows_batch -- the batch / list / shadow tests, smoke(), then config 5 with batches of 7 on 3
# contexts (the new default for --shadows) against twenty per-frame contexts, two rounds, one box.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05v; mkdir -p $O
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_batch.py tests/test_gpu_lists.py -m gpu > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pmc --shadows"
for round in 1 2; do
  for cfg in "" "--batch 0"; do
    f=$O/c5_r${round}_$(echo "x$cfg" | tr -c 'a-zA-Z0-9\n' '_').log
    timeout -k 10 300 $B $cfg > $f 2>&1 || { echo "bench failed: $cfg"; tail -20 $f; exit 1; }
    python - "$f" "config 5 ${cfg:-batch 7x3} r$round" <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(l)
print(f"{sys.argv[2]:32s} {d['ms_per_step']:.4f} ms/frame {d['value']:.0f} Mrays/s frames_equal {d.get('frames_equal')} queues {d.get('gpu_max_hw_queues')} frac {(d.get('roofline') or {}).get('frac')}")
PY
  done
done
