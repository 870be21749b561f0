#!/bin/bash
# Round 5: as gpu_r05f.sh, after pre-sizing the list buffers at a context's first (idle-schedule) frame
# then the bench frame with 20 contexts and with batches, A/B in one box, two rounds.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05h; mkdir -p $O
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_abi_c.py tests/test_gpu_batch.py tests/test_gpu_inflight.py -m gpu > $O/gpu_first.log 2>&1 || { echo "first tests failed"; tail -30 $O/gpu_first.log; exit 1; }
tail -1 $O/gpu_first.log
summ() {
  python - "$1" "$2" <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(l)
lone = d.get("lone") or {}
print(f"{sys.argv[2]:44s} {d['ms_per_step']:.4f} ms/frame {d['value']:.0f} Mrays/s frames_equal {d.get('frames_equal')} golden {d.get('golden_match')} lone {lone.get('ms')}")
PY
}
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pmc --no-extra"
for round in 1 2; do
  for cfg in "" "--batch 20 --inflight 1" "--batch 7 --inflight 3"; do
    for tune in "p0lists=0" "p0lists=1"; do
      f=$O/bench_r${round}_$(echo "$cfg $tune" | tr -c 'a-zA-Z0-9\n' '_').log
      timeout -k 10 200 $B $cfg --tune "$tune" > $f 2>&1 || { echo "bench failed: $cfg $tune"; tail -20 $f; exit 1; }
      summ $f "${cfg:-20 contexts} $tune r$round"
    done
  done
done
