#!/bin/bash
# Round 5: segmented chunk scans for frame batches (launch_scan). (1) the batch and scheduler-variant tests; (2) bench
# A/B of batches with scan_multi=0 (every scan on one workgroup, the previous code) against the default; (3) a kernel
# trace of one context submitting 20-frame batches.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05d; mkdir -p $O
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_batch.py tests/test_gpu_parity.py -m gpu > $O/pytest_batch.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest_batch.log; exit 1; }
tail -1 $O/pytest_batch.log
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pmc --no-extra"
for round in 1; do
for cfg in "--batch 20 --inflight 1" "--batch 10 --inflight 2" "--batch 7 --inflight 3"; do
  for tune in "scan_multi=0" ""; do
    f=$O/bench_r${round}_$(echo "$cfg $tune" | tr -c 'a-zA-Z0-9\n' '_').log
    timeout -k 10 200 $B $cfg ${tune:+--tune "$tune"} > $f 2>&1 || { echo "bench failed: $cfg $tune"; tail -20 $f; exit 1; }
    python - "$f" "$cfg $tune" <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(l)
print(f"{sys.argv[2]:40s} {d['ms_per_step']:.4f} ms/frame {d['value']:.0f} Mrays/s frames_equal {d.get('frames_equal')} golden {d.get('golden_match')}")
PY
  done
done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_batch20 -o ks -- python bench.py --batch 20 --inflight 1 --steps 10 --warmup 3 --no-cpu-baseline --no-pmc --no-extra --no-frame-check > $O/prof_batch20.log 2>&1; echo "prof rc=$?"
