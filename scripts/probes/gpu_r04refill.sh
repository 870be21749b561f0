#!/bin/bash
# Round 4: lane refill of the lone frame's unbounded pass (k_trace_refill): its GPU tests, then the lone frame per
# refill threshold (scripts/probes/probe_lone.py).
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/${1:-r04refill}; mkdir -p $D
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_refill.py > $D/pytest.log 2>&1 \
  || { tail -40 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
REPS=3 timeout -k 10 400 python -u scripts/probes/probe_lone.py "" "refill=8" "refill=16" "refill=32" "refill=48" "refill=64" \
  "refill=32;qsort=0" "refill=32;qwaves=1024" "refill=32;qwaves=4096" > $D/lone.log 2>&1 || { tail -20 $D/lone.log; exit 1; }
cat $D/lone.log
