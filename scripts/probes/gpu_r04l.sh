#!/bin/bash
# Round 4: the one-launch frame (k_trace_frame) -- its GPU tests, then lone-frame latency per spec (probe_ahead.py).
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/${1:-r04l}; mkdir -p $D
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_frame1.py > $D/pytest.log 2>&1 \
  || { tail -40 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
timeout -k 10 300 python -u scripts/probes/probe_ahead.py "one=0" "one=1" "one=1;budgets=24,72,216,648" "one=1;budgets=32,128,512" \
  "one=1;budgets=24,96,768" "one=1;budgets=48,192,768" > $D/one.log 2>&1 || { tail -20 $D/one.log; exit 1; }
cat $D/one.log
