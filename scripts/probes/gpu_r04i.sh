#!/bin/bash
# Round 4: the ahead stream of a lone frame -- its GPU tests, then lone-frame latency per spec (probe_ahead.py).
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/${1:-r04i}; mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ahead.py \
  tests/test_gpu_golden.py > $D/pytest.log 2>&1 || { tail -40 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
timeout -k 10 300 python -u scripts/probes/probe_ahead.py "ahead=0" "ahead=1" "ahead=1;ahead_min=128" "ahead=1;ahead_min=512" \
  "ahead=1;ahead_rpw=4" "ahead=1;ahead_rpw=16" "ahead=1;ahead_prio=0" "ahead=1;ahead_cap=4096" "ahead=1;ahead_cap=1024" > $D/ahead.log 2>&1 || { tail -20 $D/ahead.log; exit 1; }
cat $D/ahead.log
