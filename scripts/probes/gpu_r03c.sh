#!/bin/bash
# Re-entry GPU check of the adaptive schedule: -m gpu suite, default bench (CPU baseline included), lone-frame probe.
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/${1:-r03c}; mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $D/gpu_all.log 2>&1 || { tail -30 $D/gpu_all.log; exit 1; }
tail -1 $D/gpu_all.log
timeout -k 10 300 python -u bench.py > $D/bench_default.log 2>&1 || { tail -20 $D/bench_default.log; exit 1; }
tail -1 $D/bench_default.log | cut -c1-400
timeout -k 10 300 python -u scripts/probes/probe_isolated_r03.py 64 24,72,216,648 "" 48 96 > $D/isolated.log 2>&1 || { tail -20 $D/isolated.log; exit 1; }
cat $D/isolated.log
