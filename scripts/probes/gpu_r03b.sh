#!/bin/bash
# GPU check after the schedule change: -m gpu suite, ladder sweep, default and round-2-schedule bench lines.
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/${1:-r03b}; mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $D/gpu_all.log 2>&1 || { tail -30 $D/gpu_all.log; exit 1; }
tail -1 $D/gpu_all.log
scripts/probes/probe_ladder_r03.sh > $D/ladder.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $D/bench_new1.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --budgets 24,96,768 > $D/bench_old.log 2>&1 || exit 1
