#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/${1:-r03m}; mkdir -p $D
scripts/probes/probe_lone_order_r03.sh > $D/lone_order.log 2>&1 || { tail -20 $D/lone_order.log; exit 1; }
grep -v amdgpu.ids $D/lone_order.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $D/bench.log 2>&1 || { tail -20 $D/bench.log; exit 1; }
tail -1 $D/bench.log | cut -c1-300
