#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/${1:-r03p}; mkdir -p $D
scripts/probes/probe_knobs_r03.sh > $D/knobs.log 2>&1 || { tail -20 $D/knobs.log; exit 1; }
grep -v amdgpu.ids $D/knobs.log
for F in 8 12 16; do
  timeout -k 10 300 python -u bench.py --inflight $F --no-cpu-baseline --no-pmc --no-frame-check > $D/bench_f$F.log 2>&1 || { tail -20 $D/bench_f$F.log; exit 1; }
  echo "F=$F $(tail -1 $D/bench_f$F.log | cut -c1-190)"
done
