#!/bin/bash
# Round 4: fill and drain of the driver's 20-frame window, and stream priorities (scripts/probes/probe_batch.py).
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/${1:-r04t}; mkdir -p $D
for round in 1 2; do
  for m in own low hi10 hi15 hi5; do
    timeout -k 10 120 python -u scripts/probes/probe_batch.py $m >> $D/batch.log 2>&1 || { tail -20 $D/batch.log; exit 1; }
  done
done
grep -v amdgpu.ids $D/batch.log
