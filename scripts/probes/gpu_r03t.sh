#!/bin/bash
# Tail split tuning on the lone bench frame: VHX_SPLIT_TUNE = period,min_lanes,min_idle,take against the split off.
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/${1:-r03t}; mkdir -p $D
P="timeout -k 10 120 python -u scripts/probes/probe_isolated_r03.py adaptive"
VHX_SPLIT=0 $P >> $D/tune.log 2>&1 || { tail -20 $D/tune.log; exit 1; }
for t in 8,2,1,64 64,2,1,64 64,8,1,64 64,8,16,64 256,8,16,32 64,16,64,32 512,16,64,64 64,32,256,32; do
  VHX_SPLIT_TUNE=$t $P >> $D/tune.log 2>&1 || { tail -20 $D/tune.log; exit 1; }
  tail -1 $D/tune.log
done
VHX_SPLIT=0 $P >> $D/tune.log 2>&1 || { tail -20 $D/tune.log; exit 1; }
grep isolated $D/tune.log
