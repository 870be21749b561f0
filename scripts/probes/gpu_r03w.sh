#!/bin/bash
# Tail split after the first-check fix: VHX_SPLIT_WAIT x VHX_SPLIT_TUNE (period,min_lanes,min_idle,take), lone bench
# frame, against the split off (twice).
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/${1:-r03w}; mkdir -p $D
P="timeout -k 10 120 python -u scripts/probes/probe_isolated_r03.py adaptive"
VHX_SPLIT=0 $P >> $D/w.log 2>&1 || { tail -20 $D/w.log; exit 1; }
tail -1 $D/w.log
for w in 32 128 512; do
  for t in 32,2,1,64 128,2,1,64 128,8,1,32 512,8,1,32 128,16,1,64; do
    VHX_SPLIT=1 VHX_SPLIT_WAIT=$w VHX_SPLIT_TUNE=$t $P >> $D/w.log 2>&1 || { tail -20 $D/w.log; exit 1; }
    tail -1 $D/w.log
  done
done
VHX_SPLIT=0 $P >> $D/w.log 2>&1 || { tail -20 $D/w.log; exit 1; }
tail -1 $D/w.log
