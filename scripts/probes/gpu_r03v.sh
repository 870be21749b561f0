#!/bin/bash
# Tail split with a bounded number of waiting waves (VHX_SPLIT_WAIT) x split tuning, lone bench frame, vs split off.
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/${1:-r03v}; mkdir -p $D
P="timeout -k 10 120 python -u scripts/probes/probe_isolated_r03.py adaptive"
VHX_SPLIT=0 $P >> $D/wait.log 2>&1 || { tail -20 $D/wait.log; exit 1; }
for w in 8 32 128; do
  for t in 8,2,1,64 64,8,1,32 64,16,4,32 256,32,1,32; do
    VHX_SPLIT_WAIT=$w VHX_SPLIT_TUNE=$t $P >> $D/wait.log 2>&1 || { tail -20 $D/wait.log; exit 1; }
    tail -1 $D/wait.log
  done
done
VHX_SPLIT_WAIT=32 VHX_SPLIT_TUNE=64,8,1,32 VHX_SPLIT_DIAG=2 VHX_DEBUG_PASSES=1 $P > $D/diag.log 2>&1 || { tail -20 $D/diag.log; exit 1; }
grep "split slots" $D/diag.log | tail -1
VHX_SPLIT=0 $P >> $D/wait.log 2>&1 || { tail -20 $D/wait.log; exit 1; }
tail -1 $D/wait.log
