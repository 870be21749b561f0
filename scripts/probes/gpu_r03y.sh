#!/bin/bash
# Tail split with booking (a tracing wave hands rays over only to a waiting wave it booked): sweep, lone bench frame.
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/${1:-r03y}; mkdir -p $D
P="timeout -k 10 120 python -u scripts/probes/probe_isolated_r03.py adaptive"
VHX_SPLIT=0 $P >> $D/y.log 2>&1 || { tail -20 $D/y.log; exit 1; }
tail -1 $D/y.log
for w in 32 256; do
  for t in 32,2,1,32 128,2,1,32 32,2,1,64 128,8,1,32 16,2,1,32; do
    VHX_SPLIT=1 VHX_SPLIT_WAIT=$w VHX_SPLIT_TUNE=$t $P >> $D/y.log 2>&1 || { tail -20 $D/y.log; exit 1; }
    tail -1 $D/y.log
  done
done
VHX_SPLIT=1 VHX_SPLIT_WAIT=32 VHX_SPLIT_TUNE=32,2,1,32 VHX_SPLIT_DIAG=2 VHX_DEBUG_PASSES=1 $P > $D/diag.log 2>&1 || { tail -20 $D/diag.log; exit 1; }
grep "split slots" $D/diag.log | tail -1
VHX_SPLIT=0 $P >> $D/y.log 2>&1 || { tail -20 $D/y.log; exit 1; }
tail -1 $D/y.log
