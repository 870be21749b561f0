#!/bin/bash
# Tail split diagnostics: failed slot polls and waiter polls per lone frame (VHX_SPLIT_DIAG bit 1, pass-by-pass debug
# output), slot polls by atomic load against atomic read-modify-write (bit 0), timed against the split off.
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/${1:-r03u}; mkdir -p $D
P="timeout -k 10 120 python -u scripts/probes/probe_isolated_r03.py adaptive"
for dg in 2 3; do
  VHX_SPLIT_TUNE=64,8,16,64 VHX_SPLIT_DIAG=$dg VHX_DEBUG_PASSES=1 $P > $D/diag$dg.log 2>&1 || { tail -20 $D/diag$dg.log; exit 1; }
  echo "diag $dg:"; grep "split slots" $D/diag$dg.log | tail -2; grep isolated $D/diag$dg.log
done
for rep in 1 2; do
  VHX_SPLIT=0 $P >> $D/time.log 2>&1 || { tail -20 $D/time.log; exit 1; }
  for dg in 0 1; do
    VHX_SPLIT_TUNE=64,8,16,64 VHX_SPLIT_DIAG=$dg $P >> $D/time.log 2>&1 || { tail -20 $D/time.log; exit 1; }
    VHX_SPLIT_DIAG=$dg $P >> $D/time.log 2>&1 || { tail -20 $D/time.log; exit 1; }
  done
done
grep isolated $D/time.log
