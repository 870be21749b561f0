#!/bin/bash
# Tail split diagnostics: ray iterations and wave iterations of the split pass with and without hand-offs.
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/${1:-r03x}; mkdir -p $D
P="timeout -k 10 120 python -u scripts/probes/probe_isolated_r03.py adaptive"
for t in 4096,2,1,64 128,2,1,64 32,2,1,64 128,2,1,8; do
  VHX_SPLIT=1 VHX_SPLIT_WAIT=32 VHX_SPLIT_TUNE=$t VHX_SPLIT_DIAG=2 VHX_DEBUG_PASSES=1 $P > $D/d_$t.log 2>&1 || { tail -20 $D/d_$t.log; exit 1; }
  echo "tune $t:"; grep "split slots" $D/d_$t.log | tail -1; grep isolated $D/d_$t.log
done
