#!/bin/bash
# Round 4: one-launch frame occupancy (waves per SIMD 4 / 5 / 6, VHX_FRAME_WPE builds) on the lone frame.
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/${1:-r04o}; mkdir -p $D
for L in default voxelhex_amd/_lib/ab/libvhx_f5.so voxelhex_amd/_lib/ab/libvhx_f6.so; do
  E=""; [ "$L" != default ] && E="VHX_LIB=$L"
  echo "== $L" >> $D/one.log
  env $E timeout -k 10 200 python -u scripts/probes/probe_ahead.py "one=0" "one=1" "one=1;budgets=48,192,768" >> $D/one.log 2>&1 \
    || { tail -20 $D/one.log; exit 1; }
done
cat $D/one.log
