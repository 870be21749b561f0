#!/bin/bash
# A/B of kernel variants (libvhx builds under voxelhex_amd/_lib/variants/, chosen by VHX_LIB) over pass-budget
# schedules at frames in flight VHX_PROBE_F. usage: probe_variants.sh "lib1 lib2 ..." "64 16,64,512 ..."
cd "$GRAFT_REPO_ROOT" || exit 1
for l in $1; do
  lib=voxelhex_amd/_lib/libvhx.so
  [ "$l" != base ] && lib=voxelhex_amd/_lib/variants/libvhx_$l.so
  echo "== $l"
  VHX_LIB=$PWD/$lib timeout -k 10 200 python scripts/probes/probe_sched_inflight.py $2 || exit 1
done
