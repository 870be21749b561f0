#!/bin/bash
# What each pass adds to the frame: builds that stop after the first 1, 2, 3 passes (VHX_PROBE_PASSES, incomplete
# frames) against the full schedule, at frames in flight 1 and 8.   scripts/probes/probe_pass_share_r03.sh > OUT
cd "$GRAFT_REPO_ROOT" || exit 1
export VHX_PROBE_F=1,8 GPU_MAX_HW_QUEUES=12
for v in p1 p2 p3; do
  echo "passes run: $v"
  VHX_LIB=voxelhex_amd/_lib/var_$v/libvhx.so timeout -k 10 200 python -u scripts/probes/probe_sched_inflight.py 24,96,768 || exit 1
done
echo "all passes"
timeout -k 10 200 python -u scripts/probes/probe_sched_inflight.py 24,96,768 || exit 1
