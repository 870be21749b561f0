#!/bin/bash
# Lane refill in the budgeted queue passes (VHX_REFILL = thresholds of passes 1, 2) at eight frames in flight
cd "$GRAFT_REPO_ROOT" || exit 1
export GPU_MAX_HW_QUEUES=12 VHX_PROBE_F=1,8
for rf in 0,0 8,8 16,16 32,32 16,0 0,16 48,48; do
  echo "VHX_REFILL=$rf"
  VHX_REFILL=$rf timeout -k 10 120 python scripts/probes/probe_sched_inflight.py 24,96,768 2>&1 | grep -v amdgpu || exit 1
done
