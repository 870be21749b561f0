#!/bin/bash
# Sparse-wave abandonment (VHX_SPARSE, per budgeted pass) at eight frames in flight and one at a time
cd "$GRAFT_REPO_ROOT" || exit 1
export GPU_MAX_HW_QUEUES=12 VHX_PROBE_F=1,8
for sp in 0 4 8 16 4,4,4 8,8,8 16,8,4 32,16,8 8,0,0 0,8,8; do
  echo "VHX_SPARSE=$sp"
  VHX_SPARSE=$sp timeout -k 10 120 python scripts/probes/probe_sched_inflight.py 24,96,768 2>&1 | grep -v amdgpu || exit 1
done
