#!/bin/bash
# Pass-0 sparse-wave thresholds, each measured twice (eight frames in flight)
cd "$GRAFT_REPO_ROOT" || exit 1
export GPU_MAX_HW_QUEUES=12 VHX_PROBE_F=8
for rep in 1 2; do for sp in 0 8 12 16 24 32; do
  echo "VHX_SPARSE=$sp rep $rep"
  VHX_SPARSE=$sp timeout -k 10 120 python scripts/probes/probe_sched_inflight.py 24,96,768 2>&1 | grep -v amdgpu || exit 1
done; done
