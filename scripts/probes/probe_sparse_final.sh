#!/bin/bash
# Pass-0 sparse-wave threshold (VHX_SPARSE, default 12) re-checked with the final round-2 kernels at eight frames in
# flight, each setting twice (bench frame, budgets 24,96,768)
cd "$GRAFT_REPO_ROOT" || exit 1
export GPU_MAX_HW_QUEUES=12 VHX_PROBE_F=8
for rep in 1 2; do
for e in "VHX_SPARSE=12" "VHX_SPARSE=8" "VHX_SPARSE=10" "VHX_SPARSE=14" "VHX_SPARSE=16" "VHX_SPARSE=20" "VHX_SPARSE=0"; do
  echo "$e rep $rep $(env $e timeout -k 10 120 python scripts/probes/probe_sched_inflight.py 24,96,768 2>&1 | grep -v amdgpu | awk '{print $3, $4}')"
done; done
