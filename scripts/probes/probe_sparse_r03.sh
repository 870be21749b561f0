#!/bin/bash
# Sparse-wave abandonment in the budgeted queue passes (VHX_SPARSE per pass) and finer budget schedules, at frames in
# flight 1 and 8 (probe_sched_inflight.py; every line also checks that the frames are equal across contexts).
#   scripts/probes/probe_sparse_r03.sh > OUT
cd "$GRAFT_REPO_ROOT" || exit 1
export VHX_PROBE_F=1,8 GPU_MAX_HW_QUEUES=12
for sp in 12 12,8 12,8,8 12,16,16 12,4,4 12,0,8 12,0,16 12,24,24; do
  echo "VHX_SPARSE=$sp"
  VHX_SPARSE=$sp timeout -k 10 200 python -u scripts/probes/probe_sched_inflight.py 24,96,768 24,72,216,648 || exit 1
done
