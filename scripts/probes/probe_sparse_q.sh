#!/bin/bash
# Sparse-wave abandonment thresholds of the budgeted queue passes (VHX_SPARSE = pass 0, 1, 2) at eight frames in
# flight, own hardware queues, each setting twice
cd "$GRAFT_REPO_ROOT" || exit 1
export GPU_MAX_HW_QUEUES=12 VHX_PROBE_F=8
for rep in 1 2; do
for e in "12" "12,8" "12,16" "12,24" "12,16,8" "12,0,16" "12,32"; do
  echo "VHX_SPARSE=$e rep $rep $(VHX_SPARSE=$e timeout -k 10 120 python scripts/probes/probe_sched_inflight.py 24,96,768 2>&1 | grep budgets)" || exit 1
done; done
