#!/bin/bash
# Pass-budget schedules (three and four budgets) at eight frames in flight, own hardware queues, each list twice
cd "$GRAFT_REPO_ROOT" || exit 1
export GPU_MAX_HW_QUEUES=12 VHX_PROBE_F=8
L=${BUDGET_LISTS:-"24,96,768 24,96,768,3072 24,96,384,1536 24,64,256,1024 24,96,512,2048 24,128,768 24,96,1024"}
for rep in 1 2; do
  timeout -k 10 200 python scripts/probes/probe_sched_inflight.py $L 2>&1 | grep -v amdgpu || exit 1
done
