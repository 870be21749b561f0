#!/bin/bash
# Longer budget ladders (up to six budgets, VHX_MAX_BUDGETS = 6) against the five-pass default, twice each, at frames
# in flight 1 and 8, 100 frames per figure.   scripts/probes/probe_ladder_r03.sh > OUT
cd "$GRAFT_REPO_ROOT" || exit 1
export VHX_PROBE_F=1,8 GPU_MAX_HW_QUEUES=12 VHX_PROBE_K=100
for rep in 1 2; do
  timeout -k 10 300 python -u scripts/probes/probe_sched_inflight.py 24,72,216,648 24,48,96,192,384,768 \
    24,48,120,288,648 16,48,144,432,1296 24,60,150,375,940 24,72,216,648,1944 || exit 1
done
