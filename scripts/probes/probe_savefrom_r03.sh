#!/bin/bash
# Which budgeted passes save their abandoned rays' state (VHX_SAVE_FROM: passes before it keep none, the next pass
# traces those rays again from scratch), at frames in flight 1 and 8.   scripts/probes/probe_savefrom_r03.sh > OUT
cd "$GRAFT_REPO_ROOT" || exit 1
export VHX_PROBE_F=1,8 GPU_MAX_HW_QUEUES=12
for sf in 0 1 2; do
  for sp in 12 12,8; do
    echo "VHX_SAVE_FROM=$sf VHX_SPARSE=$sp"
    VHX_SAVE_FROM=$sf VHX_SPARSE=$sp timeout -k 10 200 python -u scripts/probes/probe_sched_inflight.py 24,96,768 16,96,768 || exit 1
  done
done
