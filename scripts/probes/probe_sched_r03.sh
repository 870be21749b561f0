#!/bin/bash
# Five-pass budget schedules against the default, twice each (interleaved), at frames in flight 1 and 8, 100 frames per
# figure.   scripts/probes/probe_sched_r03.sh > OUT
cd "$GRAFT_REPO_ROOT" || exit 1
export VHX_PROBE_F=1,8 GPU_MAX_HW_QUEUES=12 VHX_PROBE_K=100
for rep in 1 2; do
  timeout -k 10 300 python -u scripts/probes/probe_sched_inflight.py 24,96,768 24,48,96,768 24,64,192,768 24,72,216,648 \
    24,48,144,768 32,96,288,864 || exit 1
  VHX_SPARSE=12,4,4,4 timeout -k 10 300 python -u scripts/probes/probe_sched_inflight.py 24,72,216,648 24,48,144,768 || exit 1
done
