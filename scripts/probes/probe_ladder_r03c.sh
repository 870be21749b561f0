#!/bin/bash
# Budget ladders and pass-0 sparse thresholds under the tile-ordered queue (frames-in-flight schedule), eight frames in
# flight, two rounds.   scripts/probes/probe_ladder_r03c.sh > OUT
cd "$GRAFT_REPO_ROOT" || exit 1
export VHX_PROBE_F=8 GPU_MAX_HW_QUEUES=12 VHX_PROBE_K=100
L="24,72,216,648 24,96,768 32,96,288,864 24,48,144,432,1296 16,48,144,432 24,64,192,576 32,128,1024 24,72,216,648,1944"
for rep in 1 2; do
  timeout -k 10 300 python -u scripts/probes/probe_sched_inflight.py $L || exit 1
  for sp in 8 16 0; do
    echo "VHX_SPARSE=$sp"
    VHX_SPARSE=$sp timeout -k 10 300 python -u scripts/probes/probe_sched_inflight.py 24,72,216,648 || exit 1
  done
done
