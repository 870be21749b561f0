#!/bin/bash
# Waves of the budgeted queue passes (VHX_QWAVESM) and of the last pass (VHX_QWAVES) under the five-pass default, at
# frames in flight 1 and 8, 100 frames per figure.   scripts/probes/probe_qwaves_r03.sh > OUT
cd "$GRAFT_REPO_ROOT" || exit 1
export VHX_PROBE_F=1,8 GPU_MAX_HW_QUEUES=12 VHX_PROBE_K=100
for rep in 1 2; do
  for m in 2048 4096 8192 1024; do
    echo "VHX_QWAVESM=$m"
    VHX_QWAVESM=$m timeout -k 10 300 python -u scripts/probes/probe_sched_inflight.py 24,72,216,648 || exit 1
  done
  for w in 4096 1024; do
    echo "VHX_QWAVES=$w"
    VHX_QWAVES=$w timeout -k 10 300 python -u scripts/probes/probe_sched_inflight.py 24,72,216,648 || exit 1
  done
  echo "VHX_QBLOCK=64"
  VHX_QBLOCK=64 timeout -k 10 300 python -u scripts/probes/probe_sched_inflight.py 24,72,216,648 || exit 1
done
