#!/bin/bash
# Scheduler knobs at eight frames in flight (own hardware queues), each setting twice
cd "$GRAFT_REPO_ROOT" || exit 1
export GPU_MAX_HW_QUEUES=12 VHX_PROBE_F=8
for rep in 1 2; do
for e in "X=0" "VHX_QWAVES=1024" "VHX_QWAVES=4096" "VHX_QWAVESM=4096" "VHX_QBLOCK=64" "VHX_QBLOCK=128" "VHX_XCDG=0" "VHX_SPARSE=12,4" "VHX_QXCD=0"; do
  echo "$e rep $rep $(env $e timeout -k 10 120 python scripts/probes/probe_sched_inflight.py 24,96,768 2>&1 | grep -v amdgpu | awk '{print $3, $4}')"
done; done
