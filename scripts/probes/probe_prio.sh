#!/bin/bash
# issue priority of the queue passes (VHX_QPRIO) under frames in flight
cd "$GRAFT_REPO_ROOT" || exit 1
for p in 0 1 2 3; do
  echo "VHX_QPRIO=$p"
  VHX_QPRIO=$p timeout -k 10 120 python scripts/probes/probe_sched_inflight.py 64 32,256 16,64,512 || exit 1
done
