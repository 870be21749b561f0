#!/bin/bash
# lane-refill threshold sweep of the final pass (VHX_REFILL), frames in flight 1 and 3
cd "$GRAFT_REPO_ROOT" || exit 1
for r in 0 1 4 8 16 32 64; do
  echo "VHX_REFILL=$r"
  VHX_REFILL=$r timeout -k 10 120 python scripts/probes/probe_sched_inflight.py 64 32,256 || exit 1
done
