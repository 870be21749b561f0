#!/bin/bash
# Pass-budget schedules (incl. four budgets) and the mid-pass wave count VHX_QWAVESM at frames in flight 1 and 4
cd "$GRAFT_REPO_ROOT" || exit 1
export VHX_PROBE_F=${VHX_PROBE_F:-1,4}
timeout -k 10 200 python scripts/probes/probe_sched_inflight.py 24,96,768 16,48,192,1024 24,96,384,1536 16,64,256,1024 24,72,288,1152 32,128,512,2048 || exit 1
for w in 4096 8192; do
  echo "VHX_QWAVESM=$w"
  VHX_QWAVESM=$w timeout -k 10 200 python scripts/probes/probe_sched_inflight.py 24,96,768 16,64,256,1024 || exit 1
done
