#!/bin/bash
# Scheduler knobs with budgets 24,96,768 at four frames in flight (one env setting per line)
cd "$GRAFT_REPO_ROOT" || exit 1
export VHX_PROBE_F=4
for e in "X=0" "VHX_QWAVESM=1024" "VHX_QWAVESM=1536" "VHX_QWAVES=1024 VHX_QWAVESM=2048" "VHX_QWAVES=4096 VHX_QWAVESM=2048" "VHX_QXCD=0" "VHX_QXCD=8" "VHX_XCDG=0" "VHX_XCDG=32"; do
  echo "$e"
  env $e timeout -k 10 120 python scripts/probes/probe_sched_inflight.py 24,96,768 || exit 1
done
