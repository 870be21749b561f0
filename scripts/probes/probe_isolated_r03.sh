#!/bin/bash
# Isolated-frame latency per schedule and queue-pass wave count.   scripts/probes/probe_isolated_r03.sh > OUT
cd "$GRAFT_REPO_ROOT" || exit 1
S='"" 64 48 96 32,256 24,96,768 24,72,216,648'
for w in 2048 4096 8192; do
  eval VHX_QWAVES=$w timeout -k 10 300 python -u scripts/probes/probe_isolated_r03.py $S || exit 1
done
eval VHX_QWAVES=4096 VHX_QWAVES0=16384 timeout -k 10 300 python -u scripts/probes/probe_isolated_r03.py 64 || exit 1
eval VHX_SPARSE=0 timeout -k 10 300 python -u scripts/probes/probe_isolated_r03.py 64 24,96,768 || exit 1
