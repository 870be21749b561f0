#!/bin/bash
# Isolated-frame latency without sparse-wave abandonment (VHX_SPARSE=0), per schedule and queue-pass wave count.
cd "$GRAFT_REPO_ROOT" || exit 1
S='48 64 96 128 192 32,256 64,512 24,96,768'
for w in 2048 1024 3072; do
  eval VHX_SPARSE=0 VHX_QWAVES=$w timeout -k 10 300 python -u scripts/probes/probe_isolated_r03.py $S || exit 1
done
eval VHX_SPARSE=4 timeout -k 10 300 python -u scripts/probes/probe_isolated_r03.py 64 96 || exit 1
eval VHX_SPARSE=0 VHX_QXCD=0 timeout -k 10 300 python -u scripts/probes/probe_isolated_r03.py 64 96 || exit 1
eval VHX_SPARSE=0 VHX_XCDG=0 timeout -k 10 300 python -u scripts/probes/probe_isolated_r03.py 64 96 || exit 1
