#!/bin/bash
# Lone-frame latency of the bench frame (the adaptive lone-frame schedule) per pass-0 queue order, and the
# frames-in-flight default at F = 1, 8 once more (VHX_QORDER fixes the order of both schedules).
cd "$GRAFT_REPO_ROOT" || exit 1
for rep in 1 2; do
  for o in 0 64z 64 128z 16; do
    VHX_QORDER=$o timeout -k 10 300 python -u scripts/probes/probe_isolated_r03.py adaptive || exit 1
  done
done
