#!/bin/bash
# Rays per wave of the three queue passes (VHX_RPW = pass1,pass2,pass3; 64 = full chunks, the default) at eight
# frames in flight, each setting twice (bench frame, budgets 24,96,768)
cd "$GRAFT_REPO_ROOT" || exit 1
export GPU_MAX_HW_QUEUES=12 VHX_PROBE_F=8
for rep in 1 2; do
for e in "X=0" "VHX_RPW=32,64,64" "VHX_RPW=48,64,64" "VHX_RPW=64,48,64" "VHX_RPW=64,64,32" "VHX_RPW=64,64,48" "VHX_RPW=48,48,48"; do
  echo "$e rep $rep $(env $e timeout -k 10 120 python scripts/probes/probe_sched_inflight.py 24,96,768 2>&1 | grep -v amdgpu | awk '{print $3, $4}')"
done; done
