#!/bin/bash
# Lone-frame (isolated) latency of the bench frame: the adaptive default, then fixed lone schedules without sparse-wave
# abandonment at 8 queue waves per CU, with fewer rays per wave in the last pass (VHX_RPW: rays per wave of queue
# passes 1, 2, ...).   scripts/probes/probe_lone_r03.sh > OUT
cd "$GRAFT_REPO_ROOT" || exit 1
P="timeout -k 10 300 python -u scripts/probes/probe_isolated_r03.py"
echo "adaptive default (set_pass_budgets not called):"
timeout -k 10 300 python -u scripts/probes/probe_isolated_r03.py adaptive || exit 1
export VHX_SPARSE=0 VHX_QWAVES=2048
$P 64 64,1024 64,512 48,768 64,256,1024 || exit 1
for r in "64,8" "64,16" "64,4"; do
  VHX_RPW=$r $P 64,1024 64,512 64,2048 || exit 1
done
VHX_RPW=64,64,8 $P 64,256,1024 32,256,1024 || exit 1
VHX_RPW=64,64,4 $P 64,256,1024 || exit 1
