#!/bin/bash
# Frames-in-flight schedule knobs re-checked at sixteen frames in flight (bench frame, schedule probe, two rounds):
# pass-0 sparse threshold, first-queue-pass waves, queue waves, pass-0 queue tile, budget ladders.
cd "$GRAFT_REPO_ROOT" || exit 1
export VHX_PROBE_F=16 GPU_MAX_HW_QUEUES=20 VHX_PROBE_K=160
P="timeout -k 10 300 python -u scripts/probes/probe_sched_inflight.py"
L=24,72,216,648
for rep in 1 2; do
  echo "default"; $P $L 2>&1 | grep -v amdgpu.ids || exit 1
  echo "VHX_SPARSE=16"; VHX_SPARSE=16 $P $L 2>&1 | grep -v amdgpu.ids || exit 1
  echo "VHX_SPARSE=8"; VHX_SPARSE=8 $P $L 2>&1 | grep -v amdgpu.ids || exit 1
  echo "VHX_QWAVES0=4096"; VHX_QWAVES0=4096 $P $L 2>&1 | grep -v amdgpu.ids || exit 1
  echo "VHX_QWAVES0=16384"; VHX_QWAVES0=16384 $P $L 2>&1 | grep -v amdgpu.ids || exit 1
  echo "VHX_QWAVES=512"; VHX_QWAVES=512 $P $L 2>&1 | grep -v amdgpu.ids || exit 1
  echo "VHX_QORDER=32z"; VHX_QORDER=32z $P $L 2>&1 | grep -v amdgpu.ids || exit 1
  echo "ladders"; $P 32,96,288,864 16,48,144,432,1296 24,64,192,576,1728 2>&1 | grep -v amdgpu.ids || exit 1
done
