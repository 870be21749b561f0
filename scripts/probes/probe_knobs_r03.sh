#!/bin/bash
# Queue-pass knobs under the tile-ordered queue (frames-in-flight schedule, eight frames in flight), two rounds:
# every queue pass dealt over the XCDs, the last pass's XCD run length, queue waves per pass.
cd "$GRAFT_REPO_ROOT" || exit 1
export VHX_PROBE_F=8 GPU_MAX_HW_QUEUES=12 VHX_PROBE_K=100
P="timeout -k 10 300 python -u scripts/probes/probe_sched_inflight.py 24,72,216,648"
for rep in 1 2; do
  echo "default"; $P || exit 1
  echo "VHX_QXCD_ALL=1"; VHX_QXCD_ALL=1 $P || exit 1
  echo "VHX_QXCD=4"; VHX_QXCD=4 $P || exit 1
  echo "VHX_QXCD=64"; VHX_QXCD=64 $P || exit 1
  echo "VHX_QWAVES=2048"; VHX_QWAVES=2048 $P || exit 1
  echo "VHX_QWAVESM=2048"; VHX_QWAVESM=2048 $P || exit 1
  echo "VHX_QWAVES=512"; VHX_QWAVES=512 $P || exit 1
done
