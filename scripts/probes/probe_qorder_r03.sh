#!/bin/bash
# Pass-0 queue order A/B (VHX_QORDER: 0 output-index = row-major order; N = NxN tiles row-major; mN = Morton order of
# NxN tiles) at one and eight frames in flight under the frames-in-flight schedule, two rounds.
# usage: probe_qorder_r03.sh [ORDERS...]
cd "$GRAFT_REPO_ROOT" || exit 1
export VHX_PROBE_F=${VHX_PROBE_F:-1,8} GPU_MAX_HW_QUEUES=12 VHX_PROBE_K=100
ORDERS=${*:-0 8 16 32 64 m8 m16 m32}
for rep in ${REPS:-1 2}; do
  for o in $ORDERS; do
    echo "VHX_QORDER=$o"
    VHX_QORDER=$o timeout -k 10 300 python -u scripts/probes/probe_sched_inflight.py 24,72,216,648 || exit 1
  done
done
