#!/bin/bash
# pass-0 serialisation across frames in flight (VHX_P0SERIAL) x budgets
cd "$GRAFT_REPO_ROOT" || exit 1
for v in 0 1; do
  echo "VHX_P0SERIAL=$v"
  VHX_P0SERIAL=$v timeout -k 10 150 python scripts/probes/probe_sched_inflight.py 64 32,256 16,64,512 128 || exit 1
done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $GRAFT_REPO_ROOT/gpurun_out/tl2 -o f3 -- python3 $GRAFT_REPO_ROOT/scripts/probes/probe_inflight_trace.py 3 12 > $GRAFT_REPO_ROOT/gpurun_out/tl2.log 2>&1
