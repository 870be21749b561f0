#!/bin/bash
# Kernel trace of one bench configuration (args after the script name) under the env of the caller; per-kernel
# durations of the last traced frame (scripts/pass_times.py).
cd "$GRAFT_REPO_ROOT" || exit 1
R="$GRAFT_REPO_ROOT"; D="$R/gpurun_out/cfg_trace"; mkdir -p "$D"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace -f csv -d "$D" -o c -- python3 "$R/bench.py" --steps 4 --warmup 1 --no-cpu-baseline --no-roofline "$@" > "$D/c.log" 2>&1; rc=$?
echo "rc=$rc"; [ $rc -ne 0 ] && exit $rc
python3 "$R/scripts/pass_times.py" "$D/c_kernel_trace.csv"
