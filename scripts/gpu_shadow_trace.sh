#!/bin/bash
# Kernel trace of the config-5 bench (primary frame + hard-shadow rays), last frame's kernels.
cd "$GRAFT_REPO_ROOT" || exit 1
R="$GRAFT_REPO_ROOT"; D="$R/gpurun_out/shadow_trace"; mkdir -p "$D"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace -f csv -d "$D" -o s -- python3 "$R/bench.py" --shadows --steps 4 --warmup 1 --no-cpu-baseline > "$D/s.log" 2>&1; rc=$?
echo "rc=$rc"; [ $rc -ne 0 ] && exit $rc
python3 "$R/scripts/pass_times.py" "$D/s_kernel_trace.csv"
