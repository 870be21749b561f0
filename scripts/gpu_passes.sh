#!/bin/bash
# per-dispatch kernel durations of the multi-pass schedule (rocprofv3 kernel trace) for a few budget sets
cd "$GRAFT_REPO_ROOT" || exit 1
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for b in ${BUDGET_SET:-"" 64 32,256}; do
  VHX_BUDGETS="$b" timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d "$R/gpurun_out/passes_b$b" -o run -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/passes_b$b.log" 2>&1; rc=$?
  echo "budgets=[$b] rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
