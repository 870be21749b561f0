#!/bin/bash
# Shadow frames one at a time: kernel traces with the budgeted shadow passes dealt over the XCDs (VHX_QXCD_ALL=1) or
# not, for budgets 64 and 24,96,768 (per-pass durations: scripts/probes/pass_times.py style summary below)
cd "$GRAFT_REPO_ROOT" || exit 1
D="$GRAFT_REPO_ROOT/gpurun_out/shadow_xcd"; mkdir -p "$D"
cd /tmp && export TMPDIR=/tmp
for b in 64 24,96,768; do for a in 0 1; do
  VHX_BUDGETS=$b VHX_QXCD_ALL=$a timeout -s KILL 120 rocprofv3 --kernel-trace -f csv -d "$D" -o "b${b}_a$a" -- python3 "$GRAFT_REPO_ROOT/bench.py" --shadows --inflight 1 --steps 10 --warmup 2 --no-cpu-baseline > "$D/b${b}_a$a.log" 2>&1 || exit 1
  echo "budgets $b all=$a: $(grep -o '"ms_per_step": [0-9.]*' "$D/b${b}_a$a.log")"
done; done
