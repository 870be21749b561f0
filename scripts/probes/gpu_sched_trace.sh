#!/bin/bash
# Kernel traces of the bench frame under several multi-pass schedules ('+'-joined env items in $SCHEDULES), to see
# each pass's duration; summarised by scripts/probes/pass_times.py.
cd "$GRAFT_REPO_ROOT" || exit 1
R="$GRAFT_REPO_ROOT"; D="$R/gpurun_out/sched_trace"; mkdir -p "$D"
cd /tmp && export TMPDIR=/tmp
i=0
for item in $SCHEDULES; do
  i=$((i+1))
  envs="$(echo "$item" | tr '+' ' ')"
  for e in $envs; do export "$e"; done
  timeout -k 10 120 rocprofv3 --kernel-trace -f csv -d "$D" -o "s$i" -- python3 "$R/bench.py" --steps 4 --warmup 1 --no-cpu-baseline --no-roofline > "$D/s$i.log" 2>&1; rc=$?
  for e in $envs; do unset "${e%%=*}"; done
  echo "[$item] rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  python3 "$R/scripts/probes/pass_times.py" "$D/s${i}_kernel_trace.csv"
done
exit 0
