#!/bin/bash
# Sweep of multi-pass schedules on the bench frame (no CPU baseline). Items are env assignments joined by '+', e.g.
# "VHX_BUDGETS=64,768+VHX_RPW=64,0+VHX_TW=1024". Runs the GPU parity tests first unless SKIP_TESTS is set.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
  [ $rc -ne 0 ] && exit $rc
fi
i=0
for item in $SCHEDULES; do
  i=$((i+1))
  envs="$(echo "$item" | tr '+' ' ')"
  env $envs timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline > "gpurun_out/sched_$i.log" 2>&1; rc=$?
  echo "[$item] rc=$rc $(tail -1 "gpurun_out/sched_$i.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])" 2>&1)"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
