#!/bin/bash
# parity tests, then a sweep of multi-pass schedules on the bench frame: items "budgets/rays-per-wave",
# e.g. "32,256/64,16" = VHX_BUDGETS=32,256 VHX_RPW=64,16
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
  [ $rc -ne 0 ] && exit $rc
fi
for item in ${SCHEDULES:-"/" "64/" "32,256/"}; do
  b="${item%%/*}"; r="${item#*/}"; tag="$(echo "$item" | tr '/,' '_-')"
  VHX_BUDGETS="$b" VHX_RPW="$r" timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > "gpurun_out/bench_s$tag.log" 2>&1; rc=$?
  echo "schedule=[$item] rc=$rc $(tail -1 "gpurun_out/bench_s$tag.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])")"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
