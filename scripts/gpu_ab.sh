#!/bin/bash
# parity tests on the default kernel, then A/B bench of kernel variants
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -gt 1 ] && exit $rc
for v in 0 1; do
  VHX_PERSISTENT=$v timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_persist$v.log 2>&1; rc=$?
  echo "persistent=$v rc=$rc"; tail -1 gpurun_out/bench_persist$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
