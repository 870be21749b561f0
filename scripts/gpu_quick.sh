#!/bin/bash
# Iteration loop: GPU parity tests, bench (no CPU baseline), and the tail probe (longest rays alone).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_quick.log 2>&1; rc=$?
echo "bench rc=$rc $(tail -1 gpurun_out/bench_quick.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])")"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/probe_tail.py scratch/tail_pixels.npz 2>&1 | grep "sched=()"
