#!/bin/bash
# first GPU pass: smoke, GPU parity tests, short bench
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -5 gpurun_out/bench.log
exit $rc
