#!/bin/bash
# Tail split: the split tests, the lone bench frame with the split on / off (A/B twice), the whole
# -m gpu suite, the default bench line.   scripts/probes/gpu_r03s.sh TAG
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/${1:-r03s}; mkdir -p $D
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_split.py > $D/split_tests.log 2>&1 || { echo "split tests failed"; tail -40 $D/split_tests.log; exit 1; }
tail -2 $D/split_tests.log
for rep in 1 2; do
  timeout -k 10 300 python -u scripts/probes/probe_isolated_r03.py adaptive >> $D/lone.log 2>&1 || { tail -20 $D/lone.log; exit 1; }
  VHX_SPLIT=0 timeout -k 10 300 python -u scripts/probes/probe_isolated_r03.py adaptive >> $D/lone.log 2>&1 || { tail -20 $D/lone.log; exit 1; }
done
grep isolated $D/lone.log
timeout -k 10 900 $T tests -m gpu > $D/pytest_gpu.log 2>&1 || { echo "gpu suite failed"; tail -30 $D/pytest_gpu.log; exit 1; }
tail -2 $D/pytest_gpu.log
timeout -k 10 300 python bench.py > $D/bench.log 2>&1 || { echo "bench failed"; tail -20 $D/bench.log; exit 1; }
tail -1 $D/bench.log
