#!/bin/bash
# Final round-3 check of HEAD: the split tests, the whole -m gpu suite, kernel trace + three PMC passes of the default
# bench (gpu_profile.sh) with their summaries, then the default / orbit / config-4 bench lines.
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r03_final2}
mkdir -p gpurun_out/$TAG
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_split.py > gpurun_out/$TAG/split_tests.log 2>&1 || { echo "split tests failed"; tail -30 gpurun_out/$TAG/split_tests.log; exit 1; }
tail -1 gpurun_out/$TAG/split_tests.log
timeout -k 10 900 $T tests -m gpu > gpurun_out/$TAG/pytest_gpu.log 2>&1 || { echo "gpu suite failed"; tail -30 gpurun_out/$TAG/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest_gpu.log
scripts/probes/gpu_r03g.sh $TAG
