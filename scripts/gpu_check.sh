#!/bin/bash
# GPU check of a change: new tests first (FIRST = a -k expression), then the whole -m gpu suite, then the default
# bench, the moving-camera bench and the config-4 (strong) bench on one GPU. Every GPU step has its own time limit;
# the script stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-run}
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests -m gpu ${FIRST:+-k "$FIRST"} > gpurun_out/${TAG}_pytest_first.log 2>&1 || { echo "first tests failed"; tail -30 gpurun_out/${TAG}_pytest_first.log; exit 1; }
tail -3 gpurun_out/${TAG}_pytest_first.log
if [ -n "$FIRST" ]; then
  timeout -k 10 900 $T tests -m gpu > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { echo "gpu suite failed"; tail -30 gpurun_out/${TAG}_pytest_gpu.log; exit 1; }
  tail -3 gpurun_out/${TAG}_pytest_gpu.log
fi
[ -n "$NOBENCH" ] && exit 0
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log
timeout -k 10 300 python bench.py --orbit 0.01 --no-cpu-baseline > gpurun_out/${TAG}_bench_orbit.log 2>&1 || { echo "orbit bench failed"; tail -20 gpurun_out/${TAG}_bench_orbit.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench_orbit.log
timeout -k 10 300 python bench.py --scaling strong > gpurun_out/${TAG}_bench_strong.log 2>&1 || { echo "strong bench failed"; tail -20 gpurun_out/${TAG}_bench_strong.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench_strong.log
