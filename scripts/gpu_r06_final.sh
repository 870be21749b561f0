#!/bin/bash
# Round-6 closing check on one box: smoke, the whole -m gpu suite, the driver's bench command (--gpus 1 --steps 20
# --warmup 5) and the config-5 line, then the kernel trace + PMC passes of the driver's command (gpu_profile.sh).
# Every GPU step under its own time limit; stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r06_final}
D="$GRAFT_REPO_ROOT/gpurun_out/$TAG"; mkdir -p "$D"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $D/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $D/pytest_gpu.log 2>&1 || { echo "gpu suite failed"; tail -30 $D/pytest_gpu.log; exit 1; }
tail -1 $D/pytest_gpu.log
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $D/bench.json.log 2>&1 || { echo "bench failed"; tail -20 $D/bench.json.log; exit 1; }
tail -1 $D/bench.json.log | cut -c1-400
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 --shadows > $D/bench_shadows.json.log 2>&1 || { echo "shadow bench failed"; tail -20 $D/bench_shadows.json.log; exit 1; }
tail -1 $D/bench_shadows.json.log | cut -c1-300
bash scripts/gpu_profile.sh $TAG
