#!/bin/bash
# Round 5 check of the committed code: the whole -m gpu suite, the driver's bench command (default: batches of 7 on 3
# contexts), the 20-context line (--batch 0), config 5, and the profiles of the default command.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05x; mkdir -p $O
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests -m gpu > $O/gpu_all.log 2>&1 || { echo "gpu suite failed"; tail -30 $O/gpu_all.log; exit 1; }
tail -1 $O/gpu_all.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_default.log 2>&1 || { echo "bench failed"; tail -20 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log | cut -c1-400
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --batch 0 > $O/bench_20contexts.log 2>&1 || { echo "bench 20 failed"; tail -20 $O/bench_20contexts.log; exit 1; }
tail -1 $O/bench_20contexts.log | cut -c1-300
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --shadows > $O/c5_shadows.log 2>&1 || { echo "shadows failed"; tail -20 $O/c5_shadows.log; exit 1; }
tail -1 $O/c5_shadows.log | cut -c1-300
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 700 bash scripts/gpu_profile.sh r05_final3 || { echo "profile failed"; exit 1; }
