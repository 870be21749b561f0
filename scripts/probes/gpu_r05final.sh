#!/bin/bash
# Round 5, end: the committed tree as the driver will run it -- the whole -m gpu suite, smoke(), the driver's bench command
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05final; mkdir -p $O
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests -m gpu > $O/gpu_all.log 2>&1 || { echo "gpu suite failed"; tail -30 $O/gpu_all.log; exit 1; }
tail -1 $O/gpu_all.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench_noargs.log 2>&1 || { echo "bench failed"; tail -20 $O/bench_noargs.log; exit 1; }
tail -1 $O/bench_noargs.log | cut -c1-400
