#!/bin/bash
# Round 4: the GPU suite after removing the off-by-default lone-frame experiments, then the driver's bench command.
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/${1:-r04q}; mkdir -p $D
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $D/pytest_gpu.log 2>&1 \
  || { tail -30 $D/pytest_gpu.log; exit 1; }
tail -2 $D/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $D/bench_$r.log 2>&1 || { tail -20 $D/bench_$r.log; exit 1; }
  tail -1 $D/bench_$r.log
done
