#!/bin/bash
# Tile-layout queue order: parity of the tile / multi-GPU paths, then the one-rank vhx_mgpu bench (config 4's tile
# path) with output-index order against the default.
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/${1:-r03n}; mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_multigpu.py tests/test_gpu_mgpu_ranks.py -k "tile or untile or scheduler or mgpu or multigpu or ranks or sharded" > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for rep in 1 2; do
for o in 0 64z; do
  VHX_QORDER=$o VHX_BENCH_MGPU1=1 timeout -k 10 300 python -u bench.py --scaling strong --steps 50 --no-cpu-baseline --no-pmc > $D/mgpu1_$o.log 2>&1 || { tail -20 $D/mgpu1_$o.log; exit 1; }
  echo "mgpu1 config4 VHX_QORDER=$o: $(tail -1 $D/mgpu1_$o.log | cut -c1-200)"
done
done
scripts/probes/probe_ladder_r03c.sh > $D/ladder.log 2>&1 || { tail -20 $D/ladder.log; exit 1; }
grep -v amdgpu.ids $D/ladder.log
