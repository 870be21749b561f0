#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/${1:-r03m}; mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_inflight.py -k "shadow or scheduler or golden or inflight or ragged or full_size" > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
tail -1 $D/tests.log
scripts/probes/probe_lone_order_r03.sh > $D/lone_order.log 2>&1 || { tail -20 $D/lone_order.log; exit 1; }
grep -v amdgpu.ids $D/lone_order.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $D/bench.log 2>&1 || { tail -20 $D/bench.log; exit 1; }
tail -1 $D/bench.log | cut -c1-250
for o in 0 64z; do
  VHX_QORDER=$o timeout -k 10 300 python -u bench.py --shadows --steps 50 --no-cpu-baseline --no-pmc > $D/shadows_$o.log 2>&1 || { tail -20 $D/shadows_$o.log; exit 1; }
  echo "shadows VHX_QORDER=$o: $(tail -1 $D/shadows_$o.log | cut -c1-200)"
done
