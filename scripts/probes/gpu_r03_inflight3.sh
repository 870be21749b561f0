#!/bin/bash
# Sixteen frames in flight with 3 queue waves per CU (the new defaults): the in-flight golden tests, the bench, and an
# A/B of 3 against 4 queue waves per CU at F = 8 and F = 16 with the bench (VHX_QWAVES fixes the schedule for every
# frame, so the A/B runs both sides with it: 768 = 3 x 256 CUs, 1024 = 4 x 256).
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/${1:-r03_inflight3}; mkdir -p $D
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_inflight.py -m gpu > $D/pytest_inflight.log 2>&1 || { tail -30 $D/pytest_inflight.log; exit 1; }
tail -2 $D/pytest_inflight.log
timeout -k 10 300 python -u bench.py > $D/bench.log 2>&1 || { tail -20 $D/bench.log; exit 1; }
tail -1 $D/bench.log | cut -c1-400
J='import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d.get("frames_equal"), d.get("golden_match"))'
B="timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-pmc"
for rep in 1 2; do
  for F in 8 16; do
    for QW in 768 1024; do
      VHX_QWAVES=$QW $B --inflight $F > $D/ab_f${F}_q${QW}_$rep.log 2>&1 || { tail -20 $D/ab_f${F}_q${QW}_$rep.log; exit 1; }
      echo "F=$F QW=$QW rep $rep $(tail -1 $D/ab_f${F}_q${QW}_$rep.log | python3 -c "$J")"
    done
  done
done
