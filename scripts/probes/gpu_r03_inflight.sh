#!/bin/bash
# Frames in flight under the tile-ordered queue: the bench frame at F = 8 / 12 / 16 / 24, two rounds, A/B in one run,
# frame check on; moving camera at F = 8 / 16.
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/${1:-r03_inflight}; mkdir -p $D
B="timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-pmc"
for rep in 1 2; do
  for F in 8 12 16 24; do
    $B --inflight $F > $D/bench_f${F}_$rep.log 2>&1 || { tail -20 $D/bench_f${F}_$rep.log; exit 1; }
    echo "F=$F rep $rep $(tail -1 $D/bench_f${F}_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["frames_equal"], d["golden_match"], d["roofline"]["kernel_ms_isolated"])')"
  done
done
for F in 8 16; do
  $B --inflight $F --orbit 0.01 > $D/orbit_f$F.log 2>&1 || { tail -20 $D/orbit_f$F.log; exit 1; }
  echo "orbit F=$F $(tail -1 $D/orbit_f$F.log | cut -c1-200)"
done
