#!/bin/bash
# Frames in flight 8 / 12 / 16 with the tile-ordered queue, three rounds (bench lines without the PMC child).
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/${1:-r03q}; mkdir -p $D
for rep in 1 2 3; do
  for F in 8 12 16; do
    timeout -k 10 300 python -u bench.py --inflight $F --no-cpu-baseline --no-pmc --no-frame-check > $D/bench_f${F}_$rep.log 2>&1 || { tail -20 $D/bench_f${F}_$rep.log; exit 1; }
    echo "F=$F $(tail -1 $D/bench_f${F}_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'], d['roofline']['kernel_ms_isolated'])")"
  done
done
