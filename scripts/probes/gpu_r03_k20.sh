#!/bin/bash
# Frames in flight at the driver's bench command (--steps 20 --warmup 5: the timed region starts from an idle GPU, so
# the pipeline's fill and drain weigh more than over 100 steps): F = 8 / 12 / 16, three rounds.
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/${1:-r03_k20}; mkdir -p $D
J='import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d.get("frames_equal"), d.get("golden_match"))'
B="timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-pmc"
for rep in 1 2 3; do
  for F in 8 12 16; do
    $B --inflight $F > $D/k20_f${F}_$rep.log 2>&1 || { tail -20 $D/k20_f${F}_$rep.log; exit 1; }
    echo "K=20 F=$F rep $rep $(tail -1 $D/k20_f${F}_$rep.log | python3 -c "$J")"
  done
done
