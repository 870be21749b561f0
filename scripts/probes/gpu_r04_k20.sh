#!/bin/bash
# Frames in flight at the driver's exact bench command (--steps 20 --warmup 5): F = 8 / 12 / 16 / 20, rounds
# interleaved so that box drift hits every F alike.
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/${1:-r04_k20}; mkdir -p $D
REPS=${REPS:-2}
J='import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d.get("frames_equal"), d.get("golden_match"), d["roofline"].get("kernel_ms_isolated"), json.dumps({k: d[k] for k in ("lone", "orbit") if k in d}))'
B="timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-pmc"
for rep in $(seq 1 $REPS); do
  for F in ${FS:-8 12 16 20}; do
    $B --inflight $F $EXTRA > $D/k20_f${F}_$rep.log 2>&1 || { tail -20 $D/k20_f${F}_$rep.log; exit 1; }
    echo "K=20 F=$F rep $rep $(tail -1 $D/k20_f${F}_$rep.log | python3 -c "$J")" | tee -a $D/summary.txt
  done
done
