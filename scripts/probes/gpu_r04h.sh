#!/bin/bash
# Host submission time against the frame period at the driver's command, F = 4 / 8 / 20.
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/${1:-r04h}; mkdir -p $D
J='import json,sys; d=json.loads(sys.stdin.read()); print(d["frames_in_flight"], d["ms_per_step"], d["host_submit_ms_per_step"], d["roofline"].get("kernel_ms"))'
for F in 20 8 4; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pmc --no-extra --inflight $F > $D/f$F.log 2>&1 || { tail -20 $D/f$F.log; exit 1; }
  echo "F ms/step submit_ms/step kernel_ms: $(tail -1 $D/f$F.log | python3 -c "$J")" | tee -a $D/summary.txt
done
