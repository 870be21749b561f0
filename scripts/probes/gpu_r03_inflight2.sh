#!/bin/bash
# Where the frames-in-flight cliff is (F = 20: 24 hardware queues; F = 24 ran 0.88 ms), config 4 at F = 8 / 16, and
# queue waves of the frames-in-flight schedule at F = 16.
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/${1:-r03_inflight2}; mkdir -p $D
B="timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-pmc"
J='import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d.get("frames_equal"), d.get("golden_match"))'
for F in 16 20 16 20; do
  $B --inflight $F > $D/bench_f$F.log 2>&1 || { tail -20 $D/bench_f$F.log; exit 1; }
  echo "F=$F $(tail -1 $D/bench_f$F.log | python3 -c "$J")"
done
for F in 8 16; do
  $B --inflight $F --scaling strong > $D/strong_f$F.log 2>&1 || { tail -20 $D/strong_f$F.log; exit 1; }
  echo "strong F=$F $(tail -1 $D/strong_f$F.log | python3 -c "$J")"
done
export VHX_PROBE_F=16 GPU_MAX_HW_QUEUES=20 VHX_PROBE_K=160
P="timeout -k 10 300 python -u scripts/probes/probe_sched_inflight.py 24,72,216,648"
for rep in 1 2; do
  for QW in 1024 768 1536; do
    echo "VHX_QWAVES=$QW"; VHX_QWAVES=$QW $P 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
