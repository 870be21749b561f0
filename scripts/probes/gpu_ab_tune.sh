#!/bin/bash
# A/B/... of vhx_set_tuning specs on the driver's bench command, rounds interleaved (box drift hits every spec alike).
# usage: gpu_ab_tune.sh TAG SPEC1 SPEC2 ... ("default" = no --tune); REPS rounds (default 2); EXTRA = more bench args
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; shift
D=gpurun_out/$TAG; mkdir -p $D
J='import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; i=r.get("issue") or {}; print(d["ms_per_step"], d["value"], d.get("frames_equal"), d.get("golden_match"), r.get("kernel_ms_isolated"), i.get("valu_wave_instructions_per_frame"), json.dumps(i.get("active_lanes_per_valu")))'
for rep in $(seq 1 ${REPS:-2}); do
  k=0
  for S in "$@"; do
    k=$((k+1))
    T=""; [ "$S" != default ] && T="--tune $S"
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra $T $EXTRA > $D/s${k}_$rep.log 2>&1 \
      || { tail -20 $D/s${k}_$rep.log; exit 1; }
    echo "[$S] rep $rep $(tail -1 $D/s${k}_$rep.log | python3 -c "$J")" | tee -a $D/summary.txt
  done
done
