#!/bin/bash
# A/B of two libvhx builds on the driver's bench command, rounds interleaved (box drift hits both alike).
# usage: gpu_ab.sh TAG LIB_A LIB_B [bench args]   (LIB_* = path or "default"; REPS rounds, default 2)
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; A=$2; B=$3; shift 3
D=gpurun_out/$TAG; mkdir -p $D
J='import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; i=r.get("issue") or {}; print(d["ms_per_step"], d["value"], d.get("frames_equal"), d.get("golden_match"), r.get("kernel_ms_isolated"), i.get("valu_wave_instructions_per_frame"), json.dumps(i.get("active_lanes_per_valu")))'
for rep in $(seq 1 ${REPS:-2}); do
  for L in A B; do
    P=$A; [ $L = B ] && P=$B
    E=""; [ "$P" != default ] && E="VHX_LIB=$P"
    env $E timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra "$@" > $D/${L}_$rep.log 2>&1 \
      || { tail -20 $D/${L}_$rep.log; exit 1; }
    echo "$L rep $rep $(tail -1 $D/${L}_$rep.log | python3 -c "$J")" | tee -a $D/summary.txt
  done
done
