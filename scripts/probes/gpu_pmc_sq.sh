#!/bin/bash
# SQ counters (issue, stalls, lane utilisation, instruction fetch) of the bench frame's trace kernels and of two
# placements of the longest ray; summarised by scripts/probes/sq_summary.py.
cd "$GRAFT_REPO_ROOT" || exit 1
R="$GRAFT_REPO_ROOT"; D="$R/gpurun_out/pmc_sq"; mkdir -p "$D"
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH"
P2="SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_IFETCH SQ_IFETCH_LEVEL SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_LDS"
j=0
for P in "$P1" "$P2"; do
  j=$((j+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace -f csv -d "$D" -o "bench_p$j" -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-roofline > "$D/bench_p$j.log" 2>&1; rc=$?
  echo "bench pass $j rc=$rc"; [ $rc -ne 0 ] && exit $rc
  for cfg in "256 64" "64 64"; do
    set -- $cfg
    timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace -f csv -d "$D" -o "g$1_p$j" -- python3 "$R/scripts/probe_cfg.py" "$R/scratch/tail_pixels.npz" $1 $2 > "$D/g$1_p$j.log" 2>&1; rc=$?
    echo "probe gap=$1 pass $j rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
