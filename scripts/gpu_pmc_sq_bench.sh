#!/bin/bash
# SQ counters of the bench frame's trace kernels only (the two passes of gpu_pmc_sq.sh without the placement probes).
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
done
cd "$R" && python3 scripts/sq_summary.py "$D" bench
