#!/bin/bash
# Profiles of the default bench command for profiles/<round>/: kernel trace + stats, FETCH_SIZE (memory-side read
# bytes) and two passes of SQ counters (issue, lanes), each pass a run of its own (rocprofv3 does not split counters
# over passes; MI355X_MICROARCH.md). usage: gpu_profile.sh TAG [bench args...]
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; shift
R="$GRAFT_REPO_ROOT"; D="$R/gpurun_out/prof_$TAG"; mkdir -p "$D"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --kernel-trace --stats -f csv -d "$D" -o ks -- python3 "$R/bench.py" --no-cpu-baseline "$@" > "$D/ks.log" 2>&1 || { echo "kernel trace failed"; tail -5 "$D/ks.log"; exit 1; }
tail -1 "$D/ks.log" | cut -c1-300
P0="FETCH_SIZE"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH"
P2="SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
j=0
for P in "$P0" "$P1" "$P2"; do
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace -f csv -d "$D" -o "pmc$j" -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-roofline "$@" > "$D/pmc$j.log" 2>&1; rc=$?
  echo "pmc pass $j rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$D/pmc$j.log"; exit $rc; }
  j=$((j+1))
done
find "$D" -name "*.csv" | head -20
