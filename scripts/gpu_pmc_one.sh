#!/bin/bash
# PMC counters of single-wave traces (scripts/probe_one.py): longest ray alone, then the 64 longest in one wave
cd "$GRAFT_REPO_ROOT" || exit 1
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out/pmc_one"
cd /tmp && export TMPDIR=/tmp
i=0
for W in longest top64; do
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU" \
         "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE" \
         "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $P --kernel-trace -f csv -d "$R/gpurun_out/pmc_one" -o "${W}_p$i" -- python3 "$R/scripts/probe_one.py" "$R/scratch/tail_pixels.npz" $W > "$R/gpurun_out/pmc_one/${W}_p$i.log" 2>&1; rc=$?
  echo "$W pass $i rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
done
exit 0
