#!/bin/bash
# PMC passes (separate runs, --kernel-trace only beside --pmc) for the primary-ray kernel.
# usage: gpu_pmc.sh TAG [extra env assignments...]
cd "$GRAFT_REPO_ROOT" || exit 1
R="$GRAFT_REPO_ROOT"
TAG=${1:-cur}
mkdir -p "$R/gpurun_out/pmc_$TAG"
cd /tmp && export TMPDIR=/tmp
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU" \
         "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_VMEM_WR SQ_INST_LEVEL_VMEM SQ_INSTS_SMEM GRBM_GUI_ACTIVE" \
         "FETCH_SIZE" \
         "TCC_HIT_sum TCC_MISS_sum" \
         "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum" \
         "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $P --kernel-trace -f csv -d "$R/gpurun_out/pmc_$TAG" -o p$i -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-roofline > "$R/gpurun_out/pmc_$TAG/p$i.log" 2>&1; rc=$?
  echo "pass $i rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
