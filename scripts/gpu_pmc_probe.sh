#!/bin/bash
# SQ counters of two placements of the longest ray (probe_cfg.py): one real wave per workgroup vs four per workgroup.
cd "$GRAFT_REPO_ROOT" || exit 1
R="$GRAFT_REPO_ROOT"; D="$R/gpurun_out/pmc_probe"; mkdir -p "$D"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$D/avail.txt" 2>&1
grep -o "SQ_[A-Z0-9_]*" "$D/avail.txt" | sort -u > "$D/sq_names.txt"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
P2="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM"
for cfg in "256 64" "64 64"; do
  set -- $cfg
  j=0
  for P in "$P1" "$P2"; do
    j=$((j+1))
    ok=1; for c in $P; do grep -qx "$c" "$D/sq_names.txt" || { echo "missing counter $c"; ok=0; }; done
    [ $ok -eq 0 ] && continue
    timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace -f csv -d "$D" -o "g$1_k$2_p$j" -- python3 "$R/scripts/probe_cfg.py" "$R/scratch/tail_pixels.npz" $1 $2 > "$D/g$1_k$2_p$j.log" 2>&1; rc=$?
    echo "cfg gap=$1 k=$2 pass $j rc=$rc $(grep ms= "$D/g$1_k$2_p$j.log")"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
