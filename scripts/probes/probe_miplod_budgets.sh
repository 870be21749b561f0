#!/bin/bash
# Pass schedules for the MIP stand-in views of the headline tree (short rays: the compaction kernels are ~22 % of a
# depth-1 frame with the default {24, 96, 768}). VHX_BUDGETS: "0" = one pass.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/miplod_budgets
for d in 1 2; do
  for b in default 0 64 24,96 32,256; do
    if [ $b = default ]; then env_b=""; else env_b="VHX_BUDGETS=$b"; fi
    env $env_b timeout -k 10 200 python bench.py --mip-lod $d > gpurun_out/miplod_budgets/d${d}_b${b}.log 2>&1 || { echo "failed d=$d b=$b"; tail -5 gpurun_out/miplod_budgets/d${d}_b${b}.log; exit 1; }
    echo "depth $d budgets $b $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/miplod_budgets/d${d}_b${b}.log)"
  done
done
