#!/bin/bash
# MIP stand-in mode at the headline scale: the 1024^3 LOD parity tests, then bench --mip-lod at depths 1, 2 and 3
# (3 = every node resident, traced through the MIP kernels) beside the reference-path bench, one GPU.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/miplod
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_mips.py > gpurun_out/miplod/pytest_mips.log 2>&1 || { echo "mip tests failed"; tail -30 gpurun_out/miplod/pytest_mips.log; exit 1; }
tail -2 gpurun_out/miplod/pytest_mips.log
for d in 1 2 3; do
  timeout -k 10 300 python bench.py --mip-lod $d > gpurun_out/miplod/bench_miplod$d.log 2>&1 || { echo "bench mip-lod $d failed"; tail -20 gpurun_out/miplod/bench_miplod$d.log; exit 1; }
  tail -1 gpurun_out/miplod/bench_miplod$d.log
done
timeout -k 10 300 python bench.py --no-cpu-baseline --no-pmc > gpurun_out/miplod/bench_ref.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/miplod/bench_ref.log; exit 1; }
tail -1 gpurun_out/miplod/bench_ref.log
