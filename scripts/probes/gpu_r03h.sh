#!/bin/bash
# Randomised-tree parity (every brick_dim) on the GPU.
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/${1:-r03h}; mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_fuzz.py > $D/fuzz.log 2>&1 || { tail -40 $D/fuzz.log; exit 1; }
tail -14 $D/fuzz.log
