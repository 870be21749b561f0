#!/bin/bash
# Inner tile orders of the framebuffer queue: 64x64 tiles with 8x8 sub-tiles (64), Morton (64z) or rows (64r), and
# 32r / 128r; three rounds at eight frames in flight; then the tile-path parity tests.
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/${1:-r03o}; mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "scheduler or tile or ragged" > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
tail -1 $D/tests.log
REPS='1 2 3' VHX_PROBE_F=8 scripts/probes/probe_qorder_r03.sh 64z 64r 64 32r 128r > $D/qorder.log 2>&1 || { tail -20 $D/qorder.log; exit 1; }
grep -v amdgpu.ids $D/qorder.log
