#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/${1:-r03i}; mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "scheduler_variants or multipass or full_size_frame or ragged" > $D/parity.log 2>&1 || { tail -30 $D/parity.log; exit 1; }
tail -1 $D/parity.log
scripts/probes/probe_qorder_r03.sh $ORDERS > $D/qorder.log 2>&1 || { tail -20 $D/qorder.log; exit 1; }
grep -v amdgpu.ids $D/qorder.log
