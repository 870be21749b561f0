#!/bin/bash
# The multi-rank vhx_mgpu tests over the loopback communicator.
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/${1:-r03e}; mkdir -p $D
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_mgpu_ranks.py > $D/mgpu_ranks.log 2>&1 || { tail -60 $D/mgpu_ranks.log; exit 1; }
grep -E "PASS|FAIL|rank |root_slots" $D/mgpu_ranks.log | head -80
tail -3 $D/mgpu_ranks.log
