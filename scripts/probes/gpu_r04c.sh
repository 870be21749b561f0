#!/bin/bash
# Round 4: lead-off default check, the default bench profile (F = 20, in-flight-only PMC) and the batched streaming view
# at 4K / 1024^3 (K = 1, 4, 8).
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/${1:-r04c}; mkdir -p $D
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_lead.py \
  tests/test_gpu_inflight.py > $D/pytest.log 2>&1 || { tail -30 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
bash scripts/gpu_profile.sh ${1:-r04c} || exit 1
timeout -k 10 400 python -u scripts/bench_streaming.py 48 --inflight 8 --batches 1,4,8 --size 1024 --width 3840 \
  --height 2160 > $D/streaming.log 2>&1 || { tail -20 $D/streaming.log; exit 1; }
tail -12 $D/streaming.log
