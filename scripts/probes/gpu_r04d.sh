#!/bin/bash
# Round 4: streaming GPU tests after the deferred rebuild, then the 4K / 1024^3 streaming view one frame at a time
# (breakdown) and batched at K = 1, 4, 8 with eight frames in flight.
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/${1:-r04d}; mkdir -p $D
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_streaming.py \
  tests/test_gpu_ordering.py > $D/pytest.log 2>&1 || { tail -30 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
timeout -k 10 300 python -u scripts/bench_streaming.py 24 --size 1024 --width 3840 --height 2160 > $D/streaming_f1.log 2>&1 \
  || { tail -20 $D/streaming_f1.log; exit 1; }
tail -5 $D/streaming_f1.log
timeout -k 10 400 python -u scripts/bench_streaming.py 48 --inflight 8 --batches 1,4,8 --size 1024 --width 3840 \
  --height 2160 > $D/streaming.log 2>&1 || { tail -20 $D/streaming.log; exit 1; }
tail -12 $D/streaming.log
