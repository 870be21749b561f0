#!/bin/bash
# Round 5 check: streaming GPU tests after the incremental view-set rebuild, the 4K / 1024^3 streaming frame at K = 1
# (and K frames per upload with 8 contexts), config 5 with its roofline / CPU baseline, and the SQ counter list.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r05a
O=gpurun_out/r05a
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_streaming.py tests/test_gpu_ordering.py -m gpu > $O/pytest_streaming.log 2>&1 || { echo "streaming tests failed"; tail -30 $O/pytest_streaming.log; exit 1; }
tail -1 $O/pytest_streaming.log
timeout -k 10 300 python scripts/bench_streaming.py 100 --size 1024 --width 3840 --height 2160 > $O/streaming_k1.log 2>&1 || { echo "streaming k1 failed"; tail -20 $O/streaming_k1.log; exit 1; }
tail -4 $O/streaming_k1.log
timeout -k 10 400 python scripts/bench_streaming.py 80 --size 1024 --width 3840 --height 2160 --inflight 8 --batches 1,4,8 > $O/streaming_batches.log 2>&1 || { echo "streaming batches failed"; tail -20 $O/streaming_batches.log; exit 1; }
tail -6 $O/streaming_batches.log
timeout -k 10 400 python bench.py --shadows --steps 20 --warmup 5 > $O/c5_shadows.log 2>&1 || { echo "shadow bench failed"; tail -20 $O/c5_shadows.log; exit 1; }
tail -1 $O/c5_shadows.log | cut -c1-600
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1; echo "counter list rc=$?"
