#!/bin/bash
# Round 5: (1) the test order that lost the GPU in round 4 (loopback rank children first, then the parent's first HIP
# use), now with vhx_device_count's error text; (2) config 5 profiled like the headline (per-pass PMC incl. the shadow
# passes).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05b; mkdir -p $O
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 500 $T tests/test_gpu_mgpu_ranks.py tests/test_gpu_multigpu.py -m gpu > $O/ranks_then_multigpu.log 2>&1; echo "ranks then multigpu rc=$?"
tail -3 $O/ranks_then_multigpu.log
grep -n "vhx_device_count\|No HIP\|hipError\|libvhx error" $O/ranks_then_multigpu.log | head -10
PPASSES=5 timeout -k 10 700 bash scripts/gpu_profile.sh r05_c5 --shadows; echo "profile rc=$?"
timeout -k 10 300 python scripts/probes/probe_cumask.py > $O/cumask.log 2>&1; echo "cumask rc=$?"; tail -30 $O/cumask.log
