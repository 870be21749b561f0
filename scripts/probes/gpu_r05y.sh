#!/bin/bash
# Round 5: is pass 1's memory wait in the batch default a footprint effect (seven frames' saved states, ~280 MB,
# beyond the 256 MB Infinity Cache)? Per-pass PMC of batches of 3 on 3 contexts (~120 MB of state per batch) against
# batches of 7.
cd "$GRAFT_REPO_ROOT" || exit 1
SKIP=14 GSKIP=5 timeout -k 10 600 bash scripts/gpu_profile.sh r05_b3 --batch 3 --inflight 3 > gpurun_out/r05y_b3.log 2>&1 || { echo "b3 profile failed"; tail -5 gpurun_out/r05y_b3.log; exit 1; }
grep "pass [01]:" gpurun_out/prof_r05_b3/passes.txt
