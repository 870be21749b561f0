#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
PYTHONPATH=. timeout -k 10 300 python scripts/debug_palette3.py > gpurun_out/debug_palette.log 2>&1; rc=$?
echo "debug rc=$rc"; tail -12 gpurun_out/debug_palette.log
[ $rc -gt 1 ] && exit $rc
exit 0
echo "bench rc=$rc"; tail -2 gpurun_out/bench.log
exit $rc
