#!/bin/bash
# End-of-session GPU check: smoke, the whole -m gpu suite, and a kernel trace of the MIP stand-in bench (depth 1).
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-final}
mkdir -p gpurun_out/$TAG
R="$GRAFT_REPO_ROOT"; D="$R/gpurun_out/$TAG"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $D/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $D/pytest_gpu.log 2>&1 || { echo "gpu suite failed"; tail -30 $D/pytest_gpu.log; exit 1; }
tail -1 $D/pytest_gpu.log
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -f csv -d "$D/prof_miplod1" -o ks -- python3 "$R/bench.py" --mip-lod 1 --steps 50 --warmup 5 > "$D/prof_miplod1.log" 2>&1 || { echo "miplod trace failed"; tail -5 "$D/prof_miplod1.log"; exit 1; }
tail -1 "$D/prof_miplod1.log" | cut -c1-200
find "$D" -name "*stats*.csv"
