#!/bin/bash
# Round 5: pass-0 list parity at odd frame sizes, and smoke() (single frame + a two-frame batch against the oracle)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05u; mkdir -p $O
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_lists.py -m gpu > $O/pytest_lists.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest_lists.log; exit 1; }
tail -1 $O/pytest_lists.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
