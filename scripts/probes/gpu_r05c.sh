#!/bin/bash
# Round 5: (1) the loopback rank tests, then the first in-process HIP use through libvhx (conftest's gpu fixture no
# longer initialises torch first); (2) the whole -m gpu suite; (3) the shadow frame's first queue pass, whose waves
# wait on memory 82 % of their cycles (prof_r05_c5): XCD-dealt chunks and its wave count.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05c; mkdir -p $O
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_mgpu_ranks.py tests/test_gpu_multigpu.py -m gpu > $O/ranks_then_multigpu.log 2>&1 || { echo "subset failed"; grep -n "vhx_device_count\|No HIP\|hipError\|Error" $O/ranks_then_multigpu.log | head; tail -20 $O/ranks_then_multigpu.log; exit 1; }
tail -1 $O/ranks_then_multigpu.log
timeout -k 10 600 $T tests -m gpu > $O/gpu_all.log 2>&1 || { echo "gpu suite failed"; tail -30 $O/gpu_all.log; exit 1; }
tail -1 $O/gpu_all.log
for tune in "" "qxcd_all=1" "qwaves0=4096" "qwaves0=16384" "qxcd_all=1;qwaves0=16384"; do
  f=$O/shadows_$(echo "x$tune" | tr -c 'a-zA-Z0-9\n' '_').log
  timeout -k 10 200 python bench.py --shadows --steps 20 --warmup 5 --no-cpu-baseline --no-pmc --no-extra ${tune:+--tune "$tune"} > $f 2>&1 || { echo "shadow bench failed: $tune"; tail -20 $f; exit 1; }
  python - "$f" "$tune" <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(l)
print(f"shadows tune [{sys.argv[2]}]: {d['ms_per_step']:.4f} ms/frame, {d['value']:.0f} Mrays/s, frames_equal {d.get('frames_equal')}")
PY
done
