#!/bin/bash
# Batch mode (vhx_trace_primary_batch) on the GPU box: its tests, then the driver's bench command per batch shape, at
# the box's default hardware queues (bench.py leaves GPU_MAX_HW_QUEUES alone in batch mode). Each step has its own time
# limit; the script stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-batch}
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
if [ -z "$NOTEST" ]; then
  timeout -k 10 600 $T tests/test_gpu_batch.py -m gpu > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "batch tests failed"; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
  tail -2 gpurun_out/${TAG}_pytest.log
fi
B="python bench.py --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline --no-pmc --no-extra"
# CFGS: bench configurations separated by '|'
IFS='|' read -r -a cfgs <<< "${CFGS:---inflight 20|--batch 20 --inflight 1|--batch 20 --inflight 2|--batch 10 --inflight 2}"
for cfg in "${cfgs[@]}"; do
  name=$(echo $cfg | tr -d ' -')
  timeout -k 10 300 $B $cfg $EXTRA > gpurun_out/${TAG}_bench_$name.log 2>&1 || { echo "bench $cfg failed"; tail -20 gpurun_out/${TAG}_bench_$name.log; exit 1; }
  python - gpurun_out/${TAG}_bench_$name.log "$cfg" << 'PY'
import json, sys
l = json.loads([x for x in open(sys.argv[1]) if x.startswith("{")][-1])
print(f"{sys.argv[2]:28s} ms/frame {l['ms_per_step']:.4f}  Mrays/s {l['value']:.0f}  queues {l['gpu_max_hw_queues']}  frames_equal {l.get('frames_equal')} golden {l.get('golden_match')}")
PY
done
