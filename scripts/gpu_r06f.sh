# round 6: tile-set batches and the batched multi-GPU path (tests, then one-rank config-4 benches)
mkdir -p gpurun_out/r06f
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests -m gpu -k "tiles_batch or render_batch or bench_mgpu or one_rank or batch" > gpurun_out/r06f/pytest.log 2>&1 || { tail -40 gpurun_out/r06f/pytest.log; exit 1; }
tail -2 gpurun_out/r06f/pytest.log
for v in "" "--batch 4" "--batch 0"; do
  VHX_BENCH_MGPU1=1 timeout -k 10 300 python3 bench.py --scaling strong --steps 21 --warmup 7 --no-cpu-baseline --no-extra --no-pmc $v > gpurun_out/r06f/c4m.log 2>&1 || { tail -20 gpurun_out/r06f/c4m.log; exit 1; }
  echo "mgpu1 c4 [$v]"; grep "^{" gpurun_out/r06f/c4m.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'], d['batch'], d['contexts_in_flight'], d['multi_gpu_check'])"
done
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-pmc > gpurun_out/r06f/bench.log 2>&1 || { tail -20 gpurun_out/r06f/bench.log; exit 1; }
grep "^{" gpurun_out/r06f/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('headline', d['ms_per_step'], d['value'], d['frames_equal'], d['golden_match'], 'lone', d['lone']['ms'], 'scaling_n1', d.get('scaling_n1'))"
