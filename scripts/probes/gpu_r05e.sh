#!/bin/bash
# Round 5: pass 0 lists its abandoned rays per workgroup in the queue order (ListOrder) instead of flags + the
# count / emit kernels over every pixel. (1) the whole -m gpu suite; (2) the bench line (20 contexts), batches at 4
# queues; (3) the shadow frame's first-pass wave count.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05e; mkdir -p $O
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 120 $T tests/test_abi_c.py tests/test_gpu_batch.py -m gpu -k "consumer or golden" > $O/gpu_first.log 2>&1 || { echo "first tests failed"; tail -30 $O/gpu_first.log; exit 1; }
tail -1 $O/gpu_first.log
timeout -k 10 600 $T tests -m gpu > $O/gpu_all.log 2>&1 || { echo "gpu suite failed"; tail -30 $O/gpu_all.log; exit 1; }
tail -1 $O/gpu_all.log
summ() {
  python - "$1" "$2" <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(l)
lone = d.get("lone") or {}
print(f"{sys.argv[2]:44s} {d['ms_per_step']:.4f} ms/frame {d['value']:.0f} Mrays/s frames_equal {d.get('frames_equal')} golden {d.get('golden_match')} lone {lone.get('ms')}")
PY
}
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pmc"
for round in 1 2; do
  f=$O/bench_default_r$round.log
  timeout -k 10 300 $B > $f 2>&1 || { echo "bench failed"; tail -20 $f; exit 1; }
  summ $f "default (20 contexts) r$round"
  for cfg in "--batch 20 --inflight 1" "--batch 10 --inflight 2" "--batch 7 --inflight 3"; do
    f=$O/bench_r${round}_$(echo "$cfg" | tr -c 'a-zA-Z0-9\n' '_').log
    timeout -k 10 200 $B --no-extra $cfg > $f 2>&1 || { echo "bench failed: $cfg"; tail -20 $f; exit 1; }
    summ $f "$cfg r$round"
  done
done
for q in 2048 3072 4096 6144 8192; do
  f=$O/shadows_qw$q.log
  timeout -k 10 200 $B --no-extra --shadows --tune "qwaves0=$q" > $f 2>&1 || { echo "shadow bench failed: $q"; tail -20 $f; exit 1; }
  summ $f "shadows qwaves0=$q"
done
