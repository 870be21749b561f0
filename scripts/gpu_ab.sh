#!/bin/bash
# A/B of vhx_set_tuning specs on one box: the GPU tests first (FIRST = -k expression, skipped when empty), then for each
# spec in SPECS (";"-separated specs, "|"-separated; "-" = defaults; "+<args>" = extra bench arguments instead of a tuning
# spec, e.g. "+--shadow-mode separate"; "=<VAR=value>" = an environment setting, e.g. "=VHX_LIB=<variant .so>") the bench
# with BENCH_ARGS, twice in alternation.
# Every GPU step under its own time limit; stops at the first failure. usage: TAG=x SPECS="-|qstate=0" gpu_ab.sh
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/${TAG:-ab}; mkdir -p "$D"
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
if [ -n "$FIRST" ]; then
  timeout -k 10 600 $T tests -m gpu -k "$FIRST" > $D/pytest.log 2>&1 || { echo "tests failed"; tail -30 $D/pytest.log; exit 1; }
  tail -2 $D/pytest.log
fi
IFS='|' read -ra S <<< "${SPECS:--}"
for rep in $(seq 1 ${REPS:-2}); do
  for k in "${!S[@]}"; do
    spec=${S[$k]}
    e=""
    if [ "$spec" = "-" ]; then a=""; elif [ "${spec:0:1}" = "+" ]; then a="${spec:1}"; elif [ "${spec:0:1}" = "=" ]; then a=""; e="${spec:1}"; else a="--tune $spec"; fi
    env $e timeout -k 10 300 python3 bench.py --steps ${STEPS:-100} --warmup 10 --no-cpu-baseline --no-extra --no-pmc $BENCH_ARGS $a > $D/b${k}_$rep.log 2>&1 || { echo "bench $spec failed"; tail -5 $D/b${k}_$rep.log; exit 1; }
    python3 - "$D/b${k}_$rep.log" "$spec" <<'PY'
import json, sys
ln = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
d = json.loads(ln)
print(f"{sys.argv[2]:40s} {d['ms_per_step']:.4f} ms/step {d['value']:.0f} Mrays/s frames_equal={d.get('frames_equal')} golden={d.get('golden_match')} eq={(d.get('multi_gpu_check') or {}).get('frame_equal')}")
PY
  done
done
