#!/bin/bash
# Round 5: saved state at the pass-0 list slot (PassQ::map): the whole -m gpu suite, then A/B against the previous
# (VHX_LIB=libvhx_idxstate.so) in the batch default and the twenty-context line, two rounds, one box.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05z; mkdir -p $O
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests -m gpu > $O/gpu_all.log 2>&1 || { echo "gpu suite failed"; tail -30 $O/gpu_all.log; exit 1; }
tail -1 $O/gpu_all.log
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pmc"
for round in 1 2; do
  for lib in "" voxelhex_amd/_lib/libvhx_idxstate.so; do
    for cfg in "" "--batch 0 --no-extra"; do
      f=$O/r${round}_$(echo "x$lib$cfg" | tr -c 'a-zA-Z0-9\n' '_').log
      VHX_LIB=$lib timeout -k 10 200 $B $cfg > $f 2>&1 || { echo "bench failed: $lib $cfg"; tail -20 $f; exit 1; }
      python - "$f" "${lib:-libvhx.so (slot state)} ${cfg:-batch 7x3} r$round" <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(l)
lone = d.get("lone") or {}
print(f"{sys.argv[2]:64s} {d['ms_per_step']:.4f} ms/frame {d['value']:.0f} Mrays/s frames_equal {d.get('frames_equal')} golden {d.get('golden_match')} lone {lone.get('ms')}")
PY
    done
  done
done
