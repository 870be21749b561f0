#!/bin/bash
# Round 5: queue-kernel occupancy in the batch default: 5 waves per SIMD (94 VGPRs, no scratch; the shipped build)
# against probe builds at 6 (80 VGPRs + 60 B scratch) and 7 (72 + 104 B) -- the queue passes wait on memory 38-67 %
# of their cycles there. Two rounds, one box.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05n; mkdir -p $O
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pmc --no-extra"
for round in 1 2; do
  for lib in "" voxelhex_amd/_lib/libvhx_q6.so voxelhex_amd/_lib/libvhx_q7.so; do
    for cfg in "" "--batch 0"; do
      f=$O/r${round}_$(echo "x$lib$cfg" | tr -c 'a-zA-Z0-9\n' '_').log
      VHX_LIB=$lib timeout -k 10 200 $B $cfg > $f 2>&1 || { echo "bench failed: $lib $cfg"; tail -20 $f; exit 1; }
      python - "$f" "${lib:-libvhx.so} ${cfg:-batch 7x3} r$round" <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(l)
print(f"{sys.argv[2]:56s} {d['ms_per_step']:.4f} ms/frame {d['value']:.0f} Mrays/s frames_equal {d.get('frames_equal')} golden {d.get('golden_match')}")
PY
    done
  done
done
