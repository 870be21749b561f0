#!/bin/bash
# Round 5: pass ladders for the batch default (batches of 7 on 3 contexts): budgets, pass-0 sparse threshold, queue
# waves, and pass 0 at 8 waves per SIMD (VHX_LIB=libvhx_p0w8.so: VHX_PRIMARY_WPE=8, 64 VGPRs + 32 B scratch); two
# rounds, one box.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05k; mkdir -p $O
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pmc --no-extra"
for round in 1 2; do
  for tune in "" "budgets=32,96,288,864" "budgets=16,48,144,432,1296" "budgets=24,64,192,576" "budgets=24,96,384,1536" "budgets=24,48,96,216,648" "sparse=16" "sparse=8" "qwaves=1024" "budgets=20,60,180,540"; do
    f=$O/r${round}_$(echo "x$tune" | tr -c 'a-zA-Z0-9\n' '_').log
    timeout -k 10 200 $B ${tune:+--tune "$tune"} > $f 2>&1 || { echo "bench failed: $tune"; tail -20 $f; exit 1; }
    python - "$f" "${tune:-default} r$round" <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(l)
print(f"{sys.argv[2]:40s} {d['ms_per_step']:.4f} ms/frame {d['value']:.0f} Mrays/s frames_equal {d.get('frames_equal')} golden {d.get('golden_match')}")
PY
  done
  for lib in "" "voxelhex_amd/_lib/libvhx_p0w8.so"; do
    for cfg in "" "--batch 0"; do
      f=$O/occ_r${round}_$(echo "x$lib$cfg" | tr -c 'a-zA-Z0-9\n' '_').log
      VHX_LIB=$lib timeout -k 10 200 $B $cfg > $f 2>&1 || { echo "bench failed: $lib $cfg"; tail -20 $f; exit 1; }
      python - "$f" "${lib:-libvhx.so} ${cfg:-batch 7x3} r$round" <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(l)
print(f"{sys.argv[2]:60s} {d['ms_per_step']:.4f} ms/frame {d['value']:.0f} Mrays/s frames_equal {d.get('frames_equal')} golden {d.get('golden_match')}")
PY
    done
  done
done
