#!/bin/bash
# Round 5 (lead for round 6): per-pass L2 (TCC) hit rates of the batch default (7 x 3) and of batches of 3, to see
# what pass 1 waits on (68 % vs 48 % memory waits)
cd "$GRAFT_REPO_ROOT" || exit 1
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
for cfg in "7 3 26 4" "3 3 14 5"; do
  set -- $cfg
  D="$R/gpurun_out/prof_r05_tcc_b$1"; mkdir -p "$D"
  timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -f csv -d "$D" -o pmc0 -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --no-pmc --no-frame-check --no-extra --batch $1 --inflight $2 > "$D/pmc0.log" 2>&1 || { echo "pmc failed b$1"; tail -5 "$D/pmc0.log"; exit 1; }
  (cd "$R" && python3 scripts/pmc_passes.py "$D" "$D/passes.txt" --inflight-only --skip $4)
done
