#!/bin/bash
# Secondary BASELINE configs with the round-5 default (batches of 7 on 3 contexts at N = 1) and, for
# config 2, the twenty-context line beside it (--batch 0): small frames fill the chip better in batches.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/configs_r05
run() {
  local tag="$1"; shift
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 "$@" > "gpurun_out/configs_r05/$tag.log" 2>&1; local rc=$?
  echo "$tag rc=$rc $(tail -1 "gpurun_out/configs_r05/$tag.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d.get('cpu_baseline') or {}; r=d.get('roofline') or {}; print(d['value'], 'Mrays/s', d['ms_per_step'], 'ms', 'cpu', c.get('value'), 'frac', r.get('frac'), 'batch', d.get('batch'), 'equal', d.get('frames_equal'), d.get('golden_match'))")"
  return $rc
}
run c2_256_bd4 --size 256 --brick-dim 4 --width 1920 --height 1080 && \
run c2_256_bd4_ctx20 --size 256 --brick-dim 4 --width 1920 --height 1080 --batch 0 && \
run c2_256_bd16 --size 256 --brick-dim 16 --width 1920 --height 1080 && \
run c2_128_bd8 --size 128 --brick-dim 8 --width 1920 --height 1080 && \
run c2_512_bd8 --size 512 --brick-dim 8 --width 1920 --height 1080 && \
run c2_512_bd8_ctx20 --size 512 --brick-dim 8 --width 1920 --height 1080 --batch 0 && \
run c3_1024_bd16 --size 1024 --brick-dim 16 --no-cpu-baseline && \
run c3_heightfield --scene 6 --no-cpu-baseline && \
run c3_orbit --orbit 0.01 --no-cpu-baseline && \
run c4_strong_1gpu --scaling strong --no-cpu-baseline
