#!/bin/bash
# Secondary BASELINE configs: config 2 variants, config 3 variants, config 5 (shadows).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/configs
run() {
  local tag="$1"; shift
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 "$@" > "gpurun_out/configs/$tag.log" 2>&1; local rc=$?
  echo "$tag rc=$rc $(tail -1 "gpurun_out/configs/$tag.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d.get('cpu_baseline') or {}; r=d.get('roofline') or {}; print(d['value'], 'Mrays/s', d['ms_per_step'], 'ms', 'cpu', c.get('value'), 'frac', r.get('frac'))")"
  return $rc
}
run c2_256_bd4 --size 256 --brick-dim 4 --width 1920 --height 1080 && \
run c2_256_bd16 --size 256 --brick-dim 16 --width 1920 --height 1080 && \
run c2_128_bd8 --size 128 --brick-dim 8 --width 1920 --height 1080 && \
run c2_512_bd8 --size 512 --brick-dim 8 --width 1920 --height 1080 && \
run c3_1024_bd16 --size 1024 --brick-dim 16 --no-cpu-baseline && \
run c3_heightfield --scene 6 --no-cpu-baseline && \
run c5_shadows --shadows && \
run c5_shadows_f1 --shadows --inflight 1 && \
run c3_headline_f1 --inflight 1 --no-cpu-baseline && \
if [ -f scratch/gingerbread_house_by_kirra_luan.vox ]; then
  run c3_vox_gingerbread_bd8 --vox scratch/gingerbread_house_by_kirra_luan.vox --brick-dim 8 && \
  run c3_vox_gingerbread_bd4 --vox scratch/gingerbread_house_by_kirra_luan.vox --brick-dim 4
fi
