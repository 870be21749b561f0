#!/bin/bash
# Variant builds (scratch/var/libvhx_<name>.so) against the default build on the secondary configs (bench.py,
# 20 frames, eight frames in flight), alternating, each twice
cd "$GRAFT_REPO_ROOT" || exit 1
for rep in 1 2; do
  for cfg in "--size 256 --brick-dim 16 --width 1920 --height 1080" "--size 512 --brick-dim 8 --width 1920 --height 1080" \
             "--size 1024 --brick-dim 16" "--vox scratch/gingerbread_house_by_kirra_luan.vox --brick-dim 8"; do
    for v in base ${VARIANTS}; do
      if [ "$v" = base ]; then unset VHX_LIB; else export VHX_LIB=scratch/var/libvhx_$v.so; fi
      r=$(timeout -k 10 200 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-roofline $cfg 2>&1 | tail -1 | python -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])") || exit 1
      echo "$v | $cfg | $r ms"
    done
  done
done
