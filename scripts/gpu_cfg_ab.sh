cd "$GRAFT_REPO_ROOT" || exit 1
for env in "VHX_XCDG=16 VHX_QXCD=16" "VHX_XCDG=0 VHX_QXCD=16" "VHX_XCDG=16 VHX_QXCD=0" "VHX_XCDG=0 VHX_QXCD=0"; do
  for args in "--size 256 --brick-dim 4 --width 1920 --height 1080" "--vox scratch/gingerbread_house_by_kirra_luan.vox --brick-dim 8" "--scene 6"; do
    r=$(env $env timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline $args 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])") || exit 1
    echo "[$env] [$args] $r"
  done
done
