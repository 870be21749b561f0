#!/bin/bash
# Round 5: k_gather_chunks dispatch durations, wave-cooperative (libvhx.so) against per-chunk (libvhx_oldgather.so),
# kernel traces of the batch default and of the twenty-context line
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05s; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for lib in "" voxelhex_amd/_lib/libvhx_oldgather.so; do
  for cfg in "" "--batch 0"; do
    tag=$(echo "x$lib$cfg" | tr -c 'a-zA-Z0-9\n' '_')
    VHX_LIB=$lib timeout -s KILL 240 rocprofv3 --kernel-trace --stats -f csv -d $O/kt$tag -o ks -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pmc --no-extra --no-frame-check $cfg > $O/kt$tag.log 2>&1 || { echo "trace failed $tag"; tail -5 $O/kt$tag.log; exit 1; }
    echo "== ${lib:-new gather} ${cfg:-batch}"; grep -h "k_gather_chunks\|k_scan_counts\|k_scan_sums" $O/kt$tag/ks_kernel_stats.csv | cut -d, -f1-4
  done
done
