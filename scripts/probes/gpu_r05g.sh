#!/bin/bash
# Round 5: kernel traces of the bench frame (20 contexts) with pass-0 flags (p0lists=0) and pass-0 lists (p0lists=1)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05g; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in 0 1; do
  timeout -s KILL 240 rocprofv3 --kernel-trace --stats -f csv -d $O/kt_p0lists$v -o ks -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pmc --no-extra --no-frame-check --tune "p0lists=$v" > $O/kt_p0lists$v.log 2>&1 || { echo "trace $v failed"; tail -5 $O/kt_p0lists$v.log; exit 1; }
  tail -1 $O/kt_p0lists$v.log | cut -c1-200
  python3 scripts/trace_frames.py $O/kt_p0lists$v/ks_kernel_trace.csv 25 20 > $O/trace_frames_p0lists$v.txt 2>&1; cat $O/trace_frames_p0lists$v.txt
done
