#!/bin/bash
# Round-3 evidence of the final code, part 2: kernel trace + three PMC passes of the default bench (gpu_profile.sh),
# their summaries, then the default / orbit / config-4 bench lines.
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r03_final}
scripts/gpu_profile.sh $TAG || exit 1
D=gpurun_out/prof_$TAG
python scripts/trace_frames.py $D/ks_kernel_trace.csv 18 100 > $D/trace_frames.txt 2>&1
python scripts/pmc_passes.py $D $D/passes.txt > /dev/null 2>&1
cat $D/trace_frames.txt $D/passes.txt
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log | cut -c1-300
timeout -k 10 300 python bench.py --orbit 0.01 --no-cpu-baseline > gpurun_out/bench_${TAG}_orbit.log 2>&1 || exit 1
tail -1 gpurun_out/bench_${TAG}_orbit.log | cut -c1-300
timeout -k 10 300 python bench.py --scaling strong > gpurun_out/bench_${TAG}_strong.log 2>&1 || exit 1
tail -1 gpurun_out/bench_${TAG}_strong.log | cut -c1-300
