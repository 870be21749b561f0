#!/bin/bash
# Profiles of the driver's bench command for profiles/<round>/ (round 4: only timed, in-flight frames are summarised):
# kernel trace + stats of `bench.py --steps 20 --warmup 5`, then FETCH_SIZE (memory-side read bytes) and two passes of
# SQ counters (issue, lanes) over the same command, each pass a run of its own (rocprofv3 does not split counters over
# passes; MI355X_MICROARCH.md). The PMC runs skip the frame check and the lone / orbit extras, and pmc_passes.py keeps
# only frames-in-flight frames after the setup and warm-up frames (SKIP frames / GSKIP pass-0 groups, defaults below). PPASSES=5 with --shadows labels a frame's dispatches after the first 5 as the shadow
# trace's passes. usage: [SKIP=n] [PPASSES=p] gpu_profile.sh TAG [bench args...]
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; shift
R="$GRAFT_REPO_ROOT"; D="$R/gpurun_out/prof_$TAG"; mkdir -p "$D"
cd /tmp && export TMPDIR=/tmp
B="--steps 20 --warmup 5 --no-cpu-baseline"
timeout -s KILL 180 rocprofv3 --kernel-trace --stats -f csv -d "$D" -o ks -- python3 "$R/bench.py" $B --no-pmc "$@" > "$D/ks.log" 2>&1 || { echo "kernel trace failed"; tail -5 "$D/ks.log"; exit 1; }
tail -1 "$D/ks.log" | cut -c1-300
P0="FETCH_SIZE"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH"
P2="SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
j=0
for P in "$P0" "$P1" "$P2"; do
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace -f csv -d "$D" -o "pmc$j" -- python3 "$R/bench.py" $B --no-roofline --no-pmc --no-frame-check --no-extra "$@" > "$D/pmc$j.log" 2>&1; rc=$?
  echo "pmc pass $j rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$D/pmc$j.log"; exit $rc; }
  j=$((j+1))
done
# bench.py's default at N = 1 (round 5): batches of 7 frames on 3 contexts -- 3 setup batches + a warm-up batch of 5,
# 26 frames in 4 pass-0 groups; frames one at a time (--batch 0, --shadows): 20 setup + 5 warm-up frames
case " $* " in
  *" --shadows "*|*" --batch 0 "*) DSKIP=25; DGSKIP=25 ;;
  *) DSKIP=26; DGSKIP=4 ;;
esac
cd "$R" && python3 scripts/pmc_passes.py "$D" "$D/passes.txt" --inflight-only --skip "${GSKIP:-$DGSKIP}" ${PPASSES:+--primary-passes $PPASSES} && \
  python3 scripts/trace_frames.py "$(find "$D" -name "ks_kernel_trace.csv" | head -1)" "${SKIP:-$DSKIP}" 20 > "$D/trace_frames.txt" 2>&1
tail -5 "$D/trace_frames.txt"
