#!/bin/bash
# Lone-frame schedule sweep and the queue-wave sweep under frames in flight (evidence for ctx.hpp's Sched defaults).
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/${1:-r03d}; mkdir -p $D
scripts/probes/probe_lone_r03.sh > $D/lone.log 2>&1 || { tail -20 $D/lone.log; exit 1; }
cat $D/lone.log
scripts/probes/probe_qwaves_r03.sh > $D/qwaves.log 2>&1 || { tail -20 $D/qwaves.log; exit 1; }
cat $D/qwaves.log
