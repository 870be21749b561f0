#!/bin/bash
# Variant builds of libvhx (scratch/var/libvhx_<name>.so, e.g. compiler scheduling strategies) against the default
# build, bench frame at eight frames in flight, alternating, each twice
cd "$GRAFT_REPO_ROOT" || exit 1
export GPU_MAX_HW_QUEUES=12 VHX_PROBE_F=8
for rep in 1 2; do
  for v in base ${VARIANTS}; do
    if [ "$v" = base ]; then unset VHX_LIB; else export VHX_LIB=scratch/var/libvhx_$v.so; fi
    echo "$v $(timeout -k 10 120 python scripts/probes/probe_sched_inflight.py 24,96,768 2>&1 | grep budgets)" || exit 1
  done
done
