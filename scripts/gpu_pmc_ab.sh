#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
VHX_SIMPLE_KERNEL=1 bash scripts/gpu_pmc.sh simple || exit $?
VHX_SIMPLE_KERNEL=0 bash scripts/gpu_pmc.sh persist || exit $?
