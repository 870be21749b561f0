#!/bin/bash
# Round-3 evidence of the final code, part 1: the secondary BASELINE configs with the adaptive schedule.
cd "$GRAFT_REPO_ROOT" || exit 1
scripts/gpu_configs.sh
