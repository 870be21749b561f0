#!/bin/bash
# Round 5: block-execution counts of the traversal (VHX_PROF build) for the frames-in-flight ladder and the lone-frame
# ladder, to weight the ISA census (profiles/r05/isa/) per block.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05o; mkdir -p $O
VHX_LIB=voxelhex_amd/_lib/prof/libvhx.so timeout -k 10 300 python scripts/probes/probe_blocks.py --budgets 24,72,216,648 --json $O/blocks_busy.json > $O/blocks_busy.txt 2>&1 || { echo "probe failed"; tail -20 $O/blocks_busy.txt; exit 1; }
cat $O/blocks_busy.txt
VHX_LIB=voxelhex_amd/_lib/prof/libvhx.so timeout -k 10 300 python scripts/probes/probe_blocks.py --budgets 64 --json $O/blocks_idle.json > $O/blocks_idle.txt 2>&1 || { echo "probe failed"; tail -20 $O/blocks_idle.txt; exit 1; }
cat $O/blocks_idle.txt
