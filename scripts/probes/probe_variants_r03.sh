#!/bin/bash
# A/B of libvhx build variants on the bench frame (diagnostics): each variant (voxelhex_amd/_lib/var_<name>/libvhx.so,
# built by voxelhex_amd/_build.py with a -D define) and the default build run the bench twice, interleaved.
#   scripts/probes/probe_variants_r03.sh OUT_DIR name1 name2 ...
set -euo pipefail
out=$1; shift
mkdir -p "$out"
for rep in 1 2; do
  timeout -k 10 240 python bench.py --no-cpu-baseline --no-pmc --no-roofline --steps 300 > "$out/default_$rep.log" 2>&1
  for v in "$@"; do
    VHX_LIB=voxelhex_amd/_lib/var_$v/libvhx.so timeout -k 10 240 python bench.py --no-cpu-baseline --no-pmc \
      --no-roofline --steps 300 > "$out/${v}_$rep.log" 2>&1
  done
done
python - "$out" <<'PY'
import glob, json, os, sys
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.log"))):
    line = [l for l in open(f) if l.startswith("{")]
    if line:
        d = json.loads(line[0])
        print(f"{os.path.basename(f):24s} {d['ms_per_step']:.4f} ms  frames_equal={d.get('frames_equal')}")
PY
