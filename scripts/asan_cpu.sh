#!/bin/bash
# Host-side sanitizer run (SURVEY.md §5 "race detection / sanitizers"; GPU sanitizers are not available on this pool):
# the host C++ of libvhx (BoxTree restatement, flattener, .vox parser, streaming producer) and the oracle are built
# with -fsanitize=address,undefined into build/asan/, and the CPU test suite runs against those builds with the GCC
# sanitizer runtimes preloaded (the Python interpreter itself is not instrumented). Any ASan / UBSan report aborts the
# test process (halt_on_error), so a clean run = pytest green.
#   scripts/asan_cpu.sh [pytest args]      (default: tests -m "not gpu" -q)
# Log of the last clean run: profiles/r03/asan_cpu.log
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
OUT="$ROOT/build/asan"
SAN="-fsanitize=address,undefined -fno-omit-frame-pointer -fno-sanitize-recover=undefined -g"
mkdir -p "$OUT"
python3 - <<PY
import sys
sys.path.insert(0, "$ROOT")
from voxelhex_amd import _build
_build.build(verbose=False, force=True, lib="$OUT/libvhx.so", build_dir="$OUT/obj", host_flags=tuple("$SAN".split()))
PY
make -s -C "$ROOT/oracle" OUT="$OUT/oracle" EXTRA_CFLAGS="$SAN" >/dev/null
PRE="$(gcc -print-file-name=libasan.so):$(gcc -print-file-name=libubsan.so)"
cd "$ROOT"
if [ $# -eq 0 ]; then set -- tests -m "not gpu" -q -p no:cacheprovider; fi
export VHX_LIB="$OUT/libvhx.so" VHX_ORACLE_LIB="$OUT/oracle/liboracle.so"
export ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:abort_on_error=1:protect_shadow_gap=0:verify_asan_link_order=0"
export UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1"
echo "sanitized builds: $VHX_LIB $VHX_ORACLE_LIB; preload $PRE"
LD_PRELOAD="$PRE" python3 -m pytest "$@"
