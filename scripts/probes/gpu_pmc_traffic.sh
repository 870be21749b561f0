#!/bin/bash
# PMC passes (FETCH_SIZE, then TCC_EA0_RDREQ_sum; each beside --kernel-trace only) over the default bench command,
# summarised into profiles/traffic.json by scripts/pmc_traffic.py.
cd "$GRAFT_REPO_ROOT" || exit 1
R="$GRAFT_REPO_ROOT"
D="$R/gpurun_out/pmc_traffic"
mkdir -p "$D"
cd /tmp && export TMPDIR=/tmp
i=0
for P in FETCH_SIZE TCC_EA0_RDREQ_sum; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P --kernel-trace -f csv -d "$D" -o p$i -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-roofline > "$D/p$i.log" 2>&1; rc=$?
  echo "pmc pass $i ($P) rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
cd "$R" && python3 scripts/pmc_traffic.py "$D" "primary 3840x2160 S1 1024^3 bd4 ranks1" gpurun_out/traffic.json
