#!/bin/bash
# Round 4, first GPU check: the tuning / ordering / golden / lead tests, the lead-block probe, the driver's bench command,
# frames in flight at it.
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/${1:-r04a}; mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_lead.py \
  tests/test_gpu_tuning.py tests/test_gpu_ordering.py \
  "tests/test_gpu_golden.py::test_gpu_frame_matches_golden[c3_1024_bd4_3840x2160]" \
  tests/test_gpu_mgpu_ranks.py > $D/pytest.log 2>&1 || { tail -40 $D/pytest.log; exit 1; }
tail -3 $D/pytest.log
timeout -k 10 300 python -u scripts/probes/probe_lead.py "lead=0" "lead=1;lead_min=256" "lead=1;lead_min=512" \
  "lead=1;lead_min=1000" "lead=1;lead_min=256;lead_cap=1024" "lead=1;lead_min=128;lead_cap=512" > $D/lead.log 2>&1 \
  || { tail -20 $D/lead.log; exit 1; }
cat $D/lead.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $D/bench.log 2>&1 || { tail -20 $D/bench.log; exit 1; }
tail -1 $D/bench.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["frames_equal"], d["golden_match"], d["roofline"]["frac"], json.dumps(d.get("lone")), json.dumps(d.get("orbit")))'
REPS=2 FS="12 16 20" bash scripts/probes/gpu_r04_k20.sh ${1:-r04a}/k20 || exit 1
REPS=2 FS="16" EXTRA="--tune lead=1" bash scripts/probes/gpu_r04_k20.sh ${1:-r04a}/k20_lead
