#!/bin/bash
# Repeated bench runs of one configuration under alternating env settings ($ENVS: '+'-joined items), args after.
cd "$GRAFT_REPO_ROOT" || exit 1
for rep in 1 2 3; do
  for item in $ENVS; do
    envs="$(echo "$item" | tr '+' ' ')"
    r=$(env $envs timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-roofline "$@" 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])") || exit 1
    echo "[$item] $r"
  done
done
