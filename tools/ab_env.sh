#!/bin/bash
# Same-session A/B of env-variable knobs on bench.py (one library):
#   AB_SETS="label|ENV=V ENV2=V;label2|ENV=W" bash tools/ab_env.sh
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
IFS=';' read -ra SETS <<< "$AB_SETS"
for rep in 1 2 3; do
for set in "${SETS[@]}"; do
  IFS='|' read -r label envs <<< "$set"
  env $envs timeout -k 10 200 python bench.py --steps 1000 --warmup 100 --no-cpu-baseline --async-probe-groups 0 --ppo-updates 0 --no-time-to-90 > $OUT/abe_$label.log 2>&1 || { tail -20 $OUT/abe_$label.log; exit 1; }
  tail -1 $OUT/abe_$label.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$label', round(d['value']/1e6,1), d['kernels_ms'])"
done
done
