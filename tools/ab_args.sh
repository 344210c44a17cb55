#!/bin/bash
# A/B of bench.py argument sets: AB_SETS="label1:args1;label2:args2" bash tools/ab_args.sh
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
IFS=';' read -ra SETS <<< "$AB_SETS"
for rep in 1 2; do
for set in "${SETS[@]}"; do
  label=${set%%:*}; args=${set#*:}
  timeout -k 10 200 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --async-probe-groups 0 --ppo-updates 0 $args > $OUT/ab_$label.log 2>&1 || { tail -20 $OUT/ab_$label.log; exit 1; }
  tail -1 $OUT/ab_$label.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$label', round(d['value']/1e6,1), d['kernels_ms'])"
done
done
