#!/bin/bash
# A/B: ray lane order 1 (ray-major env blocks) vs 2 (sorted ray tasks), sort interval and bucket sizes.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
run() {  # label, env..., -- bench args
  local label=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --async-probe-groups 0 --ppo-updates 0 $BARGS > $OUT/ab_$label.log 2>&1 || { tail -20 $OUT/ab_$label.log; exit 1; }
  tail -1 $OUT/ab_$label.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$label', round(d['value']/1e6,1), d['kernels_ms'])"
}
BARGS="--ray-order 1" run o1 X=1
BARGS="--ray-order 2" run o2 X=1
BARGS="--ray-order 2 --sort-interval 8" run o2_s8 X=1
BARGS="--ray-order 2 --sort-interval 32" run o2_s32 X=1
BARGS="--ray-order 1" run o1b X=1
BARGS="--ray-order 2" run o2b X=1
timeout -k 10 200 python tools/cull_stats.py 65536 1,16 2,16 2,8 > $OUT/cull_tasks.json 2>&1 || { tail -20 $OUT/cull_tasks.json; exit 1; }
cat $OUT/cull_tasks.json
