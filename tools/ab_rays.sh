#!/bin/bash
# A/B of raycast scheduling options on the headline bench (k_rays events).
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
: > "$OUT/ab_rays.jsonl"
while IFS= read -r a; do
  [ -z "$a" ] && continue
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 300 $a > "$OUT/ab.tmp" 2>&1 || { tail -5 "$OUT/ab.tmp"; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(json.dumps({'args': sys.argv[2], 'value_M': round(d['value']/1e6,1), 'kernels_ms': d['kernels_ms']}))" "$OUT/ab.tmp" "$a" | tee -a "$OUT/ab_rays.jsonl"
done <<< "${SWEEP:-"--ray-order 0 --sort-interval 0
--ray-order 1 --sort-interval 0
--ray-order 1 --sort-interval 4
--ray-order 1 --sort-interval 16
--ray-order 1 --sort-interval 64
--ray-order 0 --sort-interval 16"}"
