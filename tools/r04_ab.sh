#!/bin/bash
# Round 4, call AB: why the driver's 20-step window runs ~8 % below the 1,000-step steady state:
# the same 20 steps after a longer burn-in (state distribution) and 20 / 60 / 200-step windows.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r04ab; mkdir -p $OUT; export TMPDIR=/tmp
run() {  # label, args
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-time-to-90 --ppo-updates 0 --selfplay-updates 0 $2 \
    > $OUT/$1.jsonl 2> $OUT/$1.err || { tail -30 $OUT/$1.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('$1', round(d['value']/1e6,1), d['ms_per_step'], d['kernels_ms'])" $OUT/$1.jsonl
}
for rep in 1 2; do
  run b100_s20_$rep "--steps 20 --warmup 5"
  run b600_s20_$rep "--steps 20 --warmup 5 --burn-in 600"
  run b100_s60_$rep "--steps 60 --warmup 5"
  run b100_s200_$rep "--steps 200 --warmup 5"
done
echo R04AB_DONE
