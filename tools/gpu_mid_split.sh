#!/bin/bash
# Mid-N kernel split (k_step2 vs its REWARD half vs the raycast alone) and the configs[1] rollout's kernels.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
for n in 4096 8192 16384; do
  timeout -k 10 120 python bench.py --envs-per-gpu $n --steps 1000 --warmup 100 --no-cpu-baseline --async-probe-groups 0 --ppo-updates 0 --no-time-to-90 > $OUT/mid_$n.log 2>&1 || { tail -20 $OUT/mid_$n.log; exit 1; }
  tail -1 $OUT/mid_$n.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($n, round(d['value']/1e6,1), d['kernels_ms'])"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/ppo_roll -o run --output-format csv -- \
  python tools/bench_ppo.py --envs 4096 --steps 128 --device-shuffle --updates 2 > $OUT/ppo_roll.log 2>&1 || { tail -20 $OUT/ppo_roll.log; exit 1; }
find $OUT/ppo_roll -name "*kernel_stats.csv" -exec cat {} \; | head -25
