#!/bin/bash
# rocprofv3 kernel stats of the configs[1] PPO update (4,096 envs x 128 steps), fp32 and bf16.
set -u
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p $OUT
for P in fp32 bf16; do
  X=""; [ $P = bf16 ] && X="--bf16"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/ppo_prof_$P -o run --output-format csv -- \
    python tools/bench_ppo.py --envs 4096 --steps 128 --device-shuffle --updates 2 $X > $OUT/ppo_prof_$P.log 2>&1 \
    || { tail -20 $OUT/ppo_prof_$P.log; exit 1; }
  tail -1 $OUT/ppo_prof_$P.log
  python tools/kstats.py $(find $OUT/ppo_prof_$P -name "*kernel_stats.csv" | head -1) 14
done
