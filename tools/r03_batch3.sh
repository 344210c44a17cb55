#!/bin/bash
# Round 3, batch 3: the optimizer / update tests after the 16-lane clip-norm fold, a
# same-session A/B of the fused minibatch step (tree vs librx_r03c = HEAD before the
# fold change), and the rocprofv3 trace of the driver's 20-step bench with the
# first-step host mark (tools/trace_window.py).
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r03; mkdir -p $OUT; export TMPDIR=/tmp
LIB=$(pwd)/self-play-racing_amd/rx/lib
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  -k "optim or ppo or golden or permutation or dist or rollout or bf16" > $OUT/pytest_b3.log 2>&1 || { tail -30 $OUT/pytest_b3.log; exit 1; }
tail -1 $OUT/pytest_b3.log
: > $OUT/ppo_micro_ab3.jsonl
for rep in 1 2; do
  for lib in librx.so librx_r03c.so; do
    RX_LIB_PATH=$LIB/$lib timeout -k 10 120 python tools/ppo_micro.py 32768 fp32 $lib >> $OUT/ppo_micro_ab3.jsonl 2> $OUT/ppo_micro.err || { tail -5 $OUT/ppo_micro.err; exit 1; }
    tail -1 $OUT/ppo_micro_ab3.jsonl
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ppoprof3 -o run -- \
  python tools/ppo_micro.py 32768 fp32 > $OUT/ppo_micro_prof3.log 2>&1 || { tail -5 $OUT/ppo_micro_prof3.log; exit 1; }
cp $(find /tmp/ppoprof3 -name '*kernel_stats.csv' | head -1) $OUT/ppo_micro_fp32_b3_kernel_stats.csv
python tools/kstats.py $OUT/ppo_micro_fp32_b3_kernel_stats.csv 4
export RX_BENCH_MARKS=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r03prof3 -o run -- \
  python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-time-to-90 --ppo-updates 0 \
  > $OUT/prof20_b3.jsonl 2> $OUT/prof20_b3.err || exit 1
TR=$(find /tmp/r03prof3 -name '*kernel_trace.csv' | head -1)
python3 tools/trace_window.py "$TR" $OUT/prof20_b3.err --out $OUT/window20_b3.json | head -12
timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-time-to-90 --no-cpu-baseline > $OUT/plain20_b3.jsonl 2> $OUT/plain20_b3.err || exit 1
grep first_step $OUT/plain20_b3.err | head -3
echo BATCH3_DONE
