#!/bin/bash
# Round 3, second GPU batch: full -m gpu suite + smoke (tools/r03_check.sh), the
# first-launch probe, k_ppo_grad stamps with the batched weight staging, a
# same-session A/B of the fused minibatch step (tree vs librx_r03a = HEAD before the
# staging change, librx_r03b = staging without the exp-form tanh), a rocprofv3 kernel summary of the tree's step, and the 2-rank gloo
# rehearsal of bench.py's own launcher on this one GPU.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r03; mkdir -p $OUT; export TMPDIR=/tmp
LIB=$(pwd)/self-play-racing_amd/rx/lib
bash tools/r03_check.sh || exit 1
timeout -k 10 120 python tools/first_launch_probe.py > $OUT/first_launch.json 2> $OUT/first_launch.err || { tail -5 $OUT/first_launch.err; exit 1; }
echo "probe done"; cat $OUT/first_launch.json
bash tools/r03_stamps.sh || exit 1
: > $OUT/ppo_micro_ab.jsonl
for rep in 1 2; do
  for prec in fp32 bf16; do
    for lib in librx.so librx_r03b.so librx_r03a.so; do
      RX_LIB_PATH=$LIB/$lib timeout -k 10 120 python tools/ppo_micro.py 32768 $prec $lib >> $OUT/ppo_micro_ab.jsonl 2> $OUT/ppo_micro.err || { tail -5 $OUT/ppo_micro.err; exit 1; }
      tail -1 $OUT/ppo_micro_ab.jsonl
    done
  done
done
for prec in fp32 bf16; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ppoprof_$prec -o run -- \
    python tools/ppo_micro.py 32768 $prec > $OUT/ppo_micro_prof_$prec.log 2>&1 || { tail -5 $OUT/ppo_micro_prof_$prec.log; exit 1; }
  cp $(find /tmp/ppoprof_$prec -name '*kernel_stats.csv' | head -1) $OUT/ppo_micro_${prec}_kernel_stats.csv
  python tools/kstats.py $OUT/ppo_micro_${prec}_kernel_stats.csv 8
done
timeout -k 10 400 python bench.py --gpus 2 --dist-backend gloo --steps 100 --warmup 10 --no-time-to-90 --ppo-updates 1 \
  > $OUT/bench_2rank_gloo.jsonl 2> $OUT/bench_2rank_gloo.err || { tail -20 $OUT/bench_2rank_gloo.err; exit 1; }
head -c 600 $OUT/bench_2rank_gloo.jsonl; echo
echo BATCH2_DONE
