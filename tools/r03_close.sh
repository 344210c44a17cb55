#!/bin/bash
# Round 3 closing evidence: the whole -m gpu suite + smoke (tools/r03_check.sh), the
# driver's bench command, its rocprofv3 kernel summary, and rocprofv3 summaries of the
# configs[1] PPO iteration (fp32, bf16).  Stops at the first failing step.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r03c; mkdir -p $OUT; export TMPDIR=/tmp
PYTEST_ARGS="" OUTDIR=$OUT bash tools/r03_check.sh || exit 1
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver20.jsonl 2> $OUT/bench_driver20.err || { tail -20 $OUT/bench_driver20.err; exit 1; }
tail -c 300 $OUT/bench_driver20.jsonl; echo
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/closeprof -o run -- \
  python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver20_rocprof.jsonl 2> $OUT/bench_rocprof.err || { tail -20 $OUT/bench_rocprof.err; exit 1; }
cp $(find /tmp/closeprof -name '*kernel_stats.csv' | head -1) $OUT/bench_driver20_kernel_stats.csv
for prec in fp32 bf16; do
  flag=""; [ $prec = bf16 ] && flag="--bf16"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ppoprof_$prec -o run -- \
    python3 tools/bench_ppo.py --mode single --envs 4096 --steps 128 --updates 3 --device-shuffle $flag > $OUT/ppo_train_${prec}_rocprof.jsonl 2> $OUT/ppo_$prec.err || { tail -20 $OUT/ppo_$prec.err; exit 1; }
  cp $(find /tmp/ppoprof_$prec -name '*kernel_stats.csv' | head -1) $OUT/ppo_train_${prec}_kernel_stats.csv
done
echo CLOSE_DONE
