#!/bin/bash
# Round 3 final check of the committed tree (after the fused re-sort histogram): the whole
# -m gpu suite + smoke, the driver's bench command, and its rocprofv3 kernel summary.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r03f; mkdir -p $OUT; export TMPDIR=/tmp
OUTDIR=$OUT bash tools/r03_check.sh || exit 1
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver20.jsonl 2> $OUT/bench_driver20.err || { tail -20 $OUT/bench_driver20.err; exit 1; }
tail -c 200 $OUT/bench_driver20.jsonl; echo
timeout -k 10 300 python3 bench.py --steps 1000 --warmup 5 --no-cpu-baseline --no-time-to-90 --ppo-updates 0 > $OUT/bench_steady1000.jsonl 2> $OUT/bench_steady.err || { tail -20 $OUT/bench_steady.err; exit 1; }
echo FINAL2_DONE
