#!/bin/bash
# Round 4, call S: the N-rank bench path rehearsed on one GPU (2 self-launched ranks over gloo:
# a path check of the driver's multi-GPU command, not a scaling number).
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r04s; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u bench.py --gpus 2 --steps 20 --warmup 5 --dist-backend gloo --no-cpu-baseline --no-time-to-90 \
  > $OUT/bench_2rank_gloo.jsonl 2> $OUT/bench_2rank_gloo.err || { tail -30 $OUT/bench_2rank_gloo.err; exit 1; }
tail -c 600 $OUT/bench_2rank_gloo.jsonl; echo
echo R04S_DONE
