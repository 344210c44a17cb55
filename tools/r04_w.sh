#!/bin/bash
# Round 4, call W: the spatial re-sort period at 65,536 envs now that a re-sort costs ~19 us
# (atomic-free scatter): bench.py --sort-interval 8 / 12 / 16 / 24 / 32, two interleaved passes.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r04w; mkdir -p $OUT; export TMPDIR=/tmp
OUT_SUB=r04w AB_SETS="s8||--sort-interval 8;s12||--sort-interval 12;s16||--sort-interval 16;s24||--sort-interval 24;s32||--sort-interval 32" \
  timeout -k 10 1100 bash tools/ab_args.sh > $OUT/ab_sort_interval.txt 2>&1 || { tail -20 $OUT/ab_sort_interval.txt; exit 1; }
cat $OUT/ab_sort_interval.txt
echo R04W_DONE
