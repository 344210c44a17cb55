#!/bin/bash
# Round 4, call X: the re-sort's scan inside the scatter (<= 8,192 bins; k_state_copy clears the
# histogram): env / full-size GPU tests incl. both scan paths, bench.py A/B against HEAD
# (librx_head.so: atomic-free scatter, scan launch) at sort intervals 16 / 12 / 8, and the sort
# kernels under rocprofv3 --kernel-trace.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r04x; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_env_gpu.py \
  tests/test_fullsize_gpu.py > $OUT/pytest_x.txt 2>&1 || { tail -60 $OUT/pytest_x.txt; exit 1; }
tail -2 $OUT/pytest_x.txt
OUT_SUB=r04x AB_SETS="head16|head|--sort-interval 16;tree16||--sort-interval 16;head12|head|--sort-interval 12;tree12||--sort-interval 12;tree8||--sort-interval 8" \
  timeout -k 10 1000 bash tools/ab_args.sh > $OUT/ab_fused_scan.txt 2>&1 || { tail -20 $OUT/ab_fused_scan.txt; exit 1; }
cat $OUT/ab_fused_scan.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_tree -o run -- python bench.py --steps 200 \
  --warmup 20 --no-cpu-baseline --async-probe-groups 0 --ppo-updates 0 --no-time-to-90 > $OUT/prof_tree.log 2>&1 \
  || { tail -20 $OUT/prof_tree.log; exit 1; }
echo R04X_DONE
