#!/bin/bash
# Round 4, call V: the re-sort's scatter without atomics (each env's rank within its bin comes back
# from the count's atomic; k_sort_scatter = cursor[bin] + rank): env / full-size / sort GPU tests,
# then bench.py A/B against HEAD's library (librx_head.so) and the sort kernels' durations under
# rocprofv3 --kernel-trace --stats for both.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r04v; mkdir -p $OUT; export TMPDIR=/tmp
LIB=$(pwd)/self-play-racing_amd/rx/lib
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_env_gpu.py \
  tests/test_fullsize_gpu.py tests/test_permutation_gpu.py tests/test_start_draws_gpu.py > $OUT/pytest_v.txt 2>&1 \
  || { tail -60 $OUT/pytest_v.txt; exit 1; }
tail -2 $OUT/pytest_v.txt
OUT_SUB=r04v AB_SETS="head|head|;tree||" timeout -k 10 1000 bash tools/ab_args.sh > $OUT/ab_scatter.txt 2>&1 \
  || { tail -20 $OUT/ab_scatter.txt; exit 1; }
cat $OUT/ab_scatter.txt
for v in head tree; do
  p=""; [ $v != tree ] && p=$LIB/librx_$v.so
  RX_LIB_PATH=$p timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$v -o run -- python bench.py --steps 200 \
    --warmup 20 --no-cpu-baseline --async-probe-groups 0 --ppo-updates 0 --no-time-to-90 > $OUT/prof_$v.log 2>&1 \
    || { tail -20 $OUT/prof_$v.log; exit 1; }
  f=$(find $OUT/prof_$v -name "*kernel_stats.csv" | head -1)
  echo "== $v"; grep -E "k_sort|k_state_copy|k_step2|k_dyn1<1, 1>" $f | cut -d, -f1-7 | cut -c1-160
done
echo R04V_DONE
