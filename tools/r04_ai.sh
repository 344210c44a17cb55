#!/bin/bash
# Round 4, call AI: k_kin1's ray-task row copied LDS -> global with every LDS read issued first
# (unrolled) vs HEAD (librx_head.so): env tests, bench.py A/B and env_probe at 4,096 / 8,192 x 2.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r04ai; mkdir -p $OUT; export TMPDIR=/tmp
LIB=$(pwd)/self-play-racing_amd/rx/lib
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_env_gpu.py \
  tests/test_fullsize_gpu.py > $OUT/pytest_ai.txt 2>&1 || { tail -40 $OUT/pytest_ai.txt; exit 1; }
tail -1 $OUT/pytest_ai.txt
OUT_SUB=r04ai AB_SETS="head|head|;tree||" timeout -k 10 900 bash tools/ab_args.sh > $OUT/ab_task_copy.txt 2>&1 || { tail -20 $OUT/ab_task_copy.txt; exit 1; }
cat $OUT/ab_task_copy.txt
for rep in 1 2; do
for v in head tree; do
  p=""; [ $v != tree ] && p=$LIB/librx_$v.so
  for cfg in "4096 1" "8192 2"; do
    RX_LIB_PATH=$p timeout -k 10 120 python -u tools/env_probe.py $cfg 400 | sed "s/^/$v /" | cut -c1-110 >> $OUT/probe_ai.txt || exit 1
  done
done
done
cat $OUT/probe_ai.txt
echo R04AI_DONE
