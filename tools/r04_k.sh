#!/bin/bash
# Round 4, call K: ray-task direction sort every k dynamics launches (RX_TASK_SORT_INTERVAL,
# A/B builds librx_ts{2,4,8}.so from tools/build_rev.py): bit-exact tests on ts4, then the
# steady-state bench and the configs[1] / two-car env probes, same session.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r04k; mkdir -p $OUT; export TMPDIR=/tmp
LIB=$(pwd)/self-play-racing_amd/rx/lib
RX_LIB_PATH=$LIB/librx_ts4.so timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread \
  tests/test_env_gpu.py tests/test_fullsize_gpu.py > $OUT/pytest_ts4.txt 2>&1 || { tail -60 $OUT/pytest_ts4.txt; exit 1; }
tail -2 $OUT/pytest_ts4.txt
OUT_SUB=r04k AB_SETS="t1||;t2|ts2|;t4|ts4|;t8|ts8|" timeout -k 10 900 bash tools/ab_args.sh > $OUT/ab_bench.txt 2>&1 || { tail -20 $OUT/ab_bench.txt; exit 1; }
cat $OUT/ab_bench.txt
for rep in 1 2; do
  for v in t1 ts2 ts4; do
    p=""; [ $v != t1 ] && p=$LIB/librx_$v.so
    for cfg in "4096 1" "65536 2" "8192 2"; do
      RX_LIB_PATH=$p timeout -k 10 120 python -u tools/env_probe.py $cfg 400 | sed "s/^/$v $cfg /" | cut -c1-150 >> $OUT/probe_ab.txt || exit 1
    done
  done
done
cat $OUT/probe_ab.txt
echo R04K_DONE
