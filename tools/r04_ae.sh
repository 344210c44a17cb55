#!/bin/bash
# Round 4, call AE: longer re-sort periods where 16 won (tools/env_probe.py, sort_interval 16 / 32 / 64 / 0 = never).
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r04ae; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_start_draws_gpu.py tests/test_rollout_gpu.py > $OUT/pytest_ae.txt 2>&1 || { tail -40 $OUT/pytest_ae.txt; exit 1; }
tail -1 $OUT/pytest_ae.txt
for rep in 1 2; do
  for cfg in "4096 1" "16384 1" "8192 2" "65536 2"; do
    for si in 16 32 64 0; do
      PROBE_SORT=$si timeout -k 10 120 python -u tools/env_probe.py $cfg 600 | cut -c1-110 >> $OUT/probe_sort_long.txt \
        || { tail -5 $OUT/probe_sort_long.txt; exit 1; }
    done
  done
done
cat $OUT/probe_sort_long.txt
echo R04AE_DONE
