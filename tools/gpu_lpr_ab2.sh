#!/bin/bash
# Lanes per ray 1 / 2 / 4 at the sizes near the crossover, plus the headline guard at 2.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_env_gpu.py -k lanes_per_ray > $OUT/t_lpr2.log 2>&1; rc=$?
tail -3 $OUT/t_lpr2.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for cfg in "8192 1" "12288 1" "16384 1" "32768 1" "4096 2" "8192 2" "16384 2"; do
  for v in 1 2 4; do
    RX_RAY_LPR=$v timeout -k 10 120 python tools/env_probe.py $cfg 400 > $OUT/lpr_probe.log 2>&1 || { tail $OUT/lpr_probe.log; exit 1; }
    echo "lpr=$v $(tail -1 $OUT/lpr_probe.log | cut -c1-200)"
  done
done
done
