#!/bin/bash
# Quad lanes per ray: exactness tests, then a same-session A/B of RX_RAY_LPR=1 vs 4
# (env_probe at mid sizes, bench_ppo at configs[1]) and the headline bench guard.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_env_gpu.py tests/test_fullsize_gpu.py > $OUT/t_lpr.log 2>&1; rc=$?
tail -3 $OUT/t_lpr.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for cfg in "2048 1" "4096 1" "8192 1" "16384 1" "2048 2" "4096 2" "8192 2"; do
  for v in 1 4; do
    RX_RAY_LPR=$v timeout -k 10 120 python tools/env_probe.py $cfg 400 > $OUT/lpr_probe.log 2>&1 || { tail $OUT/lpr_probe.log; exit 1; }
    echo "lpr=$v $(tail -1 $OUT/lpr_probe.log)"
  done
done
done
for rep in 1 2; do for v in 1 4; do
  RX_RAY_LPR=$v timeout -k 10 200 python tools/bench_ppo.py --envs 4096 --steps 128 --device-shuffle --updates 3 > $OUT/lpr_ppo.log 2>&1 || { tail -20 $OUT/lpr_ppo.log; exit 1; }
  echo "lpr=$v $(tail -1 $OUT/lpr_ppo.log)"
done; done
AB_SETS="l1|RX_RAY_LPR=1;l4|RX_RAY_LPR=4" bash tools/ab_env.sh
