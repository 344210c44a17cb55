#!/bin/bash
# Persistent rollout (k_rollout): parity tests, phase stamps and PPO throughput, this tree vs librx_rpre.so
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
LIBDIR=$(pwd)/self-play-racing_amd/rx/lib
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_rollout_gpu.py tests/test_ppo_gpu.py tests/test_ppo_golden.py > $OUT/t_roll.log 2>&1; rc=$?
tail -2 $OUT/t_roll.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  echo -n "new "; timeout -k 10 200 python tools/rollout_stamps.py 16 512 | tail -1 || exit 1
  echo -n "pre "; RSTAMPS_LIB=$LIBDIR/librx_rstamps_pre.so timeout -k 10 200 python tools/rollout_stamps.py 16 512 | tail -1 || exit 1
  echo -n "new "; timeout -k 10 200 python tools/bench_ppo.py --envs 16 --steps 2048 | tail -1 || exit 1
  echo -n "pre "; RX_LIB_PATH=$LIBDIR/librx_rpre.so timeout -k 10 200 python tools/bench_ppo.py --envs 16 --steps 2048 | tail -1 || exit 1
done
