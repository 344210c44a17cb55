#!/bin/bash
# Round 4, call J: numpy start draws (rx_set_start_draws, ABI v20), the self-play graph
# rollout fix, and the two-car env suites on the changed KIN kernel.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r04j; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/test_start_draws_gpu.py \
  tests/test_ppo_gpu.py tests/test_fullsize_gpu.py tests/test_env_gpu.py tests/test_selfplay_train_gpu.py \
  tests/test_integration_gpu.py > $OUT/pytest_j.txt 2>&1 || { tail -80 $OUT/pytest_j.txt; exit 1; }
tail -3 $OUT/pytest_j.txt
echo R04J_DONE
