#!/bin/bash
# GAE bootstrap value from the fused policy kernel: PPO tests, then the ppo_leg A/B
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${RUN_DIR:-r05g2}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ppo_gpu.py \
  tests/test_selfplay_train_gpu.py tests/test_bf16_gpu.py tests/test_rollout_gpu.py tests/test_ppo_golden.py > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
timeout -k 10 600 python -u tools/r05/g_nextvalue.py > $OUT/ab_next_value.jsonl 2> $OUT/ab.err || { tail -20 $OUT/ab.err; exit 1; }
cat $OUT/ab_next_value.jsonl
echo R05G2_DONE
