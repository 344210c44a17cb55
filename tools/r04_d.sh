#!/bin/bash
# Round 4, call D: two-car REWARD half with a lane per car -- exactness, then a same-session
# A/B at configs[3]'s 8,192 envs and at 65,536 (tools/ab_sched.py), and the self-play PPO leg.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r04d; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_env_gpu.py::test_two_car_reward_lane_per_car_is_exact tests/test_env_gpu.py::test_multi_step_vs_golden_and_oracle \
  tests/test_env_gpu.py::test_split_step_equals_one_kernel_step > $OUT/pytest_d.txt 2>&1 || { tail -60 $OUT/pytest_d.txt; exit 1; }
tail -2 $OUT/pytest_d.txt
timeout -k 10 600 python -u tools/ab_sched.py $OUT/ab_two_car_8192.jsonl --envs 8192 --agents 2 --rounds 3 --steps 300 \
  --variant rl1:reward_lpe=1 --variant rl2:reward_lpe=2 --variant rl2_lpr1:reward_lpe=2,ray_lpr=1 \
  --variant rl2_lpr4:reward_lpe=2,ray_lpr=4 > $OUT/ab_8192.log 2>&1 || { tail -30 $OUT/ab_8192.log; exit 1; }
grep summary $OUT/ab_two_car_8192.jsonl
timeout -k 10 600 python -u tools/ab_sched.py $OUT/ab_two_car_65536.jsonl --envs 65536 --agents 2 --rounds 2 --steps 200 \
  --variant rl1:reward_lpe=1 --variant rl2:reward_lpe=2 > $OUT/ab_65536.log 2>&1 || { tail -30 $OUT/ab_65536.log; exit 1; }
grep summary $OUT/ab_two_car_65536.jsonl
echo R04D_DONE
