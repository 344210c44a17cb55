#!/bin/bash
# Round 4, call A: the new GPU tests (re-sort histogram sequences, tail split, near-zero tanh,
# RCCL at world size 1, configs[3] self-play training), the ray-tail A/B sweep at 65,536 envs,
# then the whole -m gpu suite + smoke.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r04a; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_env_gpu.py::test_resort_histogram_survives_split_phase_sequences \
  tests/test_env_gpu.py::test_ray_tail_split_is_exact \
  tests/test_ppo_fused_gpu.py::test_policy_act_near_zero_preactivations \
  tests/test_dist_gpu.py::test_rccl_world1_shard_update_equals_fused \
  tests/test_selfplay_train_gpu.py \
  tests/test_rollout_gpu.py::test_rollout_steps_equals_per_step_path \
  tests/test_rollout_gpu.py::test_collect_rollout_uses_rollout_steps_and_keeps_t1_stream > $OUT/pytest_new.txt 2>&1 || { tail -60 $OUT/pytest_new.txt; exit 1; }
tail -3 $OUT/pytest_new.txt
timeout -k 10 900 python -u tools/ab_sched.py $OUT/ab_tail.jsonl --rounds 3 --steps 300 \
  --variant base:ray_tail=-1 --variant t2:ray_tail=2 --variant t3:ray_tail=3 --variant t5:ray_tail=5 \
  --variant t7:ray_tail=7 --variant t11:ray_tail=11 --variant t3x4:ray_tail=3,ray_tail_lpr=4 \
  --variant t5x4:ray_tail=5,ray_tail_lpr=4 > $OUT/ab_tail.log 2>&1 || { tail -30 $OUT/ab_tail.log; exit 1; }
grep summary $OUT/ab_tail.jsonl
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver20.jsonl 2> $OUT/bench_driver20.err \
  || { tail -30 $OUT/bench_driver20.err; exit 1; }
tail -c 400 $OUT/bench_driver20.jsonl; echo
timeout -k 10 1200 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
  > $OUT/pytest_gpu.txt 2>&1 || { tail -60 $OUT/pytest_gpu.txt; exit 1; }
tail -3 $OUT/pytest_gpu.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
echo R04A_DONE
