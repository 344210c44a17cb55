#!/bin/bash
# PPO update tests, then a same-session A/B of the fused reduce + Adam step (RX_FUSED_ADAM=0/1)
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_ppo_fused_gpu.py tests/test_optim_gpu.py tests/test_ppo_golden.py tests/test_bf16_gpu.py tests/test_permutation_gpu.py tests/test_ppo_gpu.py tests/test_dist_gpu.py > $OUT/t_adam.log 2>&1; rc=$?
tail -2 $OUT/t_adam.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for v in 0 1; do
  for a in "--envs 4096 --steps 128 --device-shuffle" "--envs 16 --steps 2048"; do
    echo -n "fused=$v $a "; RX_FUSED_ADAM=$v timeout -k 10 200 python tools/bench_ppo.py $a | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('update_ms', round(d['update_s']*1e3,2), 'train_M', round(d['train_env_steps_per_s']/1e6,2))" || exit 1
  done
done; done
