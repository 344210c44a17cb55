#!/bin/bash
# Persistent small-N rollout: parity tests, PPO tests, throughput and time-to-90% at the reference config.
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_rollout_gpu.py tests/test_ppo_gpu.py tests/test_ppo_fused_gpu.py -m gpu > gpurun_out/t_rollout.log 2>&1 || { tail -40 gpurun_out/t_rollout.log; exit 1; }
grep -E "passed|failed" gpurun_out/t_rollout.log | tail -2
timeout -k 10 200 python tools/bench_ppo.py --envs 16 --steps 2048
timeout -k 10 200 python tools/bench_ppo.py --envs 256 --steps 128
timeout -k 10 300 python tools/time_to_success.py --num-envs 16 --num-steps 2048 --eval-every 1 --max-minutes 3 2> gpurun_out/tts.err | tail -1
