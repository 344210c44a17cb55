#!/bin/bash
# r06 s: the rollout's policy fused into k_kin1 (k_kin1_act, RX_KIN_ACT) -- rollout / PPO parity tests, then
# interleaved A/B of the configs[1] PPO iteration (tools/bench_ppo.py) against the unfused build
set -o pipefail
O=gpurun_out/r06s
mkdir -p $O
L=self-play-racing_amd/rx/lib
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_rollout_gpu.py \
  tests/test_ppo_gpu.py tests/test_bf16_gpu.py tests/test_ppo_fused_gpu.py tests/test_selfplay_train_gpu.py \
  > $O/pytest.txt 2>&1 || exit 1
for r in 1 2; do
  for lib in librx.so librx_nokinact.so; do
    RX_LIB_PATH=$L/$lib timeout -k 10 200 python tools/bench_ppo.py --envs 4096 --steps 128 --device-shuffle --updates 3 --bf16 >> $O/bf16_$lib.jsonl 2>> $O/bench.err || exit 1
    RX_LIB_PATH=$L/$lib timeout -k 10 200 python tools/bench_ppo.py --envs 4096 --steps 128 --device-shuffle --updates 3 >> $O/fp32_$lib.jsonl 2>> $O/bench.err || exit 1
  done
done
