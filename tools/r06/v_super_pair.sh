#!/bin/bash
# r06 v: both sides' super boxes in one round trip at 4 lanes per ray (RX_SUPER_PAIR) -- env parity, then A/B
set -o pipefail
O=gpurun_out/r06v
mkdir -p $O
L=self-play-racing_amd/rx/lib
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_env_gpu.py \
  tests/test_fullsize_gpu.py tests/test_rollout_gpu.py > $O/pytest_env.txt 2>&1 || exit 1
for r in 1 2; do
  for cfg in "4096 1" "8192 1" "4096 2"; do
    timeout -k 10 120 python tools/env_probe.py $cfg >> $O/probe_new.jsonl 2>> $O/probe.err || exit 1
    RX_LIB_PATH=$L/librx_nopair.so timeout -k 10 120 python tools/env_probe.py $cfg >> $O/probe_old.jsonl 2>> $O/probe.err || exit 1
  done
  timeout -k 10 200 python tools/bench_ppo.py --envs 4096 --steps 128 --device-shuffle --updates 3 --bf16 >> $O/ppo_new.jsonl 2>> $O/bench.err || exit 1
  RX_LIB_PATH=$L/librx_nopair.so timeout -k 10 200 python tools/bench_ppo.py --envs 4096 --steps 128 --device-shuffle --updates 3 --bf16 >> $O/ppo_old.jsonl 2>> $O/bench.err || exit 1
done
