#!/bin/bash
# r06 p: unbalanced Feistel shuffle (no cycle walk at 2^19 rows) + the whole update as one graph over
# per-epoch batch views -- PPO / shuffle parity tests, then the configs[1] PPO iteration (tools/bench_ppo.py)
set -o pipefail
O=gpurun_out/r06p
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_permutation_gpu.py \
  tests/test_ppo_fused_gpu.py tests/test_ppo_golden.py tests/test_bf16_gpu.py tests/test_optim_gpu.py \
  tests/test_dist_gpu.py tests/test_ppo_gpu.py > $O/pytest_ppo.txt 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 200 python tools/bench_ppo.py --envs 4096 --steps 128 --device-shuffle --updates 3 --bf16 >> $O/bench_ppo_bf16.jsonl 2>> $O/bench.err || exit 1
  timeout -k 10 200 python tools/bench_ppo.py --envs 4096 --steps 128 --device-shuffle --updates 3 >> $O/bench_ppo_fp32.jsonl 2>> $O/bench.err || exit 1
done
