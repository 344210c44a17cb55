#!/bin/bash
# PPO throughput with the rollout eager (GRAPH_ROLLOUT=0) vs one captured HIP graph (1)
set -u
export TMPDIR=/tmp
for rep in 1 2; do for v in 0 1; do
  for a in "--envs 4096 --steps 128 --device-shuffle" "--mode selfplay --envs 8192 --steps 128 --device-shuffle" "--envs 1024 --steps 256 --device-shuffle" "--envs 65536 --steps 64 --device-shuffle"; do
    echo -n "graph=$v $a "; GRAPH_ROLLOUT=$v timeout -k 10 200 python tools/bench_ppo.py $a | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('rollout_ms', round(d['rollout_s']*1e3,2), 'train_M', round(d['train_env_steps_per_s']/1e6,2))" || exit 1
  done
done; done
