#!/bin/bash
# Round 4, call I: PPO GPU tests on the scalar-load k_ppo_grad, then rollout graph vs eager
# (tools/bench_ppo.py, GRAPH_ROLLOUT) at configs[1] and configs[3], same session.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r04i; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_ppo_golden.py \
  tests/test_ppo_fused_gpu.py tests/test_bf16_gpu.py tests/test_ppo_gpu.py > $OUT/pytest_ppo.txt 2>&1 || { tail -60 $OUT/pytest_ppo.txt; exit 1; }
tail -2 $OUT/pytest_ppo.txt
for rep in 1 2; do
  for g in 0 1; do
    GRAPH_ROLLOUT=$g timeout -k 10 200 python -u tools/bench_ppo.py --mode single --envs 4096 --steps 128 --updates 3 --device-shuffle >> $OUT/graph_ab.jsonl 2>> $OUT/graph_ab.err || { tail -20 $OUT/graph_ab.err; exit 1; }
    GRAPH_ROLLOUT=$g timeout -k 10 200 python -u tools/bench_ppo.py --mode selfplay --envs 8192 --steps 128 --updates 3 --device-shuffle >> $OUT/graph_ab.jsonl 2>> $OUT/graph_ab.err || { tail -20 $OUT/graph_ab.err; exit 1; }
  done
done
python3 - $OUT/graph_ab.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(d["mode"], "graph", d["graph_rollout"], "rollout_ms", round(d["rollout_s"]*1e3, 2), "gae_ms", round(d["gae_s"]*1e3, 2),
          "update_ms", round(d["update_s"]*1e3, 2), "train M/s", round(d["train_env_steps_per_s"]/1e6, 2))
PY
echo R04I_DONE
