#!/bin/bash
# Round 4, call M: both self-play policies in one launch (k_selfplay_act; the agent-row copy
# folded into it): the policy / rollout / self-play GPU tests, then tools/bench_ppo.py
# --mode selfplay against HEAD's library (librx_head.so), same session.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r04m; mkdir -p $OUT; export TMPDIR=/tmp
LIB=$(pwd)/self-play-racing_amd/rx/lib
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_selfplay_train_gpu.py \
  tests/test_ppo_fused_gpu.py tests/test_rollout_gpu.py tests/test_start_draws_gpu.py tests/test_ppo_gpu.py \
  tests/test_bf16_gpu.py > $OUT/pytest_m.txt 2>&1 || { tail -60 $OUT/pytest_m.txt; exit 1; }
tail -2 $OUT/pytest_m.txt
for rep in 1 2; do
  for v in head tree; do
    p=""; [ $v != tree ] && p=$LIB/librx_$v.so
    RX_LIB_PATH=$p timeout -k 10 300 python -u tools/bench_ppo.py --mode selfplay --envs 8192 --steps 128 --updates 3 \
      --device-shuffle | sed "s/^/$v /" >> $OUT/selfplay_ab.txt 2>> $OUT/selfplay_ab.err || { tail -20 $OUT/selfplay_ab.err; exit 1; }
  done
done
python3 - $OUT/selfplay_ab.txt <<'PY'
import json, sys
for l in open(sys.argv[1]):
    v, js = l.split(" ", 1)
    d = json.loads(js)
    print(v, "rollout_ms", round(d["rollout_s"] * 1e3, 2), "update_ms", round(d["update_s"] * 1e3, 2),
          "train M/s", round(d["train_env_steps_per_s"] / 1e6, 2))
PY
echo R04M_DONE
