#!/bin/bash
# Round 4, call R: the policy forward with its L2 weights loaded up front (rx_policy_mfma.h):
# policy / rollout / PPO GPU tests, then configs[1] fp32 / bf16 and configs[3] iterations
# against HEAD's library (librx_head.so), same session.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r04r; mkdir -p $OUT; export TMPDIR=/tmp
LIB=$(pwd)/self-play-racing_amd/rx/lib
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_ppo_fused_gpu.py \
  tests/test_rollout_gpu.py tests/test_bf16_gpu.py tests/test_selfplay_train_gpu.py tests/test_ppo_gpu.py \
  tests/test_eval_golden_gpu.py tests/test_env_gpu.py::test_task_sort_interval_is_exact > $OUT/pytest_r.txt 2>&1 \
  || { tail -60 $OUT/pytest_r.txt; exit 1; }
tail -2 $OUT/pytest_r.txt
for rep in 1 2; do
  for v in head tree; do
    p=""; [ $v != tree ] && p=$LIB/librx_$v.so
    for m in "--mode single --envs 4096" "--mode single --envs 4096 --bf16" "--mode selfplay --envs 8192"; do
      RX_LIB_PATH=$p timeout -k 10 300 python -u tools/bench_ppo.py $m --steps 128 --updates 3 --device-shuffle \
        | sed "s/^/$v /" >> $OUT/ab.txt 2>> $OUT/ab.err || { tail -20 $OUT/ab.err; exit 1; }
    done
  done
done
python3 - $OUT/ab.txt <<'PY'
import json, sys
for l in open(sys.argv[1]):
    v, js = l.split(" ", 1)
    d = json.loads(js)
    print(v, d["mode"], d["policy_dtype"], "rollout_ms", round(d["rollout_s"] * 1e3, 2), "update_ms",
          round(d["update_s"] * 1e3, 2), "train M/s", round(d["train_env_steps_per_s"] / 1e6, 2))
PY
echo R04R_DONE
