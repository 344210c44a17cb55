#!/bin/bash
# Round 4, call N: the rollout policy inside the k_kin launch (k_kin1_act, rx_rollout_steps):
# rollout / PPO GPU tests, then tools/bench_ppo.py configs[1] fp32 and bf16 against HEAD's library.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r04n; mkdir -p $OUT; export TMPDIR=/tmp
LIB=$(pwd)/self-play-racing_amd/rx/lib
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_rollout_gpu.py \
  tests/test_ppo_gpu.py tests/test_bf16_gpu.py tests/test_ppo_fused_gpu.py tests/test_ppo_golden.py \
  tests/test_eval_golden_gpu.py > $OUT/pytest_n.txt 2>&1 || { tail -60 $OUT/pytest_n.txt; exit 1; }
tail -2 $OUT/pytest_n.txt
for rep in 1 2; do
  for v in head tree; do
    p=""; [ $v != tree ] && p=$LIB/librx_$v.so
    for b in "" "--bf16"; do
      RX_LIB_PATH=$p timeout -k 10 300 python -u tools/bench_ppo.py --mode single --envs 4096 --steps 128 --updates 3 \
        --device-shuffle $b | sed "s/^/$v /" >> $OUT/single_ab.txt 2>> $OUT/single_ab.err || { tail -20 $OUT/single_ab.err; exit 1; }
    done
  done
done
python3 - $OUT/single_ab.txt <<'PY'
import json, sys
for l in open(sys.argv[1]):
    v, js = l.split(" ", 1)
    d = json.loads(js)
    print(v, d["policy_dtype"], "rollout_ms", round(d["rollout_s"] * 1e3, 2), "update_ms", round(d["update_s"] * 1e3, 2),
          "train M/s", round(d["train_env_steps_per_s"] / 1e6, 2))
PY
echo R04N_DONE
