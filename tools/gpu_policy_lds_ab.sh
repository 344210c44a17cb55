#!/bin/bash
# k_policy_act with both trunks' weights staged in LDS: policy / rollout / PPO tests, then a same-session
# A/B (HEAD lib vs this tree) of the configs[1] PPO iteration and the self-play one, rocprofv3 kernel times.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_ppo_fused_gpu.py tests/test_rollout_gpu.py tests/test_bf16_gpu.py tests/test_ppo_gpu.py tests/test_ppo_golden.py tests/test_eval_golden_gpu.py > $OUT/plds_pytest.log 2>&1; rc=$?
tail -1 $OUT/plds_pytest.log; [ $rc -eq 0 ] || exit $rc
LIBDIR=$(pwd)/self-play-racing_amd/rx/lib
for rep in 1 2; do for lib in ${LIBS:-head tree}; do
  RX_LIB_PATH=$LIBDIR/librx_$lib.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/plds_$lib -o run --output-format csv -- \
    python tools/bench_ppo.py --envs 4096 --steps 128 --device-shuffle --updates 2 > $OUT/plds_$lib.log 2>&1 || { tail -20 $OUT/plds_$lib.log; exit 1; }
  python - $lib $OUT/plds_$lib <<'PY'
import csv, glob, json, sys
f = glob.glob(sys.argv[2] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = {r["Name"]: r for r in csv.DictReader(open(f))}
pa = [r for n, r in rows.items() if "k_policy_act" in n][0]
d = json.loads([l for l in open(sys.argv[2] + ".log") if l.startswith("{")][-1])
print(sys.argv[1], "k_policy_act_us", round(float(pa["AverageNs"]) / 1e3, 2), "rollout_ms", round(d["rollout_s"] * 1e3, 3),
      "train_M", round(d["train_env_steps_per_s"] / 1e6, 2))
PY
done; done
for rep in 1 2; do for lib in ${LIBS:-head tree}; do
  RX_LIB_PATH=$LIBDIR/librx_$lib.so timeout -k 10 200 python tools/bench_ppo.py --mode selfplay --envs 8192 --steps 128 --device-shuffle --updates 2 > $OUT/plds_sp.log 2>&1 || { tail -20 $OUT/plds_sp.log; exit 1; }
  grep '^{' $OUT/plds_sp.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib selfplay rollout_ms', round(d['rollout_s']*1e3,3), 'train_M', round(d['train_env_steps_per_s']/1e6,2))"
done; done
