#!/bin/bash
# deferred Adam (rx_ppo_epoch_update): parity tests, the PPO suites it feeds, bench_ppo A/B (interleaved),
# kernel stats of the deferred configs[1] bf16 update
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${RUN_DIR:-r05t}; mkdir -p $OUT; export TMPDIR=/tmp
[ "${SKIP_TESTS:-0}" = 1 ] || timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_ppo_epoch_gpu.py \
  tests/test_ppo_fused_gpu.py tests/test_bf16_gpu.py tests/test_optim_gpu.py tests/test_ppo_golden.py \
  > $OUT/pytest.txt 2>&1 || { tail -60 $OUT/pytest.txt; exit 1; }
[ "${SKIP_TESTS:-0}" = 1 ] || tail -1 $OUT/pytest.txt
for r in 1 2; do
  for d in 0 1; do
    for p in "" "--bf16"; do
      DEFERRED_ADAM=$d timeout -k 10 150 python -u tools/bench_ppo.py --mode single --envs 4096 --device-shuffle $p > $OUT/ppo_d${d}${p}_$r.json 2> $OUT/ppo_d${d}_$r.err || { tail -20 $OUT/ppo_d${d}_$r.err; exit 1; }
      echo "defer=$d $p $(python3 -c "import json;d=json.load(open('$OUT/ppo_d${d}${p}_$r.json'));print(round(d['update_s']*1e3,3),'ms update', round(d['rollout_s']*1e3,3),'ms rollout', round(d['train_env_steps_per_s']/1e6,2),'M')")"
    done
  done
done
for d in 0 1; do
  cd /tmp && DEFERRED_ADAM=$d timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_d$d -o ppo -- python3 $GRAFT_REPO_ROOT/tools/bench_ppo.py --mode single --envs 4096 --device-shuffle --bf16 > $OUT/prof_d$d.log 2>&1 || { tail -20 $OUT/prof_d$d.log; exit 1; }
  cd $GRAFT_REPO_ROOT; echo "== rocprof defer=$d (bf16)"; python3 - <<PY
import csv,glob,re
for f in glob.glob('$OUT/prof_d$d/*kernel_stats.csv'):
    for r in csv.DictReader(open(f)):
        m=re.search(r'(k_\w+(<[^>]*>)?)', r['Name'])
        if m and ('ppo' in m.group(1) or 'adam' in m.group(1)): print(m.group(1), r['Calls'], round(float(r['AverageNs'])/1e3,2), round(float(r['TotalDurationNs'])/1e6,2))
PY
done
echo R05T_DONE
