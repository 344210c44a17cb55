#!/bin/bash
# bf16 rollout on prebuilt policy fragments (k_policy_frag once per rollout): rollout/bf16 parity tests,
# bench_ppo bf16 at configs[1], kernel stats of the same run
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${RUN_DIR:-r05s}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_rollout_gpu.py \
  tests/test_bf16_gpu.py > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
for r in 1 2; do
  timeout -k 10 150 python -u tools/bench_ppo.py --mode single --envs 4096 --bf16 > $OUT/ppo_$r.json 2> $OUT/ppo_$r.err || { tail -20 $OUT/ppo_$r.err; exit 1; }
  cat $OUT/ppo_$r.json
done
cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o ppo -- python3 $GRAFT_REPO_ROOT/tools/bench_ppo.py --mode single --envs 4096 --bf16 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT; python3 - <<PY
import csv,glob,re
for f in glob.glob('$OUT/prof/*kernel_stats.csv'):
    for r in csv.DictReader(open(f)):
        m=re.search(r'(k_\w+(<[^>]*>)?)', r['Name'])
        print(m.group(1) if m else r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,2), round(float(r['TotalDurationNs'])/1e6,2))
PY
echo R05S_DONE
