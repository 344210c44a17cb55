#!/bin/bash
# bf16 k_ppo_grad with coalesced staging (fragments built from an LDS scratch): bf16 tests, ppo_micro,
# kernel stats, phase stamps
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${RUN_DIR:-r05r}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_bf16_gpu.py \
  tests/test_ppo_fused_gpu.py > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
for r in 1 2; do
  timeout -k 10 120 python -u tools/ppo_micro.py 32768 bf16 stage$r > $OUT/micro_$r.jsonl 2> $OUT/micro_$r.err || { tail -20 $OUT/micro_$r.err; exit 1; }
  cat $OUT/micro_$r.jsonl
done
cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o micro -- python3 $GRAFT_REPO_ROOT/tools/ppo_micro.py 32768 bf16 prof > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT; python3 - <<PY
import csv,glob,re
for f in glob.glob('$OUT/prof/*kernel_stats.csv'):
    for r in csv.DictReader(open(f)):
        m=re.search(r'(k_\w+(<[^>]*>)?)', r['Name'])
        if m and ('ppo' in m.group(1) or 'adam' in m.group(1)): print(m.group(1), r['Calls'], round(float(r['AverageNs'])/1e3,2))
PY
timeout -k 10 120 python -u tools/ppo_stamps.py 32768 bf16 > $OUT/stamps_bf16.json 2> $OUT/stamps_bf16.err || { tail -20 $OUT/stamps_bf16.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/stamps_bf16.json'));r=d['runs'][-1];print('bf16', dict(zip(d['labels'], r['phase_cycles_median'])), 'total', r['wave_total_median'])"
echo R05R_DONE
