#!/bin/bash
# bf16 k_ppo_grad with two barriers per pass (double-buffered images, RX_PPO_BF_DB=1) vs four (=0):
# bf16 tests, ppo_micro interleaved x2, kernel stats of the new build
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${RUN_DIR:-r05o}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_bf16_gpu.py \
  > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
for r in 1 2; do
  for v in new bf_db0; do
    if [ $v = bf_db0 ]; then export RX_LIB_PATH=$(pwd)/build/variants/bf_db0.so; else unset RX_LIB_PATH; fi
    timeout -k 10 120 python -u tools/ppo_micro.py 32768 bf16 $v > $OUT/micro_$v$r.jsonl 2> $OUT/micro_$v$r.err || { tail -20 $OUT/micro_$v$r.err; exit 1; }
    cat $OUT/micro_$v$r.jsonl
  done
done
unset RX_LIB_PATH
cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o micro -- python3 $GRAFT_REPO_ROOT/tools/ppo_micro.py 32768 bf16 prof > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT; python3 - <<PY
import csv,glob,re
for f in glob.glob('$OUT/prof/*kernel_stats.csv'):
    for r in csv.DictReader(open(f)):
        m=re.search(r'(k_\w+(<[^>]*>)?)', r['Name'])
        if m and ('ppo' in m.group(1) or 'adam' in m.group(1)): print(m.group(1), r['Calls'], round(float(r['AverageNs'])/1e3,2))
PY
echo R05O_DONE
