#!/bin/bash
# fused minibatch tail, every tail load in one round trip: parity tests, ppo_micro, kernel stats
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${RUN_DIR:-r05i}; mkdir -p $OUT; export TMPDIR=/tmp
[ -n "${SKIP_TESTS:-}" ] || timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_ppo_fused_gpu.py \
  tests/test_dist_gpu.py tests/test_optim_gpu.py tests/test_ppo_gpu.py tests/test_bf16_gpu.py > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 1; }
tail -2 $OUT/pytest.txt
for p in fp32 bf16; do
  timeout -k 10 120 python -u tools/ppo_micro.py 32768 $p fused_tail3 > $OUT/micro_$p.jsonl 2> $OUT/micro_$p.err || { tail -20 $OUT/micro_$p.err; exit 1; }
  cat $OUT/micro_$p.jsonl
done
cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o micro -- python3 $GRAFT_REPO_ROOT/tools/ppo_micro.py 32768 fp32 prof > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT; f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1); cut -c1-220 $f | head -12
echo R05I_DONE
