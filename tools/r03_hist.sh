#!/bin/bash
# Round 3: the re-sort's histogram counted by the REWARD half (k_sort_hist launch dropped,
# single-agent split step).  Env GPU tests on the tree (sort / culling / full-size exactness),
# then same-session A/B of the 65,536-env bench (1,000 steady steps) and the driver's
# 20-step command against HEAD (librx_head.so), two passes interleaved.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r03; mkdir -p $OUT; export TMPDIR=/tmp
LIB=$(pwd)/self-play-racing_amd/rx/lib
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "env or fullsize or sort or integration or rollout" > $OUT/pytest_hist.log 2>&1 || { grep -E "FAILED|Error" $OUT/pytest_hist.log | head; tail -40 $OUT/pytest_hist.log; exit 1; }
tail -1 $OUT/pytest_hist.log
: > $OUT/hist_ab.jsonl
for rep in 1 2; do
  for v in librx.so librx_head.so; do
    RX_LIB_PATH=$LIB/$v timeout -k 10 200 python3 bench.py --steps 1000 --warmup 5 --no-cpu-baseline --no-time-to-90 --ppo-updates 0 --async-probe-groups 0 2>/dev/null | tail -1 | sed "s/^{/{\"lib\": \"$v\", /" >> $OUT/hist_ab.jsonl || exit 1
    RX_LIB_PATH=$LIB/$v timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-time-to-90 --ppo-updates 0 --async-probe-groups 0 2>/dev/null | tail -1 | sed "s/^{/{\"lib\": \"$v\", /" >> $OUT/hist_ab.jsonl || exit 1
  done
done
python3 -c "
import json
for l in open('$OUT/hist_ab.jsonl'):
    d=json.loads(l); print(d['lib'], d['steps'], round(d['value']/1e6,1), d['ms_per_step'], d['kernels_ms'].get('k_step2'))
"
