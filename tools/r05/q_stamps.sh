#!/bin/bash
# phase stamps of the bf16 (and fp32) k_ppo_grad: profiling build (-DRX_PPO_STAMPS)
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${RUN_DIR:-r05q}; mkdir -p $OUT; export TMPDIR=/tmp
for p in bf16 fp32; do
  timeout -k 10 120 python -u tools/ppo_stamps.py 32768 $p > $OUT/stamps_$p.json 2> $OUT/stamps_$p.err || { tail -20 $OUT/stamps_$p.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/stamps_$p.json'));r=d['runs'][-1];print('$p', dict(zip(d['labels'], r['phase_cycles_median'])), 'total', r['wave_total_median'], 'span', r['launch_span_cycles'], 'start_spread', r['start_spread_cycles'], 'end_spread', r['end_spread_cycles'])"
done
echo R05Q_DONE
