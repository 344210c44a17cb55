#!/bin/bash
# A/B: k_dyn1 lanes per env at 65,536 envs, plus a kernel-trace timeline of the default bench.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
for l in 1 2 4 1; do
  RX_DYN1_LPE=$l timeout -k 10 200 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --async-probe-groups 0 --ppo-updates 0 > $OUT/ab_lpe_$l.log 2>&1 || exit $?
  tail -1 $OUT/ab_lpe_$l.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('lpe', $l, d['value'], d['kernels_ms'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/trace -o run --output-format csv -- python bench.py --steps 100 --warmup 10 --no-cpu-baseline --async-probe-groups 0 --ppo-updates 0 --sample-every 1000 > $OUT/trace.log 2>&1 || exit $?
python tools/trace_gaps.py "$OUT/trace/**/*kernel_trace.csv" --last 500
