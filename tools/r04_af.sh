#!/bin/bash
# Round 4, call AF: the timed region's graph split into a 1-step head graph + the rest
# (RX_GRAPH_HEAD=1) vs one graph, driver command, interleaved, plus the window trace.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r04af; mkdir -p $OUT; export TMPDIR=/tmp
RX_GRAPH_HEAD=1 RX_BENCH_MARKS=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/winprof_h -o run -- \
  python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-time-to-90 --ppo-updates 0 \
  --selfplay-updates 0 > $OUT/window20_h.jsonl 2> $OUT/window20_h.err || { tail -20 $OUT/window20_h.err; exit 1; }
TR=$(find /tmp/winprof_h -name '*kernel_trace.csv' | head -1)
python3 tools/trace_window.py "$TR" $OUT/window20_h.err --out $OUT/window20_trace_h.json | head -8
for rep in 1 2 3; do
  for h in 0 1; do
    RX_GRAPH_HEAD=$h timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-time-to-90 \
      --ppo-updates 0 --selfplay-updates 0 > $OUT/drv_h$h$rep.jsonl 2> $OUT/drv_h$h$rep.err || { tail -30 $OUT/drv_h$h$rep.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('head$h', 'driver20', round(d['value']/1e6,1), d['ms_per_step'])" $OUT/drv_h$h$rep.jsonl
  done
done
echo R04AF_DONE
