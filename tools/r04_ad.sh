#!/bin/bash
# Round 4, call AD: graph-replayed timed region after one untimed warm replay: window trace
# (tools/trace_window.py) and the driver's command / 1,000 steps, graph on vs off, interleaved.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${AD_DIR:-r04ad}; mkdir -p $OUT; export TMPDIR=/tmp
RX_BENCH_MARKS=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/winprof_on -o run -- \
  python3 bench.py --gpus 1 --steps 20 --warmup 5 --graph on --no-cpu-baseline --no-time-to-90 --ppo-updates 0 \
  --selfplay-updates 0 > $OUT/window20_on.jsonl 2> $OUT/window20_on.err || { tail -20 $OUT/window20_on.err; exit 1; }
TR=$(find /tmp/winprof_on -name '*kernel_trace.csv' | head -1)
python3 tools/trace_window.py "$TR" $OUT/window20_on.err --out $OUT/window20_trace_on.json | head -8
for rep in 1 2 3; do
  for g in on off; do
    timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --graph $g --no-cpu-baseline --no-time-to-90 \
      --ppo-updates 0 --selfplay-updates 0 > $OUT/drv_$g$rep.jsonl 2> $OUT/drv_$g$rep.err || { tail -30 $OUT/drv_$g$rep.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('$g', 'driver20', round(d['value']/1e6,1), d['ms_per_step'])" $OUT/drv_$g$rep.jsonl
  done
done
echo R04AD_DONE
