#!/bin/bash
# Round 4, call AC: kernel trace of the driver's 20-step timed region lined up with the bench's
# host marks (tools/trace_window.py), graph-replayed (default) and per-step launches.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r04ac; mkdir -p $OUT; export TMPDIR=/tmp
export RX_BENCH_MARKS=1
for g in on off; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/winprof_$g -o run -- \
    python3 bench.py --gpus 1 --steps 20 --warmup 5 --graph $g --no-cpu-baseline --no-time-to-90 --ppo-updates 0 \
    --selfplay-updates 0 > $OUT/window20_$g.jsonl 2> $OUT/window20_$g.err || { tail -20 $OUT/window20_$g.err; exit 1; }
  TR=$(find /tmp/winprof_$g -name '*kernel_trace.csv' | head -1)
  echo "== graph $g"
  python3 tools/trace_window.py "$TR" $OUT/window20_$g.err --out $OUT/window20_trace_$g.json | head -40
done
echo R04AC_DONE
