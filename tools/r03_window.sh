#!/bin/bash
# Round 3 closing: rocprofv3 kernel trace of the driver's bench command's env-step part
# (--no-time-to-90 --no-cpu-baseline --ppo-updates 0: the same timed region), lined up
# with the bench's host marks (tools/trace_window.py): per-launch k_kin1 / k_step2 in the
# 20-step timed region vs the steady-state window after it, and the region's edge costs.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r03c; mkdir -p $OUT; export TMPDIR=/tmp
export RX_BENCH_MARKS=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/winprof -o run -- \
  python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-time-to-90 --ppo-updates 0 \
  > $OUT/window20.jsonl 2> $OUT/window20.err || { tail -20 $OUT/window20.err; exit 1; }
TR=$(find /tmp/winprof -name '*kernel_trace.csv' | head -1)
cp $(find /tmp/winprof -name '*kernel_stats.csv' | head -1) $OUT/window20_kernel_stats.csv
python3 tools/trace_window.py "$TR" $OUT/window20.err --out $OUT/window20_trace.json | head -30
