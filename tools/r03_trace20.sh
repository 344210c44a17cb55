#!/bin/bash
# Round 3: where the driver's 20-step bench line loses time against the 1,000-step
# steady state (VERDICT r02 "Next" #3).  The exact driver command, plain and under a
# rocprofv3 kernel trace with host marks at the timed region's edges (the trace is
# reduced on the box by tools/trace_window.py: the raw CSV is too big to bring back),
# then a 1,000-step run in the same session.  Stops at the first failure.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r03_trace20; mkdir -p $OUT; export TMPDIR=/tmp
export RX_BENCH_MARKS=1
timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/plain20.jsonl 2> $OUT/plain20.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r03prof -o run -- \
  python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-time-to-90 > $OUT/prof20.jsonl 2> $OUT/prof20.err || exit 1
TR=$(ls /tmp/r03prof/*/run_kernel_trace.csv 2>/dev/null | head -1); [ -z "$TR" ] && TR=$(find /tmp/r03prof -name '*kernel_trace.csv' | head -1)
python3 tools/trace_window.py "$TR" $OUT/prof20.err --out $OUT/window20.json > /dev/null || exit 1
cp $(find /tmp/r03prof -name '*kernel_stats.csv' | head -1) $OUT/prof20_kernel_stats.csv
timeout -k 10 240 python3 bench.py --gpus 1 --steps 1000 --warmup 5 --no-cpu-baseline --no-time-to-90 \
  --ppo-updates 0 > $OUT/steady1000.jsonl 2> $OUT/steady1000.err || exit 1
echo TRACE20_DONE
