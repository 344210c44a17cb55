#!/bin/bash
# Round 3: where the driver's 20-step bench line loses time against the 1,000-step
# steady state (VERDICT r02 "Next" #3).  Same session: the driver's command with the
# round-2 ordering (--refill 0: garbage collection right before timing) and the new
# default, a 1,000-step steady state, then a rocprofv3 kernel trace of the driver's
# command (CPU baseline off under the profiler: its spawned workers would inherit the
# tool; it runs before the GPU is touched, so the timed region is unchanged) with host
# marks at the timed region's edges, reduced on the box by tools/trace_window.py.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r03_trace20; mkdir -p $OUT; export TMPDIR=/tmp
export RX_BENCH_MARKS=1
for rep in 1 2; do
  timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 --refill 0 --no-time-to-90 > $OUT/old20_$rep.jsonl 2> $OUT/old20_$rep.err || exit 1
  echo "old20 rep $rep done"
  timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-time-to-90 > $OUT/new20_$rep.jsonl 2> $OUT/new20_$rep.err || exit 1
  echo "new20 rep $rep done"
done
timeout -k 10 240 python3 bench.py --gpus 1 --steps 1000 --warmup 5 --no-cpu-baseline --no-time-to-90 \
  --ppo-updates 0 > $OUT/steady1000.jsonl 2> $OUT/steady1000.err || exit 1
echo "steady done"
for mode in 0 50; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r03prof$mode -o run -- \
    python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-time-to-90 --ppo-updates 0 --refill $mode \
    > $OUT/prof20_$mode.jsonl 2> $OUT/prof20_$mode.err || exit 1
  TR=$(find /tmp/r03prof$mode -name '*kernel_trace.csv' | head -1)
  python3 tools/trace_window.py "$TR" $OUT/prof20_$mode.err --out $OUT/window20_refill$mode.json > /dev/null || exit 1
  cp $(find /tmp/r03prof$mode -name '*kernel_stats.csv' | head -1) $OUT/prof20_refill${mode}_kernel_stats.csv
  echo "prof $mode done"
done
echo TRACE20_DONE
