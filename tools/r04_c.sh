#!/bin/bash
# Round 4, call C: self-play tests after the snapshot / sequenced-rollout changes, the driver's
# bench command (FP64 compute roofline from profiles/r04/pmc_steady.json), 1,000 steady-state
# steps, and the rocprofv3 kernel trace of the driver's timed region lined up with its host marks.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r04c; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_selfplay_train_gpu.py \
  tests/test_ppo_gpu.py tests/test_ppo_golden.py > $OUT/pytest_selfplay.txt 2>&1 || { tail -60 $OUT/pytest_selfplay.txt; exit 1; }
tail -2 $OUT/pytest_selfplay.txt
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver20.jsonl 2> $OUT/bench_driver20.err \
  || { tail -30 $OUT/bench_driver20.err; exit 1; }
tail -c 300 $OUT/bench_driver20.jsonl; echo
timeout -k 10 300 python -u bench.py --steps 1000 --warmup 5 --no-cpu-baseline --no-time-to-90 --ppo-updates 0 \
  --selfplay-updates 0 > $OUT/bench_steady1000.jsonl 2> $OUT/bench_steady.err || { tail -20 $OUT/bench_steady.err; exit 1; }
tail -c 200 $OUT/bench_steady1000.jsonl; echo
export RX_BENCH_MARKS=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/winprof -o run -- \
  python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-time-to-90 --ppo-updates 0 --selfplay-updates 0 \
  --counter-steps 0 > $OUT/window20.jsonl 2> $OUT/window20.err || { tail -20 $OUT/window20.err; exit 1; }
TR=$(find /tmp/winprof -name '*kernel_trace.csv' | head -1)
cp $(find /tmp/winprof -name '*kernel_stats.csv' | head -1) $OUT/window20_kernel_stats.csv
python3 tools/trace_window.py "$TR" $OUT/window20.err --out $OUT/window20_trace.json | head -30
echo R04C_DONE
