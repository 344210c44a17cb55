#!/bin/bash
# Round 4, call E: the GPU-marked self-play / PPO tests, the driver's bench command (FP64 compute
# roofline from profiles/r04/pmc_steady.json), 1,000 steady-state steps, the rocprofv3 kernel trace
# of the driver's timed region, and the two-car schedule A/B at 4,096 and 8,192 envs.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r04e; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/test_selfplay_train_gpu.py \
  tests/test_ppo_gpu.py tests/test_ppo_golden.py > $OUT/pytest_selfplay.txt 2>&1 || { tail -60 $OUT/pytest_selfplay.txt; exit 1; }
tail -2 $OUT/pytest_selfplay.txt
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver20.jsonl 2> $OUT/bench_driver20.err \
  || { tail -30 $OUT/bench_driver20.err; exit 1; }
tail -c 300 $OUT/bench_driver20.jsonl; echo
timeout -k 10 300 python -u bench.py --steps 1000 --warmup 5 --no-cpu-baseline --no-time-to-90 --ppo-updates 0 \
  --selfplay-updates 0 > $OUT/bench_steady1000.jsonl 2> $OUT/bench_steady.err || { tail -20 $OUT/bench_steady.err; exit 1; }
tail -c 200 $OUT/bench_steady1000.jsonl; echo
timeout -k 10 600 python -u tools/ab_sched.py $OUT/ab_two_car_8192.jsonl --envs 8192 --agents 2 --rounds 3 --steps 300 \
  --variant rl1_lpr2:reward_lpe=1 --variant rl1_lpr1:reward_lpe=1,ray_lpr=1 --variant rl2_lpr1:reward_lpe=2,ray_lpr=1 \
  > $OUT/ab_8192.log 2>&1 || { tail -30 $OUT/ab_8192.log; exit 1; }
grep summary $OUT/ab_two_car_8192.jsonl
timeout -k 10 600 python -u tools/ab_sched.py $OUT/ab_two_car_4096.jsonl --envs 4096 --agents 2 --rounds 3 --steps 300 \
  --variant rl1_lpr4:reward_lpe=1 --variant rl2_lpr4:reward_lpe=2 --variant rl2_lpr2:reward_lpe=2,ray_lpr=2 \
  --variant rl2_lpr1:reward_lpe=2,ray_lpr=1 > $OUT/ab_4096.log 2>&1 || { tail -30 $OUT/ab_4096.log; exit 1; }
grep summary $OUT/ab_two_car_4096.jsonl
timeout -k 10 600 python -u tools/ab_sched.py $OUT/ab_two_car_16384.jsonl --envs 16384 --agents 2 --rounds 3 --steps 200 \
  --variant rl1:reward_lpe=1 --variant rl2:reward_lpe=2 > $OUT/ab_16384.log 2>&1 || { tail -30 $OUT/ab_16384.log; exit 1; }
grep summary $OUT/ab_two_car_16384.jsonl
export RX_BENCH_MARKS=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/winprof -o run -- \
  python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-time-to-90 --ppo-updates 0 --selfplay-updates 0 \
  --counter-steps 0 > $OUT/window20.jsonl 2> $OUT/window20.err || { tail -20 $OUT/window20.err; exit 1; }
TR=$(find /tmp/winprof -name '*kernel_trace.csv' | head -1)
cp $(find /tmp/winprof -name '*kernel_stats.csv' | head -1) $OUT/window20_kernel_stats.csv
python3 tools/trace_window.py "$TR" $OUT/window20.err --out $OUT/window20_trace.json > $OUT/window20_summary.txt
head -30 $OUT/window20_summary.txt
echo R04E_DONE
