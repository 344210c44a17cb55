#!/bin/bash
# r06 q: per-ray hit hints (RX_RAY_HINT): env parity, then interleaved A/B (seed-1 headline, 4,096 / 16,384 envs,
# two-car 8,192, stress pool)
set -o pipefail
O=gpurun_out/r06q
mkdir -p $O
L=self-play-racing_amd/rx/lib
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_env_gpu.py \
  tests/test_fullsize_gpu.py tests/test_lane_tracks_gpu.py > $O/pytest_env.txt 2>&1 || exit 1
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --ppo-updates 0 --selfplay-updates 0 --no-time-to-90 --rccl-world1 off --async-probe-groups 0 --stress off"
for r in 1 2; do
  timeout -k 10 200 $B >> $O/bench_hint.jsonl 2>> $O/bench.err || exit 1
  RX_LIB_PATH=$L/librx_nohint.so timeout -k 10 200 $B >> $O/bench_nohint.jsonl 2>> $O/bench.err || exit 1
  for cfg in "4096 1" "16384 1" "8192 2"; do
    timeout -k 10 120 python tools/env_probe.py $cfg >> $O/probe_hint.jsonl 2>> $O/probe.err || exit 1
    RX_LIB_PATH=$L/librx_nohint.so timeout -k 10 120 python tools/env_probe.py $cfg >> $O/probe_nohint.jsonl 2>> $O/probe.err || exit 1
  done
done
timeout -k 10 200 python tools/r06/stress_probe.py 65536 lane_tracks=1 >> $O/stress.jsonl 2>> $O/probe.err || exit 1
RX_LIB_PATH=$L/librx_nohint.so timeout -k 10 200 python tools/r06/stress_probe.py 65536 lane_tracks=1 >> $O/stress.jsonl 2>> $O/probe.err || exit 1
