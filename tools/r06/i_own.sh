#!/bin/bash
# r06 i: own-super leaves outward from the car's leaf (RX_OWN_OUTWARD): parity, then interleaved A/B
# RESULT (measured): outward order 871/887 M vs default 914/916 M env-steps/s, k_step2 59.1 vs 56.7 us at equal box tests; reverted.
# (seed-1 headline bench without the stress leg; stress probe for the lane-varying path)
set -o pipefail
O=gpurun_out/r06i
mkdir -p $O
L=self-play-racing_amd/rx/lib
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_env_gpu.py \
  tests/test_fullsize_gpu.py tests/test_lane_tracks_gpu.py > $O/pytest_env.txt 2>&1 || exit 1
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --ppo-updates 0 --selfplay-updates 0 --no-time-to-90 --rccl-world1 off --async-probe-groups 0 --stress off"
for r in 1 2; do
  timeout -k 10 200 $B >> $O/bench_own.jsonl 2>> $O/bench.err || exit 1
  RX_LIB_PATH=$L/ab_noown.so timeout -k 10 200 $B >> $O/bench_noown.jsonl 2>> $O/bench.err || exit 1
done
timeout -k 10 200 python tools/r06/stress_probe.py 65536 lane_tracks=1 >> $O/probe.jsonl 2>> $O/probe.err || exit 1
RX_LIB_PATH=$L/ab_noown.so timeout -k 10 200 python tools/r06/stress_probe.py 65536 lane_tracks=1 >> $O/probe.jsonl 2>> $O/probe.err || exit 1
