#!/bin/bash
# r06 j: leaf boxes of a kept super tested as one batch (RX_LEAF_BATCH): parity, then interleaved A/B
# (seed-1 headline bench without the stress leg; stress probe for the lane-varying path)
set -o pipefail
O=gpurun_out/r06j
mkdir -p $O
L=self-play-racing_amd/rx/lib
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_env_gpu.py \
  tests/test_fullsize_gpu.py tests/test_lane_tracks_gpu.py > $O/pytest_env.txt 2>&1 || exit 1
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --ppo-updates 0 --selfplay-updates 0 --no-time-to-90 --rccl-world1 off --async-probe-groups 0 --stress off"
for r in 1 2; do
  timeout -k 10 200 $B >> $O/bench_batch.jsonl 2>> $O/bench.err || exit 1
  RX_LIB_PATH=$L/librx_nobatch.so timeout -k 10 200 $B >> $O/bench_nobatch.jsonl 2>> $O/bench.err || exit 1
done
timeout -k 10 200 python tools/r06/stress_probe.py 65536 lane_tracks=1 >> $O/probe.jsonl 2>> $O/probe.err || exit 1
RX_LIB_PATH=$L/librx_nobatch.so timeout -k 10 200 python tools/r06/stress_probe.py 65536 lane_tracks=1 >> $O/probe.jsonl 2>> $O/probe.err || exit 1
for r in 1 2; do
  timeout -k 10 120 python tools/env_probe.py 4096 1 >> $O/probe4096_batch.jsonl 2>> $O/probe.err || exit 1
  RX_LIB_PATH=$L/librx_nobatch.so timeout -k 10 120 python tools/env_probe.py 4096 1 >> $O/probe4096_nobatch.jsonl 2>> $O/probe.err || exit 1
done
