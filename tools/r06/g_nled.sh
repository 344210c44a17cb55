#!/bin/bash
# r06 g: the division-free s <= 1 test as N <= D: env parity suites, then the headline bench (stress leg on)
set -o pipefail
O=gpurun_out/r06g
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_env_gpu.py tests/test_fullsize_gpu.py \
  tests/test_lane_tracks_gpu.py tests/test_rollout_gpu.py > $O/pytest_env.txt 2>&1 || exit 1
timeout -k 10 500 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --ppo-updates 0 --selfplay-updates 0 \
  --no-time-to-90 --rccl-world1 off --async-probe-groups 0 > $O/bench.json 2> $O/bench.err
