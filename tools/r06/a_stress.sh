#!/bin/bash
# r06 a: lane-varying slots -- equality tests, stress-pool oracle parity, stress bench leg
set -o pipefail
O=gpurun_out/r06a
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_lane_tracks_gpu.py \
  "tests/test_fullsize_gpu.py::test_stress_distinct_tracks_subset_bit_exact_vs_oracle" > $O/pytest_lane.txt 2>&1 && \
timeout -k 10 500 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --ppo-updates 0 --selfplay-updates 0 \
  --no-time-to-90 --rccl-world1 off --async-probe-groups 0 > $O/bench_stress.json 2> $O/bench_stress.err
