#!/bin/bash
# r06 e: bf16 G8 tests; lane-varying k_step2 without the pre-filter at 5 / 6 / 7 waves per SIMD,
# with and without quadrant box tables, on the stress pool (65,536 distinct tracks)
set -o pipefail
O=gpurun_out/r06e
mkdir -p $O
L=self-play-racing_amd/rx/lib
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_ppo_golden.py -k bf16 > $O/pytest_g8_bf16.txt 2>&1
timeout -k 10 300 python tools/r06/stress_probe.py 65536 lane_tracks=1 lane_tracks=1,box_quadrants=-1 >> $O/probe.jsonl 2>> $O/probe.err || exit 1
for v in nf6 nf7; do
  RX_LIB_PATH=$L/ab_$v.so timeout -k 10 200 python tools/r06/stress_probe.py 65536 lane_tracks=1 lane_tracks=1,box_quadrants=-1 >> $O/probe.jsonl 2>> $O/probe.err || exit 1
done
timeout -k 10 200 python tools/r06/stress_probe.py 65536 lane_tracks=1 >> $O/probe.jsonl 2>> $O/probe.err || exit 1
