#!/bin/bash
# r06 l: lane-varying leaf batch at 6 / 5 / 4 waves per SIMD (RX_STEP2_MINW_LV) vs no batch
set -o pipefail
O=gpurun_out/r06l
mkdir -p $O
L=self-play-racing_amd/rx/lib
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_lane_tracks_gpu.py \
  tests/test_fullsize_gpu.py -k "lane or stress or distinct" > $O/pytest_lv.txt 2>&1 || exit 1
for r in 1 2; do
  for lib in librx.so librx_lvw5.so librx_lvw4.so librx_nobatch.so; do
    RX_LIB_PATH=$L/$lib timeout -k 10 200 python tools/r06/stress_probe.py 65536 lane_tracks=1 >> $O/probe.jsonl 2>> $O/probe.err || exit 1
  done
done
