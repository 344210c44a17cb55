#!/bin/bash
# r06 y2: lane-varying super-box entries computed up front into LDS (RX_SUPER_ENTRY) -- LV parity, then the
# stress probe: entries (6 / 5 waves per SIMD) vs none
set -o pipefail
O=gpurun_out/r06y2
mkdir -p $O
L=self-play-racing_amd/rx/lib
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_lane_tracks_gpu.py \
  tests/test_fullsize_gpu.py -k "lane or stress or distinct" > $O/pytest_lv.txt 2>&1 || exit 1
for r in 1 2; do
  for lib in librx.so librx_entw5.so librx_noent.so; do
    RX_LIB_PATH=$L/$lib timeout -k 10 200 python tools/r06/stress_probe.py 65536 lane_tracks=1 >> $O/probe.jsonl 2>> $O/probe.err || exit 1
  done
done
