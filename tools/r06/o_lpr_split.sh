#!/bin/bash
# r06 o: leaf-box tests split over a ray's lanes (RX_LPR_BOX_SPLIT, LPR 2 / 4: few envs) -- parity, then A/B
set -o pipefail
O=gpurun_out/r06o
mkdir -p $O
L=self-play-racing_amd/rx/lib
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_env_gpu.py \
  tests/test_fullsize_gpu.py tests/test_lane_tracks_gpu.py > $O/pytest_env.txt 2>&1 || exit 1
for r in 1 2; do
  for cfg in "4096 1" "8192 1" "16384 1" "8192 2"; do
    timeout -k 10 120 python tools/env_probe.py $cfg >> $O/probe_split.jsonl 2>> $O/probe.err || exit 1
    RX_LIB_PATH=$L/librx_nosplit.so timeout -k 10 120 python tools/env_probe.py $cfg >> $O/probe_nosplit.jsonl 2>> $O/probe.err || exit 1
  done
done
