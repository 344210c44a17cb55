#!/bin/bash
# r06 x: the 1-lane leaf scan's exact-test segment data loaded with its pre-filter data (RX_SEG_PRELOAD) --
# env parity, then interleaved A/B on the seed-1 headline (20-step bench, 3 rounds)
set -o pipefail
O=gpurun_out/r06x
mkdir -p $O
L=self-play-racing_amd/rx/lib
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_env_gpu.py \
  tests/test_fullsize_gpu.py > $O/pytest_env.txt 2>&1 || exit 1
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --ppo-updates 0 --selfplay-updates 0 --no-time-to-90 --rccl-world1 off --async-probe-groups 0 --stress off"
for r in 1 2 3; do
  timeout -k 10 200 $B >> $O/bench_pre.jsonl 2>> $O/bench.err || exit 1
  RX_LIB_PATH=$L/librx_nopre.so timeout -k 10 200 $B >> $O/bench_nopre.jsonl 2>> $O/bench.err || exit 1
done
