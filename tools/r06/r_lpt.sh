#!/bin/bash
# r06 r: ray-class dispatch order diagnostic -- longest-first by the measured class durations (lpt), its reverse
# (rev), vs the default edge-first order; seed-1 headline
set -o pipefail
O=gpurun_out/r06r
mkdir -p $O
L=self-play-racing_amd/rx/lib
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --ppo-updates 0 --selfplay-updates 0 --no-time-to-90 --rccl-world1 off --async-probe-groups 0 --stress off"
for r in 1 2; do
  for lib in librx.so librx_lpt.so librx_rev.so; do
    RX_LIB_PATH=$L/$lib timeout -k 10 200 $B >> $O/bench_$lib.jsonl 2>> $O/bench.err || exit 1
  done
done
