#!/bin/bash
# r06 m: timing probe -- bf16 gradient with the weight fragments copied from a global image (garbage values)
set -o pipefail
O=gpurun_out/r06m
mkdir -p $O
L=self-play-racing_amd/rx/lib
for r in 1 2 3; do
  timeout -k 10 120 python tools/ppo_micro.py 32768 bf16 main >> $O/micro.jsonl 2>> $O/micro.err || exit 1
  RX_LIB_PATH=$L/librx_imgprobe.so timeout -k 10 120 python tools/ppo_micro.py 32768 bf16 imgprobe >> $O/micro.jsonl 2>> $O/micro.err || exit 1
done
