#!/bin/bash
# r06 f: kernel timeline of the configs[1] rollout (4,096 envs, bf16 and fp32 policy), rocprofv3 kernel trace
set -o pipefail
O=gpurun_out/r06f
mkdir -p $O
export TMPDIR=/tmp
for p in bf16 fp32; do
  F=""; [ $p = bf16 ] && F="--bf16"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tr_$p -o run --output-format csv -- \
    python tools/bench_ppo.py --envs 4096 --steps 128 --device-shuffle --updates 1 $F > $O/bench_$p.json 2> $O/bench_$p.err || exit 1
  python tools/r06/rollout_timeline.py "$O/tr_$p/**/*kernel_trace.csv" $O/timeline_$p.json || exit 1
done
