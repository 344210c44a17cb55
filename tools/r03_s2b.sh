#!/bin/bash
# Round 3, session 2, second GPU call: (1) rocprofv3 kernel trace of exactly the
# driver's bench command with host marks at the timed region's edges
# (RX_BENCH_MARKS=1; tools/trace_window.py lines the region up with the trace);
# (2) k_ppo_grad phase stamps, fp32 and bf16 (tools/ppo_stamps.py, profiling build);
# (3) the fused minibatch step timed alone (tools/ppo_micro.py).
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r03s2; mkdir -p $OUT; export TMPDIR=/tmp
export RX_BENCH_MARKS=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r03s2tr -o run -- \
  python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-time-to-90 --ppo-updates 0 \
  > $OUT/trace20.jsonl 2> $OUT/trace20.err || { tail -20 $OUT/trace20.err; exit 1; }
TR=$(find /tmp/r03s2tr -name '*kernel_trace.csv' | head -1)
python3 tools/trace_window.py "$TR" $OUT/trace20.err --out $OUT/window20.json | head -14
grep RX_FIRST $OUT/trace20.err
unset RX_BENCH_MARKS
for prec in fp32 bf16; do
  timeout -k 10 120 python tools/ppo_stamps.py 32768 $prec > $OUT/ppo_stamps_$prec.json 2> $OUT/ppo_stamps_$prec.err || { tail -20 $OUT/ppo_stamps_$prec.err; exit 1; }
  head -c 1500 $OUT/ppo_stamps_$prec.json; echo
  timeout -k 10 120 python tools/ppo_micro.py 32768 $prec > $OUT/ppo_micro_$prec.jsonl 2> $OUT/ppo_micro.err || { tail -5 $OUT/ppo_micro.err; exit 1; }
  cat $OUT/ppo_micro_$prec.jsonl
done
echo S2B_DONE
