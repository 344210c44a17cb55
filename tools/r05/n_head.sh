#!/bin/bash
# the driver's 20-step timed region: one HIP graph vs a 1- or 2-step head graph + the rest
# (the head starts the GPU while the host still submits the rest), interleaved x3
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${RUN_DIR:-r05n}; mkdir -p $OUT; export TMPDIR=/tmp
B="--gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-time-to-90 --ppo-updates 0 --selfplay-updates 0 --async-probe-groups 0 --counter-steps 0"
for r in 1 2 3; do
  for h in 0 1 2; do
    timeout -k 10 300 python -u bench.py $B --graph-head $h > $OUT/bench_h$h.$r.jsonl 2> $OUT/bench_h$h.$r.err || { tail -20 $OUT/bench_h$h.$r.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$OUT/bench_h$h.$r.jsonl').read().strip().splitlines()[-1]);print('head=$h',d['value'],d['ms_per_step'],d['steady_state']['launch'][:60])"
  done
done
echo R05N_DONE
