#!/bin/bash
# the driver's 20-step timed region: one HIP graph replay vs one rx_steps call from C++ (no graph),
# interleaved x3; then the same two forms under rocprofv3 with the bench's marks (t0 -> first kernel)
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${RUN_DIR:-r05p}; mkdir -p $OUT; export TMPDIR=/tmp
B="--gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-time-to-90 --ppo-updates 0 --selfplay-updates 0 --async-probe-groups 0 --counter-steps 0"
for r in 1 2 3; do
  for g in on off; do
    timeout -k 10 300 python -u bench.py $B --graph $g > $OUT/bench_g$g.$r.jsonl 2> $OUT/bench_g$g.$r.err || { tail -20 $OUT/bench_g$g.$r.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$OUT/bench_g$g.$r.jsonl').read().strip().splitlines()[-1]);print('graph=$g',d['value'],d['ms_per_step'],d['steady_state']['launch'][:50])"
  done
done
export RX_BENCH_MARKS=1
for g in on off; do
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/gp_$g -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py $B --graph $g --profile-steps 0 > $OUT/trace_g$g.jsonl 2> $OUT/trace_g$g.err || { tail -20 $OUT/trace_g$g.err; exit 1; }
  cd $GRAFT_REPO_ROOT
  TR=$(find /tmp/gp_$g -name '*kernel_trace.csv' | head -1)
  python3 tools/trace_window.py "$TR" $OUT/trace_g$g.err --out $OUT/window_g$g.json > /dev/null || exit 1
  python3 -c "import json;d=json.load(open('$OUT/window_g$g.json'));print('graph=$g', {k: d[k] for k in ('host_region_us','t0_to_first_kernel_us','kernel_span_us','idle_gaps_us','last_kernel_to_t1_us')})"
done
echo R05P_DONE
