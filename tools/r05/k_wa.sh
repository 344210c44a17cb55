#!/bin/bash
# write-amplification A/B -- the io rows in position order (RX_WA_POSORDER=1: every
# wave's rows one contiguous range, outputs permuted) against the product's env-order rows, bench
# interleaved + FETCH/WRITE PMC of both; then the driver command's kernel trace split by region marks
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${RUN_DIR:-r05k}; mkdir -p $OUT; export TMPDIR=/tmp
B="--steps 1000 --warmup 5 --no-cpu-baseline --no-time-to-90 --ppo-updates 0 --selfplay-updates 0 --async-probe-groups 0 --profile-steps 32 --counter-steps 0"
for r in 1 2; do
  for v in new wa_pos; do
    if [ $v = wa_pos ]; then export RX_LIB_PATH=$(pwd)/build/variants/wa_pos.so; else unset RX_LIB_PATH; fi
    timeout -k 10 300 python -u bench.py $B > $OUT/bench_$v$r.jsonl 2> $OUT/bench_$v$r.err || { tail -20 $OUT/bench_$v$r.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$OUT/bench_$v$r.jsonl').read().strip().splitlines()[-1]);print('$v',d['value'],d['ms_per_step'],d['kernels_ms'])"
  done
done
for v in new wa_pos; do
  if [ $v = wa_pos ]; then export RX_LIB_PATH=$(pwd)/build/variants/wa_pos.so; else unset RX_LIB_PATH; fi
  timeout -k 10 400 python -u tools/pmc_steady.py $OUT/pmc_$v.json --scratch /tmp/pmc_$v --passes "FETCH_SIZE;WRITE_SIZE" \
    > $OUT/pmc_$v.log 2>&1 || { tail -30 $OUT/pmc_$v.log; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/pmc_$v.json'));print('$v',{k: {c: v.get(c) for c in ('FETCH_SIZE','WRITE_SIZE')} for k, v in d.items() if 'k_step2' in k or 'k_kin1' in k})"
done
unset RX_LIB_PATH
export RX_BENCH_MARKS=1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/winprof -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-time-to-90 --ppo-updates 0 \
  --selfplay-updates 0 --async-probe-groups 0 > $OUT/window20.jsonl 2> $OUT/window20.err || { tail -20 $OUT/window20.err; exit 1; }
cd $GRAFT_REPO_ROOT
TR=$(find /tmp/winprof -name '*kernel_trace.csv' | head -1)
python3 tools/trace_window.py "$TR" $OUT/window20.err --out $OUT/window20_trace.json > /dev/null
python3 -c "import json;d=json.load(open('$OUT/window20_trace.json'));print({k: d[k] for k in ('host_region_us','t0_to_first_kernel_us','kernel_span_us','region_spans_us')});print({r: {k: v['n'] for k, v in x.items() if k.startswith('k_')} for r, x in d['regions'].items()})"
echo R05K_DONE
