#!/bin/bash
# Round 6 closing, part 2: the rocprofv3 kernel trace + stats of the driver's bench command (the stress leg
# off: its spawned 65,536-track table build stalls under the profiler; its k_step2<1,1,1,true> launches are a
# separate kernel from the headline's k_step2<1,1,1,false>), split by the bench's region marks, and the N-rank
# bench path on 2 gloo ranks.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${CLOSE_DIR:-r06z2}; mkdir -p $OUT; export TMPDIR=/tmp
export RX_BENCH_MARKS=1
cd /tmp && timeout -k 10 700 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/drvprof -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 20 --warmup 5 --stress off > $OUT/bench_driver20_rocprof.jsonl 2> $OUT/bench_driver20_rocprof.err \
  || { tail -20 $OUT/bench_driver20_rocprof.err; exit 1; }
cd $GRAFT_REPO_ROOT; unset RX_BENCH_MARKS
cp $(find /tmp/drvprof -name '*kernel_stats.csv' | head -1) $OUT/bench_driver20_kernel_stats.csv
TR=$(find /tmp/drvprof -name '*kernel_trace.csv' | head -1)
python3 tools/kstats_by_grid.py "$TR" $OUT/bench_driver20_kernel_stats_by_grid.csv > /dev/null || exit 1
python3 tools/trace_window.py "$TR" $OUT/bench_driver20_rocprof.err --out $OUT/window20_trace.json > /dev/null || exit 1
python3 -c "import json;d=json.load(open('$OUT/window20_trace.json'));print({k: d[k] for k in ('host_region_us','t0_to_first_kernel_us','kernel_span_us')});print({r: {k: (v['n'], v['mean_us']) for k, v in x.items() if k.startswith(('k_step2','k_dyn1','k_sort'))} for r, x in d['regions'].items()})"
echo R06Z_PROF_DONE
timeout -k 10 600 python -u bench.py --gpus 2 --steps 20 --warmup 5 --dist-backend gloo --no-cpu-baseline --no-time-to-90 \
  --stress off > $OUT/bench_2rank_gloo.jsonl 2> $OUT/bench_2rank_gloo.err || { tail -30 $OUT/bench_2rank_gloo.err; exit 1; }
tail -c 400 $OUT/bench_2rank_gloo.jsonl; echo
echo R06Z_RANKS_DONE
