#!/bin/bash
# Round 6 closing evidence on the committed tree: the whole -m gpu suite + smoke, the G8 host branch on this
# box, the driver's bench command (all legs, stress included), 1,000 steady-state steps, the configs[1] /
# configs[3] PPO iterations, the rocprofv3 kernel trace + stats of the driver's command split by the bench's
# region marks, and the N-rank bench path on 2 gloo ranks.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${CLOSE_DIR:-r06z}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
  > $OUT/pytest_gpu.txt 2>&1 || { tail -60 $OUT/pytest_gpu.txt; exit 1; }
tail -3 $OUT/pytest_gpu.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -3 $OUT/smoke.log
timeout -k 10 300 python -u -m pytest -q tests/test_ppo_golden.py -k reference_control_flow > $OUT/g8_host.txt 2>&1 \
  || { tail -30 $OUT/g8_host.txt; exit 1; }
grep "G8" $OUT/g8_host.txt; tail -1 $OUT/g8_host.txt
timeout -k 10 700 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver20.jsonl 2> $OUT/bench_driver20.err \
  || { tail -30 $OUT/bench_driver20.err; exit 1; }
tail -c 300 $OUT/bench_driver20.jsonl; echo
timeout -k 10 300 python -u bench.py --steps 1000 --warmup 5 --no-cpu-baseline --no-time-to-90 --ppo-updates 0 \
  --selfplay-updates 0 --stress off > $OUT/bench_steady1000.jsonl 2> $OUT/bench_steady.err || { tail -20 $OUT/bench_steady.err; exit 1; }
tail -c 200 $OUT/bench_steady1000.jsonl; echo
for m in "--mode single --envs 4096" "--mode single --envs 4096 --bf16" "--mode selfplay --envs 8192"; do
  timeout -k 10 300 python -u tools/bench_ppo.py $m --steps 128 --updates 3 --device-shuffle >> $OUT/bench_ppo.jsonl 2>> $OUT/bench_ppo.err \
    || { tail -20 $OUT/bench_ppo.err; exit 1; }
done
cat $OUT/bench_ppo.jsonl
echo R06Z_MAIN_DONE
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
