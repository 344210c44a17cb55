#!/bin/bash
# Round 4 closing evidence on the committed tree: the whole -m gpu suite + smoke, the driver's
# bench command, 1,000 steady-state steps, the rocprofv3 summary of the driver's command, and
# the configs[1] / configs[3] PPO iterations (tools/bench_ppo.py).
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${CLOSE_DIR:-r04z}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 1200 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
  > $OUT/pytest_gpu.txt 2>&1 || { tail -60 $OUT/pytest_gpu.txt; exit 1; }
tail -3 $OUT/pytest_gpu.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -3 $OUT/smoke.log
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver20.jsonl 2> $OUT/bench_driver20.err \
  || { tail -30 $OUT/bench_driver20.err; exit 1; }
tail -c 300 $OUT/bench_driver20.jsonl; echo
timeout -k 10 300 python -u bench.py --steps 1000 --warmup 5 --no-cpu-baseline --no-time-to-90 --ppo-updates 0 \
  --selfplay-updates 0 > $OUT/bench_steady1000.jsonl 2> $OUT/bench_steady.err || { tail -20 $OUT/bench_steady.err; exit 1; }
tail -c 200 $OUT/bench_steady1000.jsonl; echo
for m in "--mode single --envs 4096" "--mode single --envs 4096 --bf16" "--mode selfplay --envs 8192"; do
  timeout -k 10 300 python -u tools/bench_ppo.py $m --steps 128 --updates 3 --device-shuffle >> $OUT/bench_ppo.jsonl 2>> $OUT/bench_ppo.err \
    || { tail -20 $OUT/bench_ppo.err; exit 1; }
done
cat $OUT/bench_ppo.jsonl
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/drvprof -o run -- \
  python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver20_rocprof.jsonl 2> $OUT/bench_driver20_rocprof.err \
  || { tail -20 $OUT/bench_driver20_rocprof.err; exit 1; }
cp $(find /tmp/drvprof -name '*kernel_stats.csv' | head -1) $OUT/bench_driver20_kernel_stats.csv
TR=$(find /tmp/drvprof -name '*kernel_trace.csv' | head -1)
python3 tools/kstats_by_grid.py "$TR" $OUT/bench_driver20_kernel_stats_by_grid.csv > /dev/null || exit 1
head -12 $OUT/bench_driver20_kernel_stats.csv | cut -c1-160
echo R04Z_DONE
# the N-rank bench path rehearsed on this one GPU (2 self-launched gloo ranks: a path check, not a scaling number)
timeout -k 10 600 python -u bench.py --gpus 2 --steps 20 --warmup 5 --dist-backend gloo --no-cpu-baseline --no-time-to-90 \
  > $OUT/bench_2rank_gloo.jsonl 2> $OUT/bench_2rank_gloo.err || { tail -30 $OUT/bench_2rank_gloo.err; exit 1; }
tail -c 400 $OUT/bench_2rank_gloo.jsonl; echo
echo R04Z_RANKS_DONE
