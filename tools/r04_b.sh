#!/bin/bash
# Round 4, call B: the whole -m gpu suite + smoke, then the evidence the bench line reads
# or cites: steady-state PMC counters incl. the FP64/FP32 instruction mix
# (tools/pmc_steady.py -> profiles/r04/pmc_steady.json), a rocprofv3 kernel trace of the
# driver's bench command split by launch size, rocprofv3 of the configs[1] (fp32, bf16) and
# configs[3] PPO iterations, and a k_step2 wave profile.  Stops at the first failing step.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r04b; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
  > $OUT/pytest_gpu.txt 2>&1 || { tail -60 $OUT/pytest_gpu.txt; exit 1; }
tail -2 $OUT/pytest_gpu.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python -u tools/pmc_steady.py $OUT/pmc_steady.json --scratch /tmp/pmc_r04 > $OUT/pmc_steady.log 2>&1 \
  || { tail -30 $OUT/pmc_steady.log; exit 1; }
echo PMC_DONE
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/benchprof -o run -- \
  python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver20_rocprof.jsonl 2> $OUT/bench_rocprof.err \
  || { tail -20 $OUT/bench_rocprof.err; exit 1; }
cp $(find /tmp/benchprof -name '*kernel_stats.csv' | head -1) $OUT/bench_driver20_kernel_stats.csv
python3 tools/kstats_by_grid.py $(find /tmp/benchprof -name '*kernel_trace.csv' | head -1) $OUT/bench_driver20_kernel_stats_by_grid.csv --top 25
grep -c Aborted $OUT/bench_rocprof.err || true
for mode in fp32 bf16 selfplay; do
  args="--mode single --envs 4096 --steps 128 --updates 3 --device-shuffle"
  [ $mode = bf16 ] && args="$args --bf16"
  [ $mode = selfplay ] && args="--mode selfplay --envs 8192 --steps 128 --updates 3 --device-shuffle"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ppoprof_$mode -o run -- \
    python3 tools/bench_ppo.py $args > $OUT/ppo_${mode}_rocprof.jsonl 2> $OUT/ppo_$mode.err || { tail -20 $OUT/ppo_$mode.err; exit 1; }
  cp $(find /tmp/ppoprof_$mode -name '*kernel_stats.csv' | head -1) $OUT/ppo_${mode}_kernel_stats.csv
  python3 tools/kstats_by_grid.py $(find /tmp/ppoprof_$mode -name '*kernel_trace.csv' | head -1) $OUT/ppo_${mode}_kernel_stats_by_grid.csv --top 12
done
timeout -k 10 200 python -u tools/wave_profile.py 65536 4 > $OUT/wave_profile_65536.json 2> $OUT/wave_profile.err || { tail -20 $OUT/wave_profile.err; exit 1; }
echo R04B_DONE
