#!/bin/bash
# Round 5: the window parity tests (vs the per-step launches and the oracle), the
# integration binding, then the window on/off throughput probe and the bench.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${RUN_DIR:-r05b}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 150 --timeout-method thread -m gpu tests/test_window_gpu.py \
  tests/test_integration_gpu.py > $OUT/pytest_window.txt 2>&1 || { tail -60 $OUT/pytest_window.txt; exit 1; }
grep -E "PASS|FAIL|passed|failed" $OUT/pytest_window.txt | tail -12
timeout -k 10 300 python -u tools/window_probe.py --envs 65536 --steps 1000 --reps 3 > $OUT/probe_65536.jsonl 2> $OUT/probe.err \
  || { tail -30 $OUT/probe.err; exit 1; }
cat $OUT/probe_65536.jsonl
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-time-to-90 --ppo-updates 0 \
  --selfplay-updates 0 > $OUT/bench_driver20.jsonl 2> $OUT/bench_driver20.err || { tail -30 $OUT/bench_driver20.err; exit 1; }
python3 -c "import json;d=json.loads(open('$OUT/bench_driver20.jsonl').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['window'],d['roofline'])"
echo R05B_DONE
