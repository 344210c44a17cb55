#!/bin/bash
# Round 5, first call: the -m gpu suite on the round's first tree (dynamic task-sort LDS,
# start-draw guard), the host-aware CPU G8 test on the box's EPYC host (tolerance branch),
# and the driver's bench command as this round's baseline.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${RUN_DIR:-r05a}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
  > $OUT/pytest_gpu.txt 2>&1 || { tail -60 $OUT/pytest_gpu.txt; exit 1; }
tail -3 $OUT/pytest_gpu.txt
timeout -k 10 300 python -u -m pytest -q -rA tests/test_ppo_golden.py -k bit_exact_on_cpu -s \
  > $OUT/pytest_g8_cpu_host.txt 2>&1 || { tail -40 $OUT/pytest_g8_cpu_host.txt; exit 1; }
grep -E "branch|passed|failed" $OUT/pytest_g8_cpu_host.txt | head -6
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver20.jsonl 2> $OUT/bench_driver20.err \
  || { tail -30 $OUT/bench_driver20.err; exit 1; }
python3 -c "import json;d=json.loads(open('$OUT/bench_driver20.jsonl').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['time_to_90']['configs'][2]['value_s'])"
echo R05A_DONE
