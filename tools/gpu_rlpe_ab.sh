#!/bin/bash
# REWARD lanes per env (RX_REWARD_LPE 1 / 2 / 4): exactness tests, then bench kernel split at mid N and the headline.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_env_gpu.py -k "lanes_per" > $OUT/t_rlpe.log 2>&1; rc=$?
tail -3 $OUT/t_rlpe.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for n in 4096 8192 16384 32768 65536; do
  for v in 1 2 4; do
    RX_REWARD_LPE=$v timeout -k 10 120 python bench.py --envs-per-gpu $n --steps 1000 --warmup 100 --no-cpu-baseline --async-probe-groups 0 --ppo-updates 0 --no-time-to-90 > $OUT/rlpe.log 2>&1 || { tail -20 $OUT/rlpe.log; exit 1; }
    tail -1 $OUT/rlpe.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('rlpe=$v', $n, round(d['value']/1e6,1), d['kernels_ms'])"
  done
done
done
for v in 1 2 4; do
  RX_REWARD_LPE=$v timeout -k 10 200 python tools/bench_ppo.py --envs 4096 --steps 128 --device-shuffle --updates 3 > $OUT/rlpe_ppo.log 2>&1 || { tail -20 $OUT/rlpe_ppo.log; exit 1; }
  echo "rlpe=$v $(tail -1 $OUT/rlpe_ppo.log | cut -c1-420)"
done
