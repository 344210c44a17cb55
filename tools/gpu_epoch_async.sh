#!/bin/bash
# Async device-shuffle epochs: the equality tests, then a same-session A/B of the configs[1] update
# (EPOCH_SYNC=1: host KL check after every epoch, the previous loop; 0: one sync per update), two passes.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_permutation_gpu.py tests/test_ppo_golden.py tests/test_ppo_fused_gpu.py > $OUT/epoch_async_pytest.log 2>&1; rc=$?
grep -E "passed|failed|Error" $OUT/epoch_async_pytest.log | tail -5; [ $rc -eq 0 ] || exit $rc
: > $OUT/epoch_async_ab.jsonl
for rep in 1 2; do for es in 1 0; do
  EPOCH_SYNC=$es timeout -k 10 200 python tools/bench_ppo.py --envs 4096 --steps 128 --device-shuffle --updates 3 > $OUT/ea.log 2>&1 || { tail -20 $OUT/ea.log; exit 1; }
  grep '^{' $OUT/ea.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); d['epoch_sync']=$es; print(json.dumps(d)); import sys as s; print('sync', $es, 'update_ms', round(d['update_s']*1e3,3), 'train_M', round(d['train_env_steps_per_s']/1e6,2), file=s.stderr)" >> $OUT/epoch_async_ab.jsonl
done; done
