#!/bin/bash
# PPO-kernel GPU check: parity tests of the fused policy / update / rollout paths, then PPO throughput
# under rocprofv3 kernel stats.
set -u
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_ppo_fused_gpu.py tests/test_ppo_golden.py tests/test_rollout_gpu.py tests/test_optim_gpu.py \
  tests/test_ppo_gpu.py tests/test_dist_gpu.py tests/test_bf16_gpu.py ${PYTEST_EXTRA:-} > $OUT/pytest_ppo.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" $OUT/pytest_ppo.log | tail -60
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/ppo_prof -o run --output-format csv -- python tools/bench_ppo.py --envs 4096 --steps 128 --device-shuffle --updates 2 > $OUT/ppo_prof.log 2>&1 || { tail -20 $OUT/ppo_prof.log; exit 1; }
grep '^{' $OUT/ppo_prof.log | tail -1
python - <<'PY'
import csv,glob,os
f=glob.glob(os.environ.get("GRAFT_REPO_ROOT",".")+"/gpurun_out/ppo_prof/**/*kernel_stats.csv",recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:12]:
    print(r["Name"][:80], r["Calls"], r["AverageNs"], r["Percentage"])
PY
timeout -k 10 300 python tools/bench_ppo.py --envs 4096 --steps 128 --device-shuffle --updates 3
timeout -k 10 300 python tools/bench_ppo.py --envs 16 --steps 2048 --updates 3
timeout -k 10 300 python tools/bench_ppo.py --envs 4096 --steps 128 --device-shuffle --updates 3 --bf16
