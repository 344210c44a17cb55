#!/bin/bash
# PPO update tests, same-session A/B of the update kernels (HEAD lib vs this tree), then the default bench line.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_ppo_fused_gpu.py tests/test_optim_gpu.py tests/test_ppo_golden.py tests/test_bf16_gpu.py tests/test_ppo_gpu.py tests/test_permutation_gpu.py tests/test_dist_gpu.py > $OUT/ab2_pytest.log 2>&1; rc=$?
tail -3 $OUT/ab2_pytest.log; [ $rc -eq 0 ] || exit $rc
LIBS="head tree" bash tools/gpu_ppo_ab.sh || exit 1
for v in head tree; do python - $v $OUT <<'PY'
import csv, sys
for r in csv.DictReader(open(f"{sys.argv[2]}/ppoab_{sys.argv[1]}/run_kernel_stats.csv")):
    if any(k in r["Name"] for k in ("ppo", "adam", "perm", "adv")):
        print(sys.argv[1], r["Name"][:40], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2))
PY
done
timeout -k 10 600 python bench.py > $OUT/bench2.log 2>&1 || { tail -20 $OUT/bench2.log; exit 1; }
tail -1 $OUT/bench2.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], json.dumps(d['ppo_train']))"
