#!/bin/bash
# Round-2 closing check: PPO update tests, a same-session A/B of the update kernels (HEAD lib vs this tree),
# every -m gpu test, smoke, a 2-rank gloo rehearsal of the N-GPU bench (both ranks on this box's one GPU: the
# data-parallel PPO leg's shard update + bucket all-reduce) and a rocprofv3 summary of the configs[1] PPO
# iteration.  Stops at the first failure.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_ppo_fused_gpu.py tests/test_optim_gpu.py tests/test_ppo_golden.py tests/test_bf16_gpu.py tests/test_ppo_gpu.py tests/test_dist_gpu.py > $OUT/ab3_pytest.log 2>&1; rc=$?
tail -1 $OUT/ab3_pytest.log; [ $rc -eq 0 ] || exit $rc
LIBS="head tree" bash tools/gpu_ppo_ab.sh || exit 1
for v in head tree; do python - $v $OUT <<'PY'
import csv, sys
for r in csv.DictReader(open(f"{sys.argv[2]}/ppoab_{sys.argv[1]}/run_kernel_stats.csv")):
    if any(k in r["Name"] for k in ("ppo", "adam", "adv")):
        print(sys.argv[1], r["Name"][:40], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2))
PY
done
[ "${AB_ONLY:-0}" = 1 ] && exit 0
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -1 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --dist-backend gloo --steps 200 --warmup 10 --async-probe-groups 0 --no-cpu-baseline --no-time-to-90 > $OUT/bench_2rank_gloo.log 2>&1 || { tail -20 $OUT/bench_2rank_gloo.log; exit 1; }
tail -1 $OUT/bench_2rank_gloo.log | cut -c1-600
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/ppo_prof -o run --output-format csv -- python tools/bench_ppo.py --envs 4096 --steps 128 --device-shuffle --updates 2 > $OUT/ppo_prof.log 2>&1 || { tail -20 $OUT/ppo_prof.log; exit 1; }
tail -1 $OUT/ppo_prof.log | cut -c1-400
echo FINAL_OK
