#!/bin/bash
# the fused minibatch tail (k_ppo_reduce<true>: reduce + last-block clip/Adam) and k_kin1p's
# k_kin1-identical task order (rx_config.kin_sort): parity tests, ppo_micro, bench A/B kin_sort on/off
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${RUN_DIR:-r05h}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_kin_sort_gpu.py \
  tests/test_ppo_fused_gpu.py tests/test_dist_gpu.py tests/test_optim_gpu.py tests/test_ppo_gpu.py tests/test_bf16_gpu.py \
  tests/test_env_gpu.py tests/test_window_gpu.py > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 1; }
tail -2 $OUT/pytest.txt
for p in fp32 bf16; do
  timeout -k 10 120 python -u tools/ppo_micro.py 32768 $p fused_tail > $OUT/micro_$p.jsonl 2> $OUT/micro_$p.err || { tail -20 $OUT/micro_$p.err; exit 1; }
  cat $OUT/micro_$p.jsonl
done
B="--steps 1000 --warmup 5 --no-cpu-baseline --no-time-to-90 --ppo-updates 0 --selfplay-updates 0 --async-probe-groups 0 --profile-steps 32 --counter-steps 0"
for r in 1 2; do
  for k in 1 -1; do
    timeout -k 10 300 python -u bench.py $B --sched kin_sort=$k > $OUT/bench_k$k.$r.jsonl 2> $OUT/bench_k$k.$r.err || { tail -20 $OUT/bench_k$k.$r.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$OUT/bench_k$k.$r.jsonl').read().strip().splitlines()[-1]);print('kin_sort=$k',d['value'],d['ms_per_step'],d['kernels_ms'])"
  done
done
echo R05H_DONE
