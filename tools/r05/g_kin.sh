#!/bin/bash
# k_kin1p (workgroup-parallel ray-task ranking): the env / sort / full-size GPU tests, then an
# interleaved A/B against k_kin1 (RX_KIN_PSORT=0 build) on the bench's steady state and 4,096 envs
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${RUN_DIR:-r05g}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_env_gpu.py \
  tests/test_fullsize_gpu.py tests/test_window_gpu.py > $OUT/pytest_env.txt 2>&1 || { tail -40 $OUT/pytest_env.txt; exit 1; }
tail -2 $OUT/pytest_env.txt
B="--steps 1000 --warmup 5 --no-cpu-baseline --no-time-to-90 --ppo-updates 0 --selfplay-updates 0 --async-probe-groups 0 --profile-steps 32 --counter-steps 0"
for r in 1 2; do
  for v in new base; do
    if [ $v = base ]; then export RX_LIB_PATH=$(pwd)/build/variants/kinps0.so; else unset RX_LIB_PATH; fi
    timeout -k 10 300 python -u bench.py $B > $OUT/bench_$v$r.jsonl 2> $OUT/bench_$v$r.err || { tail -20 $OUT/bench_$v$r.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$OUT/bench_$v$r.jsonl').read().strip().splitlines()[-1]);print('$v',d['value'],d['ms_per_step'],d['kernels_ms'])"
  done
done
unset RX_LIB_PATH
# the DP update graph-captured at world 1 over RCCL (graph == eager == fused), then its bench object
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_dist_gpu.py \
  tests/test_ppo_fused_gpu.py tests/test_ppo_gpu.py tests/test_optim_gpu.py > $OUT/pytest_dist.txt 2>&1 || { tail -40 $OUT/pytest_dist.txt; exit 1; }
tail -2 $OUT/pytest_dist.txt
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-time-to-90 --selfplay-updates 0 \
  --async-probe-groups 0 > $OUT/bench_rccl.jsonl 2> $OUT/bench_rccl.err || { tail -20 $OUT/bench_rccl.err; exit 1; }
python3 -c "import json;d=json.loads(open('$OUT/bench_rccl.jsonl').read().strip().splitlines()[-1]);print(json.dumps(d.get('ppo_train_rccl_world1'))[:1500]);print(d['ppo_train']['value'])"
echo R05G_DONE
