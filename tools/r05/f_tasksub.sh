#!/bin/bash
# k_kin1's ray-task ranking with 4 counters per sector: bit-exact env / sort tests, interleaved bench A/B
# (1,000 steps at 65,536 envs; 400 steps at 4,096) against the previous tree's library
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${RUN_DIR:-r05f}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_env_gpu.py \
  tests/test_fullsize_gpu.py tests/test_kin_sort_gpu.py tests/test_integration_gpu.py > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
B="--steps 1000 --warmup 5 --no-cpu-baseline --no-time-to-90 --ppo-updates 0 --selfplay-updates 0 --async-probe-groups 0 --profile-steps 32 --counter-steps 0 --rccl-world1 off"
for r in 1 2; do
  for v in new base; do
    if [ $v = base ]; then export RX_LIB_PATH=$(pwd)/self-play-racing_amd/rx/lib/librx_base_r05f.so; else unset RX_LIB_PATH; fi
    timeout -k 10 300 python -u bench.py $B > $OUT/bench_$v$r.jsonl 2> $OUT/bench_$v$r.err || { tail -20 $OUT/bench_$v$r.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$OUT/bench_$v$r.jsonl').read().strip().splitlines()[-1]);print('$v',d['value'],d['ms_per_step'],d['kernels_ms'])"
    timeout -k 10 200 python -u bench.py $B --envs-per-gpu 4096 > $OUT/bench4k_$v$r.jsonl 2> $OUT/bench4k_$v$r.err || { tail -20 $OUT/bench4k_$v$r.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$OUT/bench4k_$v$r.jsonl').read().strip().splitlines()[-1]);print('$v 4096',d['value'],d['ms_per_step'],d['kernels_ms'])"
  done
done
unset RX_LIB_PATH
echo R05F_DONE
