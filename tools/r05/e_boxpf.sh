#!/bin/bash
# k_step2 chunk boxes one ahead through broadcast vector loads: bit-exact env tests,
# interleaved bench A/B against the previous tree's library, steady-state PMC of the new tree
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${RUN_DIR:-r05e}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_env_gpu.py \
  tests/test_fullsize_gpu.py tests/test_window_gpu.py tests/test_kin_sort_gpu.py tests/test_integration_gpu.py \
  > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 1; }
tail -2 $OUT/pytest.txt
B="--steps 1000 --warmup 5 --no-cpu-baseline --no-time-to-90 --ppo-updates 0 --selfplay-updates 0 --async-probe-groups 0 --profile-steps 32 --counter-steps 0"
for r in 1 2; do
  for v in new base; do
    if [ $v = base ]; then export RX_LIB_PATH=$(pwd)/self-play-racing_amd/rx/lib/librx_base_r05e.so; else unset RX_LIB_PATH; fi
    timeout -k 10 300 python -u bench.py $B > $OUT/bench_$v$r.jsonl 2> $OUT/bench_$v$r.err || { tail -20 $OUT/bench_$v$r.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$OUT/bench_$v$r.jsonl').read().strip().splitlines()[-1]);print('$v',d['value'],d['ms_per_step'],d['kernels_ms'])"
  done
done
unset RX_LIB_PATH
timeout -k 10 600 python -u tools/pmc_steady.py $OUT/pmc_steady.json --scratch /tmp/pmc_r05e > $OUT/pmc_steady.log 2>&1 \
  || { tail -30 $OUT/pmc_steady.log; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/pmc_steady.json'));k=[x for x in d if 'k_step2' in x];print({x: {c: d[x].get(c) for c in ('SQ_INSTS_VALU','SQ_INSTS_SALU','SQ_WAVE_CYCLES','dur_us','duration_us')} for x in k})"
echo R05E_DONE
