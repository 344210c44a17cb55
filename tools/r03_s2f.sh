#!/bin/bash
# Round 3, session 2, call 6: edge-classes-first ray-wave dispatch as the default
# (RX_RAY_DISPATCH 3): full GPU suite + smoke, two-car env A/B against mode 0
# (librx_disp0), the driver's bench command and the wave-fill profile.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r03s2f; mkdir -p $OUT; export TMPDIR=/tmp
LIB=$(pwd)/self-play-racing_amd/rx/lib
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -2 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $OUT/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
for rep in 1 2; do
  for lib in librx_disp0.so librx.so; do
    for cfg in "65536 2" "8192 2"; do
      RX_LIB_PATH=$LIB/$lib timeout -k 10 120 python tools/env_probe.py $cfg 300 > $OUT/probe.json 2> $OUT/probe.err || { tail -5 $OUT/probe.err; exit 1; }
      echo "$lib $cfg $(tail -c 400 $OUT/probe.json)"
    done
  done
done
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/driver20.jsonl 2> $OUT/driver20.err || { tail -20 $OUT/driver20.err; exit 1; }
python3 -c "import json;d=json.loads(open('$OUT/driver20.jsonl').read().splitlines()[-1]);print('driver20',d['value'],d['ms_per_step'],d['kernels_ms'],d['ppo_train']['value'],d['ppo_train_bf16']['value'],d['async_stream_groups']['value'])"
timeout -k 10 240 python3 bench.py --gpus 1 --steps 1000 --warmup 5 --no-cpu-baseline --no-time-to-90 \
  --ppo-updates 0 > $OUT/steady1000.jsonl 2> $OUT/steady1000.err || { tail -20 $OUT/steady1000.err; exit 1; }
python3 -c "import json;d=json.loads(open('$OUT/steady1000.jsonl').read().splitlines()[-1]);print('steady',d['value'],d['ms_per_step'])"
timeout -k 10 200 python tools/wave_profile.py 65536 4 > $OUT/wave_profile_65536.json 2> $OUT/wp.err || { tail -20 $OUT/wp.err; exit 1; }
echo S2F_DONE
