#!/bin/bash
# Round 3, session 2, first GPU call: re-verify the restored tree (whole -m gpu suite,
# smoke), the driver's bench command, a 1,000-step steady state, a rocprofv3 summary of
# the driver's command, and the self-launched 2-rank rehearsal (gloo, one GPU).
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r03s2; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $OUT/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/driver20.jsonl 2> $OUT/driver20.err || { tail -20 $OUT/driver20.err; exit 1; }
python3 -c "import json;d=json.loads(open('$OUT/driver20.jsonl').read().splitlines()[-1]);print('driver20',d['value'],d['ms_per_step'],d['ppo_train']['value'],d['ppo_train_bf16']['value'])"
timeout -k 10 240 python3 bench.py --gpus 1 --steps 1000 --warmup 5 --no-cpu-baseline --no-time-to-90 \
  --ppo-updates 0 > $OUT/steady1000.jsonl 2> $OUT/steady1000.err || { tail -20 $OUT/steady1000.err; exit 1; }
python3 -c "import json;d=json.loads(open('$OUT/steady1000.jsonl').read().splitlines()[-1]);print('steady',d['value'],d['ms_per_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r03s2prof -o run -- \
  python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-time-to-90 \
  > $OUT/prof20.jsonl 2> $OUT/prof20.err || { tail -20 $OUT/prof20.err; exit 1; }
cp $(find /tmp/r03s2prof -name '*kernel_stats.csv' | head -1) $OUT/prof20_kernel_stats.csv
python3 tools/kstats.py $OUT/prof20_kernel_stats.csv 12
timeout -k 10 400 python3 bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 5 --no-time-to-90 \
  > $OUT/gloo2.jsonl 2> $OUT/gloo2.err || { tail -20 $OUT/gloo2.err; exit 1; }
python3 -c "import json;d=json.loads(open('$OUT/gloo2.jsonl').read().splitlines()[-1]);print('gloo2',d['n_gpus'],d['value'],d['dist']['world_size'],d['ppo_train']['value'])"
echo S2A_DONE
