#!/bin/bash
# HIP_FORCE_DEV_KERNARG=1 (kernel arguments in device memory) vs the default, driver command and 1,000 steps
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${RUN_DIR:-r05d}; mkdir -p $OUT; export TMPDIR=/tmp
B="--warmup 5 --no-cpu-baseline --no-time-to-90 --ppo-updates 0 --selfplay-updates 0 --async-probe-groups 0 --profile-steps 0 --counter-steps 0 --rccl-world1 off"
for r in 1 2; do
  for v in dev def; do
    for n in 20 1000; do
      if [ $v = dev ]; then export HIP_FORCE_DEV_KERNARG=1; else unset HIP_FORCE_DEV_KERNARG; fi
      timeout -k 10 300 python -u bench.py $B --steps $n > $OUT/bench_${v}_${n}_$r.jsonl 2> $OUT/bench_${v}_${n}_$r.err || { tail -20 $OUT/bench_${v}_${n}_$r.err; exit 1; }
      python3 -c "import json;d=json.loads(open('$OUT/bench_${v}_${n}_$r.jsonl').read().strip().splitlines()[-1]);print('$v steps=$n',d['value'],d['ms_per_step'])"
    done
  done
done
echo R05D_DONE
