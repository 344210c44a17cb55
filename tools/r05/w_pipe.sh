#!/bin/bash
# probe: the raycast of step t on a second stream beside step t + 1's kinematics + REWARD (racy timing-only
# build, -DRX_PIPE_PROBE) against the product library, timed region as one graph and as a direct call
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${RUN_DIR:-r05w}; mkdir -p $OUT; export TMPDIR=/tmp
B="--steps 1000 --warmup 5 --no-cpu-baseline --no-time-to-90 --ppo-updates 0 --selfplay-updates 0 --async-probe-groups 0 --profile-steps 0 --counter-steps 0 --rccl-world1 off"
for r in 1 2; do
  for v in pipe base; do
    for g in on off; do
      if [ $v = pipe ]; then export RX_LIB_PATH=$(pwd)/self-play-racing_amd/rx/lib/librx_pipe.so; else unset RX_LIB_PATH; fi
      timeout -k 10 300 python -u bench.py $B --graph $g > $OUT/bench_${v}_g${g}_$r.jsonl 2> $OUT/bench_${v}_g${g}_$r.err || { tail -20 $OUT/bench_${v}_g${g}_$r.err; exit 1; }
      python3 -c "import json;d=json.loads(open('$OUT/bench_${v}_g${g}_$r.jsonl').read().strip().splitlines()[-1]);print('$v graph=$g',d['value'],d['ms_per_step'])"
    done
  done
done
echo R05W_DONE
