#!/bin/bash
# Round 4, call G: the full GPU suite on the tree (uniform operands in SGPRs: k_ppo_grad and
# k_dyn2<0> without scratch), then same-session A/Bs against HEAD's library (librx_head.so,
# tools/build_rev.py): the PPO minibatch step (tools/ppo_micro.py) and the two-car env step.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r04g; mkdir -p $OUT; export TMPDIR=/tmp
LIB=$(pwd)/self-play-racing_amd/rx/lib
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests > $OUT/pytest_gpu.txt 2>&1 \
  || { tail -60 $OUT/pytest_gpu.txt; exit 1; }
tail -3 $OUT/pytest_gpu.txt
for rep in 1 2; do
  for prec in fp32 bf16; do
    RX_LIB_PATH=$LIB/librx_head.so timeout -k 10 120 python -u tools/ppo_micro.py 32768 $prec head >> $OUT/ppo_micro_ab.jsonl 2>> $OUT/ppo_micro.err || { tail -20 $OUT/ppo_micro.err; exit 1; }
    timeout -k 10 120 python -u tools/ppo_micro.py 32768 $prec tree >> $OUT/ppo_micro_ab.jsonl 2>> $OUT/ppo_micro.err || { tail -20 $OUT/ppo_micro.err; exit 1; }
  done
done
cat $OUT/ppo_micro_ab.jsonl
for rep in 1 2; do
  for n in 8192 65536; do
    RX_LIB_PATH=$LIB/librx_head.so timeout -k 10 120 python -u tools/env_probe.py $n 2 400 | sed "s/^/head $n /" >> $OUT/env2_ab.txt || exit 1
    timeout -k 10 120 python -u tools/env_probe.py $n 2 400 | sed "s/^/tree $n /" >> $OUT/env2_ab.txt || exit 1
  done
done
cut -c1-160 $OUT/env2_ab.txt
echo R04G_DONE
