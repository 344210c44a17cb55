#!/bin/bash
# k_ppo_grad phase stamps (tools/ppo_stamps.py; the stamps build must be built here first), fp32 and bf16.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r03; mkdir -p $OUT; export TMPDIR=/tmp
for prec in fp32 bf16; do
  timeout -k 10 120 python tools/ppo_stamps.py 32768 $prec > $OUT/ppo_stamps_$prec.json 2> $OUT/ppo_stamps_$prec.err || { tail -20 $OUT/ppo_stamps_$prec.err; exit 1; }
  echo "stamps $prec done"
done
