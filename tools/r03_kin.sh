#!/bin/bash
# Round 3: k_kin1 phase stamps at 65,536 and 4,096 envs (tools/dyn_stamps.py kin).
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r03; mkdir -p $OUT; export TMPDIR=/tmp
for n in 65536 4096; do
  timeout -k 10 120 python tools/dyn_stamps.py kin $n > $OUT/kin_stamps_$n.json 2> $OUT/kin.err || { tail -5 $OUT/kin.err; exit 1; }
  cat $OUT/kin_stamps_$n.json
done
