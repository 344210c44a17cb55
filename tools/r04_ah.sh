#!/bin/bash
# Round 4, call AH: k_kin1 phase stamps at 65,536 and 4,096 envs on the final kernels
# (profiling build librx_kstamps.so, tools/dyn_stamps.py kin).
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r04ah; mkdir -p $OUT; export TMPDIR=/tmp
for n in 65536 4096; do
  timeout -k 10 180 python -u tools/dyn_stamps.py kin $n > $OUT/kin_stamps_$n.json 2> $OUT/kin_stamps_$n.err || { tail -20 $OUT/kin_stamps_$n.err; exit 1; }
  echo "== $n"; cat $OUT/kin_stamps_$n.json
done
echo R04AH_DONE
