#!/bin/bash
# Round 4, call O: issue priority for the last-dispatched ray waves (RX_RAY_PRIO A/B builds
# librx_p*.so from tools/build_rev.py), the steady-state bench at 65,536 envs, same session.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r04o; mkdir -p $OUT; export TMPDIR=/tmp
OUT_SUB=r04o AB_SETS="${AB_SETS:-base||;p1_70|p1_70|;p3_70|p3_70|;p2_50|p2_50|;p3_85|p3_85|}" timeout -k 10 1000 bash tools/ab_args.sh \
  > $OUT/ab_prio.txt 2>&1 || { tail -20 $OUT/ab_prio.txt; exit 1; }
cat $OUT/ab_prio.txt
echo R04O_DONE
