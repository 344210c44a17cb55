#!/bin/bash
# Round 4, call Q: a second priority level for the very last ray waves (RX_RAY_PRIO2 builds
# librx_c{80,85,90}.so) at 65,536 envs, and REWARD-wave priority (librx_rw1.so) on the two-car env.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r04q; mkdir -p $OUT; export TMPDIR=/tmp
LIB=$(pwd)/self-play-racing_amd/rx/lib
OUT_SUB=r04q AB_SETS="base||;c80|c80|;c85|c85|;c90|c90|;rw1|rw1|" timeout -k 10 1000 bash tools/ab_args.sh \
  > $OUT/ab_prio2.txt 2>&1 || { tail -20 $OUT/ab_prio2.txt; exit 1; }
cat $OUT/ab_prio2.txt
for rep in 1 2; do
  for v in base rw1; do
    p=""; [ $v != base ] && p=$LIB/librx_$v.so
    for cfg in "8192 2" "65536 2" "4096 1"; do
      RX_LIB_PATH=$p timeout -k 10 120 python -u tools/env_probe.py $cfg 400 | sed "s/^/$v $cfg /" | cut -c1-120 >> $OUT/probe_rw.txt || exit 1
    done
  done
done
cat $OUT/probe_rw.txt
echo R04Q_DONE
