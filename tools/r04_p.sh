#!/bin/bash
# Round 4, call P: ray-wave issue priority (librx_p1_70.so) at the other env counts, same session.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r04p; mkdir -p $OUT; export TMPDIR=/tmp
LIB=$(pwd)/self-play-racing_amd/rx/lib
for rep in 1 2; do
  for v in base p1_70; do
    p=""; [ $v != base ] && p=$LIB/librx_$v.so
    for cfg in "4096 1" "16384 1" "8192 2" "65536 2"; do
      RX_LIB_PATH=$p timeout -k 10 120 python -u tools/env_probe.py $cfg 400 | sed "s/^/$v $cfg /" | cut -c1-150 >> $OUT/probe_ab.txt || exit 1
    done
  done
done
cat $OUT/probe_ab.txt
echo R04P_DONE
