#!/bin/bash
# Same-session A/B of two-car env throughput over librx variants:
#   LIBS="base m4 m6" bash tools/ab_probe2.sh   (base = the tree's librx.so)
set -eu
LIBDIR=$(pwd)/self-play-racing_amd/rx/lib
for rep in 1 2; do for n in ${NS:-8192 65536}; do for lib in $LIBS; do
  p=""; [ "$lib" != base ] && p=$LIBDIR/librx_$lib.so
  echo -n "$lib "; RX_LIB_PATH=$p timeout -k 10 120 python tools/env_probe.py $n ${AGENTS:-2} 400
done; done; done
