#!/bin/bash
# Same-session A/B of bench.py configurations, two passes interleaved:
#   AB_SETS="label|lib|args;label2|lib2|args2" bash tools/ab_args.sh
# lib: empty = the tree's librx.so, NAME = rx/lib/librx_NAME.so (tools/build_rev.py).
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${OUT_SUB:-}; mkdir -p $OUT; export TMPDIR=/tmp
LIBDIR=$(pwd)/self-play-racing_amd/rx/lib
IFS=';' read -ra SETS <<< "$AB_SETS"
for rep in 1 2; do
for set in "${SETS[@]}"; do
  IFS='|' read -r label lib args <<< "$set"
  libpath=""; [ -n "$lib" ] && libpath=$LIBDIR/librx_$lib.so
  RX_LIB_PATH=$libpath timeout -k 10 200 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --async-probe-groups 0 --ppo-updates 0 --no-time-to-90 $args > $OUT/ab_$label.log 2>&1 || { tail -20 $OUT/ab_$label.log; exit 1; }
  tail -1 $OUT/ab_$label.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$label', round(d['value']/1e6,1), d['kernels_ms'])"
done
done
