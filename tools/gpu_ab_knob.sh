#!/bin/bash
# Env-path parity tests, culling counters and a same-session bench A/B of one env knob:
#   KNOB=RX_BUNDLE bash tools/gpu_ab_knob.sh     (A = KNOB=0, B = KNOB=1)
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
K=${KNOB:-RX_BUNDLE}
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu ${TESTS:-tests/test_env_gpu.py tests/test_fullsize_gpu.py} > $OUT/t_knob.log 2>&1; rc=$?
tail -3 $OUT/t_knob.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1; do
  env $K=$v timeout -k 10 120 python tools/cull_stats.py 65536 2,16 > $OUT/cull_$v.log 2>&1 || { tail $OUT/cull_$v.log; exit 1; }
  echo "$K=$v"; tail -8 $OUT/cull_$v.log
done
AB_SETS="a|$K=0;b|$K=1" bash tools/ab_env.sh
