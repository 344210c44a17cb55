#!/bin/bash
# k_window A/B: workgroup packing (LDS pad caps the workgroups per CU) and the parallel task ranking
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${RUN_DIR:-r05d}; mkdir -p $OUT; export TMPDIR=/tmp
for v in pad0 pad24k pad0nops; do
  RX_LIB_PATH=$(pwd)/build/variants/$v.so timeout -k 10 200 python -u tools/window_probe.py --envs 65536 --steps 400 \
    --reps 2 --label $v >> $OUT/winab.jsonl 2>> $OUT/winab.err || { tail -20 $OUT/winab.err; exit 1; }
  tail -1 $OUT/winab.jsonl | cut -c1-2000
done
