#!/bin/bash
# k_flow A/B: occupancy (6 vs 8 waves per SIMD), poll sleep, window length (sort interval 8 / 16 / 32)
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${RUN_DIR:-r05f}; mkdir -p $OUT; export TMPDIR=/tmp
run() {  # label lib interval
  RX_LIB_PATH=$2 timeout -k 10 200 python -u tools/window_probe.py --envs 65536 --steps 400 --reps 2 --mode 2 \
    --sort-interval $3 --label $1 >> $OUT/flowab.jsonl 2>> $OUT/flowab.err || { tail -20 $OUT/flowab.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$OUT/flowab.jsonl').read().strip().splitlines()[-1]);print(d['label'],d['sort_interval'],d['window_on_Msteps'],d['window_off_Msteps'],d['kernel_us_on'],d['window_workgroups']['wg_end_us_percentiles'])"
}
L=$(pwd)/self-play-racing_amd/rx/lib/librx.so
run base8 $L 8
run base16 $L 16
run base32 $L 32
run minw8_8 $(pwd)/build/variants/minw8.so 8
run minw8_16 $(pwd)/build/variants/minw8.so 16
run sleep8_8 $(pwd)/build/variants/sleep8.so 8
echo R05F_DONE
