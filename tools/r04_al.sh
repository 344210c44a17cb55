#!/bin/bash
# Round 4, call AL: k_kin1's ray-task sectors computed before the LDS atomics (angles loaded up front,
# no integer division for the agent index), the atomics back to back: env / full-size / start-draw
# GPU tests, the sort's phase stamps (librx_kstamps.so), bench.py A/B against HEAD (librx_head.so)
# and env_probe at the other sizes.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r04al; mkdir -p $OUT; export TMPDIR=/tmp
LIB=$(pwd)/self-play-racing_amd/rx/lib
timeout -k 10 700 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_env_gpu.py \
  tests/test_fullsize_gpu.py tests/test_start_draws_gpu.py > $OUT/pytest_al.txt 2>&1 || { tail -40 $OUT/pytest_al.txt; exit 1; }
tail -1 $OUT/pytest_al.txt
timeout -k 10 180 python -u tools/kin_sort_stamps.py 65536 > $OUT/kin_sort_stamps.json || exit 1
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print([r.get('ranks_scan_copy_median') for r in d['reps']])" $OUT/kin_sort_stamps.json
OUT_SUB=r04al AB_SETS="head|head|;tree||" timeout -k 10 900 bash tools/ab_args.sh > $OUT/ab_task_ranks.txt 2>&1 || { tail -20 $OUT/ab_task_ranks.txt; exit 1; }
cat $OUT/ab_task_ranks.txt
for rep in 1 2; do
for v in head tree; do
  p=""; [ $v != tree ] && p=$LIB/librx_$v.so
  for cfg in "4096 1" "16384 1" "8192 2"; do
    RX_LIB_PATH=$p timeout -k 10 120 python -u tools/env_probe.py $cfg 400 | sed "s/^/$v /" | cut -c1-110 >> $OUT/probe_al.txt || exit 1
  done
done
done
cat $OUT/probe_al.txt
echo R04AK_DONE
