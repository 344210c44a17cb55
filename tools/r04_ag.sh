#!/bin/bash
# Round 4, call AG: k_step2's REWARD workgroups dispatched after the raycast ones (librx_rl.so,
# -DRX_REWARD_LAST=1) vs the tree (REWARD first): env GPU tests on the A/B build, bench.py A/B,
# and tools/env_probe.py at the other sizes.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r04ag; mkdir -p $OUT; export TMPDIR=/tmp
LIB=$(pwd)/self-play-racing_amd/rx/lib
RX_LIB_PATH=$LIB/librx_rl.so timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread \
  tests/test_env_gpu.py -k "culling_and_sort or resort or lanes_per" > $OUT/pytest_rl.txt 2>&1 || { tail -40 $OUT/pytest_rl.txt; exit 1; }
tail -1 $OUT/pytest_rl.txt
OUT_SUB=r04ag AB_SETS="tree||;rl|rl|" timeout -k 10 900 bash tools/ab_args.sh > $OUT/ab_reward_last.txt 2>&1 || { tail -20 $OUT/ab_reward_last.txt; exit 1; }
cat $OUT/ab_reward_last.txt
for v in tree rl; do
  p=""; [ $v != tree ] && p=$LIB/librx_$v.so
  for cfg in "4096 1" "16384 1" "8192 2" "65536 2"; do
    RX_LIB_PATH=$p timeout -k 10 120 python -u tools/env_probe.py $cfg 400 | sed "s/^/$v /" | cut -c1-120 >> $OUT/probe_rl.txt || exit 1
  done
done
cat $OUT/probe_rl.txt
echo R04AG_DONE
