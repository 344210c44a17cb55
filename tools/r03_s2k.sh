#!/bin/bash
# Round 3, session 2, call 11: bf16 k_ppo_grad on pre-built operand fragments.
# Bitwise equality of gradients / fused updates against HEAD's rx_ppo.hip
# (librx_bfold), fp32 and bf16; micro timing A/B; bf16 + PPO GPU tests.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r03s2k; mkdir -p $OUT; export TMPDIR=/tmp
LIB=$(pwd)/self-play-racing_amd/rx/lib
for p in bf16 fp32; do
  RX_LIB_PATH=$LIB/librx_bfold.so timeout -k 10 120 python tools/ppo_grad_dump.py $OUT/old_$p.npz $p > /dev/null 2> $OUT/dump.err || { tail -5 $OUT/dump.err; exit 1; }
  timeout -k 10 120 python tools/ppo_grad_dump.py $OUT/new_$p.npz $p > /dev/null 2> $OUT/dump.err || { tail -5 $OUT/dump.err; exit 1; }
  python tools/ppo_grad_dump.py --compare $OUT/old_$p.npz $OUT/new_$p.npz || echo "DIFF $p"
done
for rep in 1 2; do
  for lib in librx_bfold.so librx.so; do
    for p in bf16 fp32; do
      RX_LIB_PATH=$LIB/$lib timeout -k 10 120 python tools/ppo_micro.py 32768 $p $lib 2> $OUT/micro.err || { tail -5 $OUT/micro.err; exit 1; }
    done
  done
done
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "bf16 or ppo or optim or golden" \
  > $OUT/pytest_ppo.log 2>&1; rc=$?
tail -2 $OUT/pytest_ppo.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $OUT/pytest_ppo.log | head -20; exit $rc; }
echo S2K_DONE
