#!/bin/bash
# bf16 k_ppo_grad with paired passes (an even pass runs the next pass's forward beside its own):
# bitwise dump vs the previous tree's library, interleaved ppo_micro, bf16 tests
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${RUN_DIR:-r05x}; mkdir -p $OUT; export TMPDIR=/tmp
BASE=$(pwd)/self-play-racing_amd/rx/lib/librx_base_r05x.so
for mb in 32768 2048 96; do
  timeout -k 10 120 python -u tools/ppo_grad_dump.py $OUT/new_$mb.npz bf16 $mb > /dev/null 2> $OUT/dump_new.err || { tail -20 $OUT/dump_new.err; exit 1; }
  RX_LIB_PATH=$BASE timeout -k 10 120 python -u tools/ppo_grad_dump.py $OUT/base_$mb.npz bf16 $mb > /dev/null 2> $OUT/dump_base.err || { tail -20 $OUT/dump_base.err; exit 1; }
  python3 tools/ppo_grad_dump.py --compare $OUT/new_$mb.npz $OUT/base_$mb.npz | cut -c1-300
done
for r in 1 2; do
  timeout -k 10 120 python -u tools/ppo_micro.py 32768 bf16 new$r >> $OUT/micro.jsonl 2> $OUT/micro.err || { tail -20 $OUT/micro.err; exit 1; }
  RX_LIB_PATH=$BASE timeout -k 10 120 python -u tools/ppo_micro.py 32768 bf16 base$r >> $OUT/micro.jsonl 2> $OUT/micro.err || { tail -20 $OUT/micro.err; exit 1; }
done
cat $OUT/micro.jsonl
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_bf16_gpu.py > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
echo R05X_DONE
