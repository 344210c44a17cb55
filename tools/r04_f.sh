#!/bin/bash
# Round 4, call F: two-car schedule defaults under the oracle, then the rollout-groups probe
# (tools/group_probe.py) at configs[1]'s 4,096 envs.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r04f; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread \
  tests/test_fullsize_gpu.py -k two_car tests/test_env_gpu.py > $OUT/pytest_f.txt 2>&1 || { tail -60 $OUT/pytest_f.txt; exit 1; }
tail -2 $OUT/pytest_f.txt
timeout -k 10 400 python -u tools/group_probe.py $OUT/groups_4096.jsonl --envs 4096 --groups 1,2,4 > $OUT/groups_4096.log 2>&1 \
  || { tail -30 $OUT/groups_4096.log; exit 1; }
grep summary $OUT/groups_4096.jsonl
timeout -k 10 400 python -u tools/group_probe.py $OUT/groups_4096_split.jsonl --envs 4096 --groups 2,4 --sched wide_n=-1 \
  > $OUT/groups_4096_split.log 2>&1 || { tail -30 $OUT/groups_4096_split.log; exit 1; }
grep summary $OUT/groups_4096_split.jsonl
echo R04F_DONE
