#!/bin/bash
# REWARD lanes per env at few envs: schedule A/B (ab_sched) at 4,096 and 8,192 envs
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${RUN_DIR:-r05h}; mkdir -p $OUT; export TMPDIR=/tmp
for n in 4096 8192 2560; do
  timeout -k 10 300 python -u tools/ab_sched.py $OUT/ab_rlpe_$n.jsonl --envs $n --steps 400 --rounds 3 \
    --variant rlpe2:reward_lpe=2 --variant rlpe4:reward_lpe=4 --variant rlpe1:reward_lpe=1 > $OUT/ab_rlpe_$n.log 2>&1 || { tail -20 $OUT/ab_rlpe_$n.log; exit 1; }
  grep summary $OUT/ab_rlpe_$n.jsonl
done
echo R05H_DONE
