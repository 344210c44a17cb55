#!/bin/bash
# 8 lanes per ray: the lanes-per-ray parity test, then same-session schedule A/Bs at 2,048 / 4,096 / 8,192
# envs (ray_lpr 4 vs 8) and the configs[1] rollout with either
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${RUN_DIR:-r05u}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_env_gpu.py \
  -k "lanes_per_ray" > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
for n in 4096 2048 8192; do
  timeout -k 10 300 python -u tools/ab_sched.py $OUT/ab_lpr_$n.jsonl --envs $n --steps 400 --rounds 3 \
    --variant lpr4:ray_lpr=4 --variant lpr8:ray_lpr=8 > $OUT/ab_lpr_$n.log 2>&1 || { tail -20 $OUT/ab_lpr_$n.log; exit 1; }
  grep summary $OUT/ab_lpr_$n.jsonl || tail -3 $OUT/ab_lpr_$n.jsonl
done
echo R05U_DONE
