#!/bin/bash
# Round 3, session 2, call 8: lane-parallel box prefetch in the raycast traversal:
# env/fullsize/integration GPU tests (bit-exactness), same-session A/B against
# HEAD's kernels (librx_pf0), ray-wave phase stamps.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r03s2h; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_env_gpu.py tests/test_fullsize_gpu.py tests/test_integration_gpu.py tests/test_rollout_gpu.py -m gpu -v --timeout 300 --timeout-method thread \
  > $OUT/pytest_env.log 2>&1; rc=$?
tail -2 $OUT/pytest_env.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $OUT/pytest_env.log | head -20; exit $rc; }
AB_SETS="pf0|pf0|;pf||;pf0_4k|pf0|--envs-per-gpu 4096;pf_4k||--envs-per-gpu 4096" OUT_SUB=r03s2h bash tools/ab_args.sh || exit 1
timeout -k 10 200 python tools/ray_stamps.py 65536 > $OUT/ray_stamps_65536.json 2> $OUT/rs.err || { tail -20 $OUT/rs.err; exit 1; }
python3 -c "
import json;d=json.load(open('$OUT/ray_stamps_65536.json'))
r=d['runs'][-1]; print('span',r['span_us'],'all',r['all']); print('tail',r['tail_last_25pct'])"
echo S2H_DONE
