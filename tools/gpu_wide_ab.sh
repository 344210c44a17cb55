#!/bin/bash
# Small / mid N single-agent step: segment pre-filter and wide-raycast threshold A/B (tools/env_probe.py)
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
if [ "${RUN_TESTS:-1}" = 1 ]; then
  timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_env_gpu.py tests/test_rollout_gpu.py > $OUT/t6.log 2>&1; rc=$?
  tail -3 $OUT/t6.log; [ $rc -eq 0 ] || exit $rc
fi
for rep in 1 2; do for n in ${NS:-16 256 2048 4096 8192}; do
  for cfg in "a|RX_SEG_FILTER=0" "b|RX_SEG_FILTER=1" "c|RX_SEG_FILTER=1 RX_WIDE_RAYS_N=1000000"; do
    IFS='|' read -r label envs <<< "$cfg"
    echo -n "$label $n "; env $envs timeout -k 10 120 python tools/env_probe.py $n 1 400 | tail -1 || exit 1
  done
done; done
