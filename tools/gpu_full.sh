#!/bin/bash
# Full GPU check: every -m gpu test (one process), smoke, then the default bench line.
set -u
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests ${PYTEST_EXTRA:-} > $OUT/pytest_gpu.log 2>&1; rc=$?
grep -E "passed|failed|FAIL|ERROR" $OUT/pytest_gpu.log | tail -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
[ "${NO_BENCH:-0}" = 1 ] && exit 0
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-2500
