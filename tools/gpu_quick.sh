#!/bin/bash
# Targeted GPU check: the given test files (one pytest process), then the default bench line.
set -u
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu ${TESTS} > $OUT/pytest_quick.log 2>&1; rc=$?
grep -E "passed|failed|FAIL|ERROR" $OUT/pytest_quick.log | tail -20
[ $rc -eq 0 ] || exit $rc
[ "${NO_BENCH:-0}" = 1 ] && exit 0
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-1500
