#!/bin/bash
# Round 3 GPU check: the whole -m gpu suite (one process, per-test time limit),
# smoke(), then an optional follow-up script ($1).  Stops at the first failing step.
set -u
OUT=${OUTDIR:-${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r03}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} \
  > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $OUT/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
if [ $# -ge 1 ]; then bash "$@" || exit 1; fi
echo CHECK_DONE
