#!/bin/bash
# One GPU-box round: gpu tests, smoke, bench, rocprofv3 kernel stats.
# Stops at the first step that crashes, aborts or times out (not at plain test failures).
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
STEPS=${STEPS:-tests,smoke,bench,prof}
if [[ $STEPS == *tests* ]]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q -rs ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -5 "$OUT/pytest_gpu.log"
  ok $rc || exit $rc
fi
if [[ $STEPS == *smoke* ]]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; rc=$?
  echo "smoke rc=$rc"; tail -3 "$OUT/smoke.log"
  ok $rc || exit $rc
fi
if [[ $STEPS == *bench* ]]; then
  timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > "$OUT/bench.log" 2>&1; rc=$?
  echo "bench rc=$rc"; tail -2 "$OUT/bench.log"
  [ $rc -eq 0 ] || exit $rc
fi
if [[ $STEPS == *prof* ]]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    python bench.py --steps 400 --warmup 100 --no-cpu-baseline --async-probe-groups 0 --ppo-updates 0 > "$OUT/prof.log" 2>&1; rc=$?
  echo "rocprof rc=$rc"; tail -2 "$OUT/prof.log"
  find "$OUT/prof" -name "*kernel_stats.csv" -exec cat {} \; | head -20
  [ $rc -eq 0 ] || exit $rc
fi
echo ALL_DONE
