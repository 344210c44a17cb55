#!/bin/bash
# Round-2 measurement: headline bench (steady state, CPU baseline, time-to-90), rocprofv3 kernel
# stats of the same workload, steady-state PMC passes.  Stops at the first failing step.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
STEPS=${STEPS:-bench,prof,pmc}
if [[ $STEPS == *bench* ]]; then
  timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > "$OUT/bench.log" 2>&1; rc=$?
  echo "bench rc=$rc"; tail -1 "$OUT/bench.log" | cut -c1-3000
  [ $rc -eq 0 ] || exit $rc
fi
if [[ $STEPS == *prof* ]]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    python bench.py --steps 1000 --burn-in 100 --profile-steps 0 --no-cpu-baseline --async-probe-groups 0 \
    --ppo-updates 0 --no-time-to-90 > "$OUT/prof.log" 2>&1; rc=$?
  echo "rocprof rc=$rc"; tail -1 "$OUT/prof.log" | cut -c1-400
  find "$OUT/prof" -name "*kernel_stats.csv" -exec cat {} \; | head -12
  [ $rc -eq 0 ] || exit $rc
fi
if [[ $STEPS == *pmc* ]]; then
  timeout -k 10 900 python tools/pmc_steady.py "$OUT/pmc_steady.json" > "$OUT/pmc_steady.log" 2>&1; rc=$?
  echo "pmc rc=$rc"; tail -60 "$OUT/pmc_steady.log"
  [ $rc -eq 0 ] || exit $rc
fi
echo ALL_DONE
