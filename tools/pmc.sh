#!/bin/bash
# HBM traffic of the env kernels from PMC counters (MI355X_MICROARCH.md §HBM):
# FETCH_SIZE and WRITE_SIZE in SEPARATE rocprofv3 passes (TCC slot limits), plus
# SQ_INSTS_VALU (wave-level VALU instructions: the raycast's issue roofline),
# counters only (no sys/runtime trace).  Summarised by tools/pmc_summary.py.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/pmc
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS=${PMC_BENCH_ARGS:---steps 20 --warmup 2 --no-cpu-baseline --async-probe-groups 0 --ppo-updates 0}
for C in FETCH_SIZE WRITE_SIZE SQ_INSTS_VALU; do
  timeout -k 10 600 rocprofv3 --pmc $C -d "$OUT/$C" -o run --output-format csv -- python bench.py $ARGS \
    > "$OUT/$C.log" 2>&1 || { echo "rocprofv3 $C failed rc=$?"; tail -5 "$OUT/$C.log"; exit 1; }
done
python tools/pmc_summary.py "$OUT" > "$OUT/summary.json" && cat "$OUT/summary.json"
