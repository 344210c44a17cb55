#!/bin/bash
# SQ counters (issue/wait breakdown) for the env kernels; one pass, counters only.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/pmc_sq
mkdir -p "$OUT"
export TMPDIR=/tmp
CTRS=${CTRS:-SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM}
timeout -k 10 600 rocprofv3 --pmc $CTRS -d "$OUT/run" -o run --output-format csv -- python bench.py --steps 10 --warmup 20 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/log" 2>&1 || { tail -20 "$OUT/log"; exit 1; }
python - "$OUT" <<'PY'
import csv, glob, sys, collections
root = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(root + "/run/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        k = "k_rays" if "k_rays" in n else ("k_dyn1" if "k_dyn1" in n else None)
        if k:
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    print(k, {c: round(sum(v) / len(v)) for c, v in sorted(d.items())})
PY
