#!/bin/bash
# SQ counters (issue/wait breakdown) for chosen kernels; counters only, one pass per counter set.
#   CMD="python bench.py --steps 10 --warmup 20 --no-cpu-baseline" KERNELS="k_rays k_dyn1" bash tools/pmc_sq.sh
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${PMC_NAME:-pmc_sq}
mkdir -p "$OUT"
export TMPDIR=/tmp
CMD=${CMD:-python bench.py --steps 10 --warmup 20 --no-cpu-baseline}
KERNELS=${KERNELS:-k_rays k_dyn1}
SETS=${SETS:-"SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM"}
i=0
while IFS= read -r ctrs; do
  [ -z "$ctrs" ] && continue
  i=$((i + 1))
  timeout -k 10 600 rocprofv3 --pmc $ctrs -d "$OUT/run$i" -o run --output-format csv -- $CMD > "$OUT/log$i" 2>&1 || { tail -20 "$OUT/log$i"; exit 1; }
done <<< "$SETS"
python - "$OUT" $KERNELS <<'PY'
import csv, glob, sys, collections
root, names = sys.argv[1], sys.argv[2:]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(root + "/run*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        for k in names:
            if k in n:
                acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    print(k, {c: round(sum(v) / len(v)) for c, v in sorted(d.items())})
PY
