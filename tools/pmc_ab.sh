#!/bin/bash
# SQ counters of k_rays / k_dyn1 for two bench configurations (one rocprofv3 --pmc pass each).
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
C1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM"
C2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS"
i=0
for cfg in "--ray-order 1" "--ray-order 2 --sort-interval 4"; do
  for C in "$C1" "$C2"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $C -d $OUT/pmc_ab/run$i -o run --output-format csv -- python bench.py --steps 20 --warmup 20 --no-cpu-baseline --async-probe-groups 0 --ppo-updates 0 $cfg > $OUT/pmc_ab_$i.log 2>&1 || { tail -5 $OUT/pmc_ab_$i.log; echo "pass $i failed"; }
  done
done
python - $OUT/pmc_ab <<'PY'
import csv, glob, sys, collections
for run in sorted(glob.glob(sys.argv[1] + "/run*")):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(run + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            for k in ("k_rays", "k_dyn1"):
                if k in r["Kernel_Name"]:
                    acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, d in acc.items():
        print(run.split("/")[-1], k, {c: round(sum(v) / len(v)) for c, v in sorted(d.items())})
PY
