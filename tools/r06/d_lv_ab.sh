#!/bin/bash
# r06 d: lane-varying A/B on the stress pool (65,536 distinct tracks): while-while traversals,
# k_step2 occupancy, pre-filter / quadrant boxes off; then PMC of the default LV k_step2 at 16,384 envs
set -o pipefail
O=gpurun_out/r06d
mkdir -p $O
export TMPDIR=/tmp
L=self-play-racing_amd/rx/lib
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_ppo_golden.py -k bf16 > $O/pytest_g8_bf16.txt 2>&1
timeout -k 10 300 python tools/r06/stress_probe.py 65536 lane_tracks=1 lane_tracks=1,seg_filter=-1 lane_tracks=1,box_quadrants=-1 >> $O/probe.jsonl 2>> $O/probe.err || exit 1
for v in ww_rays ww_argmin minw6 minw4; do
  RX_LIB_PATH=$L/ab_$v.so timeout -k 10 200 python tools/r06/stress_probe.py 65536 lane_tracks=1 >> $O/probe.jsonl 2>> $O/probe.err || exit 1
done
timeout -k 10 200 python tools/r06/stress_probe.py 65536 lane_tracks=1 >> $O/probe.jsonl 2>> $O/probe.err || exit 1
P="python tools/r06/stress_probe.py 16384 lane_tracks=1"
i=0
for ctrs in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAIT_ANY" "GRBM_GUI_ACTIVE"; do
  i=$((i + 1))
  RX_PROBE_WORKERS=1 timeout -k 10 240 rocprofv3 --pmc $ctrs -d $O/pmc$i -o run --output-format csv -- $P > $O/pmc$i.log 2>&1 || { tail -20 $O/pmc$i.log; exit 1; }
done
python - $O <<'PY'
import csv, glob, sys, collections, json
root = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(root + "/pmc[0-9]*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        for k in ("k_step2", "k_dyn1", "k_rays"):
            if k in n:
                key = k + ("_LV" if "ELb1E" in n else "")
                acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {k: {c: round(sum(v) / len(v)) for c, v in sorted(d.items())} for k, d in acc.items()}
json.dump(out, open(root + "/pmc_stress.json", "w"), indent=1)
print(json.dumps(out, indent=1))
PY
