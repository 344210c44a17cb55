#!/bin/bash
# r06 c: (1) lane-varying tests (while-while traversal) + stress-pool parity, schedule probe;
# (2) swizzled bf16 gradient images: bf16 / G8 / fused-update tests, bf16 PPO timing, LDS PMC;
# (3) PMC of the lane-varying k_step2 on the stress pool
set -o pipefail
O=gpurun_out/r06c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_lane_tracks_gpu.py \
  "tests/test_fullsize_gpu.py::test_stress_distinct_tracks_subset_bit_exact_vs_oracle" > $O/pytest_lane.txt 2>&1 || exit 1
timeout -k 10 400 python tools/r06/stress_probe.py 65536 > $O/probe.jsonl 2> $O/probe.err || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_bf16_gpu.py \
  tests/test_ppo_golden.py tests/test_ppo_fused_gpu.py > $O/pytest_bf16.txt 2>&1 || exit 1
timeout -k 10 300 python tools/bench_ppo.py --envs 4096 --steps 128 --device-shuffle --updates 3 --bf16 > $O/bench_ppo_bf16.json 2> $O/bench_ppo_bf16.err || exit 1
timeout -k 10 600 python tools/pmc_steady.py $O/pmc_ppo_bf16.json --last 64 --scratch $O/pmc_ppo \
  --cmd "tools/bench_ppo.py --envs 4096 --steps 128 --device-shuffle --updates 1 --bf16" \
  --passes "SQ_INSTS_VALU,SQ_INSTS_MFMA,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_WAIT_INST_LDS,SQ_INSTS_LDS,SQ_WAVE_CYCLES,SQ_WAIT_INST_ANY,GRBM_GUI_ACTIVE" \
  > $O/pmc_ppo.log 2>&1 || { tail -30 $O/pmc_ppo.log; exit 1; }
P="python tools/r06/stress_probe.py 65536 lane_tracks=1"
i=0
for ctrs in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAIT_ANY" "GRBM_GUI_ACTIVE"; do
  i=$((i + 1))
  timeout -k 10 300 rocprofv3 --pmc $ctrs -d $O/pmc$i -o run --output-format csv -- $P > $O/pmc$i.log 2>&1 || { tail -20 $O/pmc$i.log; exit 1; }
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
