#!/bin/bash
# Round 4, call U: PMC passes over the configs[1] PPO iteration, fp32 and bf16 (tools/pmc_steady.py
# over tools/bench_ppo.py; counters only, two groups within the per-pass SQ limit): what bounds
# k_ppo_grad (MFMA busy, VALU, LDS, waits).
set -u
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r04u; mkdir -p $OUT
P1="SQ_INSTS_VALU_MFMA_MOPS_F32,SQ_VALU_MFMA_BUSY_CYCLES,SQ_BUSY_CYCLES,SQ_WAVE_CYCLES,SQ_WAIT_INST_ANY,SQ_WAIT_ANY,SQ_ACTIVE_INST_VALU,SQ_INSTS_LDS,GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU,SQ_INSTS_MFMA,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_INSTS_VALU_TRANS_F32,SQ_WAIT_INST_LDS,SQ_INSTS_SALU,SQ_INSTS_VMEM_RD,GRBM_GUI_ACTIVE"
for prec in fp32 bf16; do
  b=""; [ $prec = bf16 ] && b="--bf16"
  timeout -k 10 600 python tools/pmc_steady.py $OUT/pmc_ppo_$prec.json --last 64 --scratch /tmp/pmc_ppo_$prec \
    --cmd "tools/bench_ppo.py --envs 4096 --steps 128 --device-shuffle --updates 1 $b" --passes "$P1;$P2" \
    > $OUT/pmc_ppo_$prec.log 2>&1 || { tail -30 $OUT/pmc_ppo_$prec.log; exit 1; }
done
python3 - $OUT/pmc_ppo_fp32.json $OUT/pmc_ppo_bf16.json <<'PY'
import json, sys
for f in sys.argv[1:]:
    d = json.load(open(f))
    for k, v in d.items():
        if isinstance(v, dict) and ("ppo_grad" in k or "policy_act" in k):
            print(f.split("/")[-1], k, {c: round(x) if isinstance(x, float) else x for c, x in v.items()})
PY
echo R04U_DONE
